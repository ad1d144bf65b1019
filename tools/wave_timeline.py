"""Wave timeline of the enumerated pass (diagnostic builds: variant 2 = variant 0 with stamps;
VARIANT=3 with PERT_LIB naming a -DPERT_ENUM3_STAMPS build of the three-wave pass): per workgroup the
s_memrealtime stamps (100 MHz) at entry, first-bin start and exit, plus the XCC / HW ids.
Prints the launch span, entry / exit spreads and how many waves are resident over time.
usage: python tools/wave_timeline.py CELLS [SUBDIVIDE]"""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench
from scdna_replication_tools_amd.engine import EtaCodebook, PertShard, _ptr
from scdna_replication_tools_amd.init import init_params

cells = int(sys.argv[1]) if len(sys.argv) > 1 else 1250
sub = int(sys.argv[2]) if len(sys.argv) > 2 else 1
dev = torch.device("cuda", 0)
data = bench.synth(cells, sub, 0, dev, num_reads=1e6 * sub)
reads = data["reads"].cpu().numpy(); states = data["cn"].cpu().numpy()
eta = EtaCodebook.from_states(states, 1e6, 13)
bm = np.zeros((1, 5)); bm[0, 3] = 0.5
init = init_params(2, reads, np.zeros(cells, int), 1, 13, 4, ploidy=eta.argmax_states().mean(0),
                   t_init=np.clip(data["tau"].cpu().numpy(), 0.05, 0.95), beta_means=bm, seed=0)
sh = PertShard(2, reads, data["gc"], np.zeros(cells, int), 1, 13, 4, init, eta=eta, lamb=0.75, beta_means=bm,
               device=dev, variant=int(os.environ.get("VARIANT", "2")), bins_per_tile=int(os.environ.get("LT", "0")))
L = reads.shape[0]
n_ct, n_bt = -(-cells // 64), -(-L // sh.bins_per_tile)
n_wg = n_ct * n_bt
order = int(os.environ.get("PERT_ENUM3_ORDER", "2"))
n_slots = -(-n_wg // 8) * 8 if order >= 2 else n_wg        # the 1-D grid is rounded up to 8
dbg = torch.zeros(n_slots * 4, dtype=torch.int64, device=dev)
sh._state.g_pi = _ptr(dbg)
for t in range(1, 8):
    sh._launch_step(t)
torch.cuda.synchronize()
d = dbg.cpu().numpy().reshape(n_slots, 4)
# tile of each stamp row (row = workgroup index), padding rows (no tile) dropped
i = np.arange(n_slots)
if order >= 2:
    per = -(-n_wg // 8)
    w = (i % 8) * per + i // 8
    row_wt, row_bt = (w // n_bt, w % n_bt) if order == 2 else (w % n_ct, w // n_ct)
else:
    row_wt, row_bt = i % n_ct, i // n_ct
keep = d[:, 2] > 0
d, row_wt, row_bt = d[keep], row_wt[keep], row_bt[keep]
n_wg = int(keep.sum())
t0 = d[:, 0].min()
ent, first, ex = (d[:, 0] - t0) / 100.0, (d[:, 1] - t0) / 100.0, (d[:, 2] - t0) / 100.0   # microseconds
span = ex.max()
dur = ex - ent
print("cells {} bins {} LT {} workgroups {}: span {:.1f} us".format(cells, L, sh.bins_per_tile, n_wg, span))
q = lambda a: " ".join("{:.1f}".format(v) for v in np.percentile(a, [0, 10, 50, 90, 100]))
print("entry     pct 0/10/50/90/100: ", q(ent))
print("first bin pct                :", q(first - ent))
print("exit      pct                :", q(ex))
print("wave dur  pct                :", q(dur))
grid = np.linspace(0, span, 41)
res = [int(((ent <= g) & (ex > g)).sum()) for g in grid]
print("resident waves over time (41 samples):", res)
xcc = (d[:, 3] >> 32).astype(int)
for x in range(8):
    m = xcc == x
    if m.any():
        print("xcc {} waves {} exit p50 {:.1f} p100 {:.1f} mean dur {:.1f}".format(x, m.sum(), np.median(ex[m]), ex[m].max(), dur[m].mean()))
first_round = ent < 20.0
if (~first_round).any():
    print("wave dur first round (entry < 20 us) pct:", q(dur[first_round]))
    print("wave dur later rounds pct            :", q(dur[~first_round]))
    mid = (ent > 0.3 * span) & (ex < 0.7 * span)
    if mid.any():
        print("wave dur mid-kernel pct              :", q(dur[mid]))

# where the slow waves are: by bin tile, by cell tile, by SIMD occupancy of their CU
by, wt = row_bt, row_wt
hw = (d[:, 3] & 0xffffffff).astype(np.int64)
simd = (hw >> 4) & 3
cu = (hw >> 8) & 15
sh = (hw >> 12) & 1
se = (hw >> 13) & 7
cu_key = xcc * 1000 + se * 100 + sh * 20 + cu
_, cu_idx, cu_cnt = np.unique(cu_key, return_inverse=True, return_counts=True)
waves_on_cu = cu_cnt[cu_idx]
simd_key = cu_key * 4 + simd
_, s_idx, s_cnt = np.unique(simd_key, return_inverse=True, return_counts=True)
waves_on_simd = s_cnt[s_idx]
print("CUs used {} (waves per CU: {})".format(len(cu_cnt), np.bincount(cu_cnt)))
for k in sorted(set(waves_on_simd.tolist())):
    m = waves_on_simd == k
    print("waves sharing the SIMD {}: {} waves, dur p50 {:.1f} mean {:.1f}".format(k, m.sum(), np.median(dur[m]), dur[m].mean()))
for k in sorted(set(waves_on_cu.tolist())):
    m = waves_on_cu == k
    print("waves on the CU {}: {} waves, dur p50 {:.1f} mean {:.1f}".format(k, m.sum(), np.median(dur[m]), dur[m].mean()))
nbt = by.max() + 1
for q in range(5):
    m = (by >= q * nbt / 5) & (by < (q + 1) * nbt / 5)
    print("bin tiles quintile {}: dur mean {:.1f}".format(q, dur[m].mean()))
for q in range(5):
    m = (wt >= q * n_ct / 5) & (wt < (q + 1) * n_ct / 5)
    print("cell tiles quintile {}: dur mean {:.1f}".format(q, dur[m].mean()))

# variance of the wave durations within a CU / SIMD against between CUs / XCDs (one-round launches:
# does a wave's speed follow its CU, or is it the wave's own?)
def _share(key):
    _, idx = np.unique(key, return_inverse=True)
    means = np.bincount(idx, dur) / np.bincount(idx)
    return float(np.var(means[idx]) / np.var(dur))
print("share of duration variance between XCDs {:.2f}, between CUs {:.2f}, between SIMDs {:.2f}".format(
    _share(xcc), _share(cu_key), _share(simd_key)))
if os.environ.get("DUMP"):
    np.savez(os.environ["DUMP"], d=d, wt=wt, bt=by)

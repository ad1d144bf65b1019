"""Probe: eager launch sequence vs the same sequence replayed from a HIP graph (torch.cuda.CUDAGraph)
on a small shard -- measures the per-step overhead a graph would remove.  Not a correctness path
(the captured hparams are frozen at one step)."""
import os, sys, time
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench
from scdna_replication_tools_amd.engine import EtaCodebook, PertShard
from scdna_replication_tools_amd.init import init_params

cells = int(sys.argv[1]) if len(sys.argv) > 1 else 1250
dev = torch.device("cuda", 0)
data = bench.synth(cells, 1, 0, dev)
reads = data["reads"].cpu().numpy(); states = data["cn"].cpu().numpy()
eta = EtaCodebook.from_states(states, 1e6, 13)
bm = np.zeros((1, 5)); bm[0, 3] = 0.5
init = init_params(2, reads, np.zeros(cells, int), 1, 13, 4, ploidy=eta.argmax_states().mean(0),
                   t_init=np.clip(data["tau"].cpu().numpy(), 0.05, 0.95), beta_means=bm, seed=0)
sh = PertShard(2, reads, data["gc"], np.zeros(cells, int), 1, 13, 4, init, eta=eta, lamb=0.75, beta_means=bm, device=dev)
for t in range(1, 6):
    sh._launch_step(t)
torch.cuda.synchronize()
K = 50
t0 = time.perf_counter()
for t in range(6, 6 + K):
    sh._launch_step(t)
torch.cuda.synchronize()
eager = (time.perf_counter() - t0) / K * 1e3
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    sh._launch_step(100)
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    sh._launch_step(101)
torch.cuda.synchronize()
for _ in range(3):
    g.replay()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(K):
    g.replay()
torch.cuda.synchronize()
graph = (time.perf_counter() - t0) / K * 1e3
print("cells {} eager {:.4f} ms/step graph {:.4f} ms/step".format(cells, eager, graph), flush=True)

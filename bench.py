"""PERT step-2 SVI throughput on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c4] [--scaling strong|weak]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

A step is one full ``svi_s.step`` of reference pert_model.py:801 on the step-2
(enumerated) model: the fused enumerated ELBO + analytic gradient + Adam pass over
all (bin, cell) pairs of the shard, the reductions, the RCCL all-reduce of the
shared-gradient block (N > 1), Adam on the remaining parameters, the loss record and
stopping rule of the SVI loop on the device, and the loss copied back to the host (the
float the reference returns each step; copied in chunks of 8 steps, no per-step sync).  Inputs are resident
in HBM before timing starts.  Metric: enumerated ELBO+grad cell.bins/s over the
whole job = L * N_cells * K / (max over ranks of the timed wall time).

Workload (configs[3] of BASELINE.json): synthetic
pert_simulator-style data, 10,000 S-phase cells x 5,451 500 kb bins of
notebooks/mcfrt.csv, 3 clones, P = 13, K = 4, g1_clones CN prior (weight 1e6).
Strong scaling by default: the 10k cells are split over the ranks.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (n_cells, subdivide, description)
    "c4": (10000, 1, "synthetic 10k cells x 5451 x 500kb bins (BASELINE configs[3])"),
    "c3": (2000, 1, "synthetic 2k cells x 5451 x 500kb bins (BASELINE configs[2])"),
    "c1": (400, 1, "synthetic 400 cells x 5451 bins"),
    "c5": (2000, 25, "synthetic 2k cells x 136275 x 20kb bins (BASELINE configs[4])"),
}
P, K = 13, 4
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: 8.0 TB/s spec


def bytes_per_cellbin(P: int) -> int:
    """Algorithmic HBM bytes of the fused step-2 pass per (bin, cell): reads fp32 (4) +
    eta code uint16 (2) + pi logits, Adam m, v read (12 P) and written (12 P)."""
    return 4 + 2 + 24 * P


def synth(n_total: int, subdivide: int, seed: int, device, num_reads: float = 1e6):
    """Seeded synthetic S-phase data on the GPU following pert_simulator.py:201-249."""
    from scdna_replication_tools_amd.simulator import clone_profiles, convert_rt_units, load_bins
    df = load_bins(subdivide=subdivide)
    gc = df["gc"].to_numpy(np.float64)
    rt = df["mcf7rt"].to_numpy(np.float64)
    L = gc.shape[0]
    prof = clone_profiles(L, 3)
    clone = np.arange(n_total) % 3
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    cn = torch.as_tensor(prof, device=device)[:, torch.as_tensor(clone, device=device)]
    rho = torch.as_tensor(convert_rt_units(rt), device=device)
    tau = torch.rand(n_total, generator=g, device=device, dtype=torch.float64)
    phi = 1.0 / (1.0 + torch.exp(-10.0 * (tau[None, :] - rho[:, None])))
    rep = (torch.rand(phi.shape, generator=g, device=device, dtype=torch.float64) < phi).double()
    omega = torch.exp(0.5 * torch.as_tensor(gc, device=device))[:, None]
    lam = 0.75
    u = num_reads / (1.5 * L * float(cn.mean()))
    delta = (u * cn * (1 + rep) * omega * (1 - lam) / lam).clamp(min=1.0)
    rate = torch._standard_gamma(delta) * (lam / (1 - lam))
    raw = torch.poisson(rate, generator=g)
    reads = torch.floor(raw / raw.sum(0, keepdim=True) * num_reads)
    return dict(gc=gc, reads=reads.float(), cn=cn.to(torch.int64), tau=tau.float(), clone_prof=prof, clone=clone)


def composite_problem(n_total: int, seed: int = 0, n_g: int = 600, call_noise: float = 0.02):
    """configs[3] with the reference's DEFAULT prior, g1_composite (pert_model.py:40, :299-361):
    simulated S and G1/2 tables (numpy simulator, 3 clones, 1e6 reads per cell) whose G1/2
    HMMcopy-style state calls disagree with the clone profile at ``call_noise`` of the bins
    (+-1), through the product's own prep (pivots, consensus profiles, per-cell Pearson
    matches to the clone's G1/2 cells, J = 5): eta is the product's composite code book --
    many distinct rows, so the pass reads each row from the table in global memory.
    Returns (reads (L, N) fp32, gc, eta, t_init, describe)."""
    from scdna_replication_tools_amd import prep
    from scdna_replication_tools_amd.pert_model import pert_infer_scRT
    from scdna_replication_tools_amd.simulator import simulate, to_long_form
    sim = simulate(n_s=n_total, n_g=n_g, n_clones=3, num_reads=1e6, seed=seed)
    rng = np.random.default_rng(seed + 1)
    flip = rng.random(sim.cn_g.shape) < call_noise
    step = np.where(rng.random(sim.cn_g.shape) < 0.5, -1, 1)
    sim.cn_g[:] = np.where(flip, np.clip(sim.cn_g + step, 0, P - 1), sim.cn_g)
    df_s, df_g = to_long_form(sim, n_libs=1)
    m = pert_infer_scRT(df_s, df_g, cn_prior_method="g1_composite", device="cpu", log_steps=False)
    inp = m._prepare()
    profiles = prep.consensus_clone_profiles(m.cn_g1, m.cn_state_col, keys=inp.keys_g)
    eta = m._build_etas(inp, profiles)
    t_init = np.full(inp.reads_s.shape[1], 0.5, np.float32)
    return inp.reads_s.astype(np.float32), inp.gc, eta, t_init


def cpu_share():
    """CPUs this process may use: its sched_getaffinity set, capped by a cgroup CPU quota
    (cpu.max) when one is set; plus the lscpu model name."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(float(q) / float(period)))
    except (OSError, ValueError):
        quota = None
    model = None
    try:
        import subprocess
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=20).stdout
        for line in out.splitlines():
            if line.strip().startswith("Model name:"):
                model = line.split(":", 1)[1].strip()
                break
    except (OSError, subprocess.SubprocessError):
        model = None
    if model is None:
        try:
            for line in open("/proc/cpuinfo"):
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
        except OSError:
            pass
    return {"affinity_cores": aff, "cgroup_quota_cores": quota, "cores": min(aff, quota) if quota else aff,
            "cpu_model": model}


def cpu_baseline(data, n_cells: int, steps: int):
    """The oracle (torch-CPU restatement of the tensor algebra Pyro runs: materialised
    (2, P, L, N) enumeration, autograd, torch.optim.Adam) on a bounded cell sample, on every
    CPU the process may use (cpu_share)."""
    from oracle import pert_oracle as po
    share = cpu_share()
    threads = share["cores"]
    torch.set_num_threads(threads)
    reads = data["reads"][:, :n_cells].cpu().to(torch.float32)
    L = reads.shape[0]
    states = data["cn"][:, :n_cells].cpu()
    etas = torch.ones(L, n_cells, P)
    etas.scatter_(2, states.unsqueeze(-1), 1e6)
    bm = torch.zeros(1, K + 1)
    bm[0, K - 1] = 0.5
    prob = po.OracleProblem("step2", reads, torch.as_tensor(data["gc"], dtype=torch.float32),
                            torch.zeros(n_cells, dtype=torch.long), 1, P, K, etas=etas,
                            lamb=torch.tensor([0.75]), beta_means=bm,
                            t_init=data["tau"][:n_cells].cpu().clamp(0.05, 0.95))
    z0 = po.init_params(prob, seed=0)
    po.fit(prob, z0, max_iter=1, min_iter=100, cell_chunk=64)          # warm-up
    t0 = time.perf_counter()
    po.fit(prob, z0, max_iter=steps, min_iter=100, cell_chunk=64)
    dt = time.perf_counter() - t0
    return {"value": L * n_cells * steps / dt, "unit": "cell*bins/s", "cores": threads, "kind": "port",
            "sample": "{} cells x {} bins x {} SVI steps (oracle fp32, cell-chunked autograd)".format(
                n_cells, L, steps),
            "seconds": dt, "cpu_model": share["cpu_model"], "affinity_cores": share["affinity_cores"],
            "cgroup_quota_cores": share["cgroup_quota_cores"]}


def cpu_extrapolation(sim, iters, n_sample):
    """The oracle (torch-CPU restatement of the tensor algebra Pyro runs) timed per SVI step
    on an n_sample-cell slice at full L, scaled linearly in cells and by the GPU run's
    iteration counts (C3/C4 CPU full fits are extrapolated)."""
    import torch
    from oracle import pert_oracle as po
    threads = cpu_share()["cores"]
    torch.set_num_threads(threads)
    L = sim.n_bins
    P, K = 13, 4
    n = min(n_sample, sim.reads_s.shape[1])
    gc = torch.tensor(sim.gc, dtype=torch.float32)
    # step 2 (and 3: the same model on G1 cells)
    states = torch.tensor(sim.cn_s[:, :n], dtype=torch.long)
    etas = torch.ones(L, n, P)
    etas.scatter_(2, states.unsqueeze(-1), 1e6)
    bm = torch.zeros(1, K + 1)
    bm[0, K - 1] = 0.5
    p2 = po.OracleProblem("step2", torch.tensor(sim.reads_s[:, :n], dtype=torch.float32), gc,
                          torch.zeros(n, dtype=torch.long), 1, P, K, etas=etas, lamb=torch.tensor([0.75]),
                          beta_means=bm, t_init=torch.full((n,), 0.5))
    z2 = po.init_params(p2, seed=0)
    po.fit(p2, z2, max_iter=1, min_iter=100, cell_chunk=64)
    t0 = time.perf_counter()
    po.fit(p2, z2, max_iter=2, min_iter=100, cell_chunk=64)
    t2 = (time.perf_counter() - t0) / 2 / n                        # s per step per cell
    # step 1: G1 cells doubled, cn / rep observed
    g = torch.tensor(sim.reads_g[:, :n], dtype=torch.float32)
    cg = torch.tensor(sim.cn_g[:, :n], dtype=torch.float32)
    p1 = po.OracleProblem("step1", torch.cat([g, g], 1), gc, torch.zeros(2 * n, dtype=torch.long), 1, P, K,
                          cn_obs=torch.cat([cg, cg], 1),
                          rep_obs=torch.cat([torch.zeros_like(cg), torch.ones_like(cg)], 1))
    z1 = po.init_params(p1, seed=0)
    po.fit(p1, z1, max_iter=1, min_iter=100, cell_chunk=128)
    t0 = time.perf_counter()
    po.fit(p1, z1, max_iter=2, min_iter=100, cell_chunk=128)
    t1 = (time.perf_counter() - t0) / 2 / (2 * n)
    N_s, N_g = sim.reads_s.shape[1], sim.reads_g.shape[1]
    return {"kind": "port (oracle fp32, extrapolated: per-step time on a {}-cell slice x cells x the GPU run's "
                    "iteration counts)".format(n),
            "cores": threads,
            "step1_s": t1 * 2 * N_g * iters.get("step1", 0),
            "step2_s": t2 * N_s * iters.get("step2", 0),
            "step3_s": t2 * N_g * iters.get("step3", 0),
            "per_step_s": {"step1": t1 * 2 * N_g, "step2": t2 * N_s, "step3": t2 * N_g}}


def profile_numbers(prof_dir: str, kernel: str):
    """The dominant kernel's average duration (rocprofv3 kernel trace) and HBM bytes per
    launch (PMC passes) from a tools/profile.sh run of this same command line
    (tools/pmc_summary.py's summary.json)."""
    try:
        summ = json.load(open(os.path.join(prof_dir, "summary.json")))
    except (OSError, ValueError):
        return None
    ent = summ.get("kernels", {}).get(kernel)
    if not ent or "avg_ns" not in ent:
        return None
    return {"avg_ns": ent["avg_ns"], "calls": ent.get("calls"), "hbm_bytes_per_launch": ent.get("hbm_bytes_per_launch"),
            "pmc": ent.get("pmc", {})}


def fullfit_c1():
    """configs[0] stand-in (400 S + 400 G1/2 cells x 271 bins, diploid; tests/_configs.py) under
    inference_tutorial.ipynb cell 9's call: the product's full three-step fit on the GPU
    (scRT(...).infer(level='pyro'), host prep included) and, as the measured CPU baseline, the
    same chained fit on the oracle (tests/_chain.py: the torch-CPU tensor algebra Pyro runs,
    on every CPU of the process's share) from the same prep -- both timed end to end, not
    extrapolated.  One JSON line."""
    import contextlib
    import io
    from tests._chain import oracle_chain
    from tests._configs import c1_tables, tutorial_scrt
    s, g, truth = c1_tables()
    torch.zeros(1, device="cuda")
    # the notebook's import cell (inference_tutorial cell 1: `from scdna_replication_tools.infer_scRT
    # import scRT`) before the timed cell 9 -- as the CPU baseline's modules are imported before
    # its timer; the import's own time is reported beside the fit's
    t0 = time.perf_counter()
    import scdna_replication_tools.infer_scRT  # noqa: F401
    t_import = time.perf_counter() - t0
    with contextlib.redirect_stdout(io.StringIO()):
        t0 = time.perf_counter()
        sc = tutorial_scrt(s.copy(), g.copy())
        cn_s_out, supp_s, cn_g1_out, supp_g1 = sc.infer(level='pyro')
        torch.cuda.synchronize()
        t_gpu = time.perf_counter() - t0
    m = sc.model
    share = cpu_share()
    torch.set_num_threads(share["cores"])
    m2 = tutorial_scrt(s.copy(), g.copy(), device="cpu")._pert_model()
    t0 = time.perf_counter()
    res = oracle_chain(m2, torch.float32)
    t_cpu = time.perf_counter() - t0
    iters = {k: len(res[v]) for k, v in (("step1", "losses_g"), ("step2", "losses_s"), ("step3", "losses_s2"))}
    mm = cn_s_out.merge(truth, on=["cell_id", "chr", "start"])
    rec = {"metric": "full 3-step PERT fit wall-clock, configs[0] stand-in (400+400 cells x 271 bins, max_iter 200)",
           "gpu_s": t_gpu, "gpu_import_s": t_import, "gpu_timings_s": m.timings, "gpu_iters": m.iters,
           "gpu_what": "scRT(...) + .infer(level='pyro') (inference_tutorial cell 9) in a fresh process, after the "
                       "package import (cell 1; gpu_import_s, not in gpu_s)",
           "cpu_baseline": {"seconds": t_cpu, "iters": iters, "cores": share["cores"], "cpu_model": share["cpu_model"],
                            "kind": "port", "what": "oracle chain (tests/_chain.py), fp32, measured end to end"},
           "speedup": t_cpu / t_gpu, "unit": "s", "higher_is_better": False,
           "acc_cn_vs_truth": float((mm["model_cn_state"] == mm["true_somatic_cn"]).mean()),
           "acc_rep_vs_truth": float((mm["model_rep_state"] == mm["true_rep"]).mean())}
    print(json.dumps(rec), flush=True)


class HelperLoad:
    """The host work a fit's helper thread does beside the device's steps (the tau
    initialiser's exact path, GIL-bound numpy: pert_model.py:364-423 per cell), looped on 64
    cells of the shard until stop(); the library scans made first on this thread, as a fit
    does (tau_init.prepare_host_threads)."""

    def __init__(self, reads):
        import threading
        from scdna_replication_tools_amd import tau_init
        tau_init.prepare_host_threads()
        self.cols = np.ascontiguousarray(np.asarray(reads, np.float32)[:, :64])
        self.cells = 0
        self.halt = threading.Event()
        self.thread = threading.Thread(target=self._run, name="bench-helper", daemon=True)
        self.t0 = time.perf_counter()
        self.thread.start()

    def _run(self):
        from scdna_replication_tools_amd import tau_init
        while not self.halt.is_set():
            tau_init.exact_fractions(self.cols)
            self.cells += self.cols.shape[1]

    def stop(self):
        self.halt.set()
        self.thread.join()
        dt = time.perf_counter() - self.t0
        return {"what": "tau_init.exact_fractions on 64 cells, looped on a thread", "cells": self.cells,
                "cells_per_s": round(self.cells / dt, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # K = 200 by default: a fit runs its steps as one C call, and the call's fixed costs (its first
    # launches, the final synchronisation, the interpreter lock taken back at its end) weigh 10x
    # less than at K = 20 (r05ca: 1,250 cells 0.419-0.426 ms/step at K = 200, 0.430-0.449 at 20)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c4", choices=sorted(CONFIGS))
    ap.add_argument("--scaling", default="strong", choices=["strong", "weak"])
    ap.add_argument("--bins-per-tile", type=int, default=0)
    ap.add_argument("--fit", default="step2", choices=["step1", "step2", "step3"],
                    help="which SVI fit's step to time (the metric is step 2's)")
    ap.add_argument("--variant", type=int, default=3, help="enumerated-pass kernel: 3 three-wave streamed (default), "
                    "0 two-wave LDS-DMA")
    ap.add_argument("--fused", action="store_true", help="variant 3: one launch per step (pert_enum_step)")
    ap.add_argument("--no-fused", action="store_true", help="(the default) separate finalize / adam launches")
    ap.add_argument("--cells", type=int, default=0, help="override the config's cell count (per job)")
    ap.add_argument("--subdivide", type=int, default=0, help="override the config's bin subdivision")
    ap.add_argument("--reads-per-cell", type=float, default=1e6, help="synthetic library size per cell")
    ap.add_argument("--prior", default="g1_clones", choices=["g1_clones", "g1_composite"],
                    help="CN prior of the step-2 fit: g1_clones (the tutorial's; one code per clone state) or "
                         "g1_composite (the reference's default; the product's composite code book, many rows)")
    ap.add_argument("--event-stride", type=int, default=5,
                    help="HIP events around the pass of every k-th step of the pass-timing run (1: every step)")
    ap.add_argument("--comm", default="auto", choices=["auto", "rccl", "torch", "host"],
                    help="cross-rank sum of the shared block: 'rccl' = the library's own RCCL communicator "
                         "(pert_comm, queued inside the C loop; the default on N > 1 over nccl, and at N = 1 "
                         "it times the sharded step with a one-rank all-reduce), 'torch' = torch.distributed "
                         "per step from Python, 'host' = the library's host-staged communicator (ranks sharing "
                         "a GPU: a rehearsal of the N > 1 C loop with PERT_DIST_BACKEND=gloo)")
    ap.add_argument("--comm-overlap", type=int, default=0,
                    help="1: the sharded step split so the all-reduce overlaps the per-cell finalize on a side "
                         "stream (pert_comm_allreduce_async); 0 (default; faster on ROCm 7.2): finalize, "
                         "all-reduce, Adam in sequence")
    ap.add_argument("--comm-delay-us", type=float, default=0.0,
                    help="a kernel spinning this long with every all-reduce (stand-in for an 8-rank ring's "
                         "latency at N = 1; measurement only)")
    ap.add_argument("--cpu-cells", type=int, default=640)
    ap.add_argument("--cpu-steps", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--helper-load", action="store_true",
                    help="run the tau initialiser's exact host path on a thread beside the timed steps "
                         "(what a fit's helper thread does during steps 1-2)")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    ap.add_argument("--profile", default="", help="tools/profile.sh output dir of this command: report the "
                    "roofline fraction recomputed from its kernel trace and its PMC HBM bytes")
    ap.add_argument("--fullfit-c1", action="store_true",
                    help="time the configs[0] stand-in's full fit on the GPU and on the CPU oracle, then exit")
    args = ap.parse_args()
    if args.fullfit_c1:
        fullfit_c1()
        return

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU over RCCL ("nccl"); PERT_DIST_BACKEND=gloo rehearses the same sharded
    # path with several ranks sharing the GPUs that are there (correctness runs only)
    backend = os.environ.get("PERT_DIST_BACKEND", "nccl")
    dev_index = local_rank if backend == "nccl" else local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev_index)
    device = torch.device("cuda", dev_index)
    pg = None
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)
        pg = dist

    from scdna_replication_tools_amd.engine import EtaCodebook, HostComm, PertShard, RcclComm
    from scdna_replication_tools_amd.init import init_params
    from scdna_replication_tools_amd.sharding import cell_bounds, make_allreduce

    n_cells, subdiv, desc = CONFIGS[args.config]
    if args.subdivide > 0:
        subdiv = args.subdivide
        desc = "synthetic {} cells x {} bins (--subdivide override of {})".format(n_cells, 5451 * subdiv, args.config)
    if args.cells > 0:
        n_cells = args.cells
        desc = "synthetic {} cells x {} bins (override of {})".format(n_cells, 5451 * subdiv, args.config)
    n_total = n_cells * (world if args.scaling == "weak" else 1)
    n0, n1 = cell_bounds(n_total, world)[rank]
    bm = np.zeros((1, K + 1))
    bm[0, K - 1] = 0.5                                                # betas [0.5, 0] of the simulator
    if args.prior == "g1_composite":
        if args.fit == "step1" or subdiv != 1:
            raise SystemExit("--prior g1_composite: the step-2/3 fits at 500 kb")
        reads_all, gc_all, eta_all, t_all = composite_problem(n_total)
        L = reads_all.shape[0]
        reads = np.ascontiguousarray(reads_all[:, n0:n1])
        eta = EtaCodebook(np.ascontiguousarray(eta_all.codes[:, n0:n1]), eta_all.table)
        t_init = t_all[n0:n1]
        data = {"gc": gc_all}
        states = None
        prior_desc = "g1_composite (J=5, weight 1e5; {} distinct eta rows)".format(eta_all.table.shape[0])
    else:
        data = synth(n_total, subdiv, seed=0, device=device, num_reads=args.reads_per_cell)
        L = data["reads"].shape[0]
        reads = data["reads"][:, n0:n1].cpu().numpy()
        states = data["cn"][:, n0:n1].cpu().numpy()
        eta = EtaCodebook.from_states(states, 1e6, P)                 # g1_clones prior (pert_model.py:285-296)
        t_init = np.clip(data["tau"][n0:n1].cpu().numpy(), 0.05, 0.95)
        prior_desc = "g1_clones (weight 1e6)"
    ploidy = eta.argmax_states().mean(0)
    comm, comm_error = None, None
    if args.comm == "host":
        if world < 2:
            raise SystemExit("--comm host needs torch.distributed ranks (world > 1)")
        comm = HostComm()
    elif args.comm == "rccl" or (args.comm == "auto" and world > 1 and backend == "nccl"):
        try:
            comm = RcclComm() if world > 1 else RcclComm.world1()
        except Exception as e:                     # noqa: BLE001  (then torch.distributed's all-reduce)
            if args.comm == "rccl":
                raise
            comm_error = "{}: {}".format(type(e).__name__, e)
            print("bench: the library's RCCL communicator failed ({}); all-reducing through "
                  "torch.distributed".format(comm_error), file=sys.stderr, flush=True)
    if comm is not None:
        comm.set_options(overlap=bool(args.comm_overlap), delay_us=args.comm_delay_us)
    allreduce = comm.allreduce if comm is not None else make_allreduce()
    comm_desc = (("host-staged: the library's shared-memory communicator" if args.comm == "host" else
                  "rccl: the library's own communicator") + ", all-reduce queued inside the C loop (pert_svi_run_sharded)"
                 if comm is not None else "torch.distributed all_reduce per step from Python{}".format(
                     " (pert_comm failed: {})".format(comm_error) if comm_error else "") if allreduce is not None
                 else "none (one rank)")
    libs = np.zeros(n1 - n0, int)
    common = dict(device=device, is_root=(rank == 0), allreduce=allreduce, bins_per_tile=args.bins_per_tile,
                  variant=args.variant, fused=args.fused and not args.no_fused, comm=comm)
    if args.fit == "step1":
        # step 1 (pert_model.py:718-774): the same cells as G1/2 cells, doubled with rep 0 / 1 --
        # as the product runs it, in pair mode (the columns stored once, both copies per lane)
        mr = reads.astype(np.float64).mean(0)
        init = init_params(1, None, np.zeros(2 * (n1 - n0), int), 1, P, K, seed=0,
                           mean_reads=np.concatenate([mr, mr]), n_bins=L)
        shard = PertShard(1, reads, data["gc"], np.zeros(2 * (n1 - n0), int), 1, P, K, init, cn_obs=states,
                          paired=True, n_cells_total=2 * n_total, **common)
    else:
        kind = 2 if args.fit == "step2" else 3
        init = init_params(kind, reads, libs, 1, P, K, ploidy=ploidy, t_init=t_init, beta_means=bm, seed=0)
        extra = {}
        if kind == 3:
            from scdna_replication_tools_amd.simulator import convert_rt_units, load_bins
            extra = dict(rho_fixed=convert_rt_units(load_bins(subdivide=subdiv)["mcf7rt"].to_numpy(np.float64)),
                         a_fixed=10.0)
        shard = PertShard(kind, reads, data["gc"], libs, 1, P, K, init, eta=eta, lamb=0.75, beta_means=bm,
                          n_cells_total=n_total, **extra, **common)
    del data
    torch.cuda.synchronize()

    # The fit's own loop (PertShard.run_svi, as pert_model._svi runs it): every step's loss is
    # recorded on the device, the stopping rule is evaluated there (never met here: min_iter
    # beyond the step count; the NaN check stays on) and the losses come back to the host in
    # chunks, with no per-step host synchronisation.
    # Before the timed region, in this order: (1) the loop's buffers for the warmup and both timed
    # runs (the second one's timing events too; step 1's canonical pi trajectory), as
    # run_pert_model has them ready before a fit starts, then the ranks meet; (2) the pattern's
    # HBM ceiling on this device and lease (pert_stream_ceiling: the pass's streams with no
    # arithmetic, the state left unchanged), repeated for ~100 ms of HBM load; (3) the W warmup
    # steps.  On a short shard the first timed steps otherwise run slower than the next ones:
    # r05g, 1,250 cells 0.510 ms/step in the first K steps after W = 3, 0.495 in the next K;
    # r05bm, with the warmup before the burst, the value run still 1-2.4 % behind the evented
    # run after it at 1,250-2,500 cells.
    shard.pass_events = []
    shard.pass_event_stride = max(1, args.event_stride)
    shard.reserve_svi(args.steps)
    shard.pass_events = None
    shard.reserve_svi(max(args.warmup, 0) + 2 * args.steps)   # step 1's trajectory for all three runs
    if pg is not None:
        pg.barrier()
    ceil_ms = None
    if args.fit != "step1":
        est = shard.stream_ceiling_ms(reps=3)
        ceil_ms = shard.stream_ceiling_ms(reps=int(min(200, max(10, math.ceil(100.0 / max(est, 1e-3))))))
    helper = None
    if args.helper_load:
        helper = HelperLoad(reads)
    if args.warmup > 0:
        shard.run_svi(args.warmup, min_iter=10 ** 9, rel_tol=0.0)
    # The value's region is the production loop with no timing events (one C call, pert_svi_run):
    # a HIP timing event on the stream costs the step ~50 us (r05d: 0.497 vs 0.520 ms/step at
    # 1,250 cells with events around every 5th pass).  The pass durations come from the same K
    # steps run again right after it, with events around every event_stride-th pass.
    if pg is not None:
        pg.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    losses, _ = shard.run_svi(args.steps, min_iter=10 ** 9, rel_tol=0.0)
    if len(losses) != args.steps:
        raise RuntimeError("the fit stopped after {} of {} steps (NaN loss)".format(len(losses), args.steps))
    torch.cuda.synchronize()
    if pg is not None:
        pg.barrier()
    dt = time.perf_counter() - t0
    # the pass-timing run: the next K steps, HIP events around every event_stride-th pass
    shard.pass_events = []
    shard.pass_event_stride = max(1, args.event_stride)
    shard.reserve_svi(args.steps)                     # (also creates the timing events)
    if pg is not None:
        pg.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    shard.run_svi(args.steps, min_iter=10 ** 9, rel_tol=0.0)
    torch.cuda.synchronize()
    if pg is not None:
        pg.barrier()
    dt_ev = time.perf_counter() - t1
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in shard.pass_events]))
    helper_rec = helper.stop() if helper is not None else None
    shard.pass_events = None
    t = torch.tensor([dt, kern_ms, dt_ev], dtype=torch.float64, device=device)
    if pg is not None:
        pg.all_reduce(t, op=pg.ReduceOp.MAX)
    dt, kern_ms_max, dt_ev = float(t[0]), float(t[1]), float(t[2])

    if rank == 0:
        cellbins_total = L * n_total * (2 if args.fit == "step1" else 1)
        value = cellbins_total * args.steps / dt
        step1 = args.fit == "step1"
        # step 1, pair mode: reads fp32 + observed cn u8 per G1/2 cell and bin, shared by its two
        # copies (2.5 B per fitted cell and bin)
        bpc = 2.5 if step1 else bytes_per_cellbin(P)
        local_cb = L * (n1 - n0) * (2 if step1 else 1)
        achieved = bpc * local_cb / (kern_ms * 1e-3) / 1e9
        kname = ("obs_pair_kernel<5>" if step1 else
                 "enum3_kernel<13, 0, 5>" if args.variant == 3 else
                 "enum_dma_kernel<13, 0, 5>")
        traffic, valu = None, None
        if os.path.exists(args.pmc) and args.fit == "step2":
            try:
                pm = json.load(open(args.pmc))
                if (pm.get("config") == args.config and int(pm.get("cells", -1)) == n1 - n0
                        and pm.get("kernel") == kname):
                    traffic = pm.get("hbm_bytes_per_launch")
                    valu = pm.get("valu")
            except (OSError, ValueError):
                traffic, valu = None, None
        rec = {
            "metric": ("enumerated ELBO+grad cell*bins/s (10k cells x 5.5k bins, 500kb)" if args.fit == "step2"
                       else "{} SVI step cell*bins/s".format(args.fit)),
            "value": value, "unit": "cell*bins/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True,
            "scaling": args.scaling, "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": desc, "config": args.config, "cells": n_total, "bins": L, "P": P,
                       "K": K, "cn_prior": prior_desc, "parallelism": "cell-sharded x{}".format(world),
                       "bins_per_tile": shard.bins_per_tile, "fit": args.fit, "allreduce": comm_desc,
                       "comm_overlap": bool(args.comm_overlap) if comm is not None else None,
                       "comm_delay_us": args.comm_delay_us if comm is not None else None,
                       "timed_loop": ("pert_svi_run{}: the whole loop in one GIL-free C call, no timing "
                                      "events".format("_sharded" if comm is not None else "")
                                      if comm is not None or allreduce is None
                                      else "per-iteration launches from Python")},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_unit": "bytes/launch",
                         "kernel": ("obs_kernel" if step1 else
                                    "enum3_kernel<13, STEP, 5>" if args.variant == 3 else
                                    "enum_dma_kernel<13, STEP, 5>"),
                         "kernel_ms": kern_ms,
                         "kernel_ms_events": ("HIP events on the pass's stream around every {} pass of the K steps "
                                              "run right after the timed region (ms_per_step_evented: their wall "
                                              "time; events in the value's region would cost ~50 us each)".format(
                                                  "" if args.event_stride <= 1 else "{}th".format(args.event_stride))),
                         "bytes_per_cellbin": bpc,
                         # PMC (profiles/pmc_traffic.json, tools/profile.sh): VALU issue fraction of
                         # the same kernel -- the other roofline, not the binding one here
                         "valu_issue_frac": (valu or {}).get("issue_frac")},
            "loss_first": losses[0], "loss_last": losses[-1],
        }
        rec["ms_per_step_evented"] = dt_ev / args.steps * 1e3
        if helper_rec is not None:
            rec["helper_load"] = helper_rec
        if ceil_ms is not None:
            rec["roofline"]["pattern_ceiling"] = {
                "ms": ceil_ms, "GB/s": bpc * local_cb / (ceil_ms * 1e-3) / 1e9,
                "kernel_frac_of_ceiling": ceil_ms / kern_ms,
                "what": "pert_stream_ceiling: the pass's HBM streams (x, eta code, z/m/v read + written) with no "
                        "arithmetic, same tiles, same shard, same process"}
            rec["roofline"]["pi_placement"] = dict(shard.placement or {"candidates_ms": None},
                                                   what="PertShard.choose_pi_placement: pattern time of each "
                                                        "z/m/v allocation tried at set-up (fastest kept)")
        if args.fit == "step2" and args.variant == 3 and shard.fused:
            rec["roofline"]["note"] = ("one launch per step (pert_enum_step): the pass with the reductions and "
                                       "Adam folded in; kernel_ms is that launch")
        if args.profile:
            pn = profile_numbers(args.profile, kname)
            if pn is not None:
                tk = pn["avg_ns"] * 1e-6
                ach_t = bpc * local_cb / (tk * 1e-3) / 1e9
                rec["roofline"].update({
                    "trace_kernel_ms": tk, "trace_calls": pn["calls"], "frac_trace": ach_t / HBM_PEAK_GBS,
                    "frac_vs_trace": (achieved / HBM_PEAK_GBS) / (ach_t / HBM_PEAK_GBS),
                    "trace_source": os.path.relpath(args.profile, ROOT)})
                if pn["hbm_bytes_per_launch"] is not None:
                    rec["roofline"]["traffic"] = pn["hbm_bytes_per_launch"]
                    rec["roofline"]["traffic_per_algorithmic"] = pn["hbm_bytes_per_launch"] / (bpc * local_cb)
                p = pn["pmc"]
                if p.get("SQ_WAVE_CYCLES"):
                    # where the pass's wave-cycles go (the three counters partition them): issuing,
                    # waiting on an instruction dependency / issue slot, waiting on memory (s_waitcnt)
                    wc = p["SQ_WAVE_CYCLES"]
                    rec["roofline"]["wave_cycles"] = {
                        "active_inst": p.get("SQ_ACTIVE_INST_ANY", 0.0) / wc,
                        "wait_inst": p.get("SQ_WAIT_INST_ANY", 0.0) / wc,
                        "wait_mem": p.get("SQ_WAIT_ANY", 0.0) / wc}
        if world == 1 and not args.no_cpu_baseline and args.fit == "step2" and args.prior == "g1_clones":
            data = synth(max(args.cpu_cells, 3), subdiv, seed=0, device=device)
            rec["cpu_baseline"] = cpu_baseline(data, args.cpu_cells, args.cpu_steps)
        else:
            rec["cpu_baseline"] = None
        print(json.dumps(rec), flush=True)
    if comm is not None:
        comm.close()
    if pg is not None:
        pg.destroy_process_group()


if __name__ == "__main__":
    main()

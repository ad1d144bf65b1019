"""Device-resident SVI state for one cell shard and the per-step launch sequence.

A ``PertShard`` owns every buffer of one fit (step 1, 2 or 3 of reference
``pert_model.run_pert_model``, pert_model.py:649-901) on one GPU:

* inputs: reads (L, N) fp32, gc features (L, K+1), library index (N,), the CN
  prior eta as a code book (uint16 codes (L, N) + table) for steps 2/3, the
  observed cn / rep (uint8) for step 1;
* the pi logits and their Adam moments as wave tiles [N/64][L][P][64] (steps 2/3);
* the packed non-pi parameters (layout ``pert_layout`` of include/pert_hip.h),
  their Adam moments and gradients.

``step()`` is one ``svi.step`` (pert_model.py:743 / :801 / :868): enumerated or
observed pass with the fused pi Adam update, reductions, the cross-rank
all-reduce of the shared-gradient block (rho, a, beta_stds, lambda, beta_means,
loss) when a process group is given, and Adam on the packed parameters.
Everything runs through libpert_hip.so; there is no host fallback.
"""
from __future__ import annotations

import ctypes
import contextlib
import math
import os
import threading
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, Optional

import numpy as np
import torch

from . import _native as nat

ADAM_BETAS = (0.8, 0.99)
ADAM_EPS = 1e-8
F32 = np.float32
EPS32 = float(np.finfo(np.float32).eps)
TINY32 = float(np.finfo(np.float32).tiny)

# pi-state placement search (PertShard.choose_pi_placement): candidate z / m / v allocations per
# shard (env PERT_PLACEMENT; 0 or 1 = the first allocation only), the smallest pi state searched
# (fp32 elements: 1,250 cells x 5,451 bins x 13 states is 89 M), and the pattern rate (bytes/s) at
# which a placement counts as fast and the search stops (MI355X: slow placements stream the
# pass's pattern at 5.1-5.3 TB/s, fast ones at 5.9-6.3 TB/s; profiles/r05z_sets_probe.log)
PLACEMENT_CANDIDATES = 24
PLACEMENT_MIN_FLOATS = 32 * 1024 * 1024
PLACEMENT_FAST_RATE = 5.8e12
# each try past the first moves at least this far through free HBM (a small set is followed by a
# held spacer), and the search holds at most PLACEMENT_MAX_HELD bytes of tries and spacers: the
# slow placements come in runs of ~15-45 GB of allocations (r05ab, r05ac: the 3rd 8.7 GB set, the
# 5th 4.4 GB set, the 6th-7th 2.2 GB set + spacer, the 10th-12th 1.1 GB set + spacer fast)
PLACEMENT_STRIDE = 3 << 30
PLACEMENT_MAX_HELD = 96 << 30
# fast placements come at two rates (10 k cells: pattern 2.75-2.80 ms = 6.2-6.3 TB/s, or
# 2.85-2.94 ms = 5.9-6.1 TB/s; r05z, r05ai-r05bs): the search stops at once on a set of the
# upper rate, and past the first fast set of the lower one it tries at most PLACEMENT_EXTRA
# more sets, worth at most PLACEMENT_EXTRA_BYTES (the 1,250-cell pass, bound by its one-round
# tail, runs equally fast at either rate: r05bt, up to 22 tries for the same step)
PLACEMENT_TOP_RATE = 6.15e12
PLACEMENT_EXTRA = 4
PLACEMENT_EXTRA_BYTES = 48 << 30


# --------------------------------------------------------------------------- transforms
# torch.distributions.transform_to semantics (constraint_registry.py), fp32.
def sigmoid_inv(y: torch.Tensor) -> torch.Tensor:
    y = y.clamp(min=TINY32, max=1.0 - EPS32)
    return y.log() - (-y).log1p()


def clipped_sigmoid(z: torch.Tensor) -> torch.Tensor:
    return torch.clamp(torch.sigmoid(z), min=TINY32, max=1.0 - EPS32)


def gc_features(gc: np.ndarray, K: int) -> torch.Tensor:
    """pert_model.py:460-463 evaluated like the reference (fp32 torch): [gc^K .. gc, 1]."""
    x = torch.as_tensor(np.asarray(gc), dtype=torch.float32).unsqueeze(1)
    return torch.cat([x ** i for i in reversed(range(0, K + 1))], 1)


# --------------------------------------------------------------------------- CN prior code book
@dataclass
class EtaCodebook:
    """The (L, N, P) Dirichlet concentration eta stored as uint16 row codes + table.

    Every eta builder of the reference (pert_model.py:272-361, :668-716) yields rows
    drawn from a small set (one weight on one state, or the composite sums), so the
    (L, N, P) fp32 tensor (2.8 GB at 10k cells x 5.5k bins) shrinks to 2 B per cell.bin.
    """
    codes: np.ndarray   # (L, N) uint16
    table: np.ndarray   # (n_codes, P) float32 eta rows
    # per-cell mean of the argmax states (pert_model.py:591-593), filled by the first
    # argmax_states() / ploidy() call: the fit needs it for the init, the shard and the
    # tau initialiser, and building the (L, N) states costs ~0.5 s at 10k cells
    _ploidy: Optional[np.ndarray] = field(default=None, init=False, repr=False, compare=False)

    @property
    def P(self):
        return self.table.shape[1]

    @classmethod
    def from_dense(cls, etas) -> "EtaCodebook":
        e = np.ascontiguousarray(np.asarray(etas, dtype=F32))
        L, N, P = e.shape
        table, inv = np.unique(e.reshape(-1, P), axis=0, return_inverse=True)
        if table.shape[0] > 65535:
            raise ValueError("eta has {} distinct rows; at most 65535 are supported".format(table.shape[0]))
        return cls(inv.reshape(L, N).astype(np.uint16), table.astype(F32))

    @classmethod
    def from_states(cls, states, weight: float, P: int) -> "EtaCodebook":
        """build_cn_prior (pert_model.py:272-282): ones with eta[state] = weight.  uint16
        states are taken as the codes themselves (no widening copy)."""
        s = np.asarray(states)
        if s.dtype != np.uint16:
            s = s.astype(np.int64)
        if s.size and (s.min() < 0 or s.max() >= P):
            raise ValueError("CN states must lie in [0, P) for P={}".format(P))
        table = np.ones((P, P), dtype=F32)
        table[np.arange(P), np.arange(P)] = F32(weight)
        return cls(np.ascontiguousarray(s, dtype=np.uint16), table)

    def kernel_table(self, round_site: bool = True) -> np.ndarray:
        """(n_codes, P+2): eta_k - 1, then S1 = sum_k (eta_k - 1), then A = lgamma(sum eta)
        in fp32 exactly as torch.distributions.Dirichlet.log_prob evaluates it (0 when
        ``round_site`` is off): the kernels round each element's Dirichlet value to A's grid,
        as the reference's fp32 value is rounded before it is summed (include/pert_hip.h,
        pert_math.h dir_site_round; tests/test_dirichlet_value.py)."""
        em1 = self.table.astype(np.float64) - 1.0
        t = torch.from_numpy(np.ascontiguousarray(self.table, dtype=F32))
        A = torch.lgamma(t.sum(-1)).numpy() if round_site else np.zeros(len(em1), F32)
        out = np.concatenate([em1, em1.sum(1, keepdims=True), A.astype(np.float64)[:, None]], axis=1)
        return out.astype(F32)

    def counts(self) -> np.ndarray:
        return np.bincount(self.codes.reshape(-1), minlength=self.table.shape[0])

    def dirichlet_normaliser(self, mode: str = "torch32", counts=None) -> float:
        """sum_{l,n} lgamma(sum eta) - sum lgamma(eta).  ``torch32`` evaluates each row in
        fp32 exactly as torch.distributions.Dirichlet.log_prob does on the CPU
        (dirichlet.py:93-97) -- the constant the reference adds to every loss --
        ``exact`` in fp64."""
        t = torch.from_numpy(self.table)
        if mode == "exact":
            t = t.double()
        per = (torch.lgamma(t.sum(-1)) - torch.lgamma(t).sum(-1)).double().numpy()
        return float((per * (self.counts() if counts is None else np.asarray(counts))).sum())

    def argmax_states(self) -> np.ndarray:
        """torch.argmax(etas, dim=2) (first max), pert_model.py:591-592 and :439."""
        row_arg = np.argmax(self.table, axis=1)
        states = row_arg[self.codes]
        if self._ploidy is None:
            self._ploidy = self._mean_states(states)
        return states

    @staticmethod
    def _mean_states(states) -> np.ndarray:
        # torch.mean(argmax.type(float32), dim=0) as the reference evaluates it (fp32, CPU)
        return torch.mean(torch.as_tensor(states, dtype=torch.float32), dim=0).numpy()

    def ploidy(self) -> np.ndarray:
        """(N,) float32 mean argmax state per cell (pert_model.py:591-593), cached."""
        if self._ploidy is None:
            self.argmax_states()
        return self._ploidy

    def cells(self, sl: slice) -> "EtaCodebook":
        """The code book of a contiguous range of cells (a rank's shard), ploidy cache included."""
        sub = EtaCodebook(np.ascontiguousarray(self.codes[:, sl]), self.table)
        if self._ploidy is not None:
            sub._ploidy = self._ploidy[sl]
        return sub

    def dense(self) -> np.ndarray:
        return self.table[self.codes]


def kappa_sum(reads, log_lam: Optional[float]) -> float:
    """sum over (bin, cell) of the parameter-free part of the NB log density that the
    kernels leave out: (x log lam) + (x log x - x) - lgamma(1 + x), in fp64 on the device of
    ``reads`` (a tensor: zero padding adds nothing) or on the host (an array)."""
    return kappa_and_sum(reads, log_lam)[0]


def kappa_and_sum(reads, log_lam: Optional[float]):
    """(kappa_sum, sum of reads), both fp64."""
    if isinstance(reads, torch.Tensor):
        x = reads.to(torch.float64)
    else:
        x = torch.as_tensor(np.asarray(reads), dtype=torch.float64)
    xlx = torch.where(x > 0, x * torch.log(torch.where(x > 0, x, torch.ones_like(x))), torch.zeros_like(x))
    s = float((xlx - x - torch.lgamma(1.0 + x)).sum())
    total = float(x.sum())
    if log_lam is not None:
        s += total * log_lam
    return s, total


# --------------------------------------------------------------------------- step-1 pi block
# The canonical trajectory depends only on (P, lr, betas, eps): it is computed once per
# process and shared by every step-1 fit (key -> per-step log pi~ and states).
_PI_TRAJECTORIES: Dict[tuple, dict] = {}
_PI_LOCK = threading.Lock()          # the fit's helper thread may extend it (precompute)


PI_TRAJECTORY_FILE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "pi_trajectory.npz")


def _shipped_trajectory(key: tuple) -> Optional[dict]:
    """The canonical pi trajectory for the defaults (P = 13, lr 0.05, Adam (0.8, 0.99), eps 1e-8),
    computed by CanonicalPiBlock itself and shipped with the package (tools/make_pi_trajectory.py;
    tests/test_engine_host.py checks it against the live computation bit for bit): the step-1 loop
    of every process would otherwise recompute the same 1,000 autograd steps (~0.2 s) first."""
    try:
        with np.load(PI_TRAJECTORY_FILE, allow_pickle=False) as f:
            if tuple(f["key"].tolist()) != (float(key[0]),) + tuple(key[1:]):
                return None
            lp, z, m, v = f["lp"], f["z"], f["m"], f["v"]
    except (OSError, KeyError, ValueError):
        return None
    return {"lp": [float(x) for x in lp],
            "state": [(z[i].astype(F32), m[i].astype(F32), v[i].astype(F32)) for i in range(z.shape[0])]}


class CanonicalPiBlock:
    """Step 1's expose_pi site (pert_model.py:607-613 with etas = ones, cn observed).

    pi(l, n) only enters log Categorical(cn_obs | pi) and the constant Dirichlet(1)
    density, starts at the uniform simplex for every (l, n), and Adam is
    element-wise, so every (l, n) follows the same trajectory up to a permutation
    of the states.  One P-vector reproduces all of them exactly; its loss term is
    L * N * log pi~_c(t).  The trajectory is data independent, so it is computed once
    (fp32 torch autograd + the Adam update below) and cached per (P, lr, betas, eps).
    """

    def __init__(self, P: int, lr: float, betas=ADAM_BETAS, eps=ADAM_EPS):
        self.P = P
        self.z = np.full(P, np.log(F32(1.0 / P)), dtype=F32)
        self.m = np.zeros(P, F32)
        self.v = np.zeros(P, F32)
        self.lr, self.b1, self.b2, self.eps = lr, betas[0], betas[1], eps
        self.t = 0                               # Adam steps taken

    def logp_and_grad(self):
        z = torch.from_numpy(self.z.copy()).requires_grad_(True)
        p = torch.softmax(z, 0)
        p = p / p.sum()
        lp = torch.log(torch.clamp(p, min=EPS32, max=1 - EPS32))[0]   # observed state at index 0
        lp.backward()
        return float(lp.detach()), (-z.grad).numpy().astype(F32)             # loss gradient

    def _advance(self, t: int) -> float:
        lp, g = self.logp_and_grad()
        self.m = (self.b1 * self.m + (1 - self.b1) * g).astype(F32)
        self.v = (self.b2 * self.v + (1 - self.b2) * g * g).astype(F32)
        bc1 = 1 - self.b1 ** t
        bc2 = 1 - self.b2 ** t
        denom = np.sqrt(self.v) / math.sqrt(bc2) + self.eps
        self.z = (self.z - (self.lr / bc1) * self.m / denom).astype(F32)
        return lp

    @classmethod
    def precompute(cls, P: int, lr: float, T: int, betas=ADAM_BETAS, eps=ADAM_EPS) -> None:
        """Extend the shared trajectory to T steps ahead of the fit that needs it (~0.2 ms of
        host work per step: run_pert_model starts it on its helper thread during the prep, so
        step 1's loop does not wait for it)."""
        cls(P, lr, betas, eps)._cache(T)

    def _cache(self, T: int) -> dict:
        """The shared trajectory, extended to at least T steps."""
        with _PI_LOCK:
            return self._cache_locked(T)

    def _cache_locked(self, T: int, shipped: bool = True) -> dict:
        key = (self.P, float(self.lr), float(self.b1), float(self.b2), float(self.eps))
        c = _PI_TRAJECTORIES.get(key)
        if c is None and shipped:
            c = _shipped_trajectory(key)
            if c is not None:
                _PI_TRAJECTORIES[key] = c
        if c is None:
            c = _PI_TRAJECTORIES[key] = {"lp": [], "state": [(self.__class__(self.P, self.lr, (self.b1, self.b2),
                                                                                self.eps).z, np.zeros(self.P, F32),
                                                               np.zeros(self.P, F32))]}
        if len(c["lp"]) < T:
            w = CanonicalPiBlock.__new__(CanonicalPiBlock)
            w.P, w.lr, w.b1, w.b2, w.eps = self.P, self.lr, self.b1, self.b2, self.eps
            w.z, w.m, w.v = (a.copy() for a in c["state"][-1])
            while len(c["lp"]) < T:
                c["lp"].append(w._advance(len(c["lp"]) + 1))
                c["state"].append((w.z.copy(), w.m.copy(), w.v.copy()))
        return c

    def trajectory(self, t0: int, n: int) -> np.ndarray:
        """log pi~ of steps t0 .. t0+n-1 (the values ``step`` would return), without
        advancing this block: the per-step loss term of a device-side SVI loop."""
        if t0 != self.t + 1:
            raise ValueError("the block is at step {}, not {}".format(self.t, t0 - 1))
        c = self._cache(t0 - 1 + n)
        return np.asarray(c["lp"][t0 - 1:t0 - 1 + n], dtype=np.float64)

    def step(self, t: int) -> float:
        """Adam step t (= previous step + 1); returns log pi~ before the update."""
        if t != self.t + 1:
            raise ValueError("the block is at step {}, not {}".format(self.t, t - 1))
        c = self._cache(t)
        self.z, self.m, self.v = (a.copy() for a in c["state"][t])
        self.t = t
        return c["lp"][t - 1]

    def advance_to(self, t: int) -> float:
        """Take steps up to t at once; returns the last step's log pi~."""
        c = self._cache(t)
        self.z, self.m, self.v = (a.copy() for a in c["state"][t])
        self.t = t
        return c["lp"][t - 1] if t > 0 else float("nan")


# --------------------------------------------------------------------------- ranks
def rccl_path() -> str:
    """The RCCL library this process already uses (torch's, which libtorch_hip links): the
    communicator of a sharded fit is made with the same copy."""
    try:
        with open("/proc/self/maps") as fh:
            for line in fh:
                path = line.split()[-1] if line.strip() else ""
                if "/librccl.so" in path:
                    return path
    except OSError:
        pass
    import os
    return os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")


def comm_timeout_s() -> float:
    """The deadline of a sharded fit's waits on its peers (PERT_COMM_TIMEOUT_S, default 600 s)."""
    import os
    return float(os.environ.get("PERT_COMM_TIMEOUT_S", "600"))


def _group_device(group):
    import torch.distributed as dist
    return (torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl"
            else torch.device("cpu"))


def _broadcast_bytes(data: bytes, n: int, group) -> bytes:
    """Rank 0's ``n`` bytes on every rank of ``group`` (a uint8 tensor broadcast)."""
    import torch.distributed as dist
    t = torch.zeros(n, dtype=torch.uint8)
    if data:
        t[:len(data)] = torch.tensor(list(data), dtype=torch.uint8)
    t = t.to(_group_device(group))
    dist.broadcast(t, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
    return bytes(t.cpu().tolist())


def _all_ok(ok: bool, group) -> bool:
    """True on every rank iff ``ok`` on every rank (a MIN all-reduce): the ranks of a fit take
    the same communicator, or all fall back together."""
    import torch.distributed as dist
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=_group_device(group))
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(int(t.item()))


def _segment_name() -> str:
    import os
    return "/pert-{}-{}".format(os.getpid(), os.urandom(6).hex())


class PertComm:
    """A communicator of the library's own over the ranks of a sharded fit (``pert_comm``,
    include/pert_hip.h): the library queues the per-step all-reduce of the shared block itself,
    on the fit's stream, so a sharded fit's SVI loop is one GIL-free C call
    (``pert_svi_run_sharded``) as a single-rank one is.  A rank whose loop fails raises the
    node's abort word, and every rank's loop returns within the deadline with ``CommError``."""

    handle = None
    lib = None

    def allreduce(self, t: torch.Tensor) -> None:
        """In-place sum over the ranks of an fp64 device tensor, on the current stream."""
        if t.dtype != torch.float64 or not t.is_cuda or not t.is_contiguous():
            raise ValueError("{}.allreduce takes a contiguous fp64 device tensor".format(type(self).__name__))
        nat.check(self.lib.pert_comm_allreduce_sum_f64(self.handle, t.data_ptr(), t.data_ptr(), t.numel(),
                                                        torch.cuda.current_stream(t.device).cuda_stream),
                  "pert_comm_allreduce_sum_f64")

    def set_options(self, overlap: bool = False, delay_us: float = 0.0) -> None:
        """overlap: the sharded loop's split step (the shared block's all-reduce on a side
        stream beside the per-cell finalize; off by default -- the cross-stream hops cost more
        than they hide on ROCm 7.2); delay_us > 0: a kernel
        spinning that long with every all-reduce -- a stand-in for an 8-rank ring's latency
        on a one-GPU box (measurement only)."""
        nat.check(self.lib.pert_comm_set_options(self.handle, 1 if overlap else 0, float(delay_us)),
                  "pert_comm_set_options")

    def status(self) -> int:
        """0, or the first failure this rank has seen (its own, or a peer's abort)."""
        return int(self.lib.pert_comm_status(self.handle))

    def abort(self, code: int = nat.E_COMM_ABORTED) -> None:
        nat.check(self.lib.pert_comm_abort(self.handle, int(code)), "pert_comm_abort")

    def _fault_from_env(self) -> None:
        """PERT_COMM_FAULT_AT="rank:call": the test hook below, set on that rank at creation."""
        import os
        spec = os.environ.get("PERT_COMM_FAULT_AT")
        if spec:
            r, k = (int(x) for x in spec.split(":"))
            if r == self.rank:
                self.inject_fault(k)

    def inject_fault(self, at_call: int) -> None:
        """Test hook: this rank's all-reduce call ``at_call`` (0-based, counted from the
        communicator's creation) fails at queue time."""
        nat.check(self.lib.pert_comm_inject_fault(self.handle, int(at_call)), "pert_comm_inject_fault")

    def close(self) -> None:
        if self.handle is not None and self.handle.value:
            if self.status() == 0:
                torch.cuda.synchronize()
            nat.check(self.lib.pert_comm_destroy(self.handle), "pert_comm_destroy")
        self.handle = None


class RcclComm(PertComm):
    """The product communicator: RCCL over the ranks of ``group`` (one process per GPU, xGMI),
    made collectively on the current device (rank 0's unique id broadcast over the group), with
    a node-local abort word beside it (``pert_comm_set_watchdog``).  Loading RCCL is checked on
    every rank before any rank enters the collective init, so the ranks take this communicator
    or raise together (``_Dist`` then falls back on all of them).  ``world1()`` makes a
    one-rank communicator without a process group (tests, bench)."""

    def __init__(self, group=None, *, world1: bool = False, device=None):
        self.lib = nat.lib_nogil()              # init blocks until every rank has called: GIL released
        if device is not None:
            dev = torch.device(device)
            if dev.type != "cuda" or (dev.index is not None and dev.index != torch.cuda.current_device()):
                raise ValueError("RcclComm is made on the current device ({}), not {}: set the device "
                                 "first".format(torch.cuda.current_device(), dev))
        if world1:
            self.world, self.rank, dist = 1, 0, None
        else:
            import torch.distributed as dist
            self.world, self.rank = dist.get_world_size(group), dist.get_rank(group)
        rc = self.lib.pert_comm_load(rccl_path().encode())
        if dist is not None and self.world > 1 and not _all_ok(rc == 0, group):
            raise nat.NativeLibraryError("pert_comm_load failed on {} rank(s) of the group".format(
                "this and possibly other" if rc else "another"))
        nat.check(rc, "pert_comm_load")
        uid = (ctypes.c_uint8 * 128)()
        name = b""
        if self.rank == 0:
            nat.check(self.lib.pert_comm_unique_id(uid, 128), "pert_comm_unique_id")
            name = _segment_name().encode()
        if dist is not None and self.world > 1:
            got = _broadcast_bytes(bytes(uid) + name.ljust(64, b"\0"), 128 + 64, group)
            uid = (ctypes.c_uint8 * 128)(*got[:128])
            name = got[128:].rstrip(b"\0")
        h = ctypes.c_void_p()
        rc = self.lib.pert_comm_init(uid, 128, self.world, self.rank, ctypes.byref(h))
        if dist is not None and self.world > 1 and not _all_ok(rc == 0, group):
            if rc == 0:
                self.lib.pert_comm_destroy(h)
            raise nat.NativeLibraryError("pert_comm_init failed on a rank of the group (status {})".format(rc))
        nat.check(rc, "pert_comm_init")
        self.handle = h
        rc = self.lib.pert_comm_set_watchdog(h, name if self.world > 1 else None, comm_timeout_s())
        if rc != 0:
            self.close()
            nat.check(rc, "pert_comm_set_watchdog")
        self._fault_from_env()

    @classmethod
    def world1(cls) -> "RcclComm":
        return cls(world1=True)


class HostComm(PertComm):
    """The host-staged communicator (``pert_comm_init_host``): for ranks that share a GPU (RCCL
    refuses them) -- the tests' two ranks on one device run the product's C loop
    (``pert_svi_run_sharded``) through it.  Each all-reduce is a copy to pinned memory, a host
    function that adds the ranks' blocks through POSIX shared memory in rank order, and a copy
    back, queued where the RCCL call would be.  Ranks on one node; ``max_n`` bounds the block
    (n_shared + 1 = bins + a few dozen: 2^18 covers 20 kb bins of a whole genome)."""

    def __init__(self, group=None, *, max_n: int = 1 << 18):
        import torch.distributed as dist
        self.lib = nat.lib_nogil()
        self.world, self.rank = dist.get_world_size(group), dist.get_rank(group)
        name = _broadcast_bytes(_segment_name().encode() if self.rank == 0 else b"", 64, group).rstrip(b"\0")
        self.max_n = int(max_n)
        h = ctypes.c_void_p()
        nat.check(self.lib.pert_comm_init_host(name, self.world, self.rank, self.max_n, comm_timeout_s(),
                                               ctypes.byref(h)), "pert_comm_init_host")
        self.handle = h
        self._fault_from_env()


# --------------------------------------------------------------------------- shard
def _ptr(t: Optional[torch.Tensor]) -> int:
    return 0 if t is None else int(t.data_ptr())


def placement_search(first, time_set: Callable, alloc: Callable, free_bytes: Callable, set_bytes: int,
                     pattern_bytes: float, candidates: int = PLACEMENT_CANDIDATES):
    """The loop of PertShard.choose_pi_placement, apart from the device: ``time_set(s)`` times
    the pass's stream pattern on set s (ms), ``alloc(spacer)`` returns a new set and the spacer
    allocations made before it, ``free_bytes()`` the device's free memory.  Tries sets while
    the best streams below PLACEMENT_FAST_RATE, then up to PLACEMENT_EXTRA more (at most
    PLACEMENT_EXTRA_BYTES) unless one streams at PLACEMENT_TOP_RATE (the search stops there),
    within ``candidates`` tries, PLACEMENT_MAX_HELD bytes held and 8 GB left free.  Returns the
    fastest set, every try's time (the first set's first) and the list of what was held (for
    the caller to drop once the state has moved)."""
    best = first
    best_ms = time_set(first)
    times = [best_ms]
    held = []
    spacer = max(0, PLACEMENT_STRIDE - set_bytes)
    held_bytes = 0
    step = set_bytes + spacer
    extra = None                                 # bytes tried since a fast set was first seen
    n_extra = 0
    while len(times) < candidates:
        rate = pattern_bytes / (best_ms * 1e-3)
        if rate >= PLACEMENT_TOP_RATE:
            break
        if extra is None and rate >= PLACEMENT_FAST_RATE:
            extra = 0
        if extra is not None and (extra + step > PLACEMENT_EXTRA_BYTES or n_extra >= PLACEMENT_EXTRA):
            break
        if free_bytes() < step + set_bytes + (8 << 30) or held_bytes + step > PLACEMENT_MAX_HELD:
            break
        cand, sp = alloc(spacer)
        held.extend(sp)
        held_bytes += step
        if extra is not None:
            extra += step
            n_extra += 1
        t = time_set(cand)
        times.append(t)
        if t < best_ms:
            held.append(best)
            best, best_ms = cand, t
        else:
            held.append(cand)
    return best, times, held


class PertShard:
    """One fit (kind 1/2/3) over one contiguous cell shard, resident on one GPU."""

    def __init__(self, kind: int, reads, gc, libs, n_libs: int, P: int, K: int, init: Dict[str, np.ndarray],
                 *, eta: Optional[EtaCodebook] = None, cn_obs=None, rep_obs=None,
                 lamb: Optional[float] = None, beta_means=None, rho_fixed=None, a_fixed: Optional[float] = None,
                 pi_init=None, device=None, lr: float = 0.05, betas=ADAM_BETAS, eps: float = ADAM_EPS,
                 is_root: bool = True, n_cells_total: Optional[int] = None,
                 allreduce: Optional[Callable[[torch.Tensor], None]] = None,
                 dirichlet_mode: str = "torch32", bins_per_tile: int = 0, variant: int = 3, fused: bool = False,
                 paired: bool = False, lib=None, comm: Optional[PertComm] = None,
                 placement: Optional[int] = None):
        self.lib = nat.lib() if lib is None else lib        # another build of the ABI (A/B tools)
        # the chunked SVI loop's handle: the product library through CDLL (the call releases the
        # GIL while it queues its launches); an A/B build keeps its own handle
        self._lib_chunk = nat.lib_nogil() if lib is None else (lib if hasattr(lib, "pert_svi_steps") else None)
        self.kind = int(kind)
        self.variant = int(variant)
        # one launch per SVI step (pert_enum_step): the three-wave pass of steps 2/3
        self.fused = bool(fused) and self.variant == 3 and self.kind != nat.KIND_STEP1
        self.device = torch.device(device if device is not None else "cuda")
        if self.device.type != "cuda":
            raise ValueError("PertShard needs a GPU device (got {})".format(self.device))
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        reads = np.asarray(reads)
        # step 1 pair mode (include/pert_hip.h): ``reads`` / ``cn_obs`` hold the G1/2 cells once;
        # the fit's cells are their rep-0 copies then their rep-1 copies (pert_model.py:228-251),
        # so ``libs`` and the per-cell entries of ``init`` are per copy (twice the columns)
        self.paired = bool(paired)
        if self.paired and (self.kind != nat.KIND_STEP1 or rep_obs is not None):
            raise ValueError("pair mode is step 1's doubled training set: kind 1, no rep_obs")
        L, NS = reads.shape
        N = 2 * NS if self.paired else NS
        self.L, self.N, self.P, self.K, self.K1, self.n_libs = L, N, int(P), int(K), int(K) + 1, int(n_libs)
        if not (nat.MIN_P <= self.P <= nat.MAX_P):
            raise ValueError("P={} unsupported (2..16)".format(P))
        if self.K1 > nat.MAX_K1:
            raise ValueError("K={} unsupported (K+1 <= 8)".format(K))
        self.n_cells_total = N if n_cells_total is None else int(n_cells_total)
        self.lr, self.betas, self.eps = float(lr), tuple(betas), float(eps)
        # a pert_comm communicator: the SVI loop (run_svi) queues the all-reduce in the library
        # (pert_svi_run_sharded); single steps and the set-up constants use it from here
        self.comm = comm
        self.allreduce = comm.allreduce if (comm is not None and allreduce is None) else allreduce
        self.t = 0
        self.last_launched = 0                 # iterations the last run_svi queued
        dev = self.device
        f32 = dict(dtype=torch.float32, device=dev)
        self.ldn = ldn = -(-NS // nat.BLOCK) * nat.BLOCK      # row stride: stored columns rounded up to 256

        # set-up timeline (seconds since the constructor began, per phase): timings["init"]
        _t0 = time.perf_counter()
        self.init_timings = {}
        # ---- inputs (pert_model.py:133-191 layouts)
        self.reads = self._pad_rows(torch.as_tensor(np.ascontiguousarray(reads, dtype=F32)), dev)
        self.gcf = gc_features(gc, self.K).to(dev).contiguous()
        self.libs = torch.as_tensor(np.asarray(libs).astype(np.int32), device=dev)
        mean_reads = torch.mean(torch.as_tensor(reads, dtype=torch.float32), dim=0)
        if self.paired:
            mean_reads = torch.cat([mean_reads, mean_reads])
        self.mean_reads = mean_reads.to(dev)
        if self.kind == nat.KIND_STEP1:
            ploidy = np.full(N, 2.0, dtype=F32)                                       # :595
        else:
            if eta is None:
                raise ValueError("steps 2/3 need the CN prior eta")
            if eta.P != self.P or eta.codes.shape != (L, N):
                raise ValueError("eta code book does not match (L, N, P)")
            ploidy = eta.ploidy()                                                      # :591-593
        self.ploidy = torch.as_tensor(ploidy, dtype=torch.float32, device=dev)

        self.eta = eta
        self.eta_code = self.eta_table = None
        self.cn_obs = self.rep_obs = None
        self.beta_means_t = self.rho_fixed_t = None
        lam_f = 0.0
        if self.kind == nat.KIND_STEP1:
            cn = np.asarray(cn_obs)
            if cn.min() < 0 or cn.max() >= self.P:
                raise ValueError("observed CN states must lie in [0, P)")
            self.cn_obs = self._pad_rows(torch.as_tensor(cn.astype(np.uint8)), dev)
            if not self.paired:
                self.rep_obs = self._pad_rows(torch.as_tensor(np.asarray(rep_obs).astype(np.uint8)), dev)
        else:
            self.eta_code = self._pad_rows(
                torch.as_tensor(np.ascontiguousarray(eta.codes, dtype=np.uint16).view(np.int16)), dev)
            # the site value rounded as the reference's fp32 log_prob rounds it when the host
            # adds the reference's fp32 normaliser ("torch32"), unrounded with the exact one
            self.eta_table = torch.as_tensor(eta.kernel_table(round_site=(dirichlet_mode == "torch32")),
                                             device=dev).contiguous()
            lam_f = float(np.asarray(lamb, dtype=F32).reshape(-1)[0])
            self.beta_means_t = torch.as_tensor(np.asarray(beta_means, dtype=F32).reshape(self.n_libs, self.K1),
                                                device=dev).contiguous()
            if self.kind == nat.KIND_STEP3:
                self.rho_fixed_t = torch.as_tensor(np.asarray(rho_fixed, dtype=F32).reshape(L), device=dev)
        self.lamb = lam_f

        self.init_timings["inputs"] = round(time.perf_counter() - _t0, 4)
        # ---- packed parameters (include/pert_hip.h pert_layout)
        self.lay = nat.make_layout(L, N, self.K1, self.n_libs)
        lay = self.lay
        if comm is not None and getattr(comm, "max_n", None) is not None and lay.n_shared + 1 > comm.max_n:
            raise ValueError("the shared block ({} doubles) exceeds the host communicator's max_n ({}): "
                             "make HostComm(max_n=...) larger".format(lay.n_shared + 1, comm.max_n))
        self.params = torch.zeros(lay.n_params, **f32)
        self.adam_m = torch.zeros(lay.n_params, **f32)
        self.adam_v = torch.zeros(lay.n_params, **f32)
        self.grad_shared = torch.zeros(lay.n_shared + 1, dtype=torch.float64, device=dev)
        # this shard's own shared-block sums (all-reduced into grad_shared when sharded)
        self.grad_local = torch.zeros_like(self.grad_shared) if self.allreduce is not None else self.grad_shared
        self.grad_cell = torch.zeros(lay.n_params - lay.n_shared, **f32)
        self._load_init(init)

        self.z_pi = self.m_pi = self.v_pi = None
        self.g_pi = None
        if self.kind != nat.KIND_STEP1:
            if pi_init is None:
                # AutoDelta init of the multivariate Dirichlet site: transform_to(simplex)(0) -> 1/P
                z0 = float(torch.log(torch.tensor(1.0 / self.P, dtype=torch.float32)))
                self.z_pi = torch.full((ldn // 64, L, self.P, 64), z0, **f32)
            else:
                pi0 = torch.as_tensor(np.asarray(pi_init), dtype=torch.float32)
                self.z_pi = self.to_tiles(pi0.log())                                   # SoftmaxTransform.inv
            self.m_pi = torch.zeros_like(self.z_pi)
            self.v_pi = torch.zeros_like(self.z_pi)
        self.cn_out = torch.zeros((L, ldn), dtype=torch.uint8, device=dev)
        self.rep_out = torch.zeros((L, ldn), dtype=torch.uint8, device=dev)

        self.pass_events = None      # list -> (start, end) HIP events around every pass
        self.pass_event_stride = 1   # (one-rank loop) events around every stride-th iteration's pass
        self._loop_bufs = None       # run_svi's control word / records / pinned host copy (reused)
        self._ctl_init = None

        self.init_timings["params"] = round(time.perf_counter() - _t0, 4)
        # ---- constants of the loss (added on the host, summed over ranks once)
        # (fp64 on the device, from the padded reads already there: zero columns add nothing; a
        # small shard on the host, where the device's first lgamma launch would cost more)
        big = L * NS >= 4_000_000
        src = self.reads if big else np.asarray(reads)
        if self.kind == nat.KIND_STEP1:
            copies = 2 if self.paired else 1
            kap, tot = kappa_and_sum(src, None)
            const = copies * kap + L * N * math.lgamma(self.P)   # Dirichlet(ones) normaliser
            self.sum_reads = copies * tot
            self.pi_block = CanonicalPiBlock(self.P, self.lr, self.betas, self.eps)
        else:
            # code counts from the device copy of the codes (int16 view of uint16)
            cnt = (torch.bincount((self.eta_code[:, :N].to(torch.int32) & 0xFFFF).reshape(-1),
                                  minlength=int(eta.table.shape[0])).cpu().numpy() if big else None)
            const = kappa_sum(src, math.log(lam_f)) + eta.dirichlet_normaliser(dirichlet_mode, counts=cnt)
            self.sum_reads = 0.0
            self.pi_block = None
        c = torch.tensor([const], dtype=torch.float64, device=dev)
        if self.allreduce is not None:
            self.allreduce(c)
        self.const_total = float(c.item())

        self.init_timings["constants"] = round(time.perf_counter() - _t0, 4)
        # ---- C structs
        self._prob = nat.PertProblem(
            kind=self.kind, L=L, N=N, P=self.P, K1=self.K1, n_libs=self.n_libs,
            n_codes=0 if eta is None else int(eta.table.shape[0]), ldn=ldn, is_root=1 if is_root else 0,
            reads=_ptr(self.reads), gcf=_ptr(self.gcf), libs=_ptr(self.libs), eta_code=_ptr(self.eta_code),
            eta_table=_ptr(self.eta_table), cn_obs=_ptr(self.cn_obs), rep_obs=_ptr(self.rep_obs),
            mean_reads=_ptr(self.mean_reads), ploidy=_ptr(self.ploidy), lamb=lam_f,
            log1m_lam=(math.log1p(-lam_f) if self.kind != nat.KIND_STEP1 else 0.0),
            sum_reads=self.sum_reads, a_fixed=float(a_fixed) if a_fixed is not None else 0.0,
            beta_means=_ptr(self.beta_means_t), rho_fixed=_ptr(self.rho_fixed_t))
        if bins_per_tile <= 0:
            with self._dev():
                bins_per_tile = nat.auto_bins_per_tile(self._prob, variant, self.lib)
        ncp, nbp, nblk, ncb = nat.workspace_sizes(self.kind, L, N, self.K1, self.n_libs, bins_per_tile)
        self.cell_part = torch.zeros(ncp, **f32)
        self.bin_part = torch.zeros(nbp, **f32)
        self.blk_part = torch.zeros(nblk, dtype=torch.float64, device=dev)
        self.cellblk_part = torch.zeros(ncb, dtype=torch.float64, device=dev)
        self.bins_per_tile = int(bins_per_tile)
        self._state = nat.PertState(
            lay=lay, params=_ptr(self.params), adam_m=_ptr(self.adam_m), adam_v=_ptr(self.adam_v),
            grad_shared=_ptr(self.grad_shared), grad_cell=_ptr(self.grad_cell), z_pi=_ptr(self.z_pi),
            m_pi=_ptr(self.m_pi), v_pi=_ptr(self.v_pi), g_pi=0, cn_out=_ptr(self.cn_out),
            rep_out=_ptr(self.rep_out), cell_part=_ptr(self.cell_part), bin_part=_ptr(self.bin_part),
            blk_part=_ptr(self.blk_part), cellblk_part=_ptr(self.cellblk_part),
            bins_per_tile=self.bins_per_tile, variant=int(variant))
        self._hp = nat.PertAdamHparams(lr=self.lr, beta1=self.betas[0], beta2=self.betas[1], eps=self.eps,
                                       step_size=0.0, inv_bc2_sqrt=0.0)
        self.init_timings["structs"] = round(time.perf_counter() - _t0, 4)
        self.placement = None        # the pi-state placement search's record (choose_pi_placement)
        if placement is None:
            placement = int(os.environ.get("PERT_PLACEMENT", str(PLACEMENT_CANDIDATES)))
        if placement > 1 and self.z_pi is not None and self.variant == 3 and \
                self.z_pi.numel() >= PLACEMENT_MIN_FLOATS:
            self.choose_pi_placement(placement)
        self.init_timings["placement"] = round(time.perf_counter() - _t0, 4)

    # ------------------------------------------------------------------ layouts
    def _pad_rows(self, a: torch.Tensor, dev) -> torch.Tensor:
        """(L, N) -> (L, ldn) zero-padded device copy (include/pert_hip.h row stride): the
        compact array is copied to the device and padded there."""
        out = torch.zeros((a.shape[0], self.ldn), dtype=a.dtype, device=dev)
        out[:, :a.shape[1]] = a.to(dev)
        return out

    def to_tiles(self, a: torch.Tensor) -> torch.Tensor:
        """(L, N, P) -> wave tiles (ldn/64, L, P, 64) on the device."""
        L, N, P = a.shape
        pad = torch.zeros((L, self.ldn, P), dtype=a.dtype)
        pad[:, :N] = a
        return pad.reshape(L, self.ldn // 64, 64, P).permute(1, 0, 3, 2).contiguous().to(self.device)

    def from_tiles(self, t: torch.Tensor) -> torch.Tensor:
        """Wave tiles (ldn/64, L, P, 64) -> (L, N, P)."""
        L = t.shape[1]
        return t.permute(1, 0, 3, 2).reshape(L, self.ldn, self.P)[:, :self.N]

    # ------------------------------------------------------------------ params
    def _load_init(self, init: Dict[str, np.ndarray]):
        lay, L, N, K1, nl = self.lay, self.L, self.N, self.K1, self.n_libs
        p = torch.zeros(lay.n_params, dtype=torch.float32)

        def t32(v):
            return torch.as_tensor(np.asarray(v, dtype=np.float64), dtype=torch.float32)
        if self.kind != nat.KIND_STEP3:
            p[lay.off_rho:lay.off_rho + L] = sigmoid_inv(t32(init["expose_rho"]).reshape(L))
            p[lay.off_a] = torch.log(t32(init["expose_a"]).reshape(-1)[0])
        if self.kind == nat.KIND_STEP1:
            lam = t32(init["expose_lambda"]).reshape(-1)[0]
            p[lay.off_lam] = sigmoid_inv((lam - 0.001) / 0.998)
            p[lay.off_bmeans:lay.off_bmeans + nl * K1] = t32(init["expose_beta_means"]).reshape(-1)
        p[lay.off_bstds:lay.off_bstds + nl * K1] = torch.log(t32(init["expose_beta_stds"]).reshape(-1))
        p[lay.off_u:lay.off_u + N] = t32(init["expose_u"]).reshape(N)
        p[lay.off_beta:lay.off_beta + K1 * N] = t32(init["expose_betas"]).reshape(N, K1).t().reshape(-1)
        p[lay.off_tau:lay.off_tau + N] = sigmoid_inv(t32(init["expose_tau"]).reshape(N))
        self.params.copy_(p.to(self.device))

    def set_unconstrained(self, z: Dict[str, np.ndarray]):
        """Overwrite the state with explicit unconstrained values (oracle site names)."""
        lay, L, N, K1, nl = self.lay, self.L, self.N, self.K1, self.n_libs
        p = self.params.cpu()

        def t32(v):
            return torch.as_tensor(np.asarray(v, dtype=np.float64), dtype=torch.float32)
        if "expose_rho" in z:
            p[lay.off_rho:lay.off_rho + L] = t32(z["expose_rho"]).reshape(L)
        if "expose_a" in z:
            p[lay.off_a] = t32(z["expose_a"]).reshape(-1)[0]
        if "expose_lambda" in z:
            p[lay.off_lam] = t32(z["expose_lambda"]).reshape(-1)[0]
        if "expose_beta_means" in z and self.kind == nat.KIND_STEP1:
            p[lay.off_bmeans:lay.off_bmeans + nl * K1] = t32(z["expose_beta_means"]).reshape(-1)
        p[lay.off_bstds:lay.off_bstds + nl * K1] = t32(z["expose_beta_stds"]).reshape(-1)
        p[lay.off_u:lay.off_u + N] = t32(z["expose_u"]).reshape(N)
        p[lay.off_beta:lay.off_beta + K1 * N] = t32(z["expose_betas"]).reshape(N, K1).t().reshape(-1)
        p[lay.off_tau:lay.off_tau + N] = t32(z["expose_tau"]).reshape(N)
        self.params.copy_(p.to(self.device))
        if "expose_pi" in z and self.z_pi is not None:
            self.z_pi.copy_(self.to_tiles(t32(z["expose_pi"])))

    def unconstrained(self, pi_cells=None) -> Dict[str, np.ndarray]:
        """The unconstrained fp32 storage (oracle site names; inverse of set_unconstrained).
        ``pi_cells``: include the pi logits of these cells, (L, len, P)."""
        lay, L, N, K1, nl = self.lay, self.L, self.N, self.K1, self.n_libs
        p = self.params.cpu().numpy()
        z = {}
        if self.kind != nat.KIND_STEP3:
            z["expose_rho"] = p[lay.off_rho:lay.off_rho + L].reshape(L, 1).copy()
            z["expose_a"] = p[lay.off_a:lay.off_a + 1].copy()
        if self.kind == nat.KIND_STEP1:
            z["expose_lambda"] = p[lay.off_lam:lay.off_lam + 1].copy()
            z["expose_beta_means"] = p[lay.off_bmeans:lay.off_bmeans + nl * K1].reshape(nl, K1).copy()
        z["expose_beta_stds"] = p[lay.off_bstds:lay.off_bstds + nl * K1].reshape(nl, K1).copy()
        z["expose_u"] = p[lay.off_u:lay.off_u + N].copy()
        z["expose_betas"] = p[lay.off_beta:lay.off_beta + K1 * N].reshape(K1, N).T.copy()
        z["expose_tau"] = p[lay.off_tau:lay.off_tau + N].copy()
        if pi_cells is not None and self.z_pi is not None:
            zp = self.from_tiles(self.z_pi)[:, torch.as_tensor(np.asarray(pi_cells), device=self.device)]
            z["expose_pi"] = zp.cpu().numpy()
        return z

    def constrained(self) -> Dict[str, np.ndarray]:
        """Current constrained site values (what the reference's trace exposes)."""
        lay, L, N, K1, nl = self.lay, self.L, self.N, self.K1, self.n_libs
        p = self.params.cpu()
        out = {}
        if self.kind != nat.KIND_STEP3:
            out["expose_rho"] = clipped_sigmoid(p[lay.off_rho:lay.off_rho + L]).numpy().reshape(L, 1)
            out["expose_a"] = torch.exp(p[lay.off_a:lay.off_a + 1]).numpy()
        if self.kind == nat.KIND_STEP1:
            out["expose_lambda"] = (0.001 + 0.998 * clipped_sigmoid(p[lay.off_lam:lay.off_lam + 1])).numpy()
            out["expose_beta_means"] = p[lay.off_bmeans:lay.off_bmeans + nl * K1].numpy().reshape(nl, K1)
        out["expose_beta_stds"] = torch.exp(p[lay.off_bstds:lay.off_bstds + nl * K1]).numpy().reshape(nl, K1)
        out["expose_u"] = p[lay.off_u:lay.off_u + N].numpy().copy()
        out["expose_betas"] = p[lay.off_beta:lay.off_beta + K1 * N].numpy().reshape(K1, N).T.copy()
        out["expose_tau"] = clipped_sigmoid(p[lay.off_tau:lay.off_tau + N]).numpy()
        return out

    def pi(self) -> torch.Tensor:
        """Constrained pi (L, N, P) on the device (SoftmaxTransform of the logits)."""
        return self.from_tiles(torch.softmax(self.z_pi, dim=2))   # P is dim 2 of the tiles

    # ------------------------------------------------------------------ launches
    def _stream(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream

    def _set_hparams(self, t: int):
        b1, b2 = self.betas
        self._hp.step_size = self.lr / (1.0 - b1 ** t)
        self._hp.inv_bc2_sqrt = 1.0 / math.sqrt(1.0 - b2 ** t)

    def _dev(self):
        """Device guard only when the current device differs (the common case costs nothing)."""
        if torch.cuda.current_device() == self.device.index:
            return contextlib.nullcontext()
        return torch.cuda.device(self.device)

    def _pass(self, mode: int):
        s = self._stream()
        with self._dev():
            if self.kind == nat.KIND_STEP1:
                nat.check(self.lib.pert_obs_pass(ctypes.byref(self._prob), ctypes.byref(self._state), s),
                          "pert_obs_pass")
            else:
                nat.check(self.lib.pert_enum_pass(ctypes.byref(self._prob), ctypes.byref(self._state),
                                                  ctypes.byref(self._hp), mode, s), "pert_enum_pass")

    def stream_ceiling_ms(self, reps: int = 10) -> float:
        """Mean duration (HIP events, current stream) of pert_stream_ceiling: the STEP pass's
        HBM streams with no arithmetic, on this shard's own buffers and tile grid (the state
        is unchanged).  The pass's time over this one is its fraction of the pattern's
        ceiling on the running device."""
        assert self.kind != nat.KIND_STEP1 and self.z_pi is not None
        s = self._stream()
        with self._dev():
            nat.check(self.lib.pert_stream_ceiling(ctypes.byref(self._prob), ctypes.byref(self._state), s),
                      "pert_stream_ceiling")
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                nat.check(self.lib.pert_stream_ceiling(ctypes.byref(self._prob), ctypes.byref(self._state), s),
                          "pert_stream_ceiling")
            e1.record()
            e1.synchronize()
        return e0.elapsed_time(e1) / reps

    def _set_pi_ptrs(self, z: torch.Tensor, m: torch.Tensor, v: torch.Tensor):
        self._state.z_pi, self._state.m_pi, self._state.v_pi = _ptr(z), _ptr(m), _ptr(v)

    def choose_pi_placement(self, candidates: int = PLACEMENT_CANDIDATES) -> dict:
        """Pick where the pi state (z / m / v, 97 % of the pass's bytes) lives in HBM.

        The pass's read-modify-write pattern streams at 5.1-5.3 TB/s from some physical
        placements of the three arrays and at 5.9-6.3 TB/s from others; which one an allocation
        gets is not selectable (relative offsets, contiguity and size make no difference:
        DESIGN.md section 5), but it is fixed once allocated and measurable in a few passes'
        time.  So: time pert_stream_ceiling (the pass's own streams on this shard's grid, values
        written back unchanged) on the current arrays; while that is slower than
        PLACEMENT_FAST_RATE, allocate another set (the earlier ones held, so it lands elsewhere)
        and time it, up to ``candidates`` sets, and PLACEMENT_EXTRA more (at most
        PLACEMENT_EXTRA_BYTES) once one is fast unless one streams at PLACEMENT_TOP_RATE (fast placements come at two
        rates); move the state into the fastest and free the rest
        (``placement_search``).  Results do not depend on the placement (same data, same
        kernel).  Returns (and keeps in ``self.placement``) the candidates' times and the
        choice."""
        cells = -(-self.N // 64) * 64
        pattern_bytes = float(cells) * self.L * (6.0 + 24.0 * self.P)
        set_bytes = 3 * self.z_pi.numel() * 4

        def timed() -> float:
            s = self._stream()
            with self._dev():
                nat.check(self.lib.pert_stream_ceiling(ctypes.byref(self._prob), ctypes.byref(self._state), s),
                          "pert_stream_ceiling")
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(2):
                    nat.check(self.lib.pert_stream_ceiling(ctypes.byref(self._prob), ctypes.byref(self._state),
                                                           s), "pert_stream_ceiling")
                e1.record()
                e1.synchronize()
            return e0.elapsed_time(e1) / 2

        first = (self.z_pi, self.m_pi, self.v_pi)

        def time_set(cand) -> float:
            self._set_pi_ptrs(*cand)
            return timed()

        def alloc(spacer: int):
            held = [torch.empty(spacer, dtype=torch.uint8, device=self.device)] if spacer else []
            return tuple(torch.empty_like(self.z_pi) for _ in range(3)), held

        try:
            best, times, held = placement_search(first, time_set, alloc,
                                                 lambda: torch.cuda.mem_get_info(self.device)[0],
                                                 set_bytes, pattern_bytes, candidates)
        except torch.cuda.OutOfMemoryError as e:
            # another allocation on the device (a helper's step-3 work, another fit) took the
            # room the tries assumed: keep the first set -- the search only ever speeds the
            # pass up, results do not depend on it -- and give the tries back
            self._set_pi_ptrs(*first)
            torch.cuda.synchronize(self.device)
            torch.cuda.empty_cache()
            self.placement = {"candidates_ms": None, "chosen": 0, "error": "OutOfMemoryError: {}".format(
                str(e).splitlines()[0][:200])}
            return self.placement
        best_ms = min(times)
        if best is not first:
            for dst, src in zip(best, first):
                dst.copy_(src)
        self.z_pi, self.m_pi, self.v_pi = best
        self._set_pi_ptrs(*best)
        del held, first
        if len(times) > 1:
            torch.cuda.synchronize(self.device)
            torch.cuda.empty_cache()             # the tries and spacers back to the device
        self.placement = {"candidates_ms": [round(t, 4) for t in times], "chosen": times.index(best_ms),
                          "pattern_tbs": round(pattern_bytes / (best_ms * 1e-3) / 1e12, 3)}
        return self.placement

    def _finalize(self):
        """Reductions of the pass partials; with a process group, the shard's shared block is
        written to ``grad_local`` and the all-reduce runs on a fresh copy of it, so the sum is
        idempotent: a launch the device loop has already stopped leaves grad_local unchanged
        and re-reducing it gives the same grad_shared (no world-size blow-up)."""
        st = self._state
        if self.allreduce is not None:
            st.grad_shared = _ptr(self.grad_local)
        with self._dev():
            nat.check(self.lib.pert_finalize(ctypes.byref(self._prob), ctypes.byref(st), self._stream()),
                      "pert_finalize")
        if self.allreduce is not None:
            st.grad_shared = _ptr(self.grad_shared)
            self.grad_shared.copy_(self.grad_local)
            self.allreduce(self.grad_shared)

    def step_async(self):
        """One SVI step without reading the loss back (the loss stays on the device)."""
        self.t += 1
        self._launch_step(self.t)
        if self.pi_block is not None:
            self._pi_lp = self.pi_block.step(self.t)

    def _fused_step(self):
        """Steps 2/3 with the three-wave pass: one launch (pert_enum_step) does the pass, the
        reductions and the Adam updates; sharded, the launch stops at the shared block's sums,
        which are all-reduced before pert_adam_shared."""
        st = self._state
        s = self._stream()
        with self._dev():
            if self.allreduce is None:
                nat.check(self.lib.pert_enum_step(ctypes.byref(self._prob), ctypes.byref(st), ctypes.byref(self._hp),
                                                  1, s), "pert_enum_step")
                return
            st.grad_shared = _ptr(self.grad_local)
            try:
                nat.check(self.lib.pert_enum_step(ctypes.byref(self._prob), ctypes.byref(st), ctypes.byref(self._hp),
                                                  0, s), "pert_enum_step")
            finally:
                st.grad_shared = _ptr(self.grad_shared)
            self.grad_shared.copy_(self.grad_local)
            self.allreduce(self.grad_shared)
            nat.check(self.lib.pert_adam_shared(ctypes.byref(self._prob), ctypes.byref(st), ctypes.byref(self._hp),
                                                self._stream()), "pert_adam_shared")

    def _launch_step(self, t: int):
        """Queue the launch sequence of Adam step t (1-based) on the current stream."""
        self._set_hparams(t)
        if self.fused:
            if self.pass_events is not None:
                ev0 = torch.cuda.Event(enable_timing=True)
                ev1 = torch.cuda.Event(enable_timing=True)
                ev0.record()
                self._fused_step()
                ev1.record()
                self.pass_events.append((ev0, ev1))
            else:
                self._fused_step()
            return
        if self.pass_events is not None:
            ev0 = torch.cuda.Event(enable_timing=True)
            ev1 = torch.cuda.Event(enable_timing=True)
            ev0.record()
            self._pass(nat.MODE_STEP)
            ev1.record()
            self.pass_events.append((ev0, ev1))
        else:
            self._pass(nat.MODE_STEP)
        self._finalize()
        with self._dev():
            nat.check(self.lib.pert_adam(ctypes.byref(self._prob), ctypes.byref(self._state),
                                         ctypes.byref(self._hp), self._stream()), "pert_adam")

    def _loop_buffers(self, n: int):
        """The device loop's control word, its per-iteration loss records and their pinned host
        copy, kept between fits of this shard (a pinned allocation costs far more than a step
        of a small shard); grown to the next power of two when a fit needs more."""
        cap = 0 if self._loop_bufs is None else self._loop_bufs[1].shape[0]
        if n > cap:
            cap = 1 << max(6, (n - 1).bit_length())
            self._loop_bufs = (torch.empty(2, dtype=torch.int32, device=self.device),
                               torch.empty((cap, 2), dtype=torch.float64, device=self.device),
                               torch.empty((cap, 2), dtype=torch.float64, pin_memory=True))
            self._ctl_init = torch.tensor([-1, 0], dtype=torch.int32, device=self.device)
        return self._loop_bufs

    def _adam_schedule(self, t0: int, n: int):
        """Adam's bias-corrected step sizes of steps t0+1 .. t0+n as _set_hparams computes them
        (``lr / (1 - b1^t)``, ``1 / sqrt(1 - b2^t)``, Python floats cast to fp32), from a table
        kept on the shard (a fit's call no longer loops over its steps in Python)."""
        tab = self.__dict__.get("_adam_tab")
        if tab is None or tab[0].shape[0] < t0 + n + 1:
            cap = 1 << max(10, (t0 + n).bit_length())
            b1, b2 = self.betas
            ss = np.zeros(cap + 1, dtype=F32)
            ib = np.zeros(cap + 1, dtype=F32)
            ss[1:] = [self.lr / (1.0 - b1 ** t) for t in range(1, cap + 1)]
            ib[1:] = [1.0 / math.sqrt(1.0 - b2 ** t) for t in range(1, cap + 1)]
            tab = self._adam_tab = (ss, ib)
        return tab[0][t0 + 1:t0 + n + 1], tab[1][t0 + 1:t0 + n + 1]

    def _timing_event(self):
        """A timing event from the pool reserve_svi fills (created and recorded once, so its HIP
        event exists), or a new one."""
        pool = self.__dict__.setdefault("_event_pool", [])
        if pool:
            return pool.pop()
        e = torch.cuda.Event(enable_timing=True)
        e.record()                                  # creates the HIP event behind it
        return e

    def reserve_svi(self, n: int) -> None:
        """Set up everything a run_svi(n) from the current step allocates or computes on the
        host -- its loop buffers and, for step 1, the canonical pi trajectory -- ahead of the
        call (run_pert_model computes the trajectory on its helper thread during the prep;
        bench.py calls this before its timed region)."""
        self._loop_buffers(int(n))
        self._adam_schedule(self.t, int(n))
        if self.pi_block is not None:
            self.pi_block._cache(self.t + int(n) + 1)
        if self.pass_events is not None:            # the timing events a run_svi(n) will record
            need = 2 * len(range(0, int(n), max(1, self.pass_event_stride)))
            pool = self.__dict__.setdefault("_event_pool", [])
            while len(pool) < need:
                e = torch.cuda.Event(enable_timing=True)
                e.record()
                pool.append(e)

    def run_svi(self, max_iter: int, min_iter: int, rel_tol: float, chunk: int = 8, depth: int = 8):
        """The SVI loop of pert_model.py:742-758 (:800-816, :867-883) without a per-step host
        synchronisation.  Every iteration's loss is recorded on the device and the reference's
        stopping rule (rel-tol plateau after min_iter, NaN) is evaluated there
        (include/pert_hip.h, loop_ctl); launches of iterations after the stopping one are
        no-ops.  The host queues iterations ahead, copies the loss records back every
        ``chunk`` iterations and stops queueing once a copied record shows the stop (it is
        at most ``chunk * depth`` iterations ahead: 64 by default).  On one rank that whole
        loop runs inside one C call (pert_svi_run) with the GIL released, so the helper
        thread's host work never stands between two chunks.  Returns (losses, reason) with
        reason 0 = max_iter reached, 1 = converged, 2 = NaN loss; the fit state is the one
        after the last recorded iteration, exactly as if the loop had run on the host."""
        n = int(max_iter)
        self.last_launched = 0
        if n <= 0:
            return [], 0
        dev = self.device
        ctl, rec, host = self._loop_buffers(n)
        ctl.copy_(self._ctl_init, non_blocking=True)
        offs = None
        t0 = self.t
        if self.pi_block is not None:
            lps = self.pi_block.trajectory(t0 + 1, n)
            offs = torch.as_tensor(float(self.L * self.n_cells_total) * lps, dtype=torch.float64, device=dev)
        st = self._state
        st.loop_ctl, st.loop_rec, st.loss_offset = _ptr(ctl), _ptr(rec), _ptr(offs)
        st.loss_const, st.rel_tol, st.min_iter = float(self.const_total), float(rel_tol), int(min_iter)
        # one rank, or ranks joined by a pert_comm: the whole loop is ONE C call (pert_svi_run /
        # pert_svi_run_sharded, the all-reduce queued by the library) that releases the GIL for
        # the fit's duration -- a helper thread's Python work never delays the queueing of steps;
        # per-pass timing events (pass_events, bench.py) are recorded by that call around the
        # passes of every pass_event_stride-th iteration.  Sharded over another process group
        # (gloo): per iteration from Python (torch.distributed's all-reduce sits between the
        # reductions and Adam)
        native_comm = self.comm is not None and self.allreduce == self.comm.allreduce
        native = (self.allreduce is None or native_comm) and self._lib_chunk is not None
        shard_args = (self.comm.handle, _ptr(self.grad_local)) if native_comm else ()
        b1, b2 = self.betas
        launched = 0
        pending = []
        try:
            if native:
                ss, ib = self._adam_schedule(t0, n)
                evp, sampled = None, []
                if self.pass_events is not None:
                    ptrs = [None] * (2 * n)
                    for i in range(0, n, max(1, self.pass_event_stride)):
                        e0, e1 = self._timing_event(), self._timing_event()
                        ptrs[2 * i], ptrs[2 * i + 1] = e0.cuda_event, e1.cuda_event
                        sampled.append((i, e0, e1))
                    evp = (ctypes.c_void_p * len(ptrs))(*ptrs)
                nl = ctypes.c_int32(0)
                fn = self._lib_chunk.pert_svi_run_sharded if native_comm else self._lib_chunk.pert_svi_run
                with self._dev():
                    rc = fn(ctypes.byref(self._prob), ctypes.byref(st), ctypes.byref(self._hp),
                            ss.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                            ib.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), n, chunk, depth,
                            1 if self.fused else 0, *shard_args, evp, host.data_ptr(), ctypes.byref(nl),
                            self._stream())
                launched = int(nl.value)
                self.last_launched = launched          # (also when the loop failed)
                nat.check(rc, "pert_svi_run")
                # the stop from the copied records (every launched iteration's record is in
                # pinned memory once the call returns; the first marked one is the stop --
                # loop_ctl[0] -- and a NaN loss there is reason 2), no device read-back
                marks = host[:launched, 1]
                hit = torch.nonzero(marks >= 0)
                if hit.numel():
                    j = int(hit[0, 0])
                    c = (j, 2 if math.isnan(float(host[j, 0])) else 1)
                else:
                    c = (-1, 0)
                if self.pass_events is not None:       # (iterations never queued recorded nothing)
                    self.pass_events.extend((e0, e1) for i, e0, e1 in sampled if i < launched)
                n = 0                              # nothing left for the per-iteration loop below
            for j0 in range(0, n, chunk):
                j1 = min(n, j0 + chunk)
                for i in range(j0, j1):
                    st.step = i
                    self._launch_step(t0 + i + 1)
                launched = self.last_launched = j1
                host[j0:j1].copy_(rec[j0:j1], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record()
                pending.append((j0, j1, ev))
                stop_seen = False
                while len(pending) > depth:
                    a, b, e = pending.pop(0)
                    e.synchronize()
                    stop_seen = stop_seen or bool((host[a:b, 1] >= 0).any())
                if stop_seen:
                    break
            if not native:
                c = ctl.cpu()                  # waits for every queued launch and copy
        finally:
            st.loop_ctl = st.loop_rec = st.loss_offset = None
            st.step = 0
        stop_at, reason = int(c[0]), int(c[1])
        n_done = stop_at + 1 if stop_at >= 0 else launched
        losses = host[:n_done, 0].tolist()          # (copied out: the buffer is reused by the next fit)
        self.t = t0 + n_done
        if self.pi_block is not None and n_done > 0:
            self._pi_lp = self.pi_block.advance_to(t0 + n_done)
        return losses, (reason if stop_at >= 0 else 0)

    def device_loss(self) -> float:
        """Loss of the last step: -(ELBO) with the host constants (pert_model.py:743 return value),
        accumulated in fp64 and returned as the fp32 value ``float(loss)`` gives the reference."""
        loss = float(self.grad_shared[self.lay.n_shared].item()) - self.const_total
        if self.pi_block is not None:
            loss -= self.L * self.n_cells_total * self._pi_lp
        return float(np.float32(loss))

    def step(self) -> float:
        self.step_async()
        return self.device_loss()

    def loss_and_grads(self, pi_cells=None):
        """-ELBO and d(-ELBO)/dz at the current point, without updating (parity tests).
        ``pi_cells``: return the pi-logit gradient of these cells only (L, len, P) -- the
        full (L, N, P) array is not copied to the host."""
        if self.kind != nat.KIND_STEP1:
            if self.g_pi is None:
                self.g_pi = torch.zeros_like(self.z_pi)
                self._state.g_pi = _ptr(self.g_pi)
            self._pass(nat.MODE_GRAD)
        else:
            self._pass(nat.MODE_GRAD)
        self._finalize()
        lay, L, N, K1, nl = self.lay, self.L, self.N, self.K1, self.n_libs
        gs = self.grad_shared.cpu().numpy()
        gc = self.grad_cell.cpu().numpy()
        off = lay.n_shared
        g = {}
        if self.kind != nat.KIND_STEP3:
            g["expose_rho"] = gs[lay.off_rho:lay.off_rho + L].reshape(L, 1)
            g["expose_a"] = gs[lay.off_a:lay.off_a + 1]
        if self.kind == nat.KIND_STEP1:
            g["expose_lambda"] = gs[lay.off_lam:lay.off_lam + 1]
            g["expose_beta_means"] = gs[lay.off_bmeans:lay.off_bmeans + nl * K1].reshape(nl, K1)
        g["expose_beta_stds"] = gs[lay.off_bstds:lay.off_bstds + nl * K1].reshape(nl, K1)
        g["expose_u"] = gc[lay.off_u - off:lay.off_u - off + N]
        g["expose_betas"] = gc[lay.off_beta - off:lay.off_beta - off + K1 * N].reshape(K1, N).T
        g["expose_tau"] = gc[lay.off_tau - off:lay.off_tau - off + N]
        if self.kind != nat.KIND_STEP1:
            gp = self.from_tiles(self.g_pi)
            if pi_cells is not None:
                gp = gp[:, torch.as_tensor(np.asarray(pi_cells), device=gp.device)]
            g["expose_pi"] = gp.cpu().numpy()
        loss = float(gs[lay.n_shared]) - self.const_total
        if self.pi_block is not None:
            lp, gpi = self.pi_block.logp_and_grad()
            loss -= L * self.n_cells_total * lp
        return loss, g

    def decode(self):
        """MAP (cn, rep) per (bin, cell): infer_discrete(temperature=0) (pert_model.py:820-827)."""
        if self.kind == nat.KIND_STEP1:
            raise ValueError("step 1 has no latent discrete sites")
        self._pass(nat.MODE_DECODE)
        return self.cn_out[:, :self.N], self.rep_out[:, :self.N]

"""GPU: the public entry point under torch.distributed -- pert_infer_scRT.run_pert_model()
with two gloo ranks sharing one GPU (pert_model._Dist: all three fits cell-sharded, one
all-reduce per step, the decodes gathered so every rank returns the full output tables)
against the single-process fit.  (Runs last: the spawned ranks make it the slowest GPU test.)
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _tables():
    from scdna_replication_tools_amd.simulator import simulate, to_long_form
    sim = simulate(n_s=70, n_g=60, n_bins=300, num_reads=183 * 300, seed=23)
    return to_long_form(sim, n_libs=2)


def _fit(timings=None, **extra):
    from scdna_replication_tools.pert_model import pert_infer_scRT
    s, g = _tables()
    m = pert_infer_scRT(s, g, input_col='reads', clone_col='clone_id', cn_prior_method='g1_clones',
                        max_iter=120, min_iter=30, max_iter_step1=80, max_iter_step3=60, **extra)
    out = m.run_pert_model()
    if timings is not None:
        timings.update({k: v for k, v in m.timings.items() if isinstance(v, float)})
        for k in ("tau_init_s", "tau_init_g"):          # the initialiser's cells: the rank's own
            timings[k + "_cells"] = float(m.timings.get(k, {}).get("cells", -1))
    return out


def _api_worker(rank, world, port, out_dir, comm="torch", fault=None):
    import faulthandler
    import sys
    import time
    # a hung rank shows where, well before the test's own deadline (90 s) and any runner limit
    faulthandler.dump_traceback_later(60, exit=True, file=sys.stderr)
    if comm == "host":                   # the library's C loop with its host-staged communicator
        os.environ["PERT_NATIVE_COMM"] = "host"
    if fault is not None:
        os.environ["PERT_COMM_FAULT_AT"] = fault
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:{}".format(port), rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        tm = {}
        if fault is not None:
            from scdna_replication_tools_amd._native import CommError
            try:
                _fit(timings=tm, device="cuda:0")
                got = {"raised": -1}
            except CommError as e:
                got = {"raised": e.code}
            got["t_raise"] = time.time()
            torch.save(got, os.path.join(out_dir, "fault{}.pt".format(rank)))
            return
        from scdna_replication_tools.pert_model import pert_infer_scRT
        launched = {}
        orig = pert_infer_scRT.run_pert_model

        def run(self):                    # the iterations each fit queued on this rank
            try:
                return orig(self)
            finally:
                launched.update(self.launched)
        pert_infer_scRT.run_pert_model = run
        cn_s, supp_s, cn_g, supp_g = _fit(timings=tm, device="cuda:0")
        cols = ["model_cn_state", "model_rep_state", "model_tau", "model_u", "model_rho"]
        torch.save({"s": torch.as_tensor(cn_s[cols].to_numpy(np.float64)),
                    "g": torch.as_tensor(cn_g[cols].to_numpy(np.float64)),
                    "loss_s": torch.as_tensor(supp_s.loc[supp_s.param == "loss_s", "value"].to_numpy(np.float64)),
                    "loss_g": torch.as_tensor(supp_s.loc[supp_s.param == "loss_g", "value"].to_numpy(np.float64)),
                    "timings": tm, "launched": launched},
                   os.path.join(out_dir, "api{}.pt".format(rank)))
    finally:
        dist.destroy_process_group()


def _spawn(tmp_path, comm, fault=None):
    import time
    ctx = mp.spawn(_api_worker, args=(2, _free_port(), str(tmp_path), comm, fault), nprocs=2, join=False)
    deadline = time.time() + 90           # bounded: a hung rank fails the test instead of the suite
    while not ctx.join(timeout=5):
        if time.time() > deadline:
            for p in ctx.processes:
                if p.is_alive():
                    p.kill()
            pytest.fail("the two ranks did not finish within 90 s")


def test_fault_on_rank1_stops_rank0_through_the_library_loop(tmp_path):
    """PERT_COMM_FAULT_AT=1:30: rank 1's all-reduce call 30 (inside step 1's fit) fails; rank 1
    raises CommError, raises the abort word, and rank 0 -- waiting on its stream inside the C
    loop -- raises CommError too, within 10 s, instead of hanging."""
    from scdna_replication_tools_amd import _native as nat
    _spawn(tmp_path, "host", fault="1:30")
    r = [torch.load(str(tmp_path / "fault{}.pt".format(i)), weights_only=True) for i in range(2)]
    assert r[1]["raised"] == nat.E_COMM_FAULT, r[1]
    assert r[0]["raised"] == nat.E_COMM_ABORTED, r[0]
    assert abs(r[0]["t_raise"] - r[1]["t_raise"]) < 10.0
    print("rank 0 raised {:.3f} s after rank 1".format(r[0]["t_raise"] - r[1]["t_raise"]))


@pytest.mark.parametrize("comm", ["torch", "host"])
def test_run_pert_model_two_ranks_match_single_rank(tmp_path, comm):
    """The public entry point under torch.distributed (pert_model._Dist): each fit is
    cell-sharded over the two ranks with the all-reduce per step, every rank returns the full
    output tables -- equal to the single-process fit's (losses to summation-order noise,
    calls and per-cell sites).  comm="torch": the per-step Python loop over gloo; "host": the
    product's one-call C loop (pert_svi_run_sharded) over the library's host-staged
    communicator, the loop an RCCL node runs -- and both ranks queue the same chunks."""
    _spawn(tmp_path, comm)
    r = [torch.load(str(tmp_path / "api{}.pt".format(i)), weights_only=True) for i in range(2)]
    tm1 = {}
    cn_s, supp_s, cn_g, supp_g = _fit(timings=tm1)
    from tests._bounds import write_report
    keys = ("helper_guess_times_s", "helper_guess_times_g", "helper_priors", "total", "tau_init_s_cells",
            "tau_init_g_cells")
    write_report("api_two_ranks_timings", {"one_rank": {k: tm1.get(k) for k in keys},
                                           "rank0": {k: r[0]["timings"].get(k) for k in keys},
                                           "rank1": {k: r[1]["timings"].get(k) for k in keys}})
    # each rank initialised tau for its own cells only (pert_model: per-rank host work)
    for i in range(2):
        assert r[i]["timings"]["tau_init_s_cells"] == 35 and r[i]["timings"]["tau_init_g_cells"] == 30
    cols = ["model_cn_state", "model_rep_state", "model_tau", "model_u", "model_rho"]
    for i in range(2):
        for name, ref in (("s", cn_s), ("g", cn_g)):
            got = r[i][name].numpy()
            want = ref[cols].to_numpy(np.float64)
            assert got.shape == want.shape
            assert ((got[:, 0] == want[:, 0]) & (got[:, 1] == want[:, 1])).mean() >= 0.999
            np.testing.assert_allclose(got[:, 2:], want[:, 2:], rtol=2e-3, atol=1e-4)
        ls = supp_s.loc[supp_s.param == "loss_s", "value"].to_numpy(np.float64)
        lg = supp_s.loc[supp_s.param == "loss_g", "value"].to_numpy(np.float64)
        assert len(r[i]["loss_s"]) == len(ls) and len(r[i]["loss_g"]) == len(lg)
        np.testing.assert_allclose(r[i]["loss_s"].numpy(), ls, rtol=1e-6)
        np.testing.assert_allclose(r[i]["loss_g"].numpy(), lg, rtol=1e-6)
    assert r[0]["launched"] == r[1]["launched"] and len(r[0]["launched"]) == 3, r[0]["launched"]

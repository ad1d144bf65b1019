"""Where a fresh process's C1 full fit spends its time.

configs[0] stand-in (400 + 400 cells x 271 bins, inference_tutorial cell 9 settings) through
scRT(...).infer(level='pyro') in a process that has done nothing else, as
``bench.py --fullfit-c1`` times it (import torch and one device allocation first), with:

* the wall clock of the whole call and of run_pert_model's phases (timings["phases"]);
* ``--cprofile OUT``: a cProfile of the call (host time by function, first-use imports and
  library loads included);
* ``--repeat N``: N more fits in the same process (the warm-process figure beside it).

    python tools/c1_fresh.py [--cprofile gpurun_out/c1.prof] [--repeat 1]
Prints one JSON line.
"""
import argparse
import contextlib
import io
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cprofile", default="")
    ap.add_argument("--repeat", type=int, default=1)
    a = ap.parse_args()
    t_start = time.perf_counter()
    import torch
    from tests._configs import c1_tables, tutorial_scrt
    s, g, truth = c1_tables()
    torch.zeros(1, device="cuda")
    t_ready = time.perf_counter()
    prof = None
    if a.cprofile:
        import cProfile
        prof = cProfile.Profile()
    runs = []
    for i in range(1 + a.repeat):
        with contextlib.redirect_stdout(io.StringIO()):
            if prof is not None and i == 0:
                prof.enable()
            t0 = time.perf_counter()
            sc = tutorial_scrt(s.copy(), g.copy())
            out = sc.infer(level='pyro')
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            if prof is not None and i == 0:
                prof.disable()
        m = sc.model
        runs.append({"s": dt, "run_pert_model_s": m.timings.get("total"), "phases": m.timings.get("phases"),
                     "iters": m.iters, "tau_init_s": m.timings.get("tau_init_s"),
                     "tau_init_g": m.timings.get("tau_init_g")})
    if prof is not None:
        prof.dump_stats(a.cprofile)
        import pstats
        st = io.StringIO()
        pstats.Stats(prof, stream=st).sort_stats("cumulative").print_stats(45)
        with open(a.cprofile + ".txt", "w") as fh:
            fh.write(st.getvalue())
    cn_s_out = out[0]
    mm = cn_s_out.merge(truth, on=["cell_id", "chr", "start"])
    print(json.dumps({"what": "configs[0] stand-in, fresh process: scRT(...).infer(level='pyro') end to end",
                      "import_and_device_s": t_ready - t_start, "fresh": runs[0], "warm": runs[1:],
                      "acc_cn": float((mm["model_cn_state"] == mm["true_somatic_cn"]).mean()),
                      "acc_rep": float((mm["model_rep_state"] == mm["true_rep"]).mean())}), flush=True)


if __name__ == "__main__":
    main()

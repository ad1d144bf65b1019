"""process_input_data's parts at C4 on the box's host: the block layout, the two pivots the fit
needs first (reads, states) and the sorted copy of the whole table (packaging's), per table,
each timed alone after a warm-up.

    python tools/prep_parts_probe.py [--cells 10000]
Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", type=int, default=10000)
    a = ap.parse_args()
    import numpy as np
    from scdna_replication_tools_amd import prep
    from scdna_replication_tools_amd.simulator import simulate, to_long_form
    sim = simulate(n_s=a.cells, n_g=a.cells, num_reads=1e6, seed=0)
    df_s, df_g = to_long_form(sim, n_libs=1)
    out = {"cells": a.cells}

    def timed(name, f, reps=2):
        f()
        t0 = time.perf_counter()
        for _ in range(reps):
            r = f()
        out[name] = (time.perf_counter() - t0) / reps
        return r

    cols = ("cell_id", "chr", "start")
    lay = timed("block_layout", lambda: prep._block_layout(df_s, *cols, "reads"))
    B, L, bp, q, ch0 = lay
    timed("pivot_reads", lambda: prep._block_pivot(df_s["reads"].to_numpy(), B, L, bp, q))
    timed("pivot_states", lambda: prep._block_pivot(df_s["state"].to_numpy(), B, L, bp, q))
    timed("block_table_all", lambda: prep._block_table(df_s, lay, None, "reads", "state", *cols))
    timed("process_input_data", lambda: prep.process_input_data(df_s, df_g, input_col="reads"), reps=1)
    print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in out.items()}), flush=True)


if __name__ == "__main__":
    main()

"""Where process_input_data's time goes at C4 on the box's host (tools/host_prep_profile.py
gives the stage totals): per-table _block_table time on its thread and a cProfile of one table.

    python tools/prep_split_probe.py [--cells 10000]
"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", type=int, default=10000)
    a = ap.parse_args()
    from scdna_replication_tools_amd import prep
    from scdna_replication_tools_amd.simulator import simulate, to_long_form
    sim = simulate(n_s=a.cells, n_g=a.cells, num_reads=1e6, seed=0)
    df_s, df_g = to_long_form(sim, n_libs=1)
    orig = prep._block_table

    def timed(cn, *x, **k):
        t0 = time.perf_counter()
        r = orig(cn, *x, **k)
        print("_block_table of {} rows: {:.3f} s".format(len(cn), time.perf_counter() - t0), flush=True)
        return r
    prep._block_table = timed
    t0 = time.perf_counter()
    prep.process_input_data(df_s, df_g, input_col='reads')
    print("process_input_data: {:.3f} s".format(time.perf_counter() - t0), flush=True)
    prep._block_table = orig
    lay = prep._block_layout(df_s, 'cell_id', 'chr', 'start', 'reads')
    pr = cProfile.Profile()
    pr.enable()
    orig(df_s, lay, None, 'reads', 'state', 'cell_id', 'chr', 'start')
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(15)
    print(s.getvalue())


if __name__ == "__main__":
    main()

"""One-lease strong-scaling table from bench.py lines.

Reads the JSON lines tools/shard_runs.sh collects (each a bench.py run: the 10 k-cell C4 step on one
rank, and the per-rank shard of an N-GPU run -- 10 k / N cells -- with the library's RCCL
all-reduce at world 1) and prints, per repetition, the projected N-GPU efficiency
T(10 k) / (N x T(10 k / N)) from the timed steps (HIP events on every 5th pass) and from the
same steps without events (the production loop).

    python tools/shard_table.py gpurun_out/r05d_shards.jsonl
"""
import json
import sys


def main(path):
    rows = [json.loads(l) for l in open(path) if l.strip().startswith("{")]
    # (r05d lines: ms_per_step evented, ms_per_step_no_events plain; later: ms_per_step plain,
    # ms_per_step_evented)
    ev = lambda r: r.get("ms_per_step_evented", r["ms_per_step"])
    plain = lambda r: r["ms_per_step"] if "ms_per_step_evented" in r else r.get("ms_per_step_no_events",
                                                                                r["ms_per_step"])
    groups = {}
    for r in rows:
        groups.setdefault((r["config"]["bins"], r.get("_rep")), {})[(r["config"]["cells"], bool(r.get("_fused")))] = r
    for (bins, rep), g in sorted(groups.items()):
        big = max(c for c, f in g)
        base = g.get((big, False))
        if base is None:
            continue
        t_ev, t_plain = ev(base), plain(base)
        print("rep {}: {:,} cells x {:,} bins {:.4f} ms/step (evented run {:.4f}), pass {:.4f} ms, ceiling {:.4f} ms".format(
            rep, big, bins, t_plain, t_ev, base["roofline"]["kernel_ms"], base["roofline"]["pattern_ceiling"]["ms"]))
        for (cells, fused), r in sorted(g.items()):
            if cells == big:
                continue
            n = round(big / cells)
            s_ev, s_plain = ev(r), plain(r)
            k, c = r["roofline"]["kernel_ms"], r["roofline"]["pattern_ceiling"]["ms"]
            print("  N={} shard {:5d} cells{}: {:.4f} ms/step (evented run {:.4f}), pass {:.4f} ms = {:.3f} of its "
                  "ceiling {:.4f}; efficiency {:.1%} (evented runs {:.1%}); allreduce: {}".format(
                      n, cells, " fused" if fused else "", s_plain, s_ev, k, c / k, c, t_plain / (n * s_plain),
                      t_ev / (n * s_ev), r["config"]["allreduce"][:40]))


if __name__ == "__main__":
    main(sys.argv[1])

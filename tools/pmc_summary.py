"""Summarise a tools/profile.sh run: per-kernel average duration (kernel-trace stats), the
median and warm-up-excluded mean duration over the trace's dispatches (the first
``WARMUP_FRAC`` of each kernel's dispatches dropped: cold first launches would otherwise
lift the average above the bench's own step time), per-dispatch averages of every PMC
counter, plus HBM traffic per launch.

HBM bytes per launch (MI355X_MICROARCH.md, HBM section): read bytes from the L2
memory-side request counters by request size (TCC_EA0_RDREQ_{32B,64B,128B}); FETCH_SIZE
is also reported raw and x2 (gfx950 tallies a 128-B request at 64 B).  Write bytes
from WRITE_SIZE (exact for streaming stores) and TCC_EA0_WRREQ_64B.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    for k in ("enum_kernel", "enum_dma_kernel", "enum3_kernel", "obs_kernel", "obs_pair_kernel", "finalize_kernel",
              "scalar_kernel", "tau_kmeans_em_kernel",
              "adam_kernel"):
        if k in name:
            return name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    return None


WARMUP_FRAC = 0.2


def trace_durations(d):
    """{kernel: [durations in ns, in dispatch order]} from the kernel trace."""
    dur = defaultdict(list)
    for f in glob.glob(os.path.join(d, "trace", "**", "*kernel_trace.csv"), recursive=True):
        rows = list(csv.DictReader(open(f)))
        rows.sort(key=lambda r: int(r.get("Dispatch_Id", 0) or 0))
        for row in rows:
            k = short(row.get("Kernel_Name", ""))
            if k:
                dur[k].append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    return dur


def main(d):
    out = {"kernels": {}}
    for k, ds in trace_durations(d).items():
        warm = ds[int(len(ds) * WARMUP_FRAC):] or ds
        ent = out["kernels"].setdefault(k, {})
        ent["median_ns"] = float(sorted(ds)[len(ds) // 2])
        ent["warm_mean_ns"] = float(sum(warm) / len(warm))
        ent["dispatches"] = len(ds)
    stats = glob.glob(os.path.join(d, "trace", "**", "*kernel_stats.csv"), recursive=True)
    for f in stats:
        for row in csv.DictReader(open(f)):
            k = short(row["Name"])
            if k:
                out["kernels"].setdefault(k, {})["avg_ns"] = float(row["AverageNs"])
                out["kernels"][k]["calls"] = int(row["Calls"])
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "pmc*", "**", "*counter_collection.csv"), recursive=True):
        per_dispatch = defaultdict(lambda: defaultdict(float))
        names = {}
        for row in csv.DictReader(open(f)):
            k = short(row.get("Kernel_Name", ""))
            if not k:
                continue
            did = row["Dispatch_Id"]
            per_dispatch[did][row["Counter_Name"]] += float(row["Counter_Value"])
            names[did] = k
        for did, cs in per_dispatch.items():
            for c, v in cs.items():
                acc[names[did]][c].append(v)
    for k, cs in acc.items():
        ent = out["kernels"].setdefault(k, {})
        ent["pmc"] = {c: sum(v) / len(v) for c, v in cs.items()}
        p = ent["pmc"]
        rd = None
        if "TCC_EA0_RDREQ_sum" in p:
            n32 = p.get("TCC_EA0_RDREQ_32B_sum", 0.0)
            n64 = p.get("TCC_EA0_RDREQ_64B_sum", 0.0)
            n128 = p.get("TCC_EA0_RDREQ_128B_sum", 0.0)
            rd = 32 * n32 + 64 * n64 + 128 * n128
            ent["hbm_read_bytes_by_reqsize"] = rd
        if "FETCH_SIZE" in p:
            ent["fetch_size_bytes_raw"] = p["FETCH_SIZE"] * 1024
            ent["fetch_size_bytes_x2"] = p["FETCH_SIZE"] * 2048
        wr = p["WRITE_SIZE"] * 1024 if "WRITE_SIZE" in p else None
        ent["write_size_bytes"] = wr
        if rd is not None and wr is not None:
            ent["hbm_bytes_per_launch"] = rd + wr
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main(sys.argv[1])

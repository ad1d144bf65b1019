"""Write profiles/pmc_traffic.json (read by bench.py for roofline.traffic) from a
tools/pmc_summary.py output: HBM bytes per launch of the dominant kernel.
usage: python tools/pmc_traffic.py SUMMARY.json CONFIG CELLS OUT.json"""
import json
import sys

s = json.load(open(sys.argv[1]))
name, ent = max(((k, v) for k, v in s["kernels"].items() if k.startswith("enum")), key=lambda kv: kv[1].get("avg_ns", 0))
pmc = ent.get("pmc", {})
# VALU issue: a wave64 VALU instruction occupies its SIMD for 2 cycles (MI355X_MICROARCH.md);
# GRBM_GUI_ACTIVE is summed over the 8 XCDs, 32 CUs x 4 SIMDs each
cycles = pmc.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
valu = {"insts_per_launch": pmc.get("SQ_INSTS_VALU"), "trans_insts_per_launch": pmc.get("SQ_INSTS_VALU_TRANS_F32"),
        "gpu_cycles_per_launch": cycles,
        "issue_frac": (2.0 * pmc["SQ_INSTS_VALU"] / (256 * 4 * cycles)) if cycles and pmc.get("SQ_INSTS_VALU") else None}
json.dump({"config": sys.argv[2], "cells": int(sys.argv[3]), "kernel": name, "valu": valu,
           "hbm_bytes_per_launch": ent["hbm_bytes_per_launch"],
           "hbm_read_bytes": ent["hbm_read_bytes_by_reqsize"], "hbm_write_bytes": ent["write_size_bytes"],
           "method": "TCC_EA0_RDREQ_{32,64,128}B x size + WRITE_SIZE x 1024, mean over dispatches (tools/profile.sh)",
           "avg_ns_under_profiler": ent.get("avg_ns")}, open(sys.argv[4], "w"), indent=1)

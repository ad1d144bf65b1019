"""Write profiles/pmc_traffic.json (read by bench.py for roofline.traffic) from a
tools/pmc_summary.py output: HBM bytes per launch of the dominant kernel.
usage: python tools/pmc_traffic.py SUMMARY.json CONFIG CELLS OUT.json"""
import json
import sys

s = json.load(open(sys.argv[1]))
name, ent = max(((k, v) for k, v in s["kernels"].items() if k.startswith("enum")), key=lambda kv: kv[1].get("avg_ns", 0))
json.dump({"config": sys.argv[2], "cells": int(sys.argv[3]), "kernel": name,
           "hbm_bytes_per_launch": ent["hbm_bytes_per_launch"],
           "hbm_read_bytes": ent["hbm_read_bytes_by_reqsize"], "hbm_write_bytes": ent["write_size_bytes"],
           "method": "TCC_EA0_RDREQ_{32,64,128}B x size + WRITE_SIZE x 1024, mean over dispatches (tools/profile.sh)",
           "avg_ns_under_profiler": ent.get("avg_ns")}, open(sys.argv[4], "w"), indent=1)

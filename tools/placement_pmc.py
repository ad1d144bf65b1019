"""Fast against slow z / m / v placements in the counters of tools/placement_pmc.sh: per pass,
the stream_ceiling dispatches of the counter phase mapped to their sets (placement_probe.py's
order), the sets split at 5.75 TB/s into fast and slow by that process's own timing, and each
counter's mean per launch over the fast and the slow sets (per-instance counters: also the
spread over the instances, max / mean).
    python tools/placement_pmc.py gpurun_out/TAG
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main(out):
    res = {}
    for d in sorted(glob.glob(os.path.join(out, "pmc[0-9]*"))):
        if not os.path.isdir(d):
            continue
        probe = [json.loads(l) for l in open(d + ".json") if l.startswith("{")]
        if not probe:
            continue
        probe = probe[-1]
        f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if not f:
            continue
        rows = list(csv.DictReader(open(f[0])))
        disp = defaultdict(lambda: defaultdict(list))
        order = []
        for r in rows:
            did = int(r["Dispatch_Id"])
            if did not in disp:
                order.append(did)
            disp[did][r["Counter_Name"]].append(float(r["Counter_Value"]))
        order.sort()
        n, reps = probe["sets"], probe["reps"]
        phase = order[n * probe["timing_dispatches_per_set"]:]
        cls = ["fast" if t >= 5.75 else "slow" for t in probe["tbs"]]
        acc = defaultdict(lambda: defaultdict(list))
        for j, did in enumerate(phase[:n * reps]):
            k = j // reps
            for name, vals in disp[did].items():
                acc[name][cls[k]].append((sum(vals), max(vals) / (sum(vals) / len(vals)) if sum(vals) else 0.0,
                                          len(vals)))
        pas = {"tbs": probe["tbs"], "classes": cls, "counters": {}}
        for name, byc in acc.items():
            pas["counters"][name] = {c: {"mean_per_launch": sum(v[0] for v in vs) / len(vs),
                                         "instances": vs[0][2],
                                         "max_over_mean_instance": sum(v[1] for v in vs) / len(vs)}
                                     for c, vs in byc.items()}
        res[os.path.basename(d)] = pas
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])

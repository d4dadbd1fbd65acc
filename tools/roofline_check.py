#!/usr/bin/env python3
"""Recompute every bench leg's roofline fraction from the committed rocprofv3 kernel stats:
frac = alg_bytes_per_launch / (the roofline kernel's AverageNs in profiles/<tag>_kernel_stats_<leg>.csv)
/ peak, beside the value bench.py measured with hipEvents (profiles/<tag>_bench_n1.json).

    python tools/roofline_check.py r04
"""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1] if len(sys.argv) > 1 else "r04"
line = json.loads(open(os.path.join(ROOT, "profiles", f"{tag}_bench_n1.json")).read().strip().splitlines()[-1])
legs = {"rand": line}
legs.update({k: line[k] for k in ("c2", "text", "c3", "zeros", "runs", "dna", "mix") if isinstance(line.get(k), dict)})
print(f"{'leg':6s} {'kernel':10s} {'bench kernel ms':>15s} {'rocprof avg ms':>15s} {'bench frac':>11s} {'rocprof frac':>13s}")
for leg, v in legs.items():
    r = v["roofline"]
    path = os.path.join(ROOT, "profiles", f"{tag}_kernel_stats_{leg}.csv")
    avg = None
    if not os.path.exists(path):
        continue
    rows = list(csv.DictReader(open(path)))
    name = lambda row: row["Name"].split("(")[0].replace("void ", "").replace("fcx::", "").split("<")[0]
    for row in rows:
        if name(row) == r["kernel"]:
            avg = float(row["AverageNs"]) / 1e6
    if avg is None and r["kernel"].startswith("k_match_{"):
        # several units in one call: the match stage is the sum of the units' launches per call
        # (their listed, direct and remainder kernels, the uniform unit), per k_classify call
        calls = sum(int(row["Calls"]) for row in rows if name(row) == "k_classify")
        tot = sum(float(row["TotalDurationNs"]) for row in rows if name(row).startswith("k_match") or name(row) == "k_route_mark")
        avg = tot / max(calls, 1) / 1e6
    if avg is None:
        print(f"{leg:6s} {r['kernel']:10s} (no rocprof row)")
        continue
    frac = r["alg_bytes_per_launch"] / (avg * 1e-3) / 1e9 / r["peak"]
    print(f"{leg:6s} {r['kernel']:10s} {r['kernel_ms']:15.3f} {avg:15.3f} {r['frac']:11.4f} {frac:13.4f}")

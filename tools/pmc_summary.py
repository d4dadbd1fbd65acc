#!/usr/bin/env python3
"""Summarise tools/pmc_match.sh output (SQ counter sets A and B per input kind) into
per-kernel averages per dispatch, plus the derived ratios used in DESIGN.md §4:

  busy share of wave time   = 1 - (SQ_WAIT_ANY + SQ_WAIT_INST_ANY) / SQ_WAVE_CYCLES
  LDS issue-stall share     = SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES
  LDS bank-conflict share   = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  VALU / LDS instructions per wave

    python tools/pmc_summary.py gpurun_out [--json profiles/pmc_match_rNN.json]
"""
import collections
import csv
import glob
import json
import os
import sys

base = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
out_json = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
res = {}
for d in sorted(glob.glob(os.path.join(base, "pmc_*_[AB]"))):
    kind = os.path.basename(d).split("_")[1]
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        acc = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("fcx::", "").split("<")[0]
            if not name.startswith("k_"):
                continue
            acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for name, cs in acc.items():
            slot = res.setdefault(kind, {}).setdefault(name, {})
            for c, v in cs.items():
                slot[c] = sum(v) / len(v)
for kind, ks in res.items():
    for name, c in ks.items():
        wc = c.get("SQ_WAVE_CYCLES")
        der = {}
        if wc:
            if "SQ_WAIT_ANY" in c and "SQ_WAIT_INST_ANY" in c:
                der["wait_any_share"] = c["SQ_WAIT_ANY"] / wc
                der["wait_inst_any_share"] = c["SQ_WAIT_INST_ANY"] / wc
                der["issue_share"] = 1 - der["wait_any_share"] - der["wait_inst_any_share"]
            if "SQ_WAIT_INST_LDS" in c:
                der["wait_inst_lds_share"] = c["SQ_WAIT_INST_LDS"] / wc
        if c.get("SQ_LDS_IDX_ACTIVE"):
            der["lds_bank_conflict_share"] = c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_LDS_IDX_ACTIVE"]
        if c.get("SQ_WAVES"):
            for k in ["SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM", "SQ_INSTS_BRANCH"]:
                if k in c:
                    der[k.lower().replace("sq_insts_", "") + "_per_wave"] = c[k] / c["SQ_WAVES"]
        c["derived"] = der
if out_json:
    json.dump(res, open(out_json, "w"), indent=1)
for kind, ks in sorted(res.items()):
    for name, c in sorted(ks.items()):
        if not name.startswith("k_match") and name not in ("k_emit", "k_stitch", "k_encode"):
            continue
        print(f"[{kind}] {name}")
        for k, v in sorted(c.items()):
            if k != "derived":
                print(f"    {k:24s} {v:16.1f}")
        for k, v in sorted(c["derived"].items()):
            print(f"    ~{k:23s} {v:16.4f}")

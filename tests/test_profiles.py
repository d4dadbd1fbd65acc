"""The committed round evidence is self-consistent (CPU only): every bench leg in
profiles/r05_bench_n1.json carries a roofline and a cpu_baseline, and each leg's roofline
fraction is reproducible from the rocprofv3 kernel stats committed beside it
(profiles/r05_kernel_stats_<leg>.csv, the same recomputation as tools/roofline_check.py)."""
import csv
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, "profiles")
TAG = "r05"
LEGS = ("rand", "c2", "text", "c3", "zeros", "runs", "dna")


def bench_legs():
    path = os.path.join(PROF, f"{TAG}_bench_n1.json")
    line = json.loads(open(path).read().strip().splitlines()[-1])
    legs = {"rand": line}
    legs.update({k: line[k] for k in LEGS[1:] if isinstance(line.get(k), dict)})
    return legs


def rocprof_avg_ms(leg, kernel):
    for row in csv.DictReader(open(os.path.join(PROF, f"{TAG}_kernel_stats_{leg}.csv"))):
        name = row["Name"].split("(")[0].replace("void ", "").replace("fcx::", "").split("<")[0]
        if name == kernel:
            return float(row["AverageNs"]) / 1e6
    return None


def test_every_leg_is_present():
    assert set(bench_legs()) == set(LEGS)


@pytest.mark.parametrize("leg", LEGS)
def test_leg_carries_roofline_and_cpu_baseline(leg):
    v = bench_legs()[leg]
    r, c = v["roofline"], v["cpu_baseline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "kernel", "kernel_ms", "alg_bytes_per_launch"):
        assert k in r, k
    assert r["frac"] == pytest.approx(r["achieved"] / r["peak"], rel=1e-3)
    assert c["value"] > 0 and c["cores"] >= 1 and c["kind"] in ("reference", "port")


@pytest.mark.parametrize("leg", LEGS)
def test_frac_reproducible_from_rocprof(leg):
    r = bench_legs()[leg]["roofline"]
    avg = rocprof_avg_ms(leg, r["kernel"])
    assert avg is not None, f"{r['kernel']} missing from {TAG}_kernel_stats_{leg}.csv"
    frac = r["alg_bytes_per_launch"] / (avg * 1e-3) / 1e9 / r["peak"]
    assert frac == pytest.approx(r["frac"], rel=0.05)

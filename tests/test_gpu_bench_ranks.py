"""bench.py's multi-rank path end to end on one GPU: two ranks over gloo (both on cuda:0,
FCX_BENCH_SAME_DEVICE=1) compress their block ranges of HL-rand (1 GiB, 1 MiB blocks), gather the
segments to rank 0 with the pipelined protocol, and the assembled stream must equal the reference's
file (SURVEY.md B.4 digest, checked by bench.py's own verify).  Everything the line measures besides
the timed step -- the stage profile, the cold first call -- runs between the step and that check, so
a stray write into the assembled stream shows here (round 6: the cold call did, at N > 1)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_gloo_bit_exact():
    env = dict(os.environ, FCX_BENCH_SAME_DEVICE="1", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29563", "bench.py", "--dist-backend", "gloo",
           "--steps", "2", "--warmup", "1", "--no-text", "--no-decode", "--no-host-path", "--no-cpu-baseline",
           "--no-lz78", "--no-transition", "--no-weak", "--concat", "pipe"]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]
    line = json.loads([x for x in out.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 2
    assert line["bit_exact_vs_reference"] is True, {k: line.get(k) for k in ("partition", "route", "cold_call")}
    assert line.get("cold_call") is not None   # (the cold call ran between the step and the check)

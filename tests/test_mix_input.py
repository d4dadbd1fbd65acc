"""The `mix` input (bench leg and tests/golden/make_mix_digest.py): 1 MiB blocks cycling rand / text
/ runs / dna, block i = block i // 4 of the per-kind bench streams (same seeds)."""
import hashlib

import inputs


def test_mix_blocks_are_the_per_kind_streams():
    n = 9 * inputs.MiB + 12345
    m = inputs.generate("mix", 0, n)
    assert len(m) == n
    streams = {k: inputs.generate(k, seed, 3 * inputs.MiB) for k, seed in inputs.MIX_STREAMS}
    for i in range(10):
        kind = inputs.MIX_STREAMS[i % 4][0]
        j = i // 4
        got = m[i * inputs.MiB:(i + 1) * inputs.MiB]
        assert got == streams[kind][j * inputs.MiB:j * inputs.MiB + len(got)], i


def test_mix_1GiB_input_digest():
    cfg = inputs.SURVEY_DIGESTS["mix_1GiB"]
    assert hashlib.sha256(inputs.generate("mix", 0, cfg["n"])).hexdigest() == cfg["in"]

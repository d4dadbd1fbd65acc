"""GPU parity: the HIP path (through the C ABI) against the reference's own
outputs (golden.json, made by the reference compiled in place) and against the
oracle on seeded inputs.  Integer/byte work: the bar is bit-exact.

Full-size configurations (BASELINE.json configs 2-5) are checked against the
SHA-256 digests of the reference's output; at those sizes the
oracle is not run, the digest is the size-independent check.
"""
import hashlib
import os
import random

import pytest

import inputs
import my_compress_amd as mc
import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu_compress(cuda):
    import torch

    ctxs = {}

    def run(data: bytes, block: int, mode: int = 0) -> bytes:
        if (block, mode) not in ctxs:
            ctxs[(block, mode)] = mc.Context(0, block, max(len(data), block))
            ctxs[(block, mode)].set_match_mode(mode)
        ctx = ctxs[(block, mode)]
        if not data:
            return mc.write_header(0, 0)
        d_in = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(cuda)
        cap = mc.shard_bound(len(data), block)
        d_out = torch.empty(cap, dtype=torch.uint8, device=cuda)
        n = ctx.compress_shard(d_in.data_ptr(), len(data), d_out.data_ptr(), cap,
                               torch.cuda.current_stream().cuda_stream)
        nb = (len(data) + block - 1) // block
        return mc.write_header(len(data), nb) + d_out[:n].cpu().numpy().tobytes()

    yield run
    for c in ctxs.values():
        c.close()


def _cases(golden):
    return [c for c in golden["cases"]]


def test_golden_cases_bit_exact(golden, gpu_compress):
    bad = []
    for case in _cases(golden):
        data = inputs.make(case)
        assert hashlib.sha256(data).hexdigest() == case["in_sha256"], case["name"]
        out = gpu_compress(data, case["block"])
        if hashlib.sha256(out).hexdigest() != case["out_sha256"]:
            bad.append((case["name"], len(out), case["out_bytes"]))
    assert not bad, f"GPU output differs from the reference on {bad}"


@pytest.mark.parametrize("mode", [1, 2, 4, 5, 6, 7])
def test_golden_cases_forced_match_mode(golden, gpu_compress, mode):
    """every tile through one evaluation path of k_match (1: hash buckets + run table
    for the unknowns, 2: run table for whole tiles; 4: every call through the 4-byte-key
    kernel, 5: through the kernel without the repeat filter, 6: through the kernel with the
    run-mode walk inlined, 7: through the kernel without the bucket search, whatever the
    data): the output must not change"""
    bad = []
    for case in _cases(golden):
        if case["in_bytes"] > 1 << 20:
            continue
        out = gpu_compress(inputs.make(case), case["block"], mode)
        if hashlib.sha256(out).hexdigest() != case["out_sha256"]:
            bad.append(case["name"])
    assert not bad, f"match mode {mode}: GPU output differs from the reference on {bad}"


def test_small_hex_fixtures(golden, gpu_compress):
    for case in _cases(golden):
        if "out_hex" in case:
            assert gpu_compress(inputs.make(case), case["block"]).hex() == case["out_hex"], case["name"]


def test_block_api_matches_reference(golden):
    """fcx_compress_block: the per-block drop-in for my_compress_file_lz77 (:2115)"""
    import struct

    for case in _cases(golden):
        if "out_hex" not in case or case["in_bytes"] > case["block"]:
            continue
        data = inputs.make(case)
        blob = bytes.fromhex(case["out_hex"])
        (plen,) = struct.unpack_from("<I", blob, 10)
        assert mc.my_compress_file_lz77(data) == blob[14:14 + plen], case["name"]


def test_empty_inputs(golden, cuda, tmp_path):
    """empty block and empty file through every compress entry point: the block drop-in
    returns the reference's 17-byte payload (my_compress.cpp:2115-2253, totalBytes = 0);
    a shard of 0 bytes emits no record; an empty file is the 10-byte header with
    block_num = 0 (4079-4086, 4128-4129) from the C ABI and from the CLI (one GPU and the
    -g path), and decompresses to nothing"""
    import subprocess

    import torch

    want_block = bytes.fromhex(golden["kat"]["empty_block"]["out_hex"])
    assert mc.my_compress_file_lz77(b"") == want_block
    header = oracle.compress_file(b"", 1 << 20)
    assert header == mc.write_header(0, 0)
    ctx = mc.Context(0, 1 << 20, 1 << 20)
    try:
        d_out = torch.empty(4096, dtype=torch.uint8, device=cuda)
        d_in = torch.empty(16, dtype=torch.uint8, device=cuda)
        assert ctx.compress_shard(d_in.data_ptr(), 0, d_out.data_ptr(), 4096,
                                  torch.cuda.current_stream().cuda_stream) == 0
        assert ctx.compress_host(b"") == b""
    finally:
        ctx.close()
    assert mc.compress(b"") == header
    cli = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "my_compress_amd", "bin",
                       "my_compress")
    (tmp_path / "empty").write_bytes(b"")
    for extra in ([], ["-g", "1"]):
        r = subprocess.run([cli, "-i", "empty", "-o", "e.fcx", "-c", "lz77"] + extra, cwd=tmp_path,
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stdout + r.stderr
        assert (tmp_path / "e.fcx").read_bytes() == header, extra
        r = subprocess.run([cli, "-i", "e.fcx", "-o", "back"], cwd=tmp_path, capture_output=True, text=True,
                           timeout=300)
        assert r.returncode == 0 and "SUCCESS" in r.stdout, r.stdout + r.stderr
        assert (tmp_path / "back").read_bytes() == b""


def test_random_inputs_vs_oracle(gpu_compress):
    rng = random.Random(1234)
    for it in range(40):
        n = rng.choice([1, 2, 3, 5, 17, 100, 1000, 4095, 4096, 4097, 8191, 12289, 70000, 200000, 333333])
        block = rng.choice([1, 7, 64, 1000, 4096, 4097, 65536, 262144, 1 << 20])
        if n // block > 4000:
            block = 65536
        data = inputs.mosaic(rng.randrange(1 << 30), n)
        got = gpu_compress(data, block)
        want = oracle.compress_file(data, block)
        assert got == want, f"iteration {it}: n={n} block={block}"


@pytest.mark.parametrize("groups", [2, 3, 8])
def test_pipelined_groups_same_output(cuda, groups):
    """fcx_ctx_set_groups: the shard's blocks in groups on two streams (record offsets
    continue from group to group); the bytes must equal the oracle's"""
    import torch

    data = inputs.mosaic(4321, 3 * 1000 * 1000 + 777)
    for block in (4096, 65536):
        ctx = mc.Context(0, block, len(data))
        try:
            ctx.set_groups(groups)
            d_in = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(cuda)
            cap = mc.shard_bound(len(data), block)
            d_out = torch.empty(cap, dtype=torch.uint8, device=cuda)
            n = ctx.compress_shard(d_in.data_ptr(), len(data), d_out.data_ptr(), cap,
                                   torch.cuda.current_stream().cuda_stream)
            got = mc.write_header(len(data), (len(data) + block - 1) // block) + d_out[:n].cpu().numpy().tobytes()
            assert got == oracle.compress_file(data, block), (groups, block)
            with pytest.raises(mc.FcxError):   # capacity: a later group's scan sees the overflow
                ctx.compress_shard(d_in.data_ptr(), len(data), d_out.data_ptr(), n // 2,
                                   torch.cuda.current_stream().cuda_stream)
        finally:
            ctx.close()


def test_dense_and_periodic_edges(gpu_compress):
    # long matches capped at 257, matches crossing tile borders, cap shrinking at block end
    cases = [
        b"\x00" * 5000,
        b"ab" * 40000,
        (b"xyz" * 3000) + bytes(range(256)) * 10 + b"q" * 9000,
        inputs.generate("runs", 77, 300000),
        bytes(range(256)) * 300,
        b"a" * 4097 + b"b" * 4095 + b"a" * 4096,
        # uniform tiles (one byte value over the whole window: m_uniform) between others
        b"\x07" * 20000 + inputs.generate("text", 5, 30000) + b"\xff" * 9000 + b"\x07" * 70000,
    ]
    for data in cases:
        for block in [4096, 65536, 1 << 20]:
            assert gpu_compress(data, block) == oracle.compress_file(data, block), (len(data), block)


@pytest.mark.parametrize("shift", [0, 1, 3, 6, 13])
def test_literal_tiles_read_from_input(cuda, shift):
    """all-literal tiles keep their chars in the input: k_emit marks the 64-char segments wholly
    inside them and k_encode reads those from the input at whatever alignment they have.  Random
    data with short repeats planted every few tiles puts literal tiles next to matching ones at
    every chars alignment; the device input starts at every alignment too"""
    import torch

    rng = random.Random(99 + shift)
    data = bytearray(inputs.generate("rand", 11, 3 << 20))
    for _ in range(300):
        src = rng.randrange(len(data) - 4096)
        dst, ln = src + rng.randrange(5, 2000), rng.randrange(3, 40)
        data[dst:dst + ln] = data[src:src + ln]
    data = bytes(data)
    buf = torch.zeros(len(data) + 16, dtype=torch.uint8, device=cuda)
    buf[shift:shift + len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(cuda)
    for block in (1 << 20, 65536, 10000):
        ctx = mc.Context(0, block, len(data))
        try:
            cap = mc.shard_bound(len(data), block)
            d_out = torch.empty(cap, dtype=torch.uint8, device=cuda)
            n = ctx.compress_shard(buf.data_ptr() + shift, len(data), d_out.data_ptr(), cap,
                                   torch.cuda.current_stream().cuda_stream)
            got = mc.write_header(len(data), (len(data) + block - 1) // block) + d_out[:n].cpu().numpy().tobytes()
            assert got == oracle.compress_file(data, block), (shift, block)
        finally:
            ctx.close()


@pytest.mark.parametrize("block", [1 << 20, 65536])
def test_dna_vs_oracle(gpu_compress, block):
    """'ACGT'[rand()%4]: 64 distinct 3-byte keys, ~32 same-key candidates per
    position and matches of a few bytes — the bucket budget overflows and the
    lazy evaluation path (k_stitch, wave-parallel search) carries the parse"""
    data = inputs.generate("dna", 6, 4 << 20)
    assert gpu_compress(data, block) == oracle.compress_file(data, block)


def test_round_trip_host_decoder(gpu_compress):
    for kind, seed in [("rand", 3), ("text", 4), ("runs", 5)]:
        data = inputs.generate(kind, seed, 3 << 20)
        blob = gpu_compress(data, 1 << 20)
        assert mc.decompress(blob) == data


@pytest.mark.slow
def test_cfg2_64MiB_rand_64KiB_digest(gpu_compress):
    cfg = inputs.SURVEY_DIGESTS["cfg2_rand_64MiB"]
    data = inputs.generate(cfg["kind"], cfg["seed"], cfg["n"])
    assert hashlib.sha256(data).hexdigest() == cfg["in"]
    out = gpu_compress(data, cfg["block"])
    assert len(out) == cfg["bytes"]
    assert hashlib.sha256(out).hexdigest() == cfg["out"]


@pytest.mark.slow
@pytest.mark.parametrize("name", ["hl_text_1GiB", "hl_rand_1GiB", "cfg3_text_1GiB", "cfg5a_zeros_1GiB",
                                  "cfg5b_runs_1GiB", "mix_1GiB"])
def test_full_size_digests(name, cuda):
    import torch

    cfg = inputs.SURVEY_DIGESTS[name]
    n, block = cfg["n"], cfg["block"]
    host = torch.empty(n, dtype=torch.uint8).pin_memory()
    inputs.generate_into(cfg["kind"], cfg["seed"], host.data_ptr(), n)
    d_in = host.to(cuda)
    cap = mc.shard_bound(n, block)
    d_out = torch.empty(cap, dtype=torch.uint8, device=cuda)
    ctx = mc.Context(0, block, n)
    try:
        got = ctx.compress_shard(d_in.data_ptr(), n, d_out.data_ptr(), cap, torch.cuda.current_stream().cuda_stream)
    finally:
        ctx.close()
    h = hashlib.sha256(mc.write_header(n, (n + block - 1) // block))
    out_host = d_out[:got].cpu()
    h.update(memoryview(out_host.numpy()))
    assert got + 10 == cfg["bytes"]
    assert h.hexdigest() == cfg["out"]


@pytest.mark.slow
def test_cfg4_rank_segments(cuda):
    """BASELINE config 4 (8 GiB rand seed 4 over 8 GPUs) on one GPU, rank by rank:
    rank r's 1 GiB shard is bytes [r GiB, (r+1) GiB) of the one stream, and its
    segment must equal the reference's (size + sha256 prefix, SURVEY.md B.3;
    main()'s framing my_compress.cpp:4090-4122).  The concatenation of the eight
    segments behind the 10-byte header must be the reference's 8 GiB file."""
    import torch

    n, block = 1 << 30, 1 << 20
    host = torch.empty(n, dtype=torch.uint8).pin_memory()
    d_in = torch.empty(n, dtype=torch.uint8, device=cuda)
    cap = mc.shard_bound(n, block)
    d_out = torch.empty(cap, dtype=torch.uint8, device=cuda)
    ctx = mc.Context(0, block, n)
    whole = hashlib.sha256(mc.write_header(8 * n, 8 * n // block))
    total = 10
    bad = []
    try:
        for r, (want_bytes, want_prefix) in enumerate(inputs.C4_SEGMENTS):
            inputs.rand_stream_into(4, r * n, host.data_ptr(), n)
            d_in.copy_(host)
            got = ctx.compress_shard(d_in.data_ptr(), n, d_out.data_ptr(), cap,
                                     torch.cuda.current_stream().cuda_stream)
            seg = d_out[:got].cpu().numpy()
            h = hashlib.sha256(memoryview(seg)).hexdigest()
            whole.update(memoryview(seg))
            total += got
            if got != want_bytes or h[:16] != want_prefix:
                bad.append((r, got, want_bytes, h[:16], want_prefix))
    finally:
        ctx.close()
    assert not bad, f"config-4 rank segments differ from the reference: {bad}"
    assert total == inputs.C4_FILE["bytes"]
    assert whole.hexdigest() == inputs.C4_FILE["out"]


def _small_alphabet_mix(seed: int, n: int) -> bytes:
    """small-alphabet data (dense 3-byte keys) next to text, random bytes, runs and periodic
    stretches, so 3-byte-only matches, matches capped at block ends and every tile mode occur
    in the 4-byte-key kernel"""
    rng = random.Random(seed)
    parts, left = [], n
    while left > 0:
        kind = rng.choice(["dna", "dna", "ac", "text", "rand", "runs", "period"])
        ln = min(left, rng.randrange(3000, 60000))
        if kind == "ac":   # two letters: every 3-byte key repeats constantly
            parts.append(bytes(rng.choice(b"AC") for _ in range(ln)))
        elif kind == "period":
            unit = bytes(rng.choice(b"ACGT") for _ in range(rng.randrange(3, 9)))
            parts.append((unit * (ln // len(unit) + 1))[:ln])
        else:
            parts.append(inputs.generate(kind, rng.randrange(1 << 30), ln))
        left -= ln
    return b"".join(parts)


@pytest.mark.parametrize("block", [1 << 20, 65536, 5000])
def test_key4_kernel_vs_oracle(cuda, block):
    """the 4-byte-key match unit (fcx_match_k4.hip): forced (mode 4) and routed (mode 0: 'ACGT'
    tiles go to it from the first call on), against the oracle on dna, mixed small-alphabet /
    text / random / periodic data and a ragged tail"""
    import torch

    kernel = mc.lib().fcx_ctx_match_kernel
    cases = [("dna", inputs.generate("dna", 6, 3 << 20)), ("mix", _small_alphabet_mix(5, 3 << 20)),
             ("ragged", bytes(random.Random(7).choice(b"ACGT") for _ in range(100003)))]
    for name, data in cases:
        want = oracle.compress_file(data, block)
        d_in = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(cuda)
        cap = mc.shard_bound(len(data), block)
        d_out = torch.empty(cap, dtype=torch.uint8, device=cuda)
        nb = (len(data) + block - 1) // block
        for mode, calls in ((4, 1), (0, 3)):
            ctx = mc.Context(0, block, len(data))
            try:
                ctx.set_match_mode(mode)
                for call in range(calls):
                    n = ctx.compress_shard(d_in.data_ptr(), len(data), d_out.data_ptr(), cap,
                                           torch.cuda.current_stream().cuda_stream)
                    got = mc.write_header(len(data), nb) + d_out[:n].cpu().numpy().tobytes()
                    assert got == want, (name, block, mode, call)
                    if mode == 4:
                        assert kernel(ctx._h) == 1
                    elif name == "dna":
                        assert kernel(ctx._h) == 1, (name, block, call)
                        rs = ctx.route_stats()
                        assert rs["key4"] >= rs["tiles"] - 1 and rs["rest"] == 0, (name, block, call, rs)
            finally:
                ctx.close()


@pytest.mark.parametrize("block", [1 << 20, 262144])
def test_match_units_routed(cuda, block):
    """text tiles go to the unit without the repeat filter, long-match tiles (runs) to the runs unit,
    one-byte-value windows (zeros) to the uniform unit, random data to the unit without the bucket
    search -- from a context's first call,
    decided by each tile's own bytes; the bytes equal the oracle's"""
    import torch

    kernel = mc.lib().fcx_ctx_match_kernel
    for name, data, want_kernel, lst in (("text", inputs.generate("text", 3, 3 << 20), 2, "nofilter"),
                                         ("rand", inputs.generate("rand", 4, 3 << 20), 4, "sparse"),
                                         ("runs", inputs.generate("runs", 5, 3 << 20), 3, "runs"),
                                         ("zeros", bytes(3 << 20), 5, "uniform"),
                                         ("mix", _small_alphabet_mix(9, 2 << 20), None, None)):
        want = oracle.compress_file(data, block)
        d_in = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(cuda)
        cap = mc.shard_bound(len(data), block)
        d_out = torch.empty(cap, dtype=torch.uint8, device=cuda)
        nb = (len(data) + block - 1) // block
        ctx = mc.Context(0, block, len(data))
        try:
            for call in range(3):
                n = ctx.compress_shard(d_in.data_ptr(), len(data), d_out.data_ptr(), cap,
                                       torch.cuda.current_stream().cuda_stream)
                got = mc.write_header(len(data), nb) + d_out[:n].cpu().numpy().tobytes()
                assert got == want, (name, block, call)
                rs = ctx.route_stats()
                assert rs["cold"] == (1 if call == 0 else 0), (name, call, rs)
                assert rs["tiles"] == sum((min(block, len(data) - b0) + 4095) // 4096
                                          for b0 in range(0, len(data), block)), rs
                if want_kernel is not None:
                    assert kernel(ctx._h) == want_kernel, (name, block, call)
                    # (a runs tile whose sample is one byte value goes to the uniform unit first, which
                    # hands it on to the runs list: there every hand-on is one of those)
                    assert rs[lst] == rs["tiles"] and rs["rest"] == 0, (name, call, rs)
                    assert rs["handed_on"] == (rs["uniform"] if name == "runs" else 0), (name, call, rs)
        finally:
            ctx.close()

"""GPU decoder (fcx_decompress_shard / fcx_decompress_host)
against the oracle's restatement of the reference decoder (my_decompress_file_lz77
my_compress.cpp:2255-2393, pinned in test_oracle.py) on the reference's own
streams (golden.json inputs, encoded by the oracle = the reference's bytes), plus
round trips of the GPU encoder at block sizes 1 B .. 1 MiB and at full size.
Bar: bit-exact, including the reference's single-symbol and early-stop quirks."""
import hashlib
import random

import pytest

import inputs
import my_compress_amd as mc
import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dctx(cuda):
    ctx = mc.DContext(0)
    yield ctx
    ctx.close()


def test_golden_streams(golden, dctx):
    """every golden case: the GPU decoder's bytes = the reference decoder's
    (golden.json dec_sha256, made by my_decompress_file_lz77 compiled in place)"""
    bad = []
    for case in golden["cases"]:
        data = inputs.make(case)
        blob = oracle.compress_file(data, case["block"])   # the reference's bytes (pinned in test_oracle)
        got = dctx.decompress_host(blob, len(data) + 16)
        if len(got) != case["dec_bytes"] or hashlib.sha256(got).hexdigest() != case["dec_sha256"]:
            bad.append(case["name"])
    assert not bad, f"GPU decoder differs from the reference decoder on {bad}"


def test_golden_streams_device_api(golden, dctx, cuda):
    """the same through fcx_decompress_shard on device-resident records"""
    import struct

    import torch

    bad = []
    for case in golden["cases"]:
        if case["in_bytes"] > 1 << 20:
            continue
        blob = oracle.compress_file(inputs.make(case), case["block"])
        nblk = struct.unpack_from("<H", blob, 8)[0]
        d_rec = torch.frombuffer(bytearray(blob[10:] or b"\0"), dtype=torch.uint8).to(cuda)
        d_out = torch.zeros(case["in_bytes"] + 64, dtype=torch.uint8, device=cuda)
        got = dctx.decompress_shard(d_rec.data_ptr(), len(blob) - 10, nblk, d_out.data_ptr(), d_out.numel(),
                                    torch.cuda.current_stream().cuda_stream)
        out = d_out[:got].cpu().numpy().tobytes()
        if got != case["dec_bytes"] or hashlib.sha256(out).hexdigest() != case["dec_sha256"]:
            bad.append(case["name"])
    assert not bad, f"fcx_decompress_shard differs from the reference decoder on {bad}"


def test_single_symbol_stream_decodes_as_zeros(dctx):
    # 'A' x 100000: the chars sub-stream has one distinct symbol, stored without
    # identity; the reference decodes it as zeros (SURVEY.md §8(c) fixture)
    blob = oracle.compress_file(b"A" * 100000, 1 << 20)
    assert len(blob) == 805
    assert dctx.decompress_host(blob, 100016) == b"\0" * 100000


def test_round_trip_random_mosaics(dctx):
    rng = random.Random(99)
    for it in range(30):
        n = rng.choice([1, 2, 9, 100, 4096, 4097, 9000, 70000, 200000, 600000])
        block = rng.choice([1, 7, 64, 1000, 4096, 65536, 262144, 1 << 20])
        if n // block > 4000:
            block = 65536
        data = inputs.mosaic(rng.randrange(1 << 30), n)
        blob = oracle.compress_file(data, block)
        want = oracle.decompress_file(blob, n + 16)
        assert dctx.decompress_host(blob, n + 16) == want, f"iteration {it}: n={n} block={block}"


def test_byte_code_streams(dctx):
    """chars sub-streams whose Huffman codes are all 8 bits (random bytes: a complete
    depth-8 tree) take k_dsyms' byte-substitution path; mixed with blocks whose chars
    codes vary (text) and with random blocks cut short (the stream's last partial word,
    words at every byte alignment of the record), against the oracle's restatement of
    the reference decoder (my_decompress_file_lz77 :2255-2393)"""
    rnd = inputs.generate("rand", 21, 3 * 65536 + 777)
    txt = inputs.generate("text", 22, 100000)
    cases = [(rnd, 65536), (rnd + txt + rnd[:70001], 65536), (rnd[:65536 * 2 + 13], 65536),
             (txt[:5000] + rnd, 262144), (rnd, 1 << 20)]
    for i, (data, block) in enumerate(cases):
        blob = oracle.compress_file(data, block)
        want = oracle.decompress_file(blob, len(data) + 16)
        assert dctx.decompress_host(blob, len(data) + 16) == want, f"case {i}: n={len(data)} block={block}"


def test_device_records_api(dctx, cuda):
    """GPU encode -> device records -> GPU decode, no host round trip in between"""
    import torch

    for kind, seed in [("rand", 11), ("text", 12), ("runs", 13), ("zeros", 0)]:
        n, block = 6 << 20, 1 << 20
        data = inputs.generate(kind, seed, n)
        d_in = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(cuda)
        cap = mc.shard_bound(n, block)
        d_rec = torch.empty(cap, dtype=torch.uint8, device=cuda)
        ctx = mc.Context(0, block, n)
        try:
            m = ctx.compress_shard(d_in.data_ptr(), n, d_rec.data_ptr(), cap, torch.cuda.current_stream().cuda_stream)
        finally:
            ctx.close()
        d_back = torch.empty(n, dtype=torch.uint8, device=cuda)
        got = dctx.decompress_shard(d_rec.data_ptr(), m, n // block, d_back.data_ptr(), n,
                                    torch.cuda.current_stream().cuda_stream)
        assert got == n
        assert torch.equal(d_back, d_in), kind


def test_malformed_streams_fail_cleanly(dctx):
    data = inputs.generate("text", 5, 300000)
    blob = oracle.compress_file(data, 65536)
    for cut in [11, 20, 100, len(blob) // 2, len(blob) - 1]:
        with pytest.raises(mc.FcxError):
            dctx.decompress_host(blob[:cut], len(data) + 16)
    with pytest.raises(mc.FcxError):
        dctx.decompress_host(b"NOTFCX" + blob[6:], len(data) + 16)
    with pytest.raises(mc.FcxError):   # capacity
        dctx.decompress_host(blob, 1000)
    # the context still works afterwards
    assert dctx.decompress_host(blob, len(data) + 16) == data


@pytest.mark.slow
@pytest.mark.parametrize("kind,seed", [("rand", 4), ("text", 3), ("runs", 5), ("zeros", 0)])
def test_full_size_round_trip(kind, seed, dctx, cuda):
    import torch

    n, block = 1 << 30, 1 << 20
    host = torch.empty(n, dtype=torch.uint8).pin_memory()
    inputs.generate_into(kind, seed, host.data_ptr(), n)
    d_in = host.to(cuda)
    del host
    cap = mc.shard_bound(n, block)
    d_rec = torch.empty(cap, dtype=torch.uint8, device=cuda)
    ctx = mc.Context(0, block, n)
    try:
        m = ctx.compress_shard(d_in.data_ptr(), n, d_rec.data_ptr(), cap, torch.cuda.current_stream().cuda_stream)
    finally:
        ctx.close()
    d_back = torch.empty(n, dtype=torch.uint8, device=cuda)
    got = dctx.decompress_shard(d_rec.data_ptr(), m, n // block, d_back.data_ptr(), n,
                                torch.cuda.current_stream().cuda_stream)
    assert got == n
    assert torch.equal(d_back, d_in)

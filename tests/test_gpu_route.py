"""Per-tile routing of the match search (fcx_route.hip): the unit that searches a tile is chosen
from that tile's own bytes in the same call, so the bytes -- and the speed -- do not depend on
what a context compressed before.  The reference's block codec carries no state between blocks
(my_compress.cpp:4090-4122; parse 1675-1714).  Bar: bit-exact against the oracle / the
reference's digests; the route statistics show which unit took which tiles.
"""
import hashlib
import io
import random

import pytest

import inputs
import my_compress_amd as mc
import oracle

pytestmark = pytest.mark.gpu

KINDS = ("rand", "text", "runs", "dna")


def mixed_blocks(seed: int, nblocks: int, block: int) -> bytes:
    """blocks cycling rand / text / runs / dna (the bench's `mix` leg at a smaller size)"""
    return b"".join(inputs.generate(KINDS[i % 4], seed + i, block) for i in range(nblocks))


def _compress(ctx, cuda, data: bytes, block: int) -> bytes:
    import torch

    d_in = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(cuda)
    cap = mc.shard_bound(len(data), block)
    d_out = torch.empty(cap, dtype=torch.uint8, device=cuda)
    n = ctx.compress_shard(d_in.data_ptr(), len(data), d_out.data_ptr(), cap, torch.cuda.current_stream().cuda_stream)
    return mc.write_header(len(data), (len(data) + block - 1) // block) + d_out[:n].cpu().numpy().tobytes()


@pytest.mark.parametrize("block", [1 << 20, 262144, 65536])
def test_mixed_blocks_every_unit(cuda, block):
    """one shard whose blocks cycle through four kinds: each kind's tiles go to its own unit in
    the same call, nothing is left to k_match_rest in steady state, and the bytes are exact"""
    data = mixed_blocks(11, 8, 1 << 20)
    want = oracle.compress_file(data, block)
    ctx = mc.Context(0, block, len(data))
    try:
        for call in range(3):
            assert _compress(ctx, cuda, data, block) == want, (block, call)
            rs = ctx.route_stats()
            q = rs["tiles"] // 4
            assert rs["tiles"] == len(data) // 4096
            # each kind is a quarter of the tiles (a few first-tiles of text blocks may file as sparse)
            assert abs(rs["sparse"] - q) <= 8 and rs["runs"] == q and rs["key4"] == q, rs
            assert rs["sparse"] + rs["runs"] + rs["key4"] + rs["nofilter"] + rs["uniform"] - rs["handed_on"] == rs["tiles"], rs
            assert rs["cold"] == (call == 0), rs
            if call > 0:
                assert rs["rest"] == 0, rs
    finally:
        ctx.close()


def test_kind_changes_between_calls(cuda):
    """one context, consecutive calls of different kinds: the first tiles of a kind the estimate
    did not foresee are searched by their unit's looped remainder (k_match_rest_<unit>), and the
    bytes stay exact; the call after sizes the new kind's unit from the new counts"""
    block = 1 << 20
    ctx = mc.Context(0, block, 4 << 20)
    try:
        seen_rest = 0
        for i, kind in enumerate(["rand", "text", "text", "runs", "dna", "zeros", "rand", "text"]):
            data = bytes(4 << 20) if kind == "zeros" else inputs.generate(kind, 40 + i, 4 << 20)
            got = _compress(ctx, cuda, data, block)
            assert got == oracle.compress_file(data, block), (i, kind)
            rs = ctx.route_stats()
            seen_rest += rs["rest"]
            assert rs["cold"] == (i == 0)
        assert seen_rest > 0   # the change of kind was absorbed by k_match_rest, not by a stale unit
    finally:
        ctx.close()


def test_misfiled_tiles_handed_on(cuda):
    """tiles whose sample looks random (all 256 byte values) but which repeat within the window:
    the classifier files them for the sparse unit, whose repeat filter refuses them.  The first call
    gives the sparse unit every tile directly (no hand-on branch there): its run table overflows and
    the tiles go lazy -- slow, still exact; that call's lazy tiles keep the next calls' units listed,
    where the sparse unit hands them on to the no-filter unit and no tile stays lazy"""
    data = _misfiled(5, 64)
    block = 1 << 20
    ctx = mc.Context(0, block, len(data))
    try:
        want = oracle.compress_file(data, block)
        for call in range(3):
            assert _compress(ctx, cuda, data, block) == want, call
            rs, st = ctx.route_stats(), ctx.stats()
            if call > 0:
                assert rs["handed_on"] > 0, rs
                assert st["lazy_tiles"] == 0, st
    finally:
        ctx.close()


def _misfiled(seed: int, parts: int) -> bytes:
    """tiles half a shuffled 256-byte unit repeated (sample: every byte value, few repeats 4 back),
    half text: filed for the sparse unit, whose repeat filter hands them on to the no-filter unit"""
    rng = random.Random(seed)
    perm = list(range(256))
    out = []
    for _ in range(parts):
        rng.shuffle(perm)
        out.append(bytes(perm) * 8 + inputs.generate("text", rng.randrange(1 << 20), 2048))
    return b"".join(out)


def test_late_hand_ons_after_listed_nofilter(cuda):
    """a call after one whose tiles were a third each text / runs / dna (no dominant unit, so the
    no-filter unit is launched listed with a grid sized for a third of the tiles), now on tiles the
    sparse unit's remainder (it had no estimate) hands on: those land in the no-filter list after its
    listed launch read the count, below its grid -- its remainder must start at the count it
    covered, not at its grid, or those tiles are never searched"""
    block = 1 << 20
    prev = b"".join(inputs.generate(("text", "runs", "dna")[i % 3], 80 + i, block) for i in range(3))
    data = _misfiled(9, 256)
    ctx = mc.Context(0, block, len(prev))
    try:
        assert _compress(ctx, cuda, prev, block) == oracle.compress_file(prev, block)
        rs = ctx.route_stats()
        assert min(rs["nofilter"], rs["runs"], rs["key4"]) >= 240, rs   # no unit dominant
        assert _compress(ctx, cuda, data, block) == oracle.compress_file(data, block)
        rs = ctx.route_stats()
        assert rs["handed_on"] > 0 and rs["rest"] > 0, rs
    finally:
        ctx.close()


def test_forced_unit_is_unrouted(cuda):
    """a forced unit (fcx_ctx_set_match_mode 4-7) runs unrouted over every tile: no route stats"""
    data = inputs.generate("text", 2, 1 << 20)
    ctx = mc.Context(0, 1 << 20, len(data))
    try:
        ctx.set_match_mode(7)
        assert _compress(ctx, cuda, data, 1 << 20) == oracle.compress_file(data, 1 << 20)
        with pytest.raises(mc.FcxError):
            ctx.route_stats()
        ctx.set_match_mode(0)
        assert _compress(ctx, cuda, data, 1 << 20) == oracle.compress_file(data, 1 << 20)
        assert ctx.route_stats()["nofilter"] == 256
    finally:
        ctx.close()


def test_stream_across_kinds(cuda):
    """the stream path (fcx_compress_stream) on one context over rand, then text, then runs, in
    shards smaller than each part: every shard is routed from its own bytes; the records equal
    the per-part records (independent blocks), and each part is the reference's / oracle's"""
    block = 1 << 20
    parts = [inputs.generate(k, 60 + i, 24 << 20) for i, k in enumerate(["rand", "text", "runs"])]
    data = b"".join(parts)
    ctx = mc.Context(0, block, 8 << 20)
    try:
        src, sink = io.BytesIO(data), io.BytesIO()
        tin, tout, nb = ctx.compress_stream(src, sink, 8 << 20)
        assert (tin, nb) == (len(data), len(data) // block)
        recs = sink.getvalue()
        assert len(recs) == tout
    finally:
        ctx.close()
    want = b""
    for p in parts:   # the part's records, from a fresh context (cold, routed from its own counts)
        c = mc.Context(0, block, len(p))
        try:
            want += _compress(c, cuda, p, block)[10:]
        finally:
            c.close()
    assert hashlib.sha256(recs).hexdigest() == hashlib.sha256(want).hexdigest()
    small = parts[1][: 2 << 20]
    assert _compress(mc.Context(0, block, len(small)), cuda, small, block) == oracle.compress_file(small, block)


def test_direct_every_tile_then_own_units(cuda):
    """a shard the estimate gives (nearly) all to one unit: that unit runs first over every tile with
    the unrouted kernel's code, and the few tiles of other kinds are searched again by their own
    units -- the last writer's outputs must be complete.  255 random 64 KiB blocks and one text
    block; the bytes must equal a forced unit's (every unit is exact for any tile) and the oracle's
    on the text block, and no tile may stay lazy"""
    block = 65536
    rnd = inputs.generate("rand", 71, 255 * block)
    txt = inputs.generate("text", 72, block)
    for data in (rnd + txt, rnd[: 100 * block] + txt + rnd[100 * block:]):
        ctx = mc.Context(0, block, len(data))
        ref = mc.Context(0, block, len(data))
        try:
            ref.set_match_mode(5)   # the no-filter unit for every tile, unrouted
            want = _compress(ref, cuda, data, block)
            for call in range(2):
                assert _compress(ctx, cuda, data, block) == want, call
                rs = ctx.route_stats()
                assert rs["sparse"] == 255 * 16 and rs["nofilter"] - rs["handed_on"] == 16, rs
                assert ctx.stats()["lazy_tiles"] == 0
        finally:
            ctx.close()
            ref.close()
    assert _compress(mc.Context(0, block, len(txt)), cuda, txt, block) == oracle.compress_file(txt, block)


def _uniform_cases():
    """shards whose tiles the uniform unit takes, hands on, or shares with other units: whole zero /
    0xAB blocks, zero tiles with one other byte (samples uniform, window not: handed on to the runs
    unit), zero runs that end inside a tile's window or look-ahead, a uniform stretch across a block boundary, text with zero holes, and
    random data with page-sized zero stretches (the sparse unit direct over every tile as well)
    (zero_specks: k_classify samples each tile's bytes [0, 128))"""
    rng = random.Random(17)
    txt = inputs.generate("text", 90, 1 << 20)
    rnd = inputs.generate("rand", 91, 4 << 20)
    yield "zeros", bytes(3 << 20)
    yield "ab", b"\xab" * ((2 << 20) + 5000)
    parts = []   # zero tiles with one 'A' each, away from the bytes k_classify samples: filed for the
    for t in range(512):   # uniform unit, which finds the 'A' in the window and hands the tile on
        tile = bytearray(4096)
        x = rng.randrange(200, 4000)
        while x % 1024 >= 1016:
            x = rng.randrange(200, 4000)
        tile[x] = 0x41
        parts.append(bytes(tile))
    yield "zero_specks", b"".join(parts)
    parts = []   # zero runs of 6..12 KiB ending at random offsets (inside later tiles' windows)
    while sum(map(len, parts)) < (2 << 20):
        parts.append(bytes(rng.randrange(6144, 12288)))
        parts.append(txt[rng.randrange(0, len(txt) - 300):][: rng.randrange(1, 300)])
    yield "zero_runs", b"".join(parts)
    yield "holes", b"".join(txt[i:i + 65536] + bytes(rng.choice([4096, 8192, 9000, 20000])) for i in range(0, 1 << 20, 65536))
    yield "rand_pages", b"".join(rnd[i:i + 500000] + bytes(rng.choice([8192, 16384, 12000])) for i in range(0, 4 << 20, 500000))


@pytest.mark.parametrize("block", [1 << 20, 65536])
def test_uniform_unit(cuda, block):
    """the uniform unit (fcx_match_uniform.hip) against the oracle: closed-form tiles, hand-ons to the
    runs unit where only the sample was uniform, and shards it shares with the other units"""
    for name, data in _uniform_cases():
        ctx = mc.Context(0, block, len(data))
        try:
            want = oracle.compress_file(data, block)
            for call in range(2):
                assert _compress(ctx, cuda, data, block) == want, (name, block, call)
                rs = ctx.route_stats()
                assert rs["sparse"] + rs["runs"] + rs["key4"] + rs["nofilter"] + rs["uniform"] - rs["handed_on"] == rs["tiles"], rs
                if name in ("zeros", "ab"):
                    assert rs["uniform"] == rs["tiles"] and rs["handed_on"] == 0, (name, rs)
                if name == "zero_specks":   # every tile's samples are zeros, no window is: all handed on
                    assert rs["uniform"] == rs["tiles"] and rs["handed_on"] >= rs["uniform"], (name, rs)
        finally:
            ctx.close()

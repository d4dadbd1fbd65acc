"""GPU parity of the `-c lz78` codec (fcx_lz78.hip, through the C ABI) against the
LZ78 oracle (oracle/lz78_oracle.c, itself pinned by tests/test_lz78.py against the
reference compiled in place and tests/golden/golden_lz78.json).  Integer/byte
work: bit-exact.  Reference: my_compress_file_lz78 my_compress.cpp:3127-3476,
main() -c lz78 4073-4136."""
import hashlib
import json
import os

import pytest

import inputs
import my_compress_amd as mc
import oracle

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def sha(b):
    return hashlib.sha256(b).hexdigest()


def test_golden_files():
    with open(os.path.join(HERE, "golden", "golden_lz78.json")) as f:
        g = json.load(f)
    for rec in g["cases"]:
        data = inputs.make(rec)
        out = mc.compress_lz78(data, rec["block"])
        assert len(out) == rec["out_bytes"], rec["name"]
        assert sha(out) == rec["out_sha256"], rec["name"]


@pytest.mark.parametrize("n", [1, 2, 3, 17, 255, 256, 4097, 65536, 200003])
def test_block_vs_oracle(n):
    data = inputs.mosaic(300 + n, n)
    assert mc.my_compress_file_lz78(data) == oracle.lz78_compress_block(data)


@pytest.mark.parametrize("kind", ["rand", "text", "zeros", "runs"])
def test_file_vs_oracle(kind):
    n, block = (3 << 20) + 12345, 1 << 20
    data = inputs.generate(kind, 7, n)
    assert mc.compress_lz78(data, block) == oracle.lz78_compress_file(data, block)


def test_small_blocks_many_batches_vs_oracle():
    # 64 KiB blocks: several hundred records, last one ragged
    data = inputs.mosaic(77, (20 << 20) + 999)
    assert mc.compress_lz78(data, 1 << 16) == oracle.lz78_compress_file(data, 1 << 16)


def test_edge_inputs():
    for data in [b"a", b"aaaa", b"\0\0\0", bytes(range(256)), bytes(100000), b"ab" * 50000]:
        assert mc.compress_lz78(data, 1 << 20) == oracle.lz78_compress_file(data, 1 << 20)
    assert mc.compress_lz78(b"", 1 << 20) == oracle.lz78_compress_file(b"", 1 << 20)


def test_capacity_error():
    data = inputs.generate("rand", 1, 100000)
    import ctypes
    out = ctypes.create_string_buffer(1000)
    n = ctypes.c_uint64()
    rc = mc.lib().fcx_lz78_compress_host(data, len(data), 1 << 20, out, 1000, ctypes.byref(n))
    assert rc == -2


# ---- decoder (my_decompress_file_lz78 3478-3710) ----
def test_decode_golden_files():
    with open(os.path.join(HERE, "golden", "golden_lz78.json")) as f:
        g = json.load(f)
    for rec in g["cases"]:
        data = inputs.make(rec)
        dec = mc.decompress_lz78(oracle.lz78_compress_file(data, rec["block"]))
        assert len(dec) == rec["dec_bytes"] and sha(dec) == rec["dec_sha256"], rec["name"]
        assert (dec == data) == rec["round_trip"], rec["name"]


@pytest.mark.parametrize("kind", ["rand", "text", "zeros", "runs"])
def test_decode_round_trip(kind):
    n, block = (3 << 20) + 777, 1 << 20
    data = inputs.generate(kind, 9, n)
    blob = mc.compress_lz78(data, block)
    assert mc.decompress_lz78(blob) == oracle.lz78_decompress_file(blob, n + 64)


def test_decode_small_blocks_vs_oracle():
    data = inputs.mosaic(78, (20 << 20) + 5)
    blob = mc.compress_lz78(data, 1 << 16)
    assert mc.decompress_lz78(blob) == oracle.lz78_decompress_file(blob, len(data) + 64)


def test_decode_quirks_and_malformed():
    # tail zero dropped (3701-3703), one-symbol char stream decodes as zeros
    assert mc.decompress_lz78(mc.compress_lz78(b"a")) == b""
    assert mc.decompress_lz78(mc.compress_lz78(b"aaaa")) == b"aaaa"
    assert mc.decompress_lz78(mc.compress_lz78(b"\0\0\0")) == b"\0\0"
    p = mc.my_compress_file_lz78(inputs.mosaic(5, 5000))
    assert mc.my_decompress_file_lz78(p) == oracle.lz78_decompress_block(p, 1 << 20)
    with pytest.raises(mc.FcxError):
        mc.my_decompress_file_lz78(b"\0\0\0\0")        # wcnt == 0
    with pytest.raises(mc.FcxError):
        mc.my_decompress_file_lz78(p[:len(p) // 2])    # truncated
    with pytest.raises(mc.FcxError):
        mc.decompress_lz78(mc.compress(b"abc"))         # an FCX7 stream
    # bytes after the block_num counted records are ignored, as main() does (4162-4201; the u16
    # count wraps past 65535 blocks and the reference then decodes the counted ones)
    blob = mc.compress_lz78(inputs.mosaic(6, 9000), 4096)
    assert mc.decompress_lz78(blob + b"\x07" * 37) == mc.decompress_lz78(blob)


@pytest.mark.parametrize("block", [1, 7, 1000, 4096])
def test_tiny_blocks_vs_oracle(block):
    # degenerate block sizes: thousands of records, per-block scratch bounded by the budget
    data = inputs.mosaic(90 + block, 5000 if block < 100 else 3_000_001)
    blob = mc.compress_lz78(data, block)
    assert blob == oracle.lz78_compress_file(data, block)
    assert mc.decompress_lz78(blob, len(data) + 64 * ((len(data) + block - 1) // block)) == \
        oracle.lz78_decompress_file(blob, len(data) + 64 * ((len(data) + block - 1) // block))

"""Pins the oracle (oracle/fcx_oracle.c) before anything is checked against it:
against the reference's own known-answer results and against the reference's
outputs recorded in tests/golden/golden.json (made by the reference compiled in
place, tests/golden/make_golden.py).  CPU only."""
import ctypes
import hashlib

import pytest

import inputs
import oracle


def u32arr(vals):
    return (ctypes.c_uint32 * max(len(vals), 1))(*vals)


def test_generator_matches_survey_inputs():
    # input sha256 of the 1 MiB seed-1 inputs
    want = {"rand": "48f9dbe1", "text": "164c0837", "runs": "d0ca329b", "zeros": "30e14955"}
    for kind, pre in want.items():
        seed = 0 if kind == "zeros" else 1
        assert hashlib.sha256(inputs.generate(kind, seed, 1 << 20)).hexdigest().startswith(pre), kind
    vals = (ctypes.c_int32 * 3)()
    inputs.gen_lib().fcxgen_rand_values(1, vals, 3)
    assert list(vals) == [1804289383, 846930886, 1681692777]   # glibc srand(1)


def test_generator_skip_ahead():
    G = inputs.gen_lib()
    G.fcxgen_skip.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    full = inputs.generate("rand", 4, 300000)
    for k in [0, 1, 33, 34, 1000, 299000]:
        h = G.fcxgen_create(0, 4)
        assert G.fcxgen_skip(h, k) == 0
        buf = ctypes.create_string_buffer(1000)
        G.fcxgen_fill(h, buf, 1000)
        G.fcxgen_destroy(h)
        assert buf.raw == full[k:k + 1000]


def test_sunday_kats(golden):
    # my_compress.cpp:3749-3759 (expected values in the trailing comments: 15 11 15 -1 4)
    got = []
    for main_hex, main_len, pat_hex, pat_len, ref_val in golden["kat"]["sunday"]:
        text = bytes.fromhex(main_hex) + b"\0"
        r = oracle.orc().orc_sunday_search(text, main_len, bytes.fromhex(pat_hex), pat_len)
        assert r == ref_val
        got.append(r)
    assert got == [15, 11, 15, -1, 4]


@pytest.mark.parametrize("key", ["golomb", "golomb_3_257"])
def test_golomb_kat(golden, key):
    kat = golden["kat"][key]
    words = (ctypes.c_uint32 * 4096)()
    n = oracle.orc().orc_golomb_encode(u32arr(kat["in"]), len(kat["in"]), words)
    assert [words[i] for i in range(n)] == kat["words"]
    if key == "golomb":   # the disabled self-test's printout
        assert [f"{w:08x}" for w in kat["words"]] == \
            ["fff3fd78", "ff1ffffd", "ffff5fff", "fffff9ff", "fffffdff", "fffe3fff", "017fffff"]


@pytest.mark.parametrize("key", ["combine_bits", "combine_bits_11"])
def test_combine_bits_kat(golden, key):
    kat = golden["kat"][key]
    out = (ctypes.c_uint8 * len(kat["out"]))()
    oracle.orc().orc_combine_bits(u32arr(kat["in"]), len(kat["in"]), kat["bits"], out)
    assert list(out) == kat["out"]


@pytest.mark.parametrize("key", ["huffman_tree", "huffman_tree_ties"])
def test_huffman_tree_kat(golden, key):
    kat = golden["kat"][key]
    n = len(kat["weights"])
    nodes = (ctypes.c_uint32 * (4 * (2 * n - 1)))()
    real = oracle.orc().orc_huffman_tree(u32arr(kat["weights"]), n, nodes)
    assert real == kat["real"]
    assert [list(nodes[4 * i:4 * i + 4]) for i in range(2 * n - 1)] == kat["nodes"]
    if key == "huffman_tree":  # internal nodes 14..20 (not the stale comment at 526-532)
        assert kat["nodes"][14:21] == [[8, 16, 8, 1], [15, 17, 3, 5], [19, 18, 14, 9], [29, 19, 6, 15],
                                       [42, 20, 16, 7], [58, 20, 2, 17], [100, 0, 18, 19]]


def test_lz77_token_fixtures(golden):
    for case in golden["tokens"]:
        data = inputs.make(case)
        for finder in (oracle.FINDER_EXHAUSTIVE, oracle.FINDER_SUNDAY):
            assert oracle.parse(data, finder) == case["tokens"], (case["name"], finder)
    kat = [c for c in golden["tokens"] if c["name"] == "kat30"][0]["tokens"]
    assert [(p, l, chr(c)) for p, l, c in kat] == [(0, 0, "a"), (0, 0, "a"), (0, 0, "c"), (3, 4, "b"), (3, 3, "a"),
                                                   (12, 3, "b"), (5, 4, "c"), (19, 8, "d")]


def test_oracle_matches_reference_outputs(golden):
    for case in golden["cases"]:
        data = inputs.make(case)
        assert hashlib.sha256(data).hexdigest() == case["in_sha256"], case["name"]
        out = oracle.compress_file(data, case["block"])
        assert len(out) == case["out_bytes"], case["name"]
        assert hashlib.sha256(out).hexdigest() == case["out_sha256"], case["name"]
        if "out_hex" in case:
            assert out.hex() == case["out_hex"]


def test_oracle_decoder_matches_reference_decoder(golden):
    """the oracle's decoder against my_decompress_file_lz77 (:2255-2393) itself:
    golden.json holds the reference decoder's output for every case (quirks
    included: one-symbol sub-streams decode as zeros, 930-984; a match token past
    pCnt stops the block, 2336-2339)"""
    quirky = 0
    for case in golden["cases"]:
        blob = oracle.compress_file(inputs.make(case), case["block"])   # = the reference's bytes (test above)
        dec = oracle.decompress_file(blob, case["in_bytes"] + 16)
        assert len(dec) == case["dec_bytes"], case["name"]
        assert hashlib.sha256(dec).hexdigest() == case["dec_sha256"], case["name"]
        quirky += not case["dec_is_input"]
    assert quirky >= 5   # the fixture really exercises the quirks


def test_sunday_and_exhaustive_finders_agree():
    for seed in range(6):
        data = inputs.mosaic(seed, 40000)
        assert oracle.parse(data, oracle.FINDER_SUNDAY) == oracle.parse(data, oracle.FINDER_EXHAUSTIVE)


def test_worked_example_appendix_a3():
    # bytes 03 0a 11 18 1f -> 50 bytes
    out = oracle.compress_file(bytes([3, 10, 17, 24, 31]), 1 << 20)
    assert out.hex() == ("46435837" "05000000" "0100" "24000000" "05000000" "1f" "04" "e0" "030a11181ffbfcfd"
                         "01000000" "3b060000" "00000000" "00" "00000000" "00000000")


def test_oracle_round_trip():
    for kind, seed in [("rand", 2), ("text", 2), ("runs", 2), ("zeros", 0)]:
        data = inputs.generate(kind, seed, 300000)
        blob = oracle.compress_file(data, 65536)
        assert oracle.decompress_file(blob, len(data) + 16) == data
    # single-symbol sub-streams lose their symbol (reference decoder yields zeros)
    blob = oracle.compress_file(b"A" * 100000, 1 << 20)
    assert oracle.decompress_file(blob, 100016) == b"\0" * 100000


def test_reference_build_available_here_matches_oracle():
    """when the reference is compiled in place (this container), it and the oracle agree"""
    if oracle.ref() is None:
        pytest.skip("oracle/_ref not built")
    for seed in range(3):
        data = inputs.mosaic(100 + seed, 120000)
        assert oracle.ref_compress_file(data, 32768) == oracle.compress_file(data, 32768)

"""Pins the LZ78 oracle (oracle/lz78_oracle.c, the `-c lz78` codec of
my_compress.cpp:1832-1934 / 3127-3710) before anything is checked against it:
against the reference's own self-test string (my_compress.cpp:3977-3988), against
tests/golden/golden_lz78.json (made by tests/golden/make_golden_lz78.py from the
reference compiled in place) and, when oracle/_ref is present, against the
reference directly on seeded inputs.  CPU only."""
import hashlib
import json
import os
import struct

import pytest

import inputs
import oracle

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def golden78():
    with open(os.path.join(HERE, "golden", "golden_lz78.json")) as f:
        return json.load(f)


def sha(b):
    return hashlib.sha256(b).hexdigest()


def payloads(blob):
    nb = struct.unpack_from("<H", blob, 8)[0]
    q = 10
    for _ in range(nb):
        (sz,) = struct.unpack_from("<I", blob, q)
        yield blob[q + 4:q + 4 + sz]
        q += 4 + sz


def test_textbook_string():
    # my_compress.cpp:3977-3988 runs my_LZ78_compress on "ABBCBCABABCAABCAAB";
    # the textbook parse is A|B|BC|BCA|BA|BCAA|BCAAB
    toks = oracle.lz78_parse(b"ABBCBCABABCAABCAAB")
    assert toks == [(0, 65), (0, 66), (2, 67), (3, 65), (2, 65), (4, 65), (6, 66)]


def test_tokens_golden(golden78):
    for rec in golden78["tokens"]:
        data = inputs.make(rec)
        assert sha(data) == rec["in_sha256"]
        assert [list(t) for t in oracle.lz78_parse(data)] == rec["tokens"], rec["name"]


def test_files_golden(golden78):
    for rec in golden78["cases"]:
        data = inputs.make(rec)
        assert sha(data) == rec["in_sha256"], rec["name"]
        out = oracle.lz78_compress_file(data, rec["block"])
        assert len(out) == rec["out_bytes"], rec["name"]
        assert sha(out) == rec["out_sha256"], rec["name"]
        if "out_hex" in rec:
            assert out.hex() == rec["out_hex"]
        dec = b"".join(oracle.lz78_decompress_block(p, rec["block"] + 64) for p in payloads(out))
        assert len(dec) == rec["dec_bytes"] and sha(dec) == rec["dec_sha256"], rec["name"]
        assert (dec == data) == rec["round_trip"]


def test_decoder_quirks():
    # a block whose decoded bytes end in 0x00 loses that byte (3701-3703), and a
    # single distinct token char decodes as zeros (huffman_decode_char with an
    # empty tree, 930-984): "a" -> "" ; "aaaa" round-trips only because its
    # chars are 'a' and '\0'
    assert oracle.lz78_decompress_file(oracle.lz78_compress_file(b"a", 1 << 20), 64) == b""
    assert oracle.lz78_decompress_file(oracle.lz78_compress_file(b"aaaa", 1 << 20), 64) == b"aaaa"
    assert oracle.lz78_decompress_file(oracle.lz78_compress_file(b"\0\0\0", 1 << 20), 64) == b"\0\0"


@pytest.mark.skipif(oracle.ref() is None, reason="oracle/_ref not built")
@pytest.mark.parametrize("seed", range(6))
def test_against_reference(seed):
    n = [1, 5000, 65536, 200000, 300001, 1 << 20][seed]
    data = inputs.mosaic(100 + seed, n)
    assert oracle.lz78_parse(data) == oracle.ref_lz78_tokens(data)
    a = oracle.lz78_compress_block(data)
    assert a == oracle.ref_lz78_compress_block(data)
    assert oracle.lz78_decompress_block(a, n + 64) == oracle.ref_lz78_decompress_block(a, n + 64)

"""The C-ABI library: loads, exports every symbol include/fcx.h declares, the
container helpers work, the host decoder reproduces the reference's decoder on
the golden fixtures, and — without a GPU — every compress entry point fails
loudly instead of falling back to the CPU.  CPU only (no kernel launches)."""
import ctypes
import hashlib
import os
import re
import struct
import shutil
import subprocess

import pytest

import inputs
import my_compress_amd as mc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "fcx.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(fcx_[a-z0-9_]+)\s*\(", src)))


def test_exports_every_declared_symbol():
    syms = declared_symbols()
    assert len(syms) >= 15
    L = mc.lib()
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", mc.lib_path()], capture_output=True, text=True).stdout
    for s in syms:
        assert re.search(rf"\bT {s}$", out, re.M), s


def test_library_carries_gfx950_code_object(tmp_path):
    # (llvm-objdump --offloading extracts the code objects beside its input: a copy in tmp_path)
    lib = tmp_path / "libfcx.so"
    shutil.copyfile(mc.lib_path(), lib)
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", str(lib)],
                         capture_output=True, text=True)
    assert "gfx950" in (out.stdout + out.stderr)


def test_header_roundtrip():
    h = mc.write_header(5, 1)
    assert h == b"FCX7" + struct.pack("<IH", 5, 1)
    # wraps like the reference's u32 / u16 fields (:104-105)
    assert mc.write_header(8 << 30, 8192)[4:] == struct.pack("<IH", 0, 8192)
    tot, nb, kind = ctypes.c_uint32(), ctypes.c_uint16(), ctypes.create_string_buffer(1)
    assert mc.lib().fcx_parse_header(h, ctypes.byref(tot), ctypes.byref(nb), kind) == 0
    assert (tot.value, nb.value, kind.raw) == (5, 1, b"7")
    assert mc.lib().fcx_parse_header(b"XYZ7\0\0\0\0\0\0", None, None, None) == -4


def test_shard_bound_covers_worst_case(golden):
    for case in golden["cases"]:
        payload_total = case["out_bytes"] - 10
        assert payload_total <= mc.shard_bound(case["in_bytes"], case["block"])


def test_host_decoder_matches_reference_on_fixtures(golden):
    """host decoder (fcx_decompress_block per record) on the reference's own bytes
    (out_hex) against the reference decoder's output (dec_sha256)"""
    for case in golden["cases"]:
        if "out_hex" not in case:
            continue
        got = mc.decompress(bytes.fromhex(case["out_hex"]))
        assert hashlib.sha256(got).hexdigest() == case["dec_sha256"], case["name"]


def test_host_decoder_matches_reference_decoder(golden):
    """every golden case, quirks included (one-symbol sub-streams -> zeros 930-984;
    early stop 2336-2339): bytes identical to my_decompress_file_lz77 (:2255)"""
    import oracle

    for case in golden["cases"]:
        blob = oracle.compress_file(inputs.make(case), case["block"])   # = the reference's bytes
        got = mc.decompress(blob)
        assert len(got) == case["dec_bytes"], case["name"]
        assert hashlib.sha256(got).hexdigest() == case["dec_sha256"], case["name"]


def test_no_cpu_fallback_without_gpu():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    h = ctypes.c_void_p()
    rc = mc.lib().fcx_ctx_create(ctypes.byref(h), 0, 1 << 20, 1 << 20)
    assert rc == -3   # FCX_ERR_HIP
    assert b"GPU-only" in mc.lib().fcx_last_error() or b"HIP" in mc.lib().fcx_last_error()
    out = ctypes.create_string_buffer(4096)
    assert mc.lib().fcx_compress_block(b"hello world", 11, out) == 0
    with pytest.raises(mc.FcxError):
        mc.my_compress_file_lz77(b"hello world")
    with pytest.raises(mc.FcxError):
        mc.compress(b"hello world")


def test_null_arguments_follow_reference_contract():
    # my_compress_file_lz77 returns 0 on NULL pointers (:2122-2123)
    assert mc.lib().fcx_compress_block(None, 10, None) == 0
    assert mc.lib().fcx_decompress_block(None, 0, None, 0) == -1


def test_empty_block_follows_reference(golden):
    """my_compress_file_lz77 (:2115-2253) with totalBytes = 0 is a valid call: the reference
    writes a 17-byte payload (N = 0, pCnt = 0, HUFF of one zero byte, G = 0).  The drop-in
    returns the same bytes (no device work is needed for them); the oracle agrees."""
    import oracle

    want = bytes.fromhex(golden["kat"]["empty_block"]["out_hex"])
    assert len(want) == 17
    out = ctypes.create_string_buffer(64)
    assert mc.lib().fcx_compress_block(b"", 0, out) == 17
    assert out.raw[:17] == want
    assert mc.my_compress_file_lz77(b"") == want
    assert oracle.compress_block(b"") == want
    # an empty file is the header alone: block_num = 0 (4079-4086, 4128-4129)
    assert oracle.compress_file(b"", 1 << 20) == b"FCX7" + bytes(6) == mc.compress(b"")

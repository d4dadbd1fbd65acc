/*
 * ref_harness.cpp — exposes the REFERENCE's own functions as a C ABI so tests and
 * bench.py's cpu_baseline leg can call them.  TEST INFRASTRUCTURE ONLY: it is
 * the checker, never the product.  Built by oracle/Makefile into oracle/_ref/
 * (git-ignored) straight from /root/reference/my_compress.cpp; the reference
 * source is #included where it lies, never copied.
 *
 *   ref_compress_block  -> my_compress_file_lz77   (my_compress.cpp:2115)
 *   ref_lz77_tokens     -> my_LZ77_compress        (my_compress.cpp:1675)
 *   ref_decompress_block-> my_decompress_file_lz77 (my_compress.cpp:2255)
 *   ref_sunday          -> Sunday_Search           (my_compress.cpp:1407)
 *   ref_golomb_encode   -> golomb_rice_encode      (my_compress.cpp:258)
 *   ref_combine_bits    -> combine_bits            (my_compress.cpp:1292)
 *   ref_huffman_tree    -> create_huffman_tree     (my_compress.cpp:535)
 *   ref_huffman_encode_char -> my_huffman_encode_char (my_compress.cpp:987)
 *   ref_lz78_* (below)      -> the -c lz78 block codec
 */
#define main ref_main
#include "my_compress.cpp"
#undef main

#include <fcntl.h>
#include <unistd.h>
#include <stdint.h>

static int g_saved_stdout = -1;

/* the reference printf()s per block (my_compress.cpp:2249); callers that need a
 * clean stdout (bench.py prints one JSON line) silence fd 1 around the calls. */
extern "C" void ref_set_quiet(int quiet) {
    fflush(stdout);
    if (quiet && g_saved_stdout < 0) {
        g_saved_stdout = dup(1);
        int devnull = open("/dev/null", O_WRONLY);
        dup2(devnull, 1);
        close(devnull);
    } else if (!quiet && g_saved_stdout >= 0) {
        dup2(g_saved_stdout, 1);
        close(g_saved_stdout);
        g_saved_stdout = -1;
    }
}

/* same buffer discipline as main(): zeroed input copy with slack, 2x output
 * (my_compress.cpp:4073, 4088) */
extern "C" uint32_t ref_compress_block(const uint8_t *in, uint32_t len, uint8_t *out) {
    uint32_t cap_in = len + 4096;
    uInt8 *buf = new uInt8[cap_in]();
    memcpy(buf, in, len);
    uInt8 *obuf = new uInt8[2 * (size_t)len + 4096]();
    uInt32 n = my_compress_file_lz77(buf, len, obuf);
    fflush(stdout);  /* push the per-block printf (2249) to wherever fd 1 points now */
    memcpy(out, obuf, n);
    delete[] buf;
    delete[] obuf;
    return n;
}

/* tokens of the greedy parse: p[], l[], c[] arrays of capacity len; returns N */
extern "C" uint32_t ref_lz77_tokens(const uint8_t *in, uint32_t len, uint32_t *p, uint32_t *l, uint8_t *c) {
    uInt8 *buf = new uInt8[len + 4096]();
    memcpy(buf, in, len);
    vector<stLZ77CmpCp> toks;
    my_LZ77_compress(buf, len, &toks);
    for (size_t i = 0; i < toks.size(); i++) { p[i] = toks[i].p; l[i] = toks[i].l; c[i] = toks[i].c; }
    delete[] buf;
    return (uint32_t)toks.size();
}

/* decode one block payload; returns decoded byte count (<= cap) */
extern "C" int64_t ref_decompress_block(const uint8_t *in, uint32_t len, uint8_t *out, uint64_t cap) {
    char *mem = NULL; size_t memlen = 0;
    FILE *f = open_memstream(&mem, &memlen);
    uInt8 *buf = new uInt8[(size_t)len + 4096]();
    memcpy(buf, in, len);
    uInt32 n = my_decompress_file_lz77(buf, len, f);
    fclose(f);
    int64_t r = (int64_t)n;
    if (memlen < cap) cap = memlen;
    memcpy(out, mem, cap);
    free(mem);
    delete[] buf;
    return r;
}

extern "C" int32_t ref_sunday(const uint8_t *mainStr, int32_t mainLen, const uint8_t *sub, int32_t subLen) {
    return Sunday_Search((uInt8 *)mainStr, mainLen, (uInt8 *)sub, subLen);
}

extern "C" uint32_t ref_golomb_encode(const uint32_t *vals, uint32_t n, uint32_t *words) {
    vector<uInt32> in(vals, vals + n), out;
    golomb_rice_encode(in, out);
    for (size_t i = 0; i < out.size(); i++) words[i] = out[i];
    return (uint32_t)out.size();
}

extern "C" void ref_combine_bits(const uint32_t *vals, uint32_t n, uint8_t bits, uint8_t *out) {
    combine_bits((uInt32 *)vals, n, bits, out);
}

/* node array of 2n-1 entries x {w,parent,l,r}; returns realLeafNum */
extern "C" uint32_t ref_huffman_tree(const uint32_t *weights, uint32_t n, uint32_t *nodes) {
    uInt32 real = 0;
    stHuffmanTreeNode *t = create_huffman_tree((uInt32 *)weights, n, &real);
    if (!t) return 0;
    for (uint32_t i = 0; i < 2 * n - 1; i++) {
        nodes[4 * i + 0] = t[i].weight; nodes[4 * i + 1] = t[i].parent;
        nodes[4 * i + 2] = t[i].leftChild; nodes[4 * i + 3] = t[i].rightChild;
    }
    delete[] t;
    return real;
}

extern "C" uint32_t ref_huffman_encode_char(const uint8_t *src, uint32_t n, uint8_t *out) {
    return my_huffman_encode_char((uInt8 *)src, n, out);
}

/* ---- -c lz78 ----------------------------------------------------------------
 *   ref_lz78_compress_block   -> my_compress_file_lz78   (my_compress.cpp:3127)
 *   ref_lz78_tokens           -> my_LZ78_compress        (my_compress.cpp:1832)
 *   ref_lz78_decompress_block -> my_decompress_file_lz78 (my_compress.cpp:3478)
 */
extern "C" uint32_t ref_lz78_compress_block(const uint8_t *in, uint32_t len, uint8_t *out) {
    uInt8 *buf = new uInt8[(size_t)len + 4096]();
    memcpy(buf, in, len);
    uInt8 *obuf = new uInt8[4 * (size_t)len + 65536]();
    uInt32 n = my_compress_file_lz78(buf, len, obuf);
    fflush(stdout);
    cout.flush();
    memcpy(out, obuf, n);
    delete[] buf;
    delete[] obuf;
    return n;
}

extern "C" uint32_t ref_lz78_tokens(const uint8_t *in, uint32_t len, uint32_t *idx, uint8_t *c) {
    uInt8 *buf = new uInt8[(size_t)len + 4096]();
    memcpy(buf, in, len);
    vector<stLZ78CmpCp> toks;
    my_LZ78_compress(buf, len, &toks);
    for (size_t i = 0; i < toks.size(); i++) { idx[i] = toks[i].idx; c[i] = toks[i].c; }
    delete[] buf;
    return (uint32_t)toks.size();
}

extern "C" int64_t ref_lz78_decompress_block(const uint8_t *in, uint32_t len, uint8_t *out, uint64_t cap) {
    char *mem = NULL; size_t memlen = 0;
    FILE *f = open_memstream(&mem, &memlen);
    uInt8 *buf = new uInt8[(size_t)len + 4096]();
    memcpy(buf, in, len);
    uInt32 n = my_decompress_file_lz78(buf, len, f);
    fflush(stdout);
    cout.flush();
    fclose(f);
    if (memlen < cap) cap = memlen;
    memcpy(out, mem, cap);
    free(mem);
    delete[] buf;
    return (int64_t)n;
}

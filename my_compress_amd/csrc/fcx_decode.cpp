// fcx_decode.cpp — host decoder of one FCX7 / LZ77 block payload.
//
// Replaces my_decompress_file_lz77 (my_compress.cpp:2255-2393) for the CLI's
// decompress mode and for round-trip checks.  It reproduces the reference
// decoder's observable behaviour, including the single-symbol sub-stream case:
// the reference stores no symbol identity when a sub-stream has one distinct
// byte (ts = 0, W = 0) and decodes it as zeros (930-984 with m = 0).
// The GPU decoder is the next row of the scope table.
#include <cstring>
#include <vector>

#include "fcx.h"

namespace {

struct Cursor {
    const uint8_t *p, *end;
    bool ok = true;
    uint32_t u32() {
        if (end - p < 4) { ok = false; return 0; }
        uint32_t v;
        memcpy(&v, p, 4);
        p += 4;
        return v;
    }
    const uint8_t *take(size_t n) {
        if ((size_t)(end - p) < n) { ok = false; return nullptr; }
        const uint8_t *q = p;
        p += n;
        return q;
    }
};

// one Huffman sub-stream (my_huffman_decode_char 1107-1187): tree header, W, words
bool decode_substream(Cursor &cur, uint8_t *dst, uint32_t count) {
    const uint8_t *tsb = cur.take(1);
    if (!tsb) return false;
    const uint32_t ts = *tsb, nbm = (2 * ts + 7) / 8;
    const uint8_t *bm = cur.take(nbm);
    const uint8_t *pairs = cur.take(2 * ts);
    const uint32_t nw = cur.u32();
    const uint8_t *words = cur.take(4ull * nw);
    if (!cur.ok) return false;
    // child[2*j + side]: < 256 leaf symbol, >= 256 internal node index + 256
    std::vector<uint16_t> child(2 * ts);
    const uint32_t real = ts + 1;
    for (uint32_t q = 0; q < 2 * ts; q++) {
        const bool internal = (bm[q >> 3] >> (q & 7)) & 1;
        uint32_t v = pairs[q];
        if (internal) {
            // stored as (256 - real) + k for internal node k (1042-1057)
            if (v < 256 - real || v - (256 - real) >= ts) return false;
            v = 256 + (v - (256 - real));
        }
        child[q] = (uint16_t)v;
    }
    memset(dst, 0, count);
    if (ts == 0 || count == 0) return true;
    const uint32_t root = ts - 1;
    uint32_t node = root, j = 0;
    for (uint32_t i = 0; i < nw && j < count; i++) {
        uint32_t w;
        memcpy(&w, words + 4ull * i, 4);
        for (int b = 0; b < 32 && j < count; b++, w >>= 1) {
            const uint32_t nx = child[2 * node + (w & 1)];
            if (nx < 256) { dst[j++] = (uint8_t)nx; node = root; }
            else node = nx - 256;
        }
    }
    return true;
}

}  // namespace

extern "C" int64_t fcx_decompress_block(const uint8_t *in, uint32_t len, uint8_t *out, uint64_t cap) {
    if (!in || !out) return FCX_ERR_ARG;
    Cursor cur{in, in + len};
    const uint32_t N = cur.u32();
    if (!cur.ok) return FCX_ERR_FORMAT;
    const uint32_t nb = (N + 7) / 8;
    std::vector<uint8_t> flags(nb + 1, 0), chars(N + 1, 0);
    if (nb > 1) {
        if (!decode_substream(cur, flags.data(), nb)) return FCX_ERR_FORMAT;
    } else {
        const uint8_t *raw = cur.take(nb);
        if (!cur.ok) return FCX_ERR_FORMAT;
        if (nb) flags[0] = raw[0];
    }
    if (!decode_substream(cur, chars.data(), N)) return FCX_ERR_FORMAT;
    const uint32_t pcnt = cur.u32();
    if (!cur.ok || pcnt > N) return FCX_ERR_FORMAT;
    const uint32_t pbytes = (11 * pcnt) / 8 + 1;   // :2311
    std::vector<uint8_t> pb(pbytes, 0);
    if (!decode_substream(cur, pb.data(), pbytes)) return FCX_ERR_FORMAT;
    const uint32_t G = cur.u32();
    if (!cur.ok) return FCX_ERR_FORMAT;
    std::vector<uint8_t> gb(4ull * G + 4, 0);
    if (G > 0 && !decode_substream(cur, gb.data(), 4 * G)) return FCX_ERR_FORMAT;

    // distances: decombine_bits (1315-1338), 11 bits LSB-first
    std::vector<uint32_t> dist(pcnt), mlen(pcnt);
    for (uint32_t i = 0; i < pcnt; i++) {
        const uint64_t bit = 11ull * i;
        uint32_t v = 0;
        for (uint32_t k = 0; k < 11; k++) v |= (uint32_t)((pb[(bit + k) >> 3] >> ((bit + k) & 7)) & 1) << k;
        dist[i] = v;
    }
    // lengths: golomb_rice_decode (309-358), q ones, a zero, 2 bits of r
    {
        uint64_t bit = 0;
        const uint64_t nbits = 32ull * G;
        auto get = [&](uint64_t k) { return (gb[k >> 3] >> (k & 7)) & 1; };
        for (uint32_t i = 0; i < pcnt; i++) {
            uint32_t q = 0;
            while (bit < nbits && get(bit)) { q++; bit++; }
            if (bit + 3 > nbits) return FCX_ERR_FORMAT;
            bit++;
            const uint32_t r = get(bit) | (get(bit + 1) << 1);
            bit += 2;
            mlen[i] = 4 * q + r;
        }
    }
    // tokens -> bytes (my_LZ77_decompress 1716-1735)
    uint64_t o = 0;
    uint32_t mi = 0;
    for (uint32_t t = 0; t < N; t++) {
        if (!((flags[t >> 3] >> (t & 7)) & 1)) {
            // the reference stops at the first match token it has no (p, l) for
            // ("Fatal Error!!!", break at 2331-2335) and decodes the tokens before it
            if (mi >= pcnt) break;
            const uint32_t p = dist[mi], L = mlen[mi++];
            if (p == 0 || p > o || o + L + 1 > cap) return FCX_ERR_FORMAT;
            for (uint32_t k = 0; k < L; k++, o++) out[o] = out[o - p];
        }
        if (o + 1 > cap) return FCX_ERR_CAPACITY;
        out[o++] = chars[t];
    }
    return (int64_t)o;
}

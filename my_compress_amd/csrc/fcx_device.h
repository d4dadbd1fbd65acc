// fcx_device.h — constants, batch layout and wave helpers shared by the gfx950
// kernels of the FCX7 LZ77 + Huffman compress path.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fcx {

// ---- format constants (my_compress.cpp:1261-1277, 222-224) ----------------
constexpr uint32_t kWin = 2047;     // SLIDE_WIN_LEN
constexpr uint32_t kMaxL = 258;     // CUR_BUFF_LEN: match length cap is min(258, len-i) - 1
constexpr uint32_t kMinL = 3;       // MIN_MATCH_LEN
constexpr uint32_t kPBits = 11;     // P_BITS

// ---- device work decomposition --------------------------------------------
constexpr uint32_t kTile = 4096;            // positions per match-kernel workgroup
constexpr uint32_t kMatchThreads = 512;
constexpr uint32_t kSubSeg = kTile / kMatchThreads;  // 8 positions per lane in the tile parse
constexpr uint32_t kHashBits = 13;
constexpr uint32_t kHalo = kWin;                     // left halo of a tile
constexpr uint32_t kLookAhead = 260;                 // right look-ahead bytes (>= 257)
constexpr uint32_t kTileBytes = 6464;                // >= kHalo + kTile + kLookAhead, x64
constexpr uint32_t kMaxChainSteps = 1024;            // per-position candidate budget before "unknown"
constexpr uint32_t kExtBudget = 24;                  // per-position long-match extensions before "unknown"
constexpr uint32_t kDenseUnknowns = 512;             // tile gives up all-position search past this
constexpr uint32_t kChunk = 8192;                    // symbols per histogram / encode workgroup
constexpr uint32_t kStreams = 4;                     // flags, chars, p-bits, golomb words
constexpr uint32_t kHuffHdrStride = 576;             // >= 1 + 64 + 510 bytes of tree header
constexpr uint32_t kLazyWindow = 8192;               // stitch kernel's LDS data window

// m[i] packs the match at position i: bits 0..10 distance p, bits 11..19 length L (0 = literal)
constexpr uint32_t kUnknown = 0xFFFFFFFFu;
__host__ __device__ inline uint32_t m_pack(uint32_t L, uint32_t p) { return (L << 11) | p; }
__host__ __device__ inline uint32_t m_len(uint32_t m) { return m >> 11; }
__host__ __device__ inline uint32_t m_dist(uint32_t m) { return m & 0x7FFu; }

constexpr uint32_t kTileLazy = 1u;   // tile_flags: spec parse unavailable, stitch walks it
constexpr uint32_t kTileMFull = 2u;  // tile_flags: m[] holds every match / unknown of the tile (run table ran)
constexpr uint32_t kTileUniform = 4u;  // tile_flags: the tile's window is one byte value; m is m_uniform, no m[] rows
constexpr uint32_t kTileSpan2 = 8u;    // tile_flags: m[] rows exact below kRmSpan (run-mode tiles), not just kResolveSpan

// m of block position i when the whole window [i - 2047, i + 258) and the block start
// side of it hold one byte value: every window position matches up to the cap, and the
// leftmost one wins (distance min(i, 2047)); literal at the block start and in the
// last three bytes (my_compress.cpp:1446-1514, 1675-1714)
__host__ __device__ inline uint32_t m_uniform(uint32_t i, uint32_t blen) {
    if (i == 0 || blen - i < 4) return 0u;
    const uint32_t L = (blen - i < kMaxL ? blen - i : kMaxL) - 1;
    return m_pack(L, i < kWin ? i : kWin);
}
constexpr uint32_t kResolveSpan = 256;           // k_resolve's walk limit; m[] rows always kept below it
constexpr uint32_t kRmSpan = 512;                // run-mode tiles keep m[] rows below this (kTileSpan2)
constexpr uint32_t kTileMatches = kTile / 4;     // compact match list slots per tile (a match covers >= 4)
constexpr uint32_t kConvAll = 0xFFFFu;           // tile conv record: k_emit takes every m from m[]
constexpr uint32_t kCharSeg = 64;                    // chars per segment descriptor (one k_encode lane's symbols)
constexpr uint32_t kErrScratch = 8u;                 // device error bit: inconsistent per-tile scratch (k_emit)
constexpr uint32_t kCdMixed = 0xFFFFFFFFu;       // chars segment descriptor: not a run of input bytes

// per-block results of the parse/emit stage
struct BlockInfo {
    uint32_t len;          // input bytes of the block
    uint32_t ntok;         // N
    uint32_t nmatch;       // pCnt
    uint32_t gbits;        // golomb bits
    uint32_t slen[kStreams];   // stream lengths in bytes
    uint32_t hdrlen[kStreams]; // Huffman tree header bytes (0 = stream absent / raw)
    uint32_t nwords[kStreams]; // Huffman code words W
    uint32_t words_rel[kStreams]; // byte offset of stream words inside the block record
    uint32_t rec_bytes;    // 4 + payload
    uint32_t lazy_evals;   // statistics
    uint32_t lazy_tiles;
    uint32_t pad;
};

struct Layout {
    uint64_t n;            // input bytes of the shard
    uint32_t B;            // block bytes
    uint32_t nblocks;
    uint32_t tpb;          // tiles per block
    uint32_t wpb;          // 64-bit chain words per block
    uint32_t sstride[kStreams];   // per-block stride of each stream buffer (bytes, x16)
    uint32_t cpb[kStreams];       // chunks per block per stream
    uint32_t cpb_total;           // sum of cpb
    uint32_t pad;
};

// ---- per-tile routing of the match search (fcx_route.hip) ------------------
// k_classify sorts the shard's tiles into one list per match unit; each unit's kernel then runs over
// its own list, so the unit that searches a tile depends only on that tile's bytes.
// Lists 0-3 are the match units (fcx_match_<unit>.hip); list 4 the uniform unit (fcx_match_uniform.hip:
// tiles whose sample is one byte value, checked over their whole window, the others handed on to runs).
enum : uint32_t {
    kRouteSparse = 0, kRouteRuns = 1, kRouteKey4 = 2, kRouteNoFilter = 3, kSearchUnits = 4,
    kRouteUniform = 4, kRoutes = 5
};
// route counters per block group (k_classify, the units' hand-ons, the host's cover mark): [0, kRoutes)
// list lengths, then these
constexpr uint32_t kRcNfFiled = 5;    // tiles the classifier filed as no-filter (its list grows by hand-ons)
constexpr uint32_t kRcValid = 6;      // tiles with bytes
constexpr uint32_t kRcCover = 7;      // the no-filter list's length at its listed launch
constexpr uint32_t kRcRunsFiled = 8;  // tiles the classifier filed as runs (its list grows by the uniform unit's hand-ons)
constexpr uint32_t kRouteWords = 16;
struct MatchRoute {
    const uint32_t *list = nullptr;   // the launch's tiles (null: the grid is every tile of the shard)
    const uint32_t *cnt = nullptr;    // entries in list
    uint32_t *defer_list = nullptr;   // sparse / runs units: where a tile they do not search goes (the
    uint32_t *defer_cnt = nullptr;    //   no-filter unit's list); null: their whole-tile run-table mode
    uint8_t *kind = nullptr;          // per tile: its unit (k_classify; a hand-on rewrites it).  With no
    uint32_t mine = 0;                //   list, the grid covers every tile and searches those of kind mine
};
struct RouteRest {                    // k_match_rest_<unit>: its list's entries no unit launch covered
    const uint32_t *list;
    const uint32_t *cnt;
    uint32_t start;                   // the first of them: the launch's grid (0: not launched; ~0: direct) ...
    const uint32_t *start_dev;        // ... or, when set, the smaller of it and the count read here (the
                                      //   entries the no-filter launch covered; later ones are hand-ons)
};

// ---- wave64 helpers --------------------------------------------------------
__device__ inline uint32_t lane_id() { return __lane_id(); }
// a value every lane of the wave holds alike, moved to a scalar register: loops and branches on
// it become scalar (no exec-mask bookkeeping) -- only for values that are wave-uniform
__device__ inline uint32_t uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }

__device__ inline uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        uint32_t t = __shfl_xor(v, o, 64);
        v = v > t ? v : t;
    }
    return v;
}

// sum over the 64 lanes (uniform result); every lane of the wave must be active
__device__ inline uint32_t wave_incl_scan(uint32_t v);
__device__ inline uint32_t wave_sum_u32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan(v), 63);
}

__device__ inline uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        uint32_t lo = __shfl_xor((uint32_t)v, o, 64);
        uint32_t hi = __shfl_xor((uint32_t)(v >> 32), o, 64);
        v += ((uint64_t)hi << 32) | lo;
    }
    return v;
}

// inclusive prefix sum across the 64 lanes, on the VALU through DPP lane moves (no LDS
// traffic): row_shr 1/2/4/8 within each row of 16, then row_bcast 15 / 31 carry the row
// totals upward.  Every lane of the wave must be active.
__device__ inline uint32_t wave_incl_scan(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);   // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);   // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);   // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);   // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);   // row_bcast:15 -> rows 1, 3
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);   // row_bcast:31 -> rows 2, 3
    return v;
}

// maximum over the 64 lanes (uniform), by DPP lane moves as wave_incl_scan (no LDS
// permutes); every lane of the wave must be active
__device__ inline uint32_t wave_max_dpp(uint32_t v) {
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false));   // row_shr:1
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false));   // row_shr:2
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false));   // row_shr:4
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false));   // row_shr:8
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false));   // row_bcast:15
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false));   // row_bcast:31
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// inclusive running maximum across the 64 lanes, DPP lane moves as wave_incl_scan; every lane of
// the wave must be active
__device__ inline uint32_t wave_incl_max_dpp(uint32_t v) {
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false));   // row_shr:1
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false));   // row_shr:2
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false));   // row_shr:4
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false));   // row_shr:8
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false));   // row_bcast:15
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false));   // row_bcast:31
    return v;
}

// inclusive running maximum across the 64 lanes
__device__ inline uint32_t wave_incl_max(uint32_t v) {
    const uint32_t lane = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t t = __shfl_up(v, o, 64);
        if (lane >= (uint32_t)o) v = max(v, t);
    }
    return v;
}

// unaligned 4-byte little-endian read from an LDS byte image backed by u32 words
__device__ inline uint32_t lds_ld4(const uint32_t *w, uint32_t pos) {
    uint32_t lo = w[pos >> 2], hi = w[(pos >> 2) + 1];
    return __builtin_amdgcn_alignbyte(hi, lo, pos & 3);
}
__device__ inline uint32_t lds_ld1(const uint32_t *w, uint32_t pos) {
    return (w[pos >> 2] >> ((pos & 3) * 8)) & 0xFFu;
}
__device__ inline uint32_t lds_key3(const uint32_t *w, uint32_t pos) { return lds_ld4(w, pos) & 0xFFFFFFu; }

// common-prefix length of the byte images at a and b, starting at `from`, capped at cap
__device__ inline uint32_t lds_match_len(const uint32_t *w, uint32_t a, uint32_t b, uint32_t from, uint32_t cap) {
    uint32_t L = from;
    while (L + 4 <= cap) {
        uint32_t x = lds_ld4(w, a + L) ^ lds_ld4(w, b + L);
        if (x) return L + (__builtin_ctz(x) >> 3);
        L += 4;
    }
    while (L < cap && lds_ld1(w, a + L) == lds_ld1(w, b + L)) L++;
    return L;
}


// ---- exact match over the run decomposition (dense windows: zeros, runs) ----
// Runs of equal bytes in an LDS byte image are described by a boundary bitmap
// (bit y: y == 0 or byte y != byte y-1; plus a sentinel bit at the image end),
// per-32-bit-word prefix counts, and the run table rt[k] = start | byte << 16
// (the sentinel entry carries byte 0x100).  For a query x with own run ending at
// e (r = e - x remaining bytes) and an earlier run k' of the same byte with A
// bytes available inside the window (from sp = max(start, xlo) to its end ep):
//   A <  r : the common prefix at sp is A (ep holds another byte, x + A does not);
//   A >= r : every j with ep - j > r gives exactly r (x + r holds another byte),
//            j* = ep - r gives r + ext, ext = common prefix of ep and e;
// candidates inside the own run give r.  Scanning runs left to right with a
// strict > keeps the leftmost maximum, which is the reference's choice
// (my_compress.cpp:1446-1514; SURVEY.md §0 finding 3).
constexpr uint32_t kRunBudget = 512;       // runs per window before the position stays "unknown"
constexpr uint32_t kRunTile = 1024;        // image runs up to which a tile skips the bucket search

// LDS address space: pointers of this type address LDS with 32-bit offsets (no generic-pointer
// conversion per access in out-of-line device functions)
#define FCX_LDS __attribute__((address_space(3)))

template <typename P32, typename P16>
__device__ inline uint32_t run_rank(P32 bm, P16 prc, uint32_t y) {
    // number of run boundaries at positions <= y
    const uint32_t sh = y & 31;
    const uint32_t msk = sh == 31 ? 0xFFFFFFFFu : ((2u << sh) - 1u);
    return prc[y >> 5] + (uint32_t)__builtin_popcount(bm[y >> 5] & msk);
}

// m of image position x (block position x + base), window from image position xlo,
// length cap; ok = false when the window holds more than kRunBudget runs.
__device__ inline uint32_t run_match(const uint32_t *img, const uint32_t *bm, const uint16_t *prc, const uint32_t *rt,
                                     uint32_t x, uint32_t xlo, uint32_t cap, bool &ok) {
    const uint32_t ko = run_rank(bm, prc, x) - 1;
    const uint32_t klo = run_rank(bm, prc, xlo) - 1;
    if (ko - klo > kRunBudget) { ok = false; return 0; }
    ok = true;
    const uint32_t own = rt[ko];
    const uint32_t c = own >> 16;
    const uint32_t e = rt[ko + 1] & 0xFFFFu;
    const uint32_t r = e - x;
    const bool big = r > cap;     // every same-byte candidate reaches min(A, cap)
    uint32_t bestL = 0, bestj = x;
    const uint32_t vb0 = rt[ko + 1];   // the run after the own run (query side of ext)
    bool done = false;
    uint32_t cur = rt[klo];
    for (uint32_t kk = klo; kk < ko && !done; kk += 4) {
        // four run-table entries in flight per step (rt holds >= 4 entries past the sentinel)
        const uint32_t v[5] = {cur, rt[kk + 1], rt[kk + 2], rt[kk + 3], rt[kk + 4]};
#pragma unroll
        for (uint32_t u = 0; u < 4; u++) {
            if (done || kk + u >= ko || (v[u] >> 16) != c) continue;
            const uint32_t sp = max(v[u] & 0xFFFFu, xlo), ep = v[u + 1] & 0xFFFFu;
            const uint32_t A = ep - sp;
            uint32_t Lc, j = sp;
            if (big) Lc = min(A, cap);
            else if (A < r) Lc = A;
            else {
                // ext at run granularity: equal (byte, length) runs extend it, the first
                // run that differs in length adds the shorter length and ends it.  The
                // query side meets the image end (sentinel) only past the cap.
                uint32_t ext = 0;
                if (r < cap) {
                    const uint32_t lim = cap - r;
                    uint32_t ka = kk + u + 1, kb = ko + 1, va = v[u + 1], vb = vb0;
                    for (;;) {
                        if ((va >> 16) != (vb >> 16)) break;
                        const uint32_t na = rt[ka + 1], nb = rt[kb + 1];
                        const uint32_t la = (na & 0xFFFFu) - (va & 0xFFFFu), lb = (nb & 0xFFFFu) - (vb & 0xFFFFu);
                        if (la != lb) { ext += min(la, lb); break; }
                        ext += la;
                        if (ext >= lim) break;
                        ka++; kb++; va = na; vb = nb;
                    }
                    ext = min(ext, lim);
                }
                Lc = min(r + ext, cap);
                if (ext) j = ep - r;
            }
            if (Lc > bestL) {
                bestL = Lc; bestj = j;
                done = bestL >= cap;
            }
        }
        cur = v[4];
    }
    const uint32_t sp = max(own & 0xFFFFu, xlo);
    if (bestL < cap && sp < x) {
        const uint32_t Lc = big ? cap : r;
        if (Lc > bestL) { bestL = Lc; bestj = sp; }
    }
    return bestL >= kMinL ? m_pack(bestL, x - bestj) : 0u;
}

// exact m of image position x (block position w0 + x) over the run table, by the whole wave:
// one window run per lane (64 per pass), each lane's best candidate in its run packed as
// L << 13 | (8191 - j), the wave maximum = the longest, then leftmost match (the rules of
// run_match, fcx_device.h).  ilen = block length - w0.  kUnknown: more than kRunBudget runs.
__device__ inline uint32_t run_match_wave(const FCX_LDS uint32_t *bm, const FCX_LDS uint16_t *prc,
                                          const FCX_LDS uint32_t *rt, uint32_t x, uint32_t ilen, uint32_t w0) {
    const uint32_t lane = lane_id();
    if (w0 + x == 0 || ilen - x < 4) return 0u;
    const uint32_t cap = min(kMaxL, ilen - x) - 1;
    const uint32_t xlo = max(w0 + x, kWin) - kWin - w0;
    // (x is wave-uniform and so is everything derived from it: scalar registers, scalar branches)
    const uint32_t ko = uni(run_rank(bm, prc, x) - 1), klo = uni(run_rank(bm, prc, xlo) - 1);   // one round of loads
    if (ko - klo > kRunBudget) return kUnknown;
    // second round: the own run and the run after it (the query side of ext), and each lane's
    // candidate run with the two after it, all issued together (clamped indices, no branch);
    // the first step of the ext walk needs nothing more
    const uint32_t own = uni(rt[ko]), vb0 = uni(rt[ko + 1]), vb1 = uni(rt[ko + 2]);
    const uint32_t c = own >> 16, r = (vb0 & 0xFFFFu) - x;
    const bool big = r > cap;
    uint32_t best = 0;
    for (uint32_t k0 = klo; k0 < ko; k0 += 64) {
        const uint32_t kc = min(k0 + lane, ko);
        const uint32_t v = rt[kc], nv = rt[kc + 1], nnv = rt[kc + 2];
        const uint32_t sp = max(v & 0xFFFFu, xlo), ep = nv & 0xFFFFu;
        if (k0 + lane >= ko || (v >> 16) != c || ep <= xlo) continue;
        const uint32_t A = ep - sp;
        uint32_t Lc, j = sp;
        if (big) Lc = min(A, cap);
        else if (A < r) Lc = A;
        else {
            // ext at run granularity (equal (byte, length) runs extend it, the first length
            // mismatch adds the shorter length); the query side meets the image end only past the cap
            uint32_t ext = 0;
            if (r < cap && (nv >> 16) == (vb0 >> 16)) {
                const uint32_t lim = cap - r;
                uint32_t la = (nnv & 0xFFFFu) - (nv & 0xFFFFu), lb = (vb1 & 0xFFFFu) - (vb0 & 0xFFFFu);
                if (la != lb) ext = min(la, lb);
                else {   // rare: a whole run of equal byte and length, keep walking
                    ext = la;
                    uint32_t ka = kc + 2, kb = ko + 2, va = nnv, vb = vb1;
                    while (ext < lim && (va >> 16) == (vb >> 16)) {
                        const uint32_t na = rt[ka + 1], nb = rt[kb + 1];
                        la = (na & 0xFFFFu) - (va & 0xFFFFu);
                        lb = (nb & 0xFFFFu) - (vb & 0xFFFFu);
                        if (la != lb) { ext += min(la, lb); break; }
                        ext += la;
                        ka++; kb++; va = na; vb = nb;
                    }
                }
                ext = min(ext, lim);
            }
            Lc = min(r + ext, cap);
            if (ext) j = ep - r;
        }
        best = max(best, (Lc << 13) | (8191u - j));
    }
    const uint32_t sp = max(own & 0xFFFFu, xlo);   // candidates inside the own run give r
    if (sp < x) best = max(best, ((big ? cap : r) << 13) | (8191u - sp));
    best = wave_max_dpp(best);
    const uint32_t L = best >> 13;
    return L >= kMinL ? m_pack(L, x - (8191u - (best & 0x1FFFu))) : 0u;
}

}  // namespace fcx

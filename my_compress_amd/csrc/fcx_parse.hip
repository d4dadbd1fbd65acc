// fcx_parse.hip — greedy-parse resolution across tiles and token emission (gfx950).
//
// The reference parse (my_LZ77_compress, my_compress.cpp:1675-1714) is one serial
// chain: cursor += l + 1.  k_match resolved it inside each tile under the
// assumption that a token starts at the tile's first position.  Here:
//
//   k_resolve one wave per tile, all tiles in parallel: assuming the entry is the
//             previous tile's speculative exit, walk the true chain until it meets
//             this tile's speculative chain and record the corrected counts, exit
//             and rewritten chain words.
//   k_stitch  one wave per block walks the tiles in order with the true entry
//             point.  Fast path: the entry is the one k_resolve assumed, so commit
//             its record (counts, exit, <= 4 chain words).  Slow path: walk the true chain through the tile's
//             m[] (staged in LDS) until it meets the speculative chain; positions
//             k_match left unknown (dense windows) are evaluated by the whole wave:
//             64 candidates per step, oldest first, pruned by the byte at the
//             current best length, early exit at the cap.  Per-tile token / match /
//             golomb-bit counts come from k_match's prefix counts minus the
//             speculative positions dropped before the entry, and are scanned here
//             into per-tile offsets and the block totals.
//   k_emit    writes the four streams of the block payload (make_bitMap_table
//             2073-2113, the split at 2150-2161, combine_bits 1292-1313,
//             golomb_rice_encode 258-304): bits are gathered per lane, merged in
//             LDS and stored as whole words (edge words of a tile by atomicOr);
//             chars are staged in LDS and stored as aligned dwords, except those of
//             all-literal tiles, which stay in the input: a descriptor per 64 chars
//             tells k_encode where to read them.  The tile's chars histogram goes out
//             as a row of u16 counts.
#include "fcx_device.h"

namespace fcx {

// ---------------------------------------------------------------------------
// wave-parallel exact match at position t (block-relative), window data in LDS
// image `dw` whose byte 0 is block position dbase.
__device__ uint32_t lazy_match(const uint32_t *dw, uint32_t dbase, uint32_t blen, uint32_t t) {
    if (t == 0 || blen - t < 4) return 0;
    const uint32_t lane = lane_id();
    const uint32_t cap = min(kMaxL, blen - t) - 1;
    const uint32_t x = t - dbase;
    const uint32_t xlo = (t > kWin ? t - kWin : 0) - dbase;
    const uint32_t key = lds_key3(dw, x);
    uint32_t best = kMinL - 1, bestx = x;
    for (uint32_t cb = xlo; cb < x; cb += 64) {
        const uint32_t xe = cb + lane;
        uint32_t Lc = 0;
        if (xe < x && lds_key3(dw, xe) == key &&
            (best < kMinL || lds_ld1(dw, xe + best) == lds_ld1(dw, x + best)))
            Lc = lds_match_len(dw, xe, x, kMinL, cap);
        // the step's longest, then leftmost candidate in one DPP maximum (window positions < 2^15)
        const uint32_t mk = wave_max_dpp(Lc ? (Lc << 15) | (32767u - xe) : 0u);
        if ((mk >> 15) > best) {   // strict: an earlier step's candidate wins a tie (leftmost)
            best = mk >> 15;
            bestx = 32767u - (mk & 0x7FFFu);
        }
        if (best >= cap) break;
    }
    return best >= kMinL ? m_pack(best, x - bestx) : 0u;
}

// Exact m of block position t for the stitch over a run table of its window [t - 2047, t + 258),
// built from the staged bytes dw (dw byte 0 = block position dbase): the run decomposition gives
// the leftmost-longest match in closed form (run_match, fcx_device.h), evaluated by the wave
// (run_match_wave) -- a few thousand cycles where the byte-by-byte window search (lazy_match)
// spends 10^5 on long-run data.  kUnknown when the window holds more runs than the table holds
// or than kRunBudget: the caller then searches byte by byte.
constexpr uint32_t kStRunCap = 1020;                        // run table entries (window runs + sentinel)
constexpr uint32_t kStBmWords = (kWin + kMaxL + 1) / 32 + 2;   // boundary bits 0 .. 2305
__device__ uint32_t stitch_run_match(const uint32_t *dw, uint32_t dbase, uint32_t blen, uint32_t t,
                                     FCX_LDS uint32_t *bm, FCX_LDS uint16_t *prc, FCX_LDS uint32_t *rt) {
    const uint32_t lane = lane_id();
    dbase = uni(dbase); blen = uni(blen); t = uni(t);
    const uint32_t lo = t > kWin ? t - kWin : 0;          // image position 0 = block position lo
    const uint32_t n = min(t + kMaxL, blen) - lo;         // image bytes (a match from t stays inside)
    const uint32_t ib = lo - dbase;                       // dw byte of image position 0
    for (uint32_t y0 = 0; y0 <= n; y0 += 64) {            // boundary bitmap by ballot; sentinel bit at n
        const uint32_t y = y0 + lane;
        const bool bit = y == n || (y < n && (y == 0 || lds_ld1(dw, ib + y) != lds_ld1(dw, ib + y - 1)));
        const uint64_t bal = __ballot(bit);
        if (lane == 0) { bm[y0 >> 5] = (uint32_t)bal; bm[(y0 >> 5) + 1] = (uint32_t)(bal >> 32); }
    }
    __builtin_amdgcn_wave_barrier();
    const uint32_t nw = (n >> 5) + 1;                     // words holding bits 0 .. n
    const uint32_t c0 = lane < nw ? (uint32_t)__builtin_popcount(bm[lane]) : 0u;
    const uint32_t c1 = lane + 64 < nw ? (uint32_t)__builtin_popcount(bm[lane + 64]) : 0u;
    const uint32_t i0 = wave_incl_scan(c0), i1 = wave_incl_scan(c1);
    const uint32_t t0s = (uint32_t)__builtin_amdgcn_readlane((int)i0, 63);
    const uint32_t nruns = t0s + (uint32_t)__builtin_amdgcn_readlane((int)i1, 63);
    if (nruns > kStRunCap) return kUnknown;
    const uint32_t p0 = i0 - c0, p1 = t0s + i1 - c1;
    if (lane < nw) prc[lane] = (uint16_t)p0;
    if (lane + 64 < nw) prc[lane + 64] = (uint16_t)p1;
#pragma unroll
    for (uint32_t h = 0; h < 2; h++) {                    // run table: start | byte << 16 (sentinel 0x100)
        const uint32_t w = lane + 64 * h;
        if (w >= nw) continue;
        uint32_t o = h ? p1 : p0;
        for (uint32_t v = bm[w]; v; v &= v - 1, o++) {
            const uint32_t y = 32 * w + (uint32_t)__builtin_ctz(v);
            rt[o] = y | (y < n ? lds_ld1(dw, ib + y) << 16 : 0x1000000u);
        }
    }
    __builtin_amdgcn_wave_barrier();
    return run_match_wave(bm, prc, rt, t - lo, blen - lo, lo);
}

// stage block bytes [dbase, dbase + kLazyWindow) into dw (zero padded)
__device__ void load_window(uint32_t *dw, const uint8_t *d, uint32_t dbase, uint32_t blen) {
    const uint32_t lane = lane_id();
    const uint32_t nload = min(kLazyWindow, blen - dbase);
    const uint8_t *src = d + dbase;
    if ((((uintptr_t)src) & 3) == 0) {
        const uint32_t *src4 = (const uint32_t *)src;
        const uint32_t nfull = nload >> 2;
        for (uint32_t x = lane; x < kLazyWindow / 4 + 4; x += 64) {
            uint32_t v = 0;
            if (x < nfull) v = src4[x];
            else if (x == nfull)
                for (uint32_t q = 0; q < (nload & 3); q++) v |= (uint32_t)src[4 * x + q] << (8 * q);
            dw[x] = v;
        }
    } else {
        for (uint32_t x = lane; x < kLazyWindow / 4 + 4; x += 64) {
            uint32_t v = 0;
            for (uint32_t q = 0; q < 4; q++)
                if (4 * x + q < nload) v |= (uint32_t)src[4 * x + q] << (8 * q);
            dw[x] = v;
        }
    }
}

struct Cnt3 {
    uint32_t tok, mat, gb;
    __device__ void add(uint32_t L) {
        tok++;
        if (L) { mat++; gb += (L >> 2) + 3; }
    }
};

// counts of the speculative chain positions in [t0, t0 + rel): k_match's prefix
// for the word plus the set bits of the (original) word below rel.  Wave-wide.
__device__ Cnt3 spec_prefix(const uint64_t *pfx, const uint32_t *mt, const uint64_t *mb, uint64_t orig_word,
                            uint32_t rel, bool uni, uint32_t t0, uint32_t blen) {
    const uint32_t lane = lane_id();
    const uint32_t w = rel >> 6, r = rel & 63;
    const uint64_t p = pfx[w];
    Cnt3 c{(uint32_t)(p & 0x1FFFu), (uint32_t)((p >> 13) & 0x7FFu), (uint32_t)((p >> 24) & 0x1FFFu)};
    const uint64_t below = r ? (orig_word & ((1ull << r) - 1)) : 0ull;
    uint32_t mt_ = 0, gb = 0;
    if ((below >> lane) & (mb[w] >> lane) & 1ull) {
        const uint32_t L = m_len(uni ? m_uniform(t0 + w * 64 + lane, blen) : mt[w * 64 + lane]);
        if (L) { mt_ = 1; gb = (L >> 2) + 3; }
    }
    c.tok += (uint32_t)__popcll(below);
    c.mat += wave_sum_u32(mt_);
    c.gb += wave_sum_u32(gb);
    return c;
}

// the same counts for a tile whose m[] rows stop at kResolveSpan: the dropped
// speculative match tokens are the first entries of the tile's compact match list
// (k_match writes them in chain order), so their golomb bits come from there
__device__ Cnt3 spec_prefix_c(const uint64_t *pfx, const uint32_t *mtt, const uint64_t *mb, uint64_t orig_word,
                              uint32_t rel) {
    const uint32_t lane = lane_id();
    const uint32_t w = rel >> 6, r = rel & 63;
    const uint64_t p = pfx[w];
    Cnt3 c{(uint32_t)(p & 0x1FFFu), (uint32_t)((p >> 13) & 0x7FFu), (uint32_t)((p >> 24) & 0x1FFFu)};
    const uint64_t below = r ? (orig_word & ((1ull << r) - 1)) : 0ull;
    const uint32_t nm = (uint32_t)__popcll(below & mb[w]);   // no unknowns: mbits = matches
    uint32_t gb = 0;
    if (lane < nm) {
        const uint32_t L = m_len(mtt[c.mat + lane]);
        gb = (L >> 2) + 3;
    }
    c.tok += (uint32_t)__popcll(below);
    c.mat += nm;
    c.gb += wave_sum_u32(gb);
    return c;
}

// Fast-path resolution per tile, for all tiles in parallel ahead of the
// sequential stitch.  Assume the true entry is the previous tile's speculative
// exit (it is whenever the previous tile was resolved this way) and walk the
// greedy chain from it until it meets this tile's speculative chain — usually
// within a few tokens.  Recorded per tile (fp[8*tix]):
//   [0] ok | rel << 1 (assumed entry - t0) | nmod << 16 (chain words rewritten)
//   [1] tokens | matches << 32, [2] golomb bits | conv << 32 (the tile's final counts;
//       conv = rel | dropped speculative matches << 16 where the walk met the
//       speculative chain, kConvAll if it walked to the tile end)
//   [3] exit (first chain position >= t1)
//   [4..11] the rewritten chain words 0..nmod-1 (positions t0 .. t0 + 64 nmod - 1)
// The walk reaches kResolveSpan positions, kRmSpan on run-mode tiles (their m rows are exact that
// far: long tokens take longer to meet the speculative chain).  ok = 0 when the walk needs more,
// meets an unknown position, or a neighbour is lazy: the stitch then walks the tile itself.
constexpr uint32_t kFpStride = 12;               // u64 per tile record
constexpr uint32_t kResW = kRmSpan / 64;         // chain words a walk may rewrite
static_assert(kFpStride >= 4 + kResW && kRmSpan >= kResolveSpan, "resolve record");

__global__ __launch_bounds__(64) void k_resolve(Layout L, const uint32_t *__restrict__ m,
                                                const uint64_t *__restrict__ mbits,
                                                const uint64_t *__restrict__ chain,
                                                const uint64_t *__restrict__ chain_pfx,
                                                const uint32_t *__restrict__ tinfo, uint64_t *__restrict__ fp) {
    const uint32_t lane = threadIdx.x, tix = blockIdx.x;
    const uint32_t b = tix / L.tpb, k = tix % L.tpb;
    const uint64_t bstart = (uint64_t)b * L.B;
    const uint32_t blen = (uint32_t)min((uint64_t)L.B, L.n - bstart);
    const uint32_t t0 = k * kTile;
    if (t0 >= blen) return;
    const uint32_t t1 = min(blen, t0 + kTile);
    uint64_t *out = fp + (uint64_t)kFpStride * tix;
    // this tile's flags, the previous one's flags and exit, and this tile's chain and mbits words (one
    // per lane: in the block's words for every lane), all read before the first branch: the compiler
    // does not move a load above one (the conditional form waited for six dependent round trips)
    const uint32_t *ti = tinfo + 8ull * tix, *tp = tinfo + 8ull * (k > 0 ? tix - 1 : tix);
    const uint32_t f0 = ti[0], pf0 = tp[0], pexit = tp[1];
    const uint64_t *cw = chain + (uint64_t)b * L.wpb + (uint64_t)k * (kTile / 64);
    const uint64_t *mb = mbits + (uint64_t)b * L.wpb + (uint64_t)k * (kTile / 64);
    uint64_t wv = cw[lane], mv = mb[lane];
    asm volatile("" ::"s"(f0), "s"(pf0), "s"(pexit), "v"(wv), "v"(mv));
    const bool uni = (f0 & kTileUniform) != 0;   // m = m_uniform, no rows
    const uint32_t span = (f0 & kTileSpan2) ? kRmSpan : kResolveSpan;   // m rows exact below it
    const uint32_t ea = k > 0 ? pexit : t0;
    // (a uniform tile's record is never used: k_stitch commits uniform tiles in closed form; skipping
    // its walk took zeros' resolve + stitch from 0.207 to 0.117 ms per GiB)
    bool ok = (f0 & (kTileLazy | kTileUniform)) == 0 && (k == 0 || (pf0 & kTileLazy) == 0) && ea < t1 && ea - t0 < span;
    if (!ok) {
        if (lane == 0) out[0] = 0;
        return;
    }
    const uint32_t rel0 = ea - t0;
    const uint32_t *mt = m + bstart + t0;
    const uint32_t nw = min(span / 64, (t1 - t0 + 63) / 64);
    // chain + mbits words below the span (lanes 0..nw-1); m of those positions below
    if (lane >= nw) { wv = 0; mv = 0; }
    // chain / mbits words stay distributed (lane q holds word q); the walk reads word q of the
    // wave-uniform position by readlane, and lane q keeps the walked bits of word q
    auto word_at = [](uint64_t v, uint32_t q) -> uint64_t {
        return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)q) |
               ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), (int)q) << 32);
    };
    // the assumed entry on the speculative chain (the previous tile's exit is t0 and the chain
    // starts there: random data's tiles): the walk ends before it starts, no m row is needed
    const bool at_chain = rel0 < t1 - t0 && ((word_at(wv, fcx::uni(rel0 >> 6)) >> (rel0 & 63)) & 1ull);
    uint32_t mreg[kResW];
#pragma unroll
    for (uint32_t q = 0; q < kResW; q++) {
        const uint32_t x = 64 * q + lane;
        const uint64_t mbq = __shfl(mv, q, 64);
        mreg[q] = (!at_chain && q < nw && x < t1 - t0 && ((mbq >> lane) & 1ull)) ? (uni ? m_uniform(t0 + x, blen) : mt[x])
                                                                                : 0u;
    }
    uint64_t nwb = 0;
    // walk from the assumed entry until it meets the speculative chain (uniform over the wave)
    Cnt3 walked{0, 0, 0};
    uint32_t rel = rel0, exitv = 0;
    bool conv = false;
    for (;;) {
        if (rel >= t1 - t0) { exitv = t0 + rel; break; }
        if (rel >= span) { ok = false; break; }
        const uint32_t q = fcx::uni(rel >> 6), r = rel & 63;
        const uint64_t o = word_at(wv, q), mbq = word_at(mv, q);
        if ((o >> r) & 1ull) { conv = true; break; }
        uint32_t mm = 0;
        if ((mbq >> r) & 1ull) {
            uint32_t v = mreg[0];
#pragma unroll
            for (uint32_t u = 1; u < kResW; u++) if (q == u) v = mreg[u];
            mm = __shfl(v, r, 64);
        }
        if (mm == kUnknown) { ok = false; break; }
        if (lane == q) nwb |= 1ull << r;
        walked.add(m_len(mm));
        rel += m_len(mm) + 1;
    }
    if (!ok) {
        if (lane == 0) out[0] = 0;
        return;
    }
    Cnt3 fin = walked;
    uint32_t keep_from = rel;   // speculative bits at positions >= keep_from stay
    uint32_t convrec = kConvAll;
    if (conv) {
        const Cnt3 drop = rel ? spec_prefix(chain_pfx + (uint64_t)tix * (kTile / 64), mt, mb, word_at(wv, fcx::uni(rel >> 6)),
                                            rel, uni, t0, blen)
                              : Cnt3{0, 0, 0};
        fin.tok += ti[2] - drop.tok;
        fin.mat += ti[3] - drop.mat;
        fin.gb += ti[4] - drop.gb;
        exitv = ti[1];
        convrec = rel | (drop.mat << 16);
    } else {
        keep_from = t1 - t0;   // the walk covered the rest of the tile
    }
    // rewritten words: walked bits below keep_from, speculative bits from keep_from on
    const uint32_t nmod = min(nw, (min(keep_from, span) + 63) / 64);
    if (lane < nmod) {
        const uint32_t lo = 64 * lane;
        uint64_t keepmask;
        if (keep_from <= lo) keepmask = ~0ull;
        else if (keep_from >= lo + 64) keepmask = 0;
        else keepmask = ~0ull << (keep_from - lo);
        out[4 + lane] = (wv & keepmask) | nwb;
    }
    if (lane == 0) {
        out[0] = 1ull | ((uint64_t)rel0 << 1) | ((uint64_t)nmod << 16);
        out[1] = (uint64_t)fin.tok | ((uint64_t)fin.mat << 32);
        out[2] = fin.gb | ((uint64_t)convrec << 32);
        out[3] = exitv;
    }
    (void)conv;
}

// one tile's m rows (16 x 16 B per lane), mbits word and chain word (lane < nw), all in
// flight together
__device__ inline void fetch_tile(const uint32_t *mt, const uint64_t *mb, const uint64_t *cw, uint32_t nt, uint32_t nw,
                                  uint4 *v, uint64_t &mbw, uint64_t &cwv) {
    const uint32_t lane = lane_id();
#pragma unroll
    for (uint32_t q = 0; q < kTile / 256; q++) {
        const uint32_t x = 4 * (lane + 64 * q);
        v[q] = x + 4 <= nt ? ((const uint4 *)mt)[lane + 64 * q] : make_uint4(0, 0, 0, 0);
    }
    mbw = lane < nw ? mb[lane] : 0ull;
    cwv = lane < nw ? cw[lane] : 0ull;
}

// k_emit ORs each tile's two edge words of the flags, distance and golomb streams (the
// words it shares with its neighbours); the stitch zeroes them at every tile boundary
// (and the word after the block's last bit: the distance stream's (11 pCnt)/8 + 1 bytes
// reach one byte past its bits), so the streams need no memset.  Lanes 8..13.
__device__ inline void zero_edges(uint8_t *s_flags, uint8_t *s_p, uint8_t *s_golomb, const Layout &L, uint32_t b,
                                  uint32_t tok, uint32_t mat, uint32_t gb) {
    const uint32_t lane = lane_id();
    if (lane < 8 || lane >= 14) return;
    const uint32_t k = lane - 8, st = k >> 1;
    const uint32_t pos = st == 0 ? tok : st == 1 ? kPBits * mat : gb;   // bit position of the boundary
    if ((k & 1) == 0 && pos == 0) return;
    const uint32_t wd = (k & 1) ? pos >> 5 : (pos - 1) >> 5;
    uint8_t *base = st == 0 ? s_flags : st == 1 ? s_p : s_golomb;
    ((uint32_t *)(base + (uint64_t)b * L.sstride[st == 0 ? 0 : st == 1 ? 2 : 3]))[wd] = 0u;
}

// the same six words, all from the calling lane (the batched fast path: one lane per tile)
__device__ inline void zero_edges_lane(uint8_t *s_flags, uint8_t *s_p, uint8_t *s_golomb, const Layout &L, uint32_t b,
                                       uint32_t tok, uint32_t mat, uint32_t gb) {
#pragma unroll
    for (uint32_t st = 0; st < 3; st++) {
        const uint32_t pos = st == 0 ? tok : st == 1 ? kPBits * mat : gb;
        uint32_t *w = (uint32_t *)((st == 0 ? s_flags : st == 1 ? s_p : s_golomb) +
                                   (uint64_t)b * L.sstride[st == 0 ? 0 : st == 1 ? 2 : 3]);
        if (pos) w[(pos - 1) >> 5] = 0u;
        w[pos >> 5] = 0u;
    }
}

__global__ __launch_bounds__(64) void k_stitch(const uint8_t *__restrict__ in, Layout L, uint32_t *__restrict__ m,
                                               const uint64_t *__restrict__ mbits, uint64_t *__restrict__ chain, const uint64_t *__restrict__ chain_pfx,
                                               const uint32_t *__restrict__ tinfo, const uint64_t *__restrict__ fp,
                                               const uint32_t *__restrict__ mtok, uint32_t *__restrict__ tile_off,
                                               uint32_t *__restrict__ tconv, BlockInfo *__restrict__ binfo,
                                               uint8_t *__restrict__ s_flags, uint8_t *__restrict__ s_p,
                                               uint8_t *__restrict__ s_golomb) {
    __shared__ uint32_t mL[kTile];
    __shared__ uint32_t sti[64][6];          // per tile of the batch: flags, exit, totals, k_resolve verdict
    __shared__ uint32_t sfp[64][5];          // k_resolve: final counts, exit, conv record
    __shared__ uint64_t sfw[64][kResW];      // k_resolve: rewritten chain words
    __shared__ uint64_t bmL[kTile / 64];
    __shared__ uint64_t mbL[kTile / 64];
    __shared__ uint32_t dw[kLazyWindow / 4 + 4];
    __shared__ uint32_t srm_bm[kStBmWords], srm_rt[kStRunCap + 4];   // stitch_run_match's run table
    __shared__ uint16_t srm_prc[kStBmWords];

    const uint32_t lane = threadIdx.x;
    const uint32_t b = blockIdx.x;
    const uint64_t bstart = (uint64_t)b * L.B;
    const uint32_t blen = (uint32_t)min((uint64_t)L.B, L.n - bstart);
    const uint8_t *d = in + bstart;
    const uint32_t ntiles = (blen + kTile - 1) / kTile;
    uint32_t e = 0, dbase = 0xFFFFFFFFu, nlazy = 0, lazy_tiles = 0;
    Cnt3 run{0, 0, 0};
    uint4 pv[kTile / 256];   // prefetched rows / mbits / chain word of tile pk
    uint64_t pmb = 0, pcw = 0;
    uint32_t pk = 0xFFFFFFFFu;

    for (uint32_t k = 0; k < ntiles; k++) {
        const uint32_t t0 = k * kTile, t1 = min(blen, t0 + kTile);
        const uint32_t tix = b * L.tpb + k;
        const uint32_t j = k & 63;
        if (j == 0) {   // prefetch the next 64 tiles' info (independent loads, one tile per lane)
            __syncthreads();
            const uint32_t kk = k + lane;
            if (kk < ntiles) {
                const uint32_t *tq = tinfo + 8ull * (b * L.tpb + kk);
                const uint64_t *fq = fp + (uint64_t)kFpStride * (b * L.tpb + kk);
                sti[lane][0] = tq[0]; sti[lane][1] = tq[1]; sti[lane][2] = tq[2];
                sti[lane][3] = tq[3]; sti[lane][4] = tq[4];
                const uint64_t f0 = fq[0];
                // (nmod <= kResW by construction; clamped so that a bad record cannot index past
                // the tile's chain words)
                const uint32_t nmod = min((uint32_t)(f0 >> 16) & 0xFFu, kResW);
                sti[lane][5] = ((uint32_t)f0 & 0xFFFFu) | (nmod << 16);
                if (f0 & 1ull) {
                    const uint64_t f1 = fq[1];
                    sfp[lane][0] = (uint32_t)f1; sfp[lane][1] = (uint32_t)(f1 >> 32);
                    const uint64_t f2 = fq[2];
                    sfp[lane][2] = (uint32_t)f2; sfp[lane][3] = (uint32_t)fq[3]; sfp[lane][4] = (uint32_t)(f2 >> 32);
                    for (uint32_t u = 0; u < nmod; u++) sfw[lane][u] = fq[4 + u];
                }
            }
            __syncthreads();
        }
        {   // batched fast path: the leading tiles of the batch whose k_resolve record applies
            // (each one's assumed entry is its predecessor's recorded exit, starting from e)
            // are committed at once, one lane per tile, counts by a wave prefix sum
            const uint32_t u = lane, jj = j + u, kk = k + u;
            bool ok = jj < 64 && kk < ntiles;
            uint32_t ct = 0, cm = 0, cg = 0;
            if (ok) {
                const uint32_t t0u = kk * kTile, t1u = min(blen, t0u + kTile);
                const uint32_t eu = u == 0 ? e : sfp[jj - 1][3];
                const uint32_t fpv = sti[jj][5];
                ok = (sti[jj][0] & kTileUniform) == 0 && (fpv & 1u) && eu >= t0u && eu < t1u &&
                     eu - t0u == ((fpv >> 1) & 0x7FFFu);
            }
            const uint64_t okm = __ballot(ok);
            const uint32_t F = ~okm ? (uint32_t)__builtin_ctzll(~okm) : 64u;   // leading committed tiles
            if (F >= 2) {
                if (u < F) { ct = sfp[jj][0]; cm = sfp[jj][1]; cg = sfp[jj][2]; }
                const uint32_t it = wave_incl_scan(ct), im = wave_incl_scan(cm), ig = wave_incl_scan(cg);
                if (u < F) {
                    const uint32_t tixu = tix + u;
                    const uint32_t pt = run.tok + it - ct, pm = run.mat + im - cm, pg = run.gb + ig - cg;
                    tile_off[3 * tixu + 0] = pt;
                    tile_off[3 * tixu + 1] = pm;
                    tile_off[3 * tixu + 2] = pg;
                    zero_edges_lane(s_flags, s_p, s_golomb, L, b, pt, pm, pg);
                    const uint32_t fpv = sti[jj][5], nmod = fpv >> 16;
                    uint64_t *cwu = chain + (uint64_t)b * L.wpb + (uint64_t)kk * (kTile / 64);
                    for (uint32_t w = 0; w < nmod; w++) cwu[w] = sfw[jj][w];
                    tconv[tixu] = (sti[jj][0] & kTileMFull) ? kConvAll : sfp[jj][4];
                }
                run.tok += (uint32_t)__builtin_amdgcn_readlane((int)it, (int)(F - 1));
                run.mat += (uint32_t)__builtin_amdgcn_readlane((int)im, (int)(F - 1));
                run.gb += (uint32_t)__builtin_amdgcn_readlane((int)ig, (int)(F - 1));
                e = sfp[j + F - 1][3];
                k += F - 1;
                continue;
            }
        }
        {   // batched uniform tiles: where every token is 258 long (one byte value, no block
            // start, >= 258 bytes to the block end) the chain from e is e + 258 m, so the
            // leading such tiles of the batch are committed at once in closed form
            constexpr uint32_t kStep = kMaxL;                 // L = 257, cursor += 258
            constexpr uint32_t kGb = ((kMaxL - 1) >> 2) + 3;  // golomb bits of one such token
            const uint32_t u = lane, jj = j + u, kk = k + u;
            const uint32_t t0u = kk * kTile, t1u = min(blen, t0u + kTile);
            const bool ok = jj < 64 && kk < ntiles && (sti[jj][0] & kTileUniform) && t0u >= 1 && t1u + kMaxL - 1 <= blen &&
                            e >= t0 && e < t1;
            const uint64_t okm = __ballot(ok);
            const uint32_t F = ~okm ? (uint32_t)__builtin_ctzll(~okm) : 64u;
            if (F >= 2) {
                uint32_t nt = 0, eu = 0;
                if (u < F) {
                    eu = u == 0 ? e : e + kStep * ((t0u - e + kStep - 1) / kStep);   // first chain position >= t0u
                    nt = (t1u - eu + kStep - 1) / kStep;
                }
                const uint32_t it = wave_incl_scan(nt);
                if (u < F) {
                    const uint32_t tixu = tix + u;
                    const uint32_t pt = run.tok + it - nt, pm = run.mat + it - nt, pg = run.gb + kGb * (it - nt);
                    tile_off[3 * tixu + 0] = pt;
                    tile_off[3 * tixu + 1] = pm;
                    tile_off[3 * tixu + 2] = pg;
                    zero_edges_lane(s_flags, s_p, s_golomb, L, b, pt, pm, pg);
                    tconv[tixu] = kConvAll;
                }
                // the tiles' chain words, tile by tile with one word per lane (coalesced stores; one
                // lane per tile looping over its 64 words stored 64 lines per instruction)
                for (uint32_t i = 0; i < F; i++) {
                    const uint32_t eui = (uint32_t)__builtin_amdgcn_readlane((int)eu, (int)i);
                    const uint32_t t0i = (k + i) * kTile, t1i = min(blen, t0i + kTile), lo = t0i + 64 * lane;
                    if (lo < t1i) {
                        const uint32_t p = lo <= eui ? eui : eui + kStep * ((lo - eui + kStep - 1) / kStep);
                        chain[(uint64_t)b * L.wpb + (uint64_t)(k + i) * (kTile / 64) + lane] =
                            p < min(lo + 64, t1i) ? 1ull << (p - lo) : 0ull;
                    }
                }
                const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)it, (int)(F - 1));
                run.tok += tot;
                run.mat += tot;
                run.gb += kGb * tot;
                const uint32_t eF = (uint32_t)__builtin_amdgcn_readlane((int)eu, (int)(F - 1)),
                               nF = (uint32_t)__builtin_amdgcn_readlane((int)nt, (int)(F - 1));
                e = eF + kStep * nF;
                k += F - 1;
                continue;
            }
        }
        const bool lazy = (sti[j][0] & kTileLazy) != 0;
        const bool mfull = (sti[j][0] & kTileMFull) != 0;   // else m[] rows stop at kResolveSpan
        const bool uni = (sti[j][0] & kTileUniform) != 0;  // m = m_uniform, no rows
        const uint32_t span = (sti[j][0] & kTileSpan2) ? kRmSpan : kResolveSpan;   // m rows exact below it
        uint64_t *cw = chain + (uint64_t)b * L.wpb + (uint64_t)k * (kTile / 64);
        const uint64_t *pfx = chain_pfx + (uint64_t)tix * (kTile / 64);
        const uint64_t *mb = mbits + (uint64_t)b * L.wpb + (uint64_t)k * (kTile / 64);
        const uint32_t *mt = m + bstart + t0;
        const uint32_t nw = (t1 - t0 + 63) / 64;
        if (lane < 3) tile_off[3 * tix + lane] = lane == 0 ? run.tok : lane == 1 ? run.mat : run.gb;
        zero_edges(s_flags, s_p, s_golomb, L, b, run.tok, run.mat, run.gb);
        if (e >= t1) {  // a match spans the whole tile
            for (uint32_t w = lane; w < nw; w += 64) cw[w] = 0;
            if (lane == 0) tconv[tix] = kConvAll;
            continue;
        }
        if (uni) {
            // one byte value: the chain from e follows from m_uniform.  Every lane walks it
            // to the tile end (<= 17 tokens, ALU only) counting the tokens and keeping the
            // bits of its chain word
            Cnt3 w{0, 0, 0};
            uint64_t wv = 0;
            const uint32_t lo = t0 + 64 * lane;
            uint32_t t = e;
            while (t < t1) {
                const uint32_t Lm = m_len(m_uniform(t, blen));
                w.add(Lm);
                if (t - lo < 64) wv |= 1ull << (t - lo);
                t += Lm + 1;
            }
            if (lane < nw) cw[lane] = wv;
            if (lane == 0) tconv[tix] = kConvAll;
            run.tok += w.tok; run.mat += w.mat; run.gb += w.gb;
            e = t;
            continue;
        }
        const Cnt3 tot{sti[j][2], sti[j][3], sti[j][4]};
        const uint32_t fpv = sti[j][5];
        if ((fpv & 1u) && e - t0 == ((fpv >> 1) & 0x7FFFu)) {   // entry = the one k_resolve assumed
            run.tok += sfp[j][0];
            run.mat += sfp[j][1];
            run.gb += sfp[j][2];
            const uint32_t nmod = fpv >> 16;
            if (lane < nmod) cw[lane] = sfw[j][lane];
            if (lane == 0) tconv[tix] = mfull ? kConvAll : sfp[j][4];
            e = sfp[j][3];
            continue;
        }
        // ---- slow path ----
        lazy_tiles += lazy ? 1 : 0;
        const uint32_t nt = t1 - t0;
        const bool vec = (((uintptr_t)mt) & 15) == 0;
        if (vec) {
            // this tile's rows, mbits and chain words: prefetched during the previous tile's
            // walk (run-table tiles, whose entries rarely match k_resolve's), else loaded now
            if (pk != k) fetch_tile(mt, mb, cw, nt, nw, pv, pmb, pcw);
            mbL[lane] = pmb;
            bmL[lane] = pcw;
#pragma unroll
            for (uint32_t q = 0; q < kTile / 256; q++) {
                const uint32_t x = 4 * (lane + 64 * q);
                const uint64_t mw = __shfl(pmb, (lane >> 4) + 4 * q, 64);   // mbits word of x
                if (x >= nt) continue;
                const uint32_t mbw = (uint32_t)(mw >> (x & 63)) & 0xFu;
                const uint32_t vv[4] = {pv[q].x, pv[q].y, pv[q].z, pv[q].w};
#pragma unroll
                for (uint32_t u = 0; u < 4; u++)
                    if (x + u < nt)
                        mL[x + u] = ((mbw >> u) & 1u) ? (mfull || x + u < span ? (x + 4 <= nt ? vv[u] : mt[x + u])
                                                                                      : kUnknown)
                                                      : 0u;
            }
            pk = 0xFFFFFFFFu;
            if (k + 1 < ntiles && j + 1 < 64 && (sti[j + 1][0] & (kTileMFull | kTileUniform)) == kTileMFull) {
                const uint32_t u0 = t1, u1 = min(blen, u0 + kTile);
                fetch_tile(m + bstart + u0, mb + kTile / 64, cw + kTile / 64, u1 - u0, (u1 - u0 + 63) / 64, pv, pmb, pcw);
                pk = k + 1;
            }
        } else {
            mbL[lane] = lane < nw ? mb[lane] : 0ull;   // one mbits word per lane (64 words per tile)
            __syncthreads();
            for (uint32_t x = lane; x < nt; x += 64)   // m only where the position's mbits bit is set
                mL[x] = ((mbL[x >> 6] >> (x & 63)) & 1ull) ? (mfull || x < span ? mt[x] : kUnknown) : 0u;
            for (uint32_t w = lane; w < kTile / 64; w += 64) bmL[w] = w < nw ? cw[w] : 0ull;
        }
        __syncthreads();
        // the walk is wave-uniform and reads only LDS written above: no barrier per token.
        // Lane w keeps the walked chain bits of word w; the speculative bits stay from the
        // stop point (conv point, or the tile end) on.
        uint64_t nwb = 0;
        uint32_t t = e, exitv, convrec = kConvAll, stop;
        Cnt3 walked{0, 0, 0};
        for (;;) {
            const uint32_t rel = t - t0;
            if (!lazy && ((bmL[rel >> 6] >> (rel & 63)) & 1ull)) {
                // converged: the speculative chain from here on is the true one
                const Cnt3 drop = mfull ? spec_prefix(pfx, mt, mb, cw[rel >> 6], rel, false, t0, blen)
                                        : spec_prefix_c(pfx, mtok + (uint64_t)tix * kTileMatches, mb, cw[rel >> 6], rel);
                if (!mfull) convrec = rel | (drop.mat << 16);
                walked.tok += tot.tok - drop.tok;
                walked.mat += tot.mat - drop.mat;
                walked.gb += tot.gb - drop.gb;
                exitv = sti[j][1];
                stop = rel;
                break;
            }
            uint32_t mm = mL[rel];
            if (mm == kUnknown) {
                const uint32_t lo = t > kWin ? t - kWin : 0;
                if (dbase == 0xFFFFFFFFu || lo < dbase || t + kMaxL + 8 > dbase + kLazyWindow) {
                    __syncthreads();
                    dbase = lo & ~3u;
                    load_window(dw, d, dbase, blen);
                    __syncthreads();
                }
                mm = stitch_run_match(dw, dbase, blen, t, (FCX_LDS uint32_t *)srm_bm, (FCX_LDS uint16_t *)srm_prc,
                                      (FCX_LDS uint32_t *)srm_rt);
                if (mm == kUnknown) mm = lazy_match(dw, dbase, blen, t);
                nlazy++;
                if (lane == 0) m[bstart + t] = mm;
            }
            walked.add(m_len(mm));
            if (lane == (rel >> 6)) nwb |= 1ull << (rel & 63);
            t += m_len(mm) + 1;
            if (t >= t1) { exitv = t; stop = nt; break; }
        }
        if (lane < nw) {
            const uint32_t lo = 64 * lane;
            const uint64_t keep = stop <= lo ? ~0ull : stop >= lo + 64 ? 0ull : ~0ull << (stop - lo);
            cw[lane] = (bmL[lane] & keep) | nwb;
        }
        if (lane == 0) tconv[tix] = convrec;
        __syncthreads();
        run.tok += walked.tok; run.mat += walked.mat; run.gb += walked.gb;
        e = exitv;
    }
    zero_edges(s_flags, s_p, s_golomb, L, b, run.tok, run.mat, run.gb);
    if (lane == 0) {
        BlockInfo &bi = binfo[b];
        bi.len = blen;
        bi.ntok = run.tok;
        bi.nmatch = run.mat;
        bi.gbits = run.gb;
        bi.slen[0] = (run.tok + 7) / 8;                 // flags bytes (2078-2079)
        bi.slen[1] = run.tok;                           // chars
        bi.slen[2] = (kPBits * run.mat) / 8 + 1;        // (11*pCnt)/8 + 1 (2192)
        bi.slen[3] = 4 * ((run.gb + 31) / 32);          // golomb words as bytes
        bi.lazy_evals = nlazy;
        bi.lazy_tiles = lazy_tiles;
    }
}

// ---------------------------------------------------------------------------
// block-wide exclusive scan of 3 counters (256 threads); returns totals in tot
__device__ inline void block_scan3(uint32_t v[3], uint32_t tot[3], uint32_t *sh /* >= 12 */) {
    const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
    uint32_t inc[3];
#pragma unroll
    for (int q = 0; q < 3; q++) inc[q] = wave_incl_scan(v[q]);
    if (lane == 63)
        for (int q = 0; q < 3; q++) sh[q * 4 + wv] = inc[q];
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 3; q++) {
        uint32_t pre = 0, all = 0;
        for (uint32_t w = 0; w < 4; w++) {
            const uint32_t x = sh[q * 4 + w];
            if (w < wv) pre += x;
            all += x;
        }
        v[q] = pre + inc[q] - v[q];
        tot[q] = all;
    }
    __syncthreads();
}

// block-wide (256 threads) exclusive scan of one counter in place, with the total
__device__ inline void block_scan1t(uint32_t &v, uint32_t &total, uint32_t *sh /* >= 4 */) {
    const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
    const uint32_t inc = wave_incl_scan(v);
    if (lane == 63) sh[wv] = inc;
    __syncthreads();
    uint32_t pre = 0, all = 0;
    for (uint32_t w = 0; w < 4; w++) {
        const uint32_t x = sh[w];
        if (w < wv) pre += x;
        all += x;
    }
    v = pre + inc - v;
    total = all;
    __syncthreads();
}

// LDS staging capacities per tile (words)
constexpr uint32_t kFlagW = kTile / 32 + 2;
constexpr uint32_t kPW = (kPBits * (kTile / 4 + 1)) / 32 + 4;
constexpr uint32_t kGW = 128;
constexpr uint32_t kCharW = kTile / 4 + 2;

// OR the low n (<= 64) bits of v at absolute bit pos into staged words (index relative to wbase)
__device__ inline void or_bits64(uint32_t *w, uint32_t wbase, uint64_t pos, uint64_t v, uint32_t n) {
    if (n == 0) return;
    uint32_t wi = (uint32_t)(pos >> 5) - wbase, sh = (uint32_t)(pos & 31);
    atomicOr(&w[wi], (uint32_t)(v << sh));
    uint32_t done = 32 - sh;
    while (done < n) {
        wi++;
        atomicOr(&w[wi], (uint32_t)(v >> done));
        done += 32;
    }
}

// store staged words [0, nw) at global word index gw0: edge words OR'd, interior stored
__device__ inline void flush_words(uint32_t *g, uint32_t gw0, const uint32_t *w, uint32_t nw, uint32_t tid) {
    for (uint32_t x = tid; x < nw; x += 256) {
        const uint32_t v = w[x];
        if (x == 0 || x == nw - 1) { if (v) atomicOr(&g[gw0 + x], v); }
        else g[gw0 + x] = v;
    }
}

// all-literal tile (random data): the tile's chars are its input bytes (staged in LDS), its flags
// all ones.  k_encode reads the chars of the segments that lie wholly inside the tile [sa, sz) straight
// from the input (their descriptors say so), so only the chars outside them go to the stream: the
// head and tail partial segments as byte stores.  (sa >= sz: every char, as dwords on the stream's
// dword grid by alignbyte, the partial dwords at the two ends as byte stores.)
__device__ void emit_literal_tile(const uint32_t *lin, uint32_t nt, uint32_t tok0, uint32_t sa, uint32_t sz, uint8_t *chars,
                                  uint32_t *flags) {
    const uint32_t tid = threadIdx.x;
    const uint32_t f0 = tok0, f1 = tok0 + nt;
    for (uint32_t w = (f0 >> 5) + tid; w <= ((f1 - 1) >> 5); w += 256) {
        const uint32_t lo = max(f0, 32 * w), hi = min(f1, 32 * w + 32);
        if (hi - lo == 32) flags[w] = ~0u;
        else atomicOr(&flags[w], ((1u << (hi - lo)) - 1u) << (lo - 32 * w));
    }
    const uint8_t *lb = (const uint8_t *)lin;
    if (sa < sz) {
        if (tid < sa - tok0) chars[tok0 + tid] = lb[tid];
        if (tid < f1 - sz) chars[sz + tid] = lb[sz - tok0 + tid];
        return;
    }
    const uint32_t e = (4u - (tok0 & 3u)) & 3u;             // input byte of the first whole output dword
    const uint32_t nfull = nt >= e ? (nt - e) >> 2 : 0u;      // whole output dwords
    uint32_t *c4 = (uint32_t *)chars + ((tok0 + e) >> 2);
#pragma unroll
    for (uint32_t u = 0; u < kTile / 4 / 256; u++) {
        const uint32_t j = tid + 256 * u;
        if (j < nfull) c4[j] = __builtin_amdgcn_alignbyte(lin[j + 1], lin[j], e);
    }
    const uint32_t zf = e + 4 * nfull;
    if (tid < min(e, nt)) chars[tok0 + tid] = lb[tid];
    if (tid < nt - min(zf, nt)) chars[tok0 + zf + tid] = lb[zf + tid];
}

// ---- the chars histogram (my_huffman_encode_char's count, my_compress.cpp:998-1000), built here
// while the tile's chars are in LDS or registers: one row of u16 counts per tile (one plain 512-B
// store), summed by k_tree.  The flag / distance / golomb streams are short (text: 0.33 MB per
// MiB) and k_tree counts their bytes straight from the finished streams.
__device__ inline void hist_bytes16(const uint32_t in4[4], uint32_t n, uint32_t *h) {   // the first n of 16 bytes
#pragma unroll
    for (uint32_t q = 0; q < 16; q++)
        if (q < n) atomicAdd(&h[(in4[q >> 2] >> (8 * (q & 3))) & 0xFFu], 1u);
}

constexpr uint32_t kInW = (kTile + kLookAhead) / 4 + 2;   // tile input + look-ahead (dwords)

// Latency shape: every load that does not depend on another goes out first (tile
// offsets, conv record, chain and mbits words, the tile's input + look-ahead into LDS);
// after one block scan, the second and last round of loads (m rows, the compact match
// list into LDS); everything after that is LDS work and stores.
// kDev = true carries development exits (timing of the paths, output discarded: fcx_debug_emit_bits);
// the product launches k_emit<false>
template <bool kDev>
__global__ __launch_bounds__(256) void k_emit(const uint8_t *__restrict__ in, Layout L, const uint32_t *__restrict__ m,
                                              const uint64_t *__restrict__ mbits, const uint64_t *__restrict__ chain, const uint32_t *__restrict__ tile_off,
                                              const BlockInfo *__restrict__ binfo, const uint32_t *__restrict__ mtok,
                                              const uint32_t *__restrict__ tconv, const uint32_t *__restrict__ tinfo,
                                              uint8_t *__restrict__ s_flags, uint8_t *__restrict__ s_chars,
                                              uint8_t *__restrict__ s_p, uint8_t *__restrict__ s_golomb,
                                              uint16_t *__restrict__ thist, uint32_t *__restrict__ sdesc,
                                              uint32_t *__restrict__ err, uint32_t dbg_in) {
    const uint32_t dbg = kDev ? dbg_in : 0u;
    __shared__ uint32_t sh[16];
    __shared__ uint32_t hc[256];             // this tile's chars counts
    __shared__ uint32_t lf[kFlagW], lp[kPW], lg[kGW], lc[kCharW];
    __shared__ uint32_t lin[kInW];           // input bytes [t0, t0 + kTile + kLookAhead) of the block
    __shared__ uint32_t lmt[kTileMatches];   // the tile's compact match list from its conv point
    const uint32_t tid = threadIdx.x;
    const uint32_t b = blockIdx.x / L.tpb, k = blockIdx.x % L.tpb;
    const uint64_t bstart = (uint64_t)b * L.B;
    const uint32_t blen = (uint32_t)min((uint64_t)L.B, L.n - bstart);
    const uint32_t t0 = k * kTile;
    if (t0 >= blen) return;
    const uint32_t t1 = min(blen, t0 + kTile);
    const uint32_t tix = blockIdx.x;
    hc[tid] = 0;   // (every path's barriers order it)
    uint16_t *trow = thist + (uint64_t)tix * 256;

    // ---- round 1: independent loads.  Every scalar the tile needs is read unconditionally (tile_off
    // has a tile of slack past the shard's last; every tile reads its block's record), and the check
    // below combines its compares without short circuits: the compiler does not move a load above a
    // branch, so the short-circuit form waited for seven dependent round trips before the first
    // vector load.  The chain and mbits words are in the block's words for every lane. ----
    const bool last = t1 == blen;
    const uint32_t cv = tconv[tix];
    const uint4 ti4 = *(const uint4 *)(tinfo + 8ull * tix);   // flags [0], match tokens of the speculative chain [3]
    const uint32_t ti0 = ti4.x, nspec = ti4.w;
    const uint32_t tok0 = tile_off[3 * tix + 0], mi0 = tile_off[3 * tix + 1], g0 = tile_off[3 * tix + 2];
    const uint32_t tn0 = tile_off[3 * tix + 3], tn1 = tile_off[3 * tix + 4];
    const uint32_t bnt = binfo[b].ntok, bnm = binfo[b].nmatch;
    const uint32_t s = t0 + tid * 16;   // this lane's 16 positions: one quarter of a chain word
    const uint64_t wi = (uint64_t)b * L.wpb + (uint64_t)k * (kTile / 64) + (tid >> 2);
    uint64_t cwv = chain[wi], mbv = mbits[wi];
    asm volatile("" ::"s"(tok0), "s"(mi0), "s"(g0), "s"(tn0), "s"(tn1), "s"(bnt), "s"(bnm), "s"(cv), "s"(ti0), "s"(nspec),
                 "v"(cwv), "v"(mbv));   // (all of them in flight before the check's branch)
    const uint32_t tk1 = last ? bnt : tn0, mk1 = last ? bnm : tn1;
    const bool uni = (ti0 & kTileUniform) != 0;   // m = m_uniform, no rows
    // the tile's offsets and counts come from scratch the earlier kernels wrote: one inconsistent
    // value (a kernel that did not run, a bug) sets an error bit instead of indexing the streams
    // or the match list out of bounds (uniform values: scalar compares)
    const bool bad = (tk1 > blen) | (tok0 > tk1) | (tk1 - tok0 > t1 - t0) | (mi0 > mk1) | (mk1 - mi0 > tk1 - tok0) |
                     (mk1 > tk1) | (nspec > kTileMatches) | ((cv >> 16) > kTileMatches) | (g0 > 8u * L.sstride[3]);
    if (bad) {
        if (tid == 0) atomicOr(err, kErrScratch);
        return;
    }
    if (s >= t1) { cwv = 0; mbv = 0; }
    const uint8_t *d = in + bstart;
    const bool al = (((uintptr_t)d) & 15) == 0;
    // (the loads above are waited for by the check: a uniform tile -- zeros -- skips the input loads,
    // its one byte value is read below; 1 GiB of zeros no longer re-reads its GiB here)
    uint32_t in4[4] = {0u, 0u, 0u, 0u};
    if (uni) {
    } else if (al && s + 16 <= blen) {
        const uint4 v4 = *(const uint4 *)(d + s);
        in4[0] = v4.x; in4[1] = v4.y; in4[2] = v4.z; in4[3] = v4.w;
    } else {
#pragma unroll
        for (uint32_t q = 0; q < 4; q++) {
            uint32_t w = 0;
            for (uint32_t j = 0; j < 4; j++)
                if (s + 4 * q + j < blen) w |= (uint32_t)d[s + 4 * q + j] << (8 * j);
            in4[q] = w;
        }
    }
    // descriptors of the chars segments (kCharSeg chars: one k_encode lane's symbols) that start in this
    // tile: a segment wholly inside an all-literal tile (as many tokens as positions, no match; the
    // block's last segment may end past the stream) is the input bytes from char + t0 - tok0
    const bool lit = tk1 - tok0 == t1 - t0 && mk1 == mi0;
    const uint32_t sa = (tok0 + kCharSeg - 1) / kCharSeg * kCharSeg, sz = last ? tk1 : tk1 / kCharSeg * kCharSeg;   // inside: [sa, sz)
    if (tid < (tk1 + kCharSeg - 1) / kCharSeg - sa / kCharSeg) {
        const uint32_t g = sa / kCharSeg + tid;
        sdesc[(uint64_t)b * ((L.B + kCharSeg - 1) / kCharSeg) + g] = lit && kCharSeg * g < sz ? t0 - tok0 : kCdMixed;
    }
    uint32_t la = 0;   // look-ahead dword (match chars past the tile end)
    const uint32_t xa = t0 + kTile + 4 * tid;
    if (!uni && tid < kInW - kTile / 4 && xa < blen) {
        if (al && xa + 4 <= blen) la = *(const uint32_t *)(d + xa);
        else
            for (uint32_t j = 0; j < 4 && xa + j < blen; j++) la |= (uint32_t)d[xa + j] << (8 * j);
    }
    if (uni) {
        // one byte value over the tile and its window (zeros): a token's m is m_uniform, its
        // char the tile's byte (at i + L, inside the uniform window); no input staging, no
        // m rows, no match list, just the few tokens' bits
        uint32_t bits = 0;
        if (s < t1) {
            bits = (uint32_t)(cwv >> (16 * (tid & 3))) & 0xFFFFu;
            if (t1 - s < 16) bits &= (1u << (t1 - s)) - 1u;
        }
        const uint8_t ub = d[t0];   // the tile's byte value
        uint32_t v[3] = {(uint32_t)__builtin_popcount(bits), 0, 0}, tot[3];
        for (uint32_t bb = bits; bb; bb &= bb - 1) {
            const uint32_t Lm = m_len(m_uniform(s + __builtin_ctz(bb), blen));
            if (Lm) { v[1]++; v[2] += (Lm >> 2) + 3; }
        }
        for (uint32_t w = tid; w < kFlagW; w += 256) lf[w] = 0;
        for (uint32_t w = tid; w < kPW; w += 256) lp[w] = 0;
        for (uint32_t w = tid; w < kGW; w += 256) lg[w] = 0;
        block_scan3(v, tot, sh);   // (its barriers also order the zeroing before the ORs)
        const uint32_t fw0 = tok0 >> 5, pw0 = (uint32_t)(((uint64_t)kPBits * mi0) >> 5), gw0 = g0 >> 5;
        uint8_t *chars = s_chars + (uint64_t)b * L.sstride[1];
        uint32_t fl = 0, nt_lane = 0, np_lane = 0, goff = g0 + v[2];
        uint64_t pacc = 0;
        for (uint32_t bb = bits; bb; bb &= bb - 1) {
            const uint32_t mu = m_uniform(s + __builtin_ctz(bb), blen), Lm = m_len(mu);
            chars[tok0 + v[0] + nt_lane] = ub;
            if (Lm == 0) {
                fl |= 1u << nt_lane;
            } else {
                pacc |= (uint64_t)m_dist(mu) << (kPBits * np_lane);
                np_lane++;
                const uint32_t qq = Lm >> 2, r = Lm & 3;   // q one-bits, a zero bit, r (2 bits)
                uint32_t pos = goff, left = qq;
                while (left) {
                    const uint32_t sh_ = pos & 31, n = min(left, 32 - sh_);
                    atomicOr(&lg[(pos >> 5) - gw0], (n == 32 ? ~0u : ((1u << n) - 1)) << sh_);
                    pos += n;
                    left -= n;
                }
                if (r) or_bits64(lg, gw0, pos + 1, r, 2);
                goff += qq + 3;
            }
            nt_lane++;
        }
        or_bits64(lf, fw0, tok0 + v[0], fl, nt_lane);
        or_bits64(lp, pw0, (uint64_t)kPBits * (mi0 + v[1]), pacc, kPBits * np_lane);
        __syncthreads();
        const uint32_t nfw = tot[0] ? ((tok0 + tot[0] - 1) >> 5) - fw0 + 1 : 0;
        const uint32_t npw = tot[1] ? (uint32_t)(((uint64_t)kPBits * (mi0 + tot[1]) - 1) >> 5) - pw0 + 1 : 0;
        const uint32_t ngw = tot[2] ? ((g0 + tot[2] - 1) >> 5) - gw0 + 1 : 0;
        flush_words((uint32_t *)(s_flags + (uint64_t)b * L.sstride[0]), fw0, lf, nfw, tid);
        flush_words((uint32_t *)(s_p + (uint64_t)b * L.sstride[2]), pw0, lp, npw, tid);
        flush_words((uint32_t *)(s_golomb + (uint64_t)b * L.sstride[3]), gw0, lg, ngw, tid);
        trow[tid] = tid == ub ? (uint16_t)tot[0] : (uint16_t)0;   // every token's char is the tile's byte
        return;
    }
#pragma unroll
    for (uint32_t q = 0; q < 4; q++) lin[4 * tid + q] = in4[q];
    if (tid < kInW - kTile / 4) lin[kTile / 4 + tid] = la;

    if (lit) {   // no match token in the tile
        if (dbg & 1u) { if (s < t1 && (in4[0] ^ (uint32_t)cwv) == 0x12345u) trow[tid] = 1; return; }   // (timing)
        __syncthreads();
        emit_literal_tile(lin, t1 - t0, tok0, sa, sz, s_chars + (uint64_t)b * L.sstride[1],
                          (uint32_t *)(s_flags + (uint64_t)b * L.sstride[0]));
        // chars = the tile's bytes; every whole flag byte is 0xFF
        hist_bytes16(in4, s < t1 ? min(16u, t1 - s) : 0u, hc);
        __syncthreads();
        trow[tid] = (uint16_t)hc[tid];
        return;
    }

    if (dbg & 2u) { if (s < t1 && (in4[0] ^ (uint32_t)cwv ^ (uint32_t)mbv ^ cv) == 0x12345u) trow[tid] = 1; return; }
    uint32_t bits = 0, mbs = 0;
    if (s < t1) {
        bits = (uint32_t)(cwv >> (16 * (tid & 3))) & 0xFFFFu;
        mbs = (uint32_t)(mbv >> (16 * (tid & 3))) & 0xFFFFu;
        const uint32_t valid = min(16u, t1 - s);
        if (valid < 16) bits &= (1u << valid) - 1;
    }
    // positions from the tile's conv point on (where the final chain joined the
    // speculative one) take their matches from the compact list, in order; the others
    // read m[] (first kResolveSpan positions, the stitch's walks, run-table tiles)
    const uint32_t crel = cv & 0xFFFFu;   // conv rel | dropped speculative matches << 16
    uint32_t post = 0;
    if (crel != kConvAll) {
        const uint32_t rel0 = s - t0;
        post = rel0 >= crel ? 0xFFFFu : rel0 + 16 > crel ? (0xFFFFu << (crel - rel0)) & 0xFFFFu : 0u;
    }
    const uint32_t rd = bits & mbs & ~post;   // chain positions whose m is in m[]
    const uint32_t rc = bits & mbs & post;    // chain matches in the compact list

    // ---- round 2: m rows and the compact list, issued before the scan (they need only round-1
    // values: the list from the conv point holds at most the speculative matches not dropped) ----
    const uint32_t *mt = m + bstart + s;
    uint32_t mm[16];
    if (uni) {
#pragma unroll
        for (uint32_t q = 0; q < 16; q++) mm[q] = ((rd >> q) & 1u) ? m_uniform(s + q, blen) : 0u;
    } else if (rd && ((uintptr_t)mt & 15) == 0) {   // whole 64-B row as four 16-B loads
#pragma unroll
        for (uint32_t q = 0; q < 4; q++) {
            const uint4 w4 = ((const uint4 *)mt)[q];
            mm[4 * q] = w4.x; mm[4 * q + 1] = w4.y; mm[4 * q + 2] = w4.z; mm[4 * q + 3] = w4.w;
        }
    } else {
#pragma unroll
        for (uint32_t q = 0; q < 16; q++) mm[q] = ((rd >> q) & 1u) ? mt[q] : 0u;
    }
    uint32_t cbase = (uint32_t)__builtin_popcount(rc), ncomp;
    {   // the list starts at the tile's first speculative position: skip the matches the
        // final chain dropped before the conv point
        const uint32_t *mct = mtok + (uint64_t)tix * kTileMatches + (cv >> 16);
        const uint32_t nl = crel != kConvAll && nspec > (cv >> 16) ? nspec - (cv >> 16) : 0u;
        uint32_t cl[kTileMatches / 256];
#pragma unroll
        for (uint32_t u = 0; u < kTileMatches / 256; u++) cl[u] = tid + 256 * u < nl ? mct[tid + 256 * u] : 0u;
        block_scan1t(cbase, ncomp, sh + 12);       // (also publishes lin)
#pragma unroll
        for (uint32_t u = 0; u < kTileMatches / 256; u++) lmt[tid + 256 * u] = cl[u];
    }
    for (uint32_t w = tid; w < kFlagW; w += 256) lf[w] = 0;
    for (uint32_t w = tid; w < kPW; w += 256) lp[w] = 0;
    for (uint32_t w = tid; w < kGW; w += 256) lg[w] = 0;
    for (uint32_t w = tid; w < kCharW; w += 256) lc[w] = 0;
    __syncthreads();
    if (dbg & 4u) { if (lmt[tid] == 0x12345u && mm[0] == 7u) trow[tid] = 1; return; }   // (timing: + round 2)

    uint32_t v[3] = {(uint32_t)__builtin_popcount(bits), 0, 0};
#pragma unroll
    for (uint32_t q = 0; q < 16; q++) {
        const uint32_t ci = cbase + (uint32_t)__builtin_popcount(rc & ((1u << q) - 1u));
        mm[q] = ((rd >> q) & 1u) ? mm[q] : ((rc >> q) & 1u) ? lmt[ci] : 0u;
        const uint32_t Lq = m_len(mm[q]);
        if (((bits >> q) & 1u) && Lq) { v[1]++; v[2] += (Lq >> 2) + 3; }
    }
    uint32_t tot[3];
    const uint32_t nm_lane = v[1];
    block_scan3(v, tot, sh);
    tot[0] = fcx::uni(tot[0]); tot[1] = fcx::uni(tot[1]); tot[2] = fcx::uni(tot[2]);
    const uint32_t tokA = tok0 + v[0], miA = mi0 + v[1];
    const uint32_t fw0 = tok0 >> 5, pw0 = (uint32_t)(((uint64_t)kPBits * mi0) >> 5), gw0 = g0 >> 5;
    const uint32_t cw0 = tok0 >> 2;   // chars staged on the global dword grid

    const uint8_t *lb = (const uint8_t *)lin;
    uint8_t *lcb = (uint8_t *)lc;
    uint32_t fl = 0, nt_lane = 0;
    uint64_t pacc = 0;
    uint32_t np_lane = 0;
    if (bits == 0xFFFFu && nm_lane == 0) {
        // 16 literal tokens: the chars are the input bytes; shifted dword stores into the
        // staging, the two words shared with the neighbouring lanes by atomicOr
        const uint32_t bo = tokA - 4 * cw0, sb = 8 * (bo & 3), w0 = bo >> 2;
        uint32_t prev = 0;
#pragma unroll
        for (uint32_t q = 0; q < 5; q++) {
            const uint32_t cur = q < 4 ? lin[4 * tid + q] : 0u;
            const uint32_t o = sb ? (cur << sb) | (prev >> (32 - sb)) : cur;
            prev = cur;
            if (q == 0 || q >= 3) { if (o) atomicOr(&lc[w0 + q], o); }
            else lc[w0 + q] = o;
        }
        fl = 0xFFFFu;
        nt_lane = 16;
        const uint32_t r4[4] = {lin[4 * tid], lin[4 * tid + 1], lin[4 * tid + 2], lin[4 * tid + 3]};
        hist_bytes16(r4, 16, hc);
    } else
#pragma unroll
    for (uint32_t q = 0; q < 16; q++) {
        if ((bits >> q) & 1u) {
            const uint32_t Lm = m_len(mm[q]);
            const uint8_t ch = lb[s - t0 + q + Lm];
            lcb[tokA + nt_lane - 4 * cw0] = ch;
            atomicAdd(&hc[ch], 1u);
            if (Lm == 0) {
                fl |= 1u << nt_lane;
            } else {
                pacc |= (uint64_t)m_dist(mm[q]) << (kPBits * np_lane);
                np_lane++;
                // the golomb code's offset and length go to the match's slot of lmt (free since the
                // m values were resolved); the codes are written match-parallel below
                lmt[miA - mi0 + np_lane - 1] = Lm;
            }
            nt_lane++;
        }
    }
    or_bits64(lf, fw0, tokA, fl, nt_lane);
    or_bits64(lp, pw0, (uint64_t)kPBits * miA, pacc, kPBits * nm_lane);
    __syncthreads();
    // the golomb codes (qq one-bits, a zero bit, r in 2 bits), four consecutive matches per lane, their
    // offsets from one block scan: inside the token loop their word loop held k_emit at 78 VGPRs (6
    // waves per SIMD; 62 and 8 waves without it).  tot[1] <= kTileMatches = 4 x 256.
    if (tot[1]) {
        uint32_t lm4[4], gsum = 0;
#pragma unroll
        for (uint32_t u = 0; u < 4; u++) {
            lm4[u] = 4 * tid + u < tot[1] ? lmt[4 * tid + u] : 0u;
            gsum += lm4[u] ? (lm4[u] >> 2) + 3 : 0u;
        }
        uint32_t gtot;
        block_scan1t(gsum, gtot, sh + 12);
        uint32_t pos = g0 + gsum;
#pragma unroll
        for (uint32_t u = 0; u < 4; u++) {
            const uint32_t Lm = lm4[u], r = Lm & 3u;
            if (!Lm) continue;
            uint32_t left = Lm >> 2;
            while (left) {
                const uint32_t sh_ = pos & 31, n = min(left, 32 - sh_);
                atomicOr(&lg[(pos >> 5) - gw0], (n == 32 ? ~0u : ((1u << n) - 1)) << sh_);
                pos += n;
                left -= n;
            }
            if (r) or_bits64(lg, gw0, pos + 1, r, 2);
            pos += 3;
        }
    }
    __syncthreads();
    if (dbg & 8u) { if (lf[tid & 63] == 0x12345u) trow[tid] = 1; return; }   // (timing: + token loop)

    // chars: aligned dwords inside the tile's range, bytes at its two edges
    uint8_t *chars = s_chars + (uint64_t)b * L.sstride[1];
    const uint32_t ce = tok0 + tot[0];   // end (exclusive) of this tile's chars
    if (tot[0]) {
        const uint32_t a = (tok0 + 3) & ~3u, z = ce & ~3u;   // [a, z) whole dwords
        if (a < z) {
            uint32_t *c4 = (uint32_t *)chars;
            for (uint32_t w = (a >> 2) + tid; w < (z >> 2); w += 256) c4[w] = lc[w - cw0];
        }
        const uint32_t head_end = min(a, ce);
        if (tid < head_end - tok0) chars[tok0 + tid] = lcb[tok0 + tid - 4 * cw0];
        if (z >= a && tid < ce - z) chars[z + tid] = lcb[z + tid - 4 * cw0];
    }
    const uint32_t nfw = tot[0] ? ((tok0 + tot[0] - 1) >> 5) - fw0 + 1 : 0;
    const uint32_t npw = tot[1] ? (uint32_t)(((uint64_t)kPBits * (mi0 + tot[1]) - 1) >> 5) - pw0 + 1 : 0;
    const uint32_t ngw = tot[2] ? ((g0 + tot[2] - 1) >> 5) - gw0 + 1 : 0;
    flush_words((uint32_t *)(s_flags + (uint64_t)b * L.sstride[0]), fw0, lf, nfw, tid);
    flush_words((uint32_t *)(s_p + (uint64_t)b * L.sstride[2]), pw0, lp, npw, tid);
    flush_words((uint32_t *)(s_golomb + (uint64_t)b * L.sstride[3]), gw0, lg, ngw, tid);
    trow[tid] = (uint16_t)hc[tid];   // (the barrier after the token loop ordered the counts)
}

void launch_parse(const uint8_t *in, const Layout &L, uint32_t *m, const uint64_t *mbits, uint64_t *chain,
                  const uint64_t *chain_pfx, const uint32_t *tinfo, const uint32_t *mtok, uint64_t *fp,
                  uint32_t *tile_off, uint32_t *tconv, BlockInfo *binfo, uint8_t *s_flags, uint8_t *s_chars,
                  uint8_t *s_p, uint8_t *s_golomb, uint16_t *thist, uint32_t *sdesc, uint32_t *err, hipStream_t st,
                  hipEvent_t *ev, uint32_t emit_dbg) {
    const uint32_t ntiles = L.nblocks * L.tpb;
    hipLaunchKernelGGL(k_resolve, dim3(ntiles), dim3(64), 0, st, L, m, mbits, chain, chain_pfx, tinfo, fp);
    hipLaunchKernelGGL(k_stitch, dim3(L.nblocks), dim3(64), 0, st, in, L, m, mbits, chain, chain_pfx, tinfo, fp, mtok,
                       tile_off, tconv, binfo, s_flags, s_p, s_golomb);
    if (ev) (void)hipEventRecord(ev[0], st);
    emit_dbg &= 0xFFFFu;   // (bits 16.. are k_tree's)
    if (emit_dbg == 0)
        hipLaunchKernelGGL(k_emit<false>, dim3(ntiles), dim3(256), 0, st, in, L, m, mbits, chain, tile_off, binfo, mtok,
                           tconv, tinfo, s_flags, s_chars, s_p, s_golomb, thist, sdesc, err, 0u);
    else
        hipLaunchKernelGGL(k_emit<true>, dim3(ntiles), dim3(256), 0, st, in, L, m, mbits, chain, tile_off, binfo, mtok,
                           tconv, tinfo, s_flags, s_chars, s_p, s_golomb, thist, sdesc, err, emit_dbg);
    if (ev) (void)hipEventRecord(ev[1], st);
}

}  // namespace fcx

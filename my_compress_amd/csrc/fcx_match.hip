// fcx_match.hip — all-position LZ77 match search + tile-local greedy parse (gfx950).
//
// Replaces the inner loop of my_LZ77_compress (my_compress.cpp:1675-1714), i.e.
// longest_match_sunday (1446-1514) driven by Sunday_Search (1407-1443).  The
// reference's result at cursor i is the LEFTMOST j in [max(0,i-2047), i) with the
// MAXIMUM common prefix L, L capped at min(258, len-i)-1, literal if L < 3
// (SURVEY.md §0 finding 3).  Here one 256-lane workgroup owns a tile of 4096
// positions of one block:
//
//   1. stage [t0-2048, t1+260) of the block in LDS (coalesced, dword loads);
//   2. insert every window position into a 4096-bucket hash table of 3-byte keys,
//      in 256-position passes separated by barriers, so a chain runs newest pass
//      first; query the pass's tile positions right after it is inserted — a
//      chain walk then meets exactly the window candidates, and stops as soon as
//      it reaches a pass lying wholly below i-2047;
//   3. exact max-length / min-position selection over the key-equal candidates
//      (dword compares in LDS); a position whose window holds more than
//      kMaxChainSteps candidates is left "unknown" for the stitch kernel's
//      wave-parallel evaluation (runs / zeros: long matches, few tokens);
//   4. greedy parse of the tile assuming a token starts at t0: each lane walks
//      its 16 positions, then lanes agree on sub-segment entry points by a
//      Jacobi fixed point (entry_k+1 = exit of walking sub-segment k from entry_k)
//      that converges in a few rounds because greedy chains resynchronise.
//
// Outputs: m[i] for every position, the tile's chain bitmap (positions that start
// a token if a token starts at t0), and the tile's exit (first chain position
// >= t1).  Tiles with unknown positions are flagged lazy.
#include "fcx_device.h"

namespace fcx {

__global__ __launch_bounds__(kMatchThreads) void k_match(const uint8_t *__restrict__ in, Layout L,
                                                        uint32_t *__restrict__ m, uint64_t *__restrict__ chain,
                                                        uint32_t *__restrict__ tile_exit,
                                                        uint32_t *__restrict__ tile_flags) {
    __shared__ uint32_t sdw[kTileBytes / 4 + 4];           // byte image of the window
    __shared__ uint32_t head[1u << kHashBits];             // bucket -> newest local index + 1
    __shared__ uint16_t nxt[kHalo + 1 + kTile];            // older entry of the same bucket (+1)
    __shared__ uint16_t step[kTile];                       // L+1 per tile position, 0 = unknown
    __shared__ uint32_t Gs[kMatchThreads + 1];             // sub-segment entry points
    __shared__ uint32_t Xs[kMatchThreads];                 // speculative sub-segment exits
    __shared__ uint32_t Vs[kMatchThreads];                 // speculative visit masks
    __shared__ uint32_t s_unknown;
    __shared__ uint32_t s_chg[2];

    const uint32_t tid = threadIdx.x;
    const uint32_t b = blockIdx.x / L.tpb, k = blockIdx.x % L.tpb;
    const uint64_t bstart = (uint64_t)b * L.B;
    const uint32_t blen = (uint32_t)min((uint64_t)L.B, L.n - bstart);
    const uint32_t t0 = k * kTile;
    if (t0 >= blen) return;  // uniform
    const uint32_t t1 = min(blen, t0 + kTile);
    const uint8_t *d = in + bstart;
    const uint32_t w0 = t0 >= 2048 ? t0 - 2048 : 0;  // 4-aligned relative to the block
    const uint32_t dend = min(blen, t1 + kLookAhead);
    const uint32_t nload = dend - w0;

    // ---- 1. stage bytes (zero padded) ----
    const uint8_t *src = d + w0;
    if ((((uintptr_t)src) & 3) == 0) {
        const uint32_t *src4 = (const uint32_t *)src;
        const uint32_t nfull = nload >> 2;
        for (uint32_t x = tid; x < kTileBytes / 4 + 4; x += kMatchThreads) {
            uint32_t v = 0;
            if (x < nfull) v = src4[x];
            else if (x == nfull) {
                for (uint32_t q = 0; q < (nload & 3); q++) v |= (uint32_t)src[4 * x + q] << (8 * q);
            }
            sdw[x] = v;
        }
    } else {
        for (uint32_t x = tid; x < kTileBytes / 4 + 4; x += kMatchThreads) {
            uint32_t v = 0;
            for (uint32_t q = 0; q < 4; q++)
                if (4 * x + q < nload) v |= (uint32_t)src[4 * x + q] << (8 * q);
            sdw[x] = v;
        }
    }
    for (uint32_t x = tid; x < (1u << kHashBits); x += kMatchThreads) head[x] = 0;
    if (tid == 0) { s_unknown = 0; s_chg[0] = 0; s_chg[1] = 0; }
    __syncthreads();

    // ---- 2/3. insert + query in passes of 256 positions ----
    const uint32_t npos = t1 - w0;
    const uint32_t q0 = t0 - w0;
    for (uint32_t base = 0; base < npos; base += kMatchThreads) {
        const uint32_t x = base + tid;
        const uint32_t j = w0 + x;
        if (x < npos && j + 3 <= blen) {
            const uint32_t h = hash3(lds_key3(sdw, x));
            const uint32_t old = atomicExch(&head[h], x + 1);
            nxt[x] = (uint16_t)old;
        }
        __syncthreads();
        if (x >= q0 && x < npos) {
            const uint32_t i = j;
            uint32_t res = 0, st = 1;
            if (i != 0 && blen - i >= 4) {
                if (s_unknown > kDenseUnknowns) {
                    res = kUnknown; st = 0;   // dense tile: leave the rest to the stitch kernel
                } else {
                    const uint32_t cap = min(kMaxL, blen - i) - 1;
                    const uint32_t key = lds_key3(sdw, x);
                    const uint32_t xlo = (i > kWin ? i - kWin : 0) - w0;
                    uint32_t best = kMinL - 1, bestx = 0xFFFFFFFFu, steps = 0;
                    bool unk = false;
                    for (uint32_t c = head[hash3(key)]; c != 0;) {
                        const uint32_t xe = c - 1;
                        if ((xe | (kMatchThreads - 1)) < xlo) break;  // whole pass below the window
                        if (xe < x && xe >= xlo) {
                            if (++steps > kMaxChainSteps) { unk = true; break; }
                            if (lds_key3(sdw, xe) == key) {
                                bool cand;
                                if (best < kMinL) cand = true;
                                else if (xe < bestx)   // may tie: needs L >= best
                                    cand = lds_ld1(sdw, xe + best - 1) == lds_ld1(sdw, x + best - 1);
                                else                   // must beat: needs L > best
                                    cand = best < cap && lds_ld1(sdw, xe + best) == lds_ld1(sdw, x + best);
                                if (cand) {
                                    const uint32_t Lc = lds_match_len(sdw, xe, x, kMinL, cap);
                                    if (Lc > best || (Lc == best && xe < bestx)) { best = Lc; bestx = xe; }
                                }
                            }
                        }
                        c = nxt[xe];
                    }
                    if (unk) { res = kUnknown; st = 0; atomicAdd(&s_unknown, 1u); }
                    else if (best >= kMinL) { res = m_pack(best, x - bestx); st = best + 1; }
                }
            }
            m[bstart + i] = res;
            step[i - t0] = (uint16_t)st;
        }
        __syncthreads();
    }

    // ---- 4. tile-local greedy parse ----
    uint64_t *cw = chain + (uint64_t)b * L.wpb + (uint64_t)k * (kTile / 64);
    const uint32_t nwords = (t1 - t0 + 63) / 64;
    if (s_unknown != 0) {
        for (uint32_t w = tid; w < nwords; w += kMatchThreads) cw[w] = 0;
        if (tid == 0) { tile_flags[blockIdx.x] = kTileLazy; tile_exit[blockIdx.x] = 0; }
        return;
    }
    const uint32_t s = t0 + tid * kSubSeg;
    const uint32_t se = min(s + kSubSeg, t1);
    uint32_t V = 0, X = s;
    if (s < t1) {
        uint32_t t = s;
        while (t < se) { V |= 1u << (t - s); t += step[t - t0]; }
        X = t;
    }
    Vs[tid] = V;
    Xs[tid] = X;
    Gs[tid + 1] = X;
    if (tid == 0) Gs[0] = t0;
    __syncthreads();
    uint32_t T = 0;
    for (uint32_t r = 0;; r++) {
        const uint32_t e = Gs[tid];
        uint32_t ex;
        if (s >= t1 || e >= se) {
            ex = e; T = 0;
        } else if ((V >> (e - s)) & 1u) {
            ex = X; T = V & (~0u << (e - s));
        } else {
            T = 0;
            uint32_t t = e;
            while (t < se && !((V >> (t - s)) & 1u)) { T |= 1u << (t - s); t += step[t - t0]; }
            if (t < se) { ex = X; T |= V & (~0u << (t - s)); }
            else ex = t;
        }
        __syncthreads();
        if (ex != Gs[tid + 1]) { Gs[tid + 1] = ex; s_chg[r & 1] = 1; }
        if (tid == 0) s_chg[(r + 1) & 1] = 0;
        __syncthreads();
        if (!s_chg[r & 1]) break;
    }
    Vs[tid] = T;
    __syncthreads();
    for (uint32_t w = tid; w < nwords; w += kMatchThreads) {
        const uint64_t word = (uint64_t)Vs[4 * w] | ((uint64_t)Vs[4 * w + 1] << 16) |
                              ((uint64_t)Vs[4 * w + 2] << 32) | ((uint64_t)Vs[4 * w + 3] << 48);
        cw[w] = word;
    }
    if (tid == 0) {
        const uint32_t nsub = (t1 - t0 + kSubSeg - 1) / kSubSeg;
        tile_flags[blockIdx.x] = 0;
        tile_exit[blockIdx.x] = Gs[nsub];
    }
}

void launch_match(const uint8_t *in, const Layout &L, uint32_t *m, uint64_t *chain, uint32_t *tile_exit,
                  uint32_t *tile_flags, hipStream_t st) {
    const uint32_t grid = L.nblocks * L.tpb;
    hipLaunchKernelGGL(k_match, dim3(grid), dim3(kMatchThreads), 0, st, in, L, m, chain, tile_exit, tile_flags);
}

}  // namespace fcx

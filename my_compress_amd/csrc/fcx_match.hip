// fcx_match.hip — all-position LZ77 match search + tile-local greedy parse (gfx950).
//
// Replaces the inner loop of my_LZ77_compress (my_compress.cpp:1675-1714), i.e.
// longest_match_sunday (1446-1514) driven by Sunday_Search (1407-1443).  The
// reference's result at cursor i is the LEFTMOST j in [max(0,i-2047), i) with the
// MAXIMUM common prefix L, L capped at min(258, len-i)-1, literal if L < 3
// (SURVEY.md §0 finding 3).  One 512-lane workgroup owns a tile of 4096
// positions of one block:
//
//   1. stage [t0-2048, t1+260) of the block in LDS (dword loads);
//   2. counting-sort every window position by the bucket of its 3-byte key: the
//      key is split by a bijection of Z/2^24 into (12-bit bucket, 12-bit tag), an
//      entry {tag, position} identifies the key exactly, and a bucket is one
//      contiguous LDS range (count by LDS atomics, block scan, scatter);
//   3. every tile position scans its bucket range (independent LDS loads, no
//      pointer chase; four queries interleaved per lane) and keeps the
//      max-length / min-position candidate among entries in its window (stored
//      to m[] only where a match or "unknown" results, flagged per position in
//      the mbits bitmap by one ballot per wave: random data writes almost no m).  A
//      candidate's length is read off two dword compares against the query's
//      preloaded bytes 3..10; only a match reaching 11 bytes enters the extension
//      loop.  A bucket with more than kMaxChainSteps entries makes the position
//      "unknown" at once, for the stitch kernel's wave-parallel evaluation
//      (runs / zeros: long matches, few tokens);
//   4. greedy parse of the tile assuming a token starts at t0: each lane walks
//      its 8 positions, lanes agree on sub-segment entries by a Jacobi fixed
//      point (entry_{k+1} = exit of sub-segment k walked from entry_k) that
//      converges in one or two rounds because greedy chains resynchronise; then
//      the tile's chain bitmap, per-64-position prefix counts (tokens, matches,
//      golomb bits) and totals are published for the stitch kernel.
#include <cstdlib>

#include "fcx_device.h"

namespace fcx {

constexpr uint32_t kWinPos = kHalo + 1 + kTile;      // 6144 window positions per tile
constexpr uint32_t kMT = kMatchThreads;              // 512
constexpr uint32_t kSeg = kTile / kMT;               // 8 positions per lane in the parse
constexpr uint32_t kQPL = kTile / kMT;               // 8 queries per lane
constexpr uint32_t kIlp = 4;                         // interleaved chain walks per lane
constexpr uint32_t kWaves = kMT / 64;

__device__ inline uint32_t key_mix(uint32_t key) { return (key * 0x9E3779B1u) & 0xFFFFFFu; }  // bijective mod 2^24

struct Walk {   // one query: bucket range [c, c + steps), window [xlo, x), cap, key tag, bytes 3..10
    uint32_t c, x, xlo, cap, tag, best, bestx, steps, q1, q2;
    bool unk;
};

__global__ __launch_bounds__(kMT) void k_match(const uint8_t *__restrict__ in, Layout L, uint32_t *__restrict__ m,
                                              uint64_t *__restrict__ mbits, uint64_t *__restrict__ chain,
                                              uint64_t *__restrict__ chain_pfx,
                                              uint32_t *__restrict__ tinfo, uint32_t dbg) {
    __shared__ uint32_t sdw[kTileBytes / 4 + 4];           // byte image of the window
    __shared__ uint32_t head[(1u << kHashBits) + 4];       // bucket -> count, then start of its range;
                                                           // after the queries: step[] + parse scratch
    __shared__ uint32_t node[kWinPos];                     // entries sorted by bucket: (tag << 13) | position
    __shared__ uint32_t s_unknown;
    __shared__ uint32_t s_chg[2];
    __shared__ uint32_t s_red[3 * kWaves];   // cross-wave scan partials

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
        for (uint32_t x = tid; x < kTileBytes / 4 + 4; x += kMT) {
            uint32_t v = 0;
            if (x < nfull) v = src4[x];
            else if (x == nfull)
                for (uint32_t q = 0; q < (nload & 3); q++) v |= (uint32_t)src[4 * x + q] << (8 * q);
            sdw[x] = v;
        }
    } else {
        for (uint32_t x = tid; x < kTileBytes / 4 + 4; x += kMT) {
            uint32_t v = 0;
            for (uint32_t q = 0; q < 4; q++)
                if (4 * x + q < nload) v |= (uint32_t)src[4 * x + q] << (8 * q);
            sdw[x] = v;
        }
    }
    for (uint32_t x = tid; x < (1u << kHashBits) + 4; x += kMT) head[x] = 0;
    if (tid == 0) { s_unknown = 0; s_chg[0] = 0; s_chg[1] = 0; }
    __syncthreads();

    // ---- 2. counting sort of the window positions by bucket ----
    const uint32_t npos = t1 - w0;
    const uint32_t q0 = t0 - w0;
    const uint32_t ins_end = min(npos, blen >= 3 ? blen - 2 - w0 : 0);  // j + 3 <= blen
    constexpr uint32_t kIns = (kWinPos + kMT - 1) / kMT;               // 12 per lane
    uint32_t ins_h[kIns], ins_r[kIns];
#pragma unroll
    for (uint32_t r = 0; r < kIns; r++) {
        const uint32_t x = tid + kMT * r;
        ins_h[r] = 0xFFFFFFFFu;
        if (x < ins_end) {
            ins_h[r] = key_mix(lds_key3(sdw, x));
            ins_r[r] = atomicAdd(&head[ins_h[r] >> 12], 1u);
        }
    }
    __syncthreads();
    {   // exclusive scan of the 4096 bucket counts: 8 consecutive buckets per lane
        constexpr uint32_t kPer = (1u << kHashBits) / kMT;
        uint32_t cnt[kPer], sum = 0;
#pragma unroll
        for (uint32_t q = 0; q < kPer; q++) { cnt[q] = head[tid * kPer + q]; sum += cnt[q]; }
        const uint32_t inc = wave_incl_scan(sum);
        const uint32_t lane = tid & 63, wv = tid >> 6;
        if (lane == 63) s_red[wv] = inc;
        __syncthreads();
        uint32_t run = inc - sum;
        for (uint32_t w = 0; w < wv; w++) run += s_red[w];
#pragma unroll
        for (uint32_t q = 0; q < kPer; q++) { head[tid * kPer + q] = run; run += cnt[q]; }
        if (tid == kMT - 1) head[1u << kHashBits] = run;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t r = 0; r < kIns; r++)
        if (ins_h[r] != 0xFFFFFFFFu)
            node[head[ins_h[r] >> 12] + ins_r[r]] = ((ins_h[r] & 0xFFFu) << 13) | (tid + kMT * r);
    __syncthreads();

    // ---- 3. queries: position i = w0 + q0 + tid + kMT*r, kIlp at a time ----
    uint32_t st_reg[kQPL];
#pragma unroll
    for (uint32_t g = 0; g < kQPL; g += kIlp) {
        Walk W[kIlp];
        uint32_t nmax = 0;
#pragma unroll
        for (uint32_t u = 0; u < kIlp; u++) {
            Walk &w = W[u];
            w.x = q0 + tid + kMT * (g + u);
            w.c = 0; w.best = kMinL - 1; w.bestx = 0xFFFFFFFFu; w.steps = 0; w.unk = false;
            w.cap = 0; w.xlo = 0; w.tag = 0; w.q1 = 0; w.q2 = 0;
            if (w.x < npos) {
                const uint32_t i = w0 + w.x;
                if (i != 0 && blen - i >= 4 && !(dbg & 1u)) {
                    w.cap = min(kMaxL, blen - i) - 1;
                    const uint32_t h = key_mix(lds_key3(sdw, w.x));
                    w.tag = h & 0xFFFu;
                    w.xlo = (i > kWin ? i - kWin : 0) - w0;
                    w.q1 = lds_ld4(sdw, w.x + 3);
                    w.q2 = lds_ld4(sdw, w.x + 7);
                    w.c = head[h >> 12];                       // range start
                    w.steps = head[(h >> 12) + 1] - w.c;      // range length
                    if (w.steps > kMaxChainSteps) { w.unk = true; w.steps = 0; }
                    nmax = max(nmax, w.steps);
                }
            }
        }
        for (uint32_t j = 0; j < nmax; j++) {
#pragma unroll
            for (uint32_t u = 0; u < kIlp; u++) {
                Walk &w = W[u];
                if (j >= w.steps) continue;
                const uint32_t nd = node[w.c + j];
                const uint32_t xe = nd & 0x1FFFu;
                if ((nd >> 13) != w.tag || xe >= w.x || xe < w.xlo) continue;
                // common prefix with the query: bytes 0..2 equal by the key
                uint32_t Lc;
                const uint32_t a = lds_ld4(sdw, xe + 3) ^ w.q1;
                if (a) {
                    Lc = 3 + (__builtin_ctz(a) >> 3);
                } else {
                    const uint32_t bb = lds_ld4(sdw, xe + 7) ^ w.q2;
                    if (bb) Lc = 7 + (__builtin_ctz(bb) >> 3);
                    else Lc = (w.cap > 11 && !(dbg & 2u)) ? lds_match_len(sdw, xe, w.x, 11, w.cap) : 11;
                }
                Lc = min(Lc, w.cap);
                if (Lc > w.best || (Lc == w.best && xe < w.bestx)) { w.best = Lc; w.bestx = xe; }
            }
        }
#pragma unroll
        for (uint32_t u = 0; u < kIlp; u++) {
            Walk &w = W[u];
            uint32_t st = 1, res = 0;
            if (w.x < npos) {
                if (w.unk) { res = kUnknown; st = 0; s_unknown = 1; }
                else if (w.best >= kMinL) { res = m_pack(w.best, w.x - w.bestx); st = w.best + 1; }
                if (res) m[bstart + w0 + w.x] = res;   // m is stored only where mbits says so
            }
            // the wave's 64 lanes hold 64 consecutive positions = one mbits word
            const uint64_t mb = __ballot(res != 0);
            const uint32_t xw = q0 + (tid & ~63u) + kMT * (g + u);
            if ((tid & 63) == 0 && xw < npos) mbits[(uint64_t)b * L.wpb + ((w0 + xw) >> 6)] = mb;
            st_reg[g + u] = st;
        }
    }
    __syncthreads();   // head[] is dead from here on

    uint64_t *cw = chain + (uint64_t)b * L.wpb + (uint64_t)k * (kTile / 64);
    uint32_t *ti = tinfo + 8ull * blockIdx.x;
    const uint32_t nwords = (t1 - t0 + 63) / 64;
    if (s_unknown != 0) {
        for (uint32_t w = tid; w < nwords; w += kMT) cw[w] = 0;
        if (tid == 0) { ti[0] = kTileLazy; ti[1] = 0; ti[2] = ti[3] = ti[4] = 0; }
        return;
    }

    // ---- 4. tile-local greedy parse ----
    uint16_t *step = (uint16_t *)head;                 // 8 KB
    uint32_t *Gs = head + kTile / 2;                   // kMT + 1 entries
    uint32_t *Xs = Gs + kMT + 1;
    uint32_t *Vs = Xs + kMT;
#pragma unroll
    for (uint32_t r = 0; r < kQPL; r++) step[tid + kMT * r] = (uint16_t)st_reg[r];
    __syncthreads();
    const uint32_t s = t0 + tid * kSeg;
    const uint32_t se = min(s + kSeg, t1);
    uint32_t V = 0, X = s;
    if (s < t1) {
        uint32_t t = s;
        while (t < se) { V |= 1u << (t - s); t += step[t - t0]; }
        X = t;
    }
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
    // counts of this lane's chain positions, prefix over lanes
    uint32_t cnt[3] = {(uint32_t)__builtin_popcount(T), 0, 0};
    for (uint32_t bits = T; bits; bits &= bits - 1) {
        const uint32_t Lm = step[s - t0 + __builtin_ctz(bits)] - 1u;
        if (Lm) { cnt[1]++; cnt[2] += (Lm >> 2) + 3; }
    }
    const uint32_t lane = tid & 63, wv = tid >> 6;
    uint32_t inc[3];
#pragma unroll
    for (int q = 0; q < 3; q++) inc[q] = wave_incl_scan(cnt[q]);
    if (lane == 63)
        for (int q = 0; q < 3; q++) s_red[q * kWaves + wv] = inc[q];
    Vs[tid] = T;
    __syncthreads();
    uint32_t pre[3], tot[3];
#pragma unroll
    for (int q = 0; q < 3; q++) {
        uint32_t p = 0, a = 0;
        for (uint32_t w = 0; w < kWaves; w++) {
            const uint32_t v = s_red[q * kWaves + w];
            if (w < wv) p += v;
            a += v;
        }
        pre[q] = p + inc[q] - cnt[q];
        tot[q] = a;
    }
    constexpr uint32_t kLanesPerWord = 64 / kSeg;   // 8
    if ((tid % kLanesPerWord) == 0 && tid / kLanesPerWord < nwords) {
        const uint32_t w = tid / kLanesPerWord;
        uint64_t word = 0;
#pragma unroll
        for (uint32_t q = 0; q < kLanesPerWord; q++) word |= (uint64_t)Vs[tid + q] << (kSeg * q);
        cw[w] = word;
        chain_pfx[(uint64_t)blockIdx.x * (kTile / 64) + w] =
            (uint64_t)pre[0] | ((uint64_t)pre[1] << 13) | ((uint64_t)pre[2] << 24);
    }
    if (tid == 0) {
        const uint32_t nsub = (t1 - t0 + kSeg - 1) / kSeg;
        ti[0] = 0;
        ti[1] = Gs[nsub];
        ti[2] = tot[0];
        ti[3] = tot[1];
        ti[4] = tot[2];
    }
}

void launch_match(const uint8_t *in, const Layout &L, uint32_t *m, uint64_t *mbits, uint64_t *chain, uint64_t *chain_pfx,
                  uint32_t *tinfo, hipStream_t st) {
    // FCX_MATCH_DBG (experiments only, output invalid when set): bit0 skip searches, bit1 skip long extension
    static const uint32_t dbg = getenv("FCX_MATCH_DBG") ? (uint32_t)atoi(getenv("FCX_MATCH_DBG")) : 0u;
    const uint32_t grid = L.nblocks * L.tpb;
    hipLaunchKernelGGL(k_match, dim3(grid), dim3(kMT), 0, st, in, L, m, mbits, chain, chain_pfx, tinfo, dbg);
}

}  // namespace fcx

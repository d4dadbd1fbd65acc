// fcx_match_uniform.hip — the uniform unit: the match search of a tile whose window is one byte value.
//
// Where the window [t0 - 2048, t1 + 260) of a tile holds one byte value, every position's match is
// known in closed form (m_uniform, fcx_device.h: the leftmost of the equal candidates at the length
// cap; literal at the block start and in the last three bytes -- my_compress.cpp:1446-1514,
// 1675-1714), and the general units write it as such (uniform_tile_out, fcx_match.hip) after
// staging the window in 39 KB of LDS and counting its runs in a 512-lane workgroup.  Here one wave
// per tile checks the window from registers (seven 16-byte loads per lane) and writes the same
// outputs: a tenth of the LDS-bound launch's cost on zeros.
//
// k_classify files a tile here when its 128-byte sample has no byte change and the next tile of its
// block starts with the same byte (that sample lies in this tile's look-ahead); a tile whose window is not
// uniform after all goes on to the runs list (the runs unit is launched after this kernel).  The kernel
// is looped (few VGPRs: no occupancy cost), so any grid covers the whole list: each XCD takes a
// contiguous eighth of it, so the overlapping windows of neighbouring tiles meet in that XCD's L2.
#include "fcx_device.h"

namespace fcx {

constexpr uint32_t kUniLoads = (kTileBytes + 1023) / 1024;   // 16-byte loads per lane over the window

__global__ __launch_bounds__(64, 8) void k_match_uniform(const uint8_t *__restrict__ in, Layout L,
                                                      uint64_t *__restrict__ mbits, uint64_t *__restrict__ chain,
                                                      uint64_t *__restrict__ chain_pfx, uint32_t *__restrict__ tinfo,
                                                      const uint32_t *__restrict__ list, const uint32_t *__restrict__ cnt,
                                                      uint32_t *__restrict__ runs_list, uint32_t *__restrict__ runs_cnt,
                                                      uint8_t *__restrict__ tkind) {
    const uint32_t lane = threadIdx.x;
    const uint32_t c = *cnt;
    const uint32_t xcd = blockIdx.x & 7, slot = blockIdx.x >> 3, nslot = gridDim.x >> 3;   // (grid: x 8)
    const uint32_t p1 = (uint32_t)((uint64_t)c * (xcd + 1) / 8);
    for (uint32_t p = (uint32_t)((uint64_t)c * xcd / 8) + slot; p < p1; p += nslot) {
        const uint32_t bx = list[p];
        const uint32_t b = bx / L.tpb, k = bx % L.tpb;
        const uint64_t bstart = (uint64_t)b * L.B;
        const uint32_t blen = (uint32_t)min((uint64_t)L.B, L.n - bstart);
        const uint32_t t0 = k * kTile, t1 = min(blen, t0 + kTile);
        const uint32_t w0 = t0 >= 2048 ? t0 - 2048 : 0, nload = min(blen, t1 + kLookAhead) - w0;
        const uint8_t *src = in + bstart + w0;
        const uint32_t rep = (uint32_t)src[0] * 0x01010101u;
        // every load in flight at once: a chunk past the window's end reads the window's last 16 bytes
        // instead (the tile has >= 128 bytes, k_classify), so no load is conditional
        uint32_t w[kUniLoads][4], diff = 0;
#pragma unroll
        for (uint32_t r = 0; r < kUniLoads; r++)
            __builtin_memcpy(w[r], src + min(16 * lane + 1024 * r, nload - 16), 16);   // (any byte address)
#pragma unroll
        for (uint32_t r = 0; r < kUniLoads; r++) diff |= (w[r][0] ^ rep) | (w[r][1] ^ rep) | (w[r][2] ^ rep) | (w[r][3] ^ rep);
        if (__ballot(diff != 0)) {   // not one byte value: the runs unit searches it
            if (lane == 0) {
                runs_list[atomicAdd(runs_cnt, 1u)] = bx;   // (one atomic: the count of these is the list's
                tkind[bx] = (uint8_t)kRouteRuns;            //  growth past the classifier's kRcRunsFiled)
            }
            continue;
        }
        // mbits: m_uniform is a match except at the block's first position and where fewer than 4 bytes
        // remain; lane w writes word w
        const uint32_t nw = (t1 - t0 + 63) / 64, a = t0 + 64 * lane;
        if (lane < nw) {
            const uint32_t lo = blen >= 3 ? blen - 3 : 0u;   // literal from lo on
            uint64_t word = t1 - a < 64 ? (1ull << (t1 - a)) - 1 : ~0ull;
            if (a == 0) word &= ~1ull;
            if (lo < a + 64) word &= lo <= a ? 0ull : (1ull << (lo - a)) - 1;
            mbits[(uint64_t)b * L.wpb + (a >> 6)] = word;
        }
        // the speculative chain from t0: a step is min(258, bytes left) (1 at the block start), so each
        // lane jumps its walk to its word over the full-length steps at once, then walks the word
        auto ustep = [&](uint32_t q) -> uint32_t { return m_len(m_uniform(q, blen)) + 1; };
        uint32_t q = t0;
        if (q == 0 && a > 0) q = 1;
        if (q < a && blen - q >= kMaxL) {
            const uint32_t kmax = (blen - q - kMaxL) / kMaxL + 1, ks = (a - q + kMaxL - 1) / kMaxL;
            q += kMaxL * min(kmax, ks);
        }
        uint64_t T = 0;
        uint32_t cn[3] = {0, 0, 0};
        if (lane < nw) {
            while (q < a) q += ustep(q);
            const uint32_t se = min(a + 64, t1);
            while (q < se) {
                T |= 1ull << (q - a);
                const uint32_t Lm = ustep(q) - 1;
                cn[0]++;
                if (Lm) { cn[1]++; cn[2] += (Lm >> 2) + 3; }
                q += Lm + 1;
            }
        }
        uint32_t inc[3];
#pragma unroll
        for (uint32_t u = 0; u < 3; u++) inc[u] = wave_incl_scan(cn[u]);
        if (lane < nw) {
            chain[(uint64_t)b * L.wpb + (uint64_t)k * (kTile / 64) + lane] = T;
            chain_pfx[(uint64_t)bx * (kTile / 64) + lane] = (uint64_t)(inc[0] - cn[0]) |
                                                            ((uint64_t)(inc[1] - cn[1]) << 13) |
                                                            ((uint64_t)(inc[2] - cn[2]) << 24);
        }
        const uint32_t ex = (uint32_t)__builtin_amdgcn_readlane((int)q, (int)(nw - 1));   // the tile's exit
        const uint32_t tot0 = (uint32_t)__builtin_amdgcn_readlane((int)inc[0], 63),
                       tot1 = (uint32_t)__builtin_amdgcn_readlane((int)inc[1], 63),
                       tot2 = (uint32_t)__builtin_amdgcn_readlane((int)inc[2], 63);
        if (lane < 5)
            tinfo[8ull * bx + lane] = lane == 0 ? kTileUniform | kTileMFull : lane == 1 ? ex : lane == 2 ? tot0
                                    : lane == 3 ? tot1 : tot2;
    }
}

void launch_match_uniform(const uint8_t *in, const Layout &L, uint64_t *mbits, uint64_t *chain, uint64_t *chain_pfx,
                          uint32_t *tinfo, const uint32_t *list, const uint32_t *cnt, uint32_t *runs_list,
                          uint32_t *runs_cnt, uint8_t *tkind, uint32_t grid, hipStream_t st) {
    hipLaunchKernelGGL(k_match_uniform, dim3(grid), dim3(64), 0, st, in, L, mbits, chain, chain_pfx, tinfo, list, cnt,
                       runs_list, runs_cnt, tkind);
}

}  // namespace fcx

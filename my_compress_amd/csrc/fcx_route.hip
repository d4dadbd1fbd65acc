// fcx_route.hip — which match unit searches which tile, decided from the tile's own bytes.
//
// The match search is compiled as four units (fcx_match*.hip), each fastest on one
// kind of data and exact on any.  The reference's block codec carries no state from one block to the
// next (my_compress.cpp:4090-4122; the parse 1675-1714 depends on the block in hand only), so the
// choice is made per call from the call's input: k_classify reads a 128-byte sample at the start of
// every 4096-position tile and files the tile into one list per unit, in tile order:
//
//   uniform   no byte change in the sample (zeros, padding): the uniform unit checks the whole
//             window and writes the closed form, else hands the tile on to the runs list
//   runs      few byte changes (≤ 1 per 8 sampled bytes: the tile's window then has ≲ 1024 runs
//             and takes the run-mode closed form; zeros, runs)
//   4-byte    ≤ 6 of the 64 byte-value buckets (v >> 2) seen ('ACGT' data: dense 3-byte keys)
//   sparse    ≥ 40 buckets seen and ≤ 1 byte in 16 equal to the byte 4 back (random data: ~55
//             buckets in 128 bytes, 1 in 256; text ~13 buckets)
//   no-filter everything else (text, mixed)
//
// The counts are per-lane register work (no LDS atomics) reduced over the tile's 4 lanes by lane
// shuffles.
//
// A wrong guess costs time only.  The sparse and runs units hand a tile they cannot search in their
// own modes to the no-filter unit's list (MatchRoute::defer_list), which is launched after them, so
// no tile reaches the whole-tile run table it could overflow; the uniform unit hands a tile whose
// window is not one byte value to the runs list.  The host launches each unit over its list with a
// grid estimated from a recent call (the counts come back asynchronously; a context's first call
// waits for this call's counts instead), and each unit's looped remainder kernel
// (k_match_rest_<unit>) takes the entries past its grid.  The output bytes do not depend on any of
// this.
#include "fcx_device.h"

namespace fcx {

constexpr uint32_t kClsLanes = 1024;                     // lanes per classify workgroup
constexpr uint32_t kClsPerTile = 4;                      // lanes per tile, 32 sampled bytes each
constexpr uint32_t kClsRound = kClsLanes / kClsPerTile;  // 256 tiles per round
constexpr uint32_t kClsRounds = 4;                       // rounds per workgroup: 1024 tiles (4 MiB)
constexpr uint32_t kClsWgTiles = kClsRound * kClsRounds;
constexpr uint32_t kClsSample = 32 * kClsPerTile;        // 128 bytes sampled per tile (1/32 of the input)
static_assert(kClsWgTiles <= kClsLanes, "one lane per tile for the ranks");

// cnt: [0, kRoutes) list lengths (the no-filter and runs lists grow by the hand-ons later),
// [kRcNfFiled] tiles the classifier filed as no-filter, [kRcValid] tiles with bytes (a block's tail
// tiles past its length have none).
// A workgroup takes kClsWgTiles consecutive tiles in rounds of kClsRound (the next round's sample
// loads issued before this round's counting), then files them with one global atomic per list:
// few workgroups (one per CU for a GiB), because atomics on one address from every XCD serialise in
// the fabric (256 lanes per 32 tiles and one atomic set per workgroup: 0.20-0.29 ms per GiB).
__global__ __launch_bounds__(kClsLanes) void k_classify(const uint8_t *__restrict__ in, Layout L, uint32_t nt,
                                                        uint32_t *__restrict__ lists, uint32_t stride,
                                                        uint32_t *__restrict__ cnt, uint8_t *__restrict__ tkind,
                                                        const uint32_t R) {
    __shared__ uint8_t s_kind[kClsWgTiles];
    __shared__ uint16_t s_ub[kClsWgTiles];   // uniform sample: 0x100 | its byte, else 0
    __shared__ uint32_t s_wsum[kClsWgTiles / 64][kRoutes + 1];
    __shared__ uint32_t s_base[kRoutes];
    const uint32_t tid = threadIdx.x, tl = tid / kClsPerTile, sub = tid % kClsPerTile;
    const uint32_t lane = tid & 63, wv = tid >> 6;
    const uint32_t wgt = kClsRound * R;   // this launch's tiles per workgroup (R <= kClsRounds rounds)
    const uint32_t tile0 = blockIdx.x * wgt;
    const uint32_t o = 32 * sub;   // this lane's sampled bytes [o, o + 32) of its tile

    // sample of round r's tile (zero past len; len 0: no tile / no bytes)
    auto load = [&](uint32_t r, uint32_t (&w)[8]) -> uint32_t {
        const uint32_t bx = tile0 + kClsRound * r + tl;
        uint32_t len = 0;
        const uint8_t *src = in;
        if (bx < nt) {
            const uint32_t b = bx / L.tpb, k = bx % L.tpb;
            const uint64_t bstart = (uint64_t)b * L.B;
            const uint32_t blen = (uint32_t)min((uint64_t)L.B, L.n - bstart), t0 = k * kTile;
            if (t0 < blen) {
                len = min(kClsSample, blen - t0);
                src = in + bstart + t0;
            }
        }
        if (o + 32 <= len && (((uintptr_t)(src + o)) & 15) == 0) {
            const uint4 a = ((const uint4 *)(src + o))[0], c = ((const uint4 *)(src + o))[1];
            w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w; w[4] = c.x; w[5] = c.y; w[6] = c.z; w[7] = c.w;
        } else {
#pragma unroll
            for (uint32_t q = 0; q < 8; q++) {
                w[q] = 0;
#pragma unroll
                for (uint32_t j = 0; j < 4; j++)
                    if (o + 4 * q + j < len) w[q] |= (uint32_t)src[o + 4 * q + j] << (8 * j);
            }
        }
        return len;
    };
    const uint32_t rounds = min(R, (nt - tile0 + kClsRound - 1) / kClsRound);
    // every round's sample loads in flight at once (one memory latency per workgroup)
    uint32_t ws[kClsRounds][8], lens[kClsRounds];
#pragma unroll
    for (uint32_t r = 0; r < kClsRounds; r++) lens[r] = r < rounds ? load(r, ws[r]) : 0u;
#pragma unroll
    for (uint32_t r = 0; r < kClsRounds; r++) {
        if (r >= rounds) break;
        const uint32_t(&w)[8] = ws[r];
        const uint32_t len = lens[r];
        // the previous lane's last dword (the byte before o, and the bytes 4 back of o .. o + 3);
        // the lanes of a tile are consecutive in the wave
        const uint32_t pw = __shfl_up(w[7], 1, 64);
        // per lane, over its sampled bytes x in [o, o + 32) ∩ [1, len): byte changes (d[x] != d[x-1]),
        // repeats 4 back (d[x] == d[x-4], x >= 4) and the byte values' 64 buckets (v >> 2) seen
        uint32_t changes = 0, eq4 = 0;
        uint64_t seen = 0;
#pragma unroll
        for (uint32_t q = 0; q < 8; q++) {
            const uint32_t cur = w[q], prev = q ? w[q - 1] : pw;
            const uint32_t d1 = cur ^ ((cur << 8) | (prev >> 24)), d4 = cur ^ prev;
#pragma unroll
            for (uint32_t j = 0; j < 4; j++) {
                const uint32_t x = o + 4 * q + j;
                if (x < len) {
                    seen |= 1ull << ((cur >> (8 * j + 2)) & 63u);
                    changes += x >= 1 && ((d1 >> (8 * j)) & 0xFFu) != 0;
                    eq4 += x >= 4 && ((d4 >> (8 * j)) & 0xFFu) == 0;
                }
            }
        }
        uint32_t slo = (uint32_t)seen, shi = (uint32_t)(seen >> 32);
#pragma unroll
        for (uint32_t sft = 1; sft < kClsPerTile; sft <<= 1) {
            changes += __shfl_xor(changes, sft, 64);
            eq4 += __shfl_xor(eq4, sft, 64);
            slo |= __shfl_xor(slo, sft, 64);
            shi |= __shfl_xor(shi, sft, 64);
        }
        const uint32_t buckets = (uint32_t)__builtin_popcount(slo) + (uint32_t)__builtin_popcount(shi);
        uint32_t kind = kRoutes;   // no bytes: no list
        if (len) {
            if (changes == 0 && len == kClsSample) kind = kRouteUniform;
            else if (8 * changes <= len) kind = kRouteRuns;
            else if (buckets <= 6) kind = kRouteKey4;
            else if (buckets >= 40 && 16 * eq4 <= len) kind = kRouteSparse;
            else kind = kRouteNoFilter;
        }
        if (sub == 0) {
            s_kind[kClsRound * r + tl] = (uint8_t)kind;
            s_ub[kClsRound * r + tl] = kind == kRouteUniform ? (uint16_t)(0x100u | (w[0] & 0xFFu)) : (uint16_t)0;
        }
    }
    __syncthreads();
    // file the workgroup's tiles in tile order: lane t holds tile tile0 + t; ranks by ballot.  A uniform
    // sample goes to the uniform unit only when the next tile of its block starts with the same byte
    // too (that tile's sample lies inside this tile's look-ahead, so a uniform window has it; on runs
    // data a 128-byte run is common, two at 4 KiB are not, and each misfiled tile costs the uniform
    // unit a window read and a same-address atomic)
    uint32_t kind = tid < rounds * kClsRound ? (uint32_t)s_kind[tid] : kRoutes;
    if (kind == kRouteUniform && tid + 1 < rounds * kClsRound && tile0 + tid + 1 < nt) {
        const uint32_t bx = tile0 + tid, b = bx / L.tpb, k = bx % L.tpb;
        const uint64_t bstart = (uint64_t)b * L.B;
        const uint32_t blen = (uint32_t)min((uint64_t)L.B, L.n - bstart);
        if (k + 1 < L.tpb && (k + 1) * kTile < blen && s_ub[tid + 1] != s_ub[tid]) kind = kRouteRuns;
    }
    uint32_t rank = 0;
    if (tid < wgt) {
#pragma unroll
        for (uint32_t u = 0; u <= kRoutes; u++) {
            const uint64_t bal = __ballot(kind == u);
            if (kind == u)
                rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
            if (lane == 0) s_wsum[wv][u] = (uint32_t)__popcll(bal);
        }
    }
    __syncthreads();
    if (tid <= kRoutes) {
        uint32_t tot = 0;
        for (uint32_t q = 0; q < wgt / 64; q++) tot += s_wsum[q][tid];
        if (tid < kRoutes) {
            s_base[tid] = tot ? atomicAdd(&cnt[tid], tot) : 0u;
            if (tid == kRouteNoFilter && tot) atomicAdd(&cnt[kRcNfFiled], tot);
            if (tid == kRouteRuns && tot) atomicAdd(&cnt[kRcRunsFiled], tot);
        } else {   // tiles with bytes: all but the no-list ones
            const uint32_t valid = wgt - tot;   // (lanes past the shard's tiles count as no-list)
            if (valid) atomicAdd(&cnt[kRcValid], valid);
        }
    }
    __syncthreads();
    if (tid < wgt && tile0 + tid < nt) tkind[tile0 + tid] = (uint8_t)kind;   // (the direct launch's filter)
    if (tid < wgt && kind < kRoutes) {
        uint32_t pos = s_base[kind] + rank;
        for (uint32_t q = 0; q < wv; q++) pos += s_wsum[q][kind];
        lists[(uint64_t)kind * stride + pos] = tile0 + tid;
    }
}

// the no-filter list's count just before its listed launch: the launch covers its entries up to
// min(grid, that count); the sparse / runs remainders hand on later tiles past it, which the
// no-filter remainder then takes (fcx_capi.hip)
__global__ void k_route_mark(uint32_t *__restrict__ dst, const uint32_t *__restrict__ src) {
    if (threadIdx.x == 0) *dst = *src;
}

void launch_route_mark(uint32_t *dst, const uint32_t *src, hipStream_t st) {
    hipLaunchKernelGGL(k_route_mark, dim3(1), dim3(64), 0, st, dst, src);
}

void launch_classify(const uint8_t *in, const Layout &L, uint32_t *lists, uint32_t stride, uint32_t *cnt,
                     uint8_t *tkind, hipStream_t st) {
    const uint32_t nt = L.nblocks * L.tpb;
    // rounds per workgroup: 4 from 256 workgroups on (a GiB), fewer below, so a small shard (C2: 64 MiB)
    // still spreads over 64 workgroups
    const uint32_t R = std::min(kClsRounds, std::max(1u, nt / (256u * kClsRound)));
    hipLaunchKernelGGL(k_classify, dim3((nt + kClsRound * R - 1) / (kClsRound * R)), dim3(kClsLanes), 0, st, in, L, nt,
                       lists, stride, cnt, tkind, R);
}

}  // namespace fcx

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
//   2. counting-sort every window position by the bucket of its 3-byte key (a
//      bijection of Z/2^24 gives a 13-bit bucket; 16-bit entries keep the position
//      and 3 more hash bits, the rare collisions are rejected by comparing key
//      bytes); a bucket is one contiguous LDS range (16-bit counters by LDS
//      atomics, block scan, scatter), its entries in slab order (12 barrier-
//      separated insertion passes of 512 positions), and the bucket counters
//      sampled during the passes bound each query's window [x - 2047, x) inside
//      its bucket;
//   3. every tile position scans that part of its bucket (independent LDS loads, no
//      pointer chase; four queries interleaved per lane) and keeps the
//      max-length / min-position candidate among entries in its window (stored
//      to m[] only where a match or "unknown" results, flagged per position in
//      the mbits bitmap by one ballot per wave: random data writes almost no m).  A
//      candidate's key check and length come from three dword compares against
//      the query's preloaded bytes 0..11; only a match reaching 12 bytes enters
//      the extension loop.  A candidate right of the current best is skipped when
//      it cannot be longer (best at the cap, or its byte at the best length
//      differs).  A bucket with more than kMaxChainSteps entries, or a query with
//      more than kExtBudget long extensions (periodic data), leaves the position
//      "unknown" for the run table / the stitch kernel's wave-parallel evaluation
//      (runs / zeros / short periods: long matches, few tokens);
//   4. greedy parse of the tile assuming a token starts at t0: each lane walks
//      its 8 positions, lanes agree on sub-segment entries by a Jacobi fixed
//      point (entry_{k+1} = exit of sub-segment k walked from entry_k) that
//      converges in one or two rounds because greedy chains resynchronise; then
//      the tile's chain bitmap, per-64-position prefix counts (tokens, matches,
//      golomb bits) and totals are published for the stitch kernel.
#include <cstdlib>

#include "fcx_device.h"

#ifndef FCX_MATCH_EXIT
#define FCX_MATCH_EXIT 0u   // development: a dbg timing-exit bit compiled into the product kernel (tools/phase_libs.sh)
#endif

// FCX_KEY4 (fcx_match_k4.hip): the same kernel with the bucket search over 4-byte keys, for shards of
// dense keys (small alphabets such as 'ACGT' data: 64 distinct 3-byte keys, ~32 candidates per
// query).  A match of length >= 4 shares its query's first four bytes, so the 4-byte bucket holds
// every candidate of a longest match >= 4 (a quarter of the 3-byte candidates on 'ACGT' data); a
// query without one takes the leftmost 3-byte match by a window scan.  The context picks this
// translation unit per call from the previous call's share of small-alphabet blocks (k_tree);
// both units give the same bytes.  The K3 unit's source is unchanged by the K4 branches below
// (preprocessor): k_match's register allocation moves with any edit of its source.
#ifndef FCX_KEY4
#define FCX_KEY4 0
#endif
// FCX_NOFILTER (fcx_match_nf.hip): the kernel without the repeat sample, the repeat filter, the
// sparse search and the run count, for shards of match-dense blocks (text: every tile takes the
// bucket search there, so the sampled filter that sends random-data tiles to the sparse search and
// the run count that sends long-run tiles to the run mode are wasted work, ~0.8 ms per GiB).
// Chosen per call like the 4-byte-key unit; the same bytes either way.
#ifndef FCX_NOFILTER
#define FCX_NOFILTER 0
#endif
// FCX_RUNS (fcx_match_runs.hip): the kernel with the run-mode walk inlined, for shards of long-match
// blocks (runs, zeros).  Out of line, the walk saves callee-saved VGPRs to scratch on every run-mode
// tile (16 KB per tile, written to HBM); inlined, the other tile modes' register allocation moves,
// which only this unit's shards pay.
#ifndef FCX_RUNS
#define FCX_RUNS 0
#endif
// FCX_SPARSE (fcx_match_sparse.hip): the kernel without the bucket search, the repeat sample and the
// run count, for shards of few-match blocks (random data: every tile takes the sparse search).  Every
// tile runs the repeat filter; a tile it does not send to the sparse search takes the whole-tile
// run-table mode instead (exact for any tile, slow where the runs overflow the table:
// fcx_ctx_set_match_mode 2); the sparse search is inlined.  Rand k_match 2.64 -> 2.31 ms per GiB
// (DESIGN.md §4).
#ifndef FCX_SPARSE
#define FCX_SPARSE 0
#endif
// FCX_NOBUCKET: no bucket search; a tile the repeat filter does not send to the sparse search takes
// the whole-tile run-table mode (the sparse unit)
#ifndef FCX_NOBUCKET
#define FCX_NOBUCKET FCX_SPARSE
#endif
// FCX_SHORTK (the no-filter unit): waves whose longest bucket range is at most this many entries skip
// the K search and pass B of the bucket scan (0: never)
#ifndef FCX_SHORTK
#define FCX_SHORTK 0
#endif
// FCX_REST (fcx_match_rest_<unit>.hip): the unit's tile body in k_match_rest_<unit>, a loop over the
// entries of the unit's list that its launch did not cover (fcx_route.hip).  Its own translation
// unit, so the unit's k_match keeps its code generation.
#ifndef FCX_REST
#define FCX_REST 0
#endif
#ifndef FCX_REST_WAVES
#define FCX_REST_WAVES 8
#endif
#if FCX_SPARSE   // (the sparse search inline in its own unit: rand k_match 2.43 -> 2.31 ms per GiB)
#define FCX_SPARSE_CALL __forceinline__
#else
#define FCX_SPARSE_CALL __noinline__
#endif
#if !FCX_NOFILTER && !FCX_SPARSE && !FCX_RUNS
#define FCX_SAMPLE 1   // the repeat sample decides whether the filter runs
#else
#define FCX_SAMPLE 0
#endif
// the unit's kernel and launcher names (a unit may combine switches: the 4-byte-key unit also drops
// the filter and the run count)
#if FCX_KEY4
#define k_match k_match_k4
#define launch_match launch_match_k4
#define launch_match_listed launch_match_k4_listed
#define launch_match_direct launch_match_k4_direct
#define k_match_rest k_match_rest_k4
#define launch_match_rest launch_match_rest_k4
#elif FCX_NOFILTER
#define k_match k_match_nf
#define launch_match launch_match_nf
#define launch_match_listed launch_match_nf_listed
#define launch_match_direct launch_match_nf_direct
#define k_match_rest k_match_rest_nf
#define launch_match_rest launch_match_rest_nf
#elif FCX_SPARSE
#define k_match k_match_sparse
#define launch_match launch_match_sparse
#define launch_match_listed launch_match_sparse_listed
#define launch_match_direct launch_match_sparse_direct
#define k_match_rest k_match_rest_sparse
#define launch_match_rest launch_match_rest_sparse
#elif FCX_RUNS
#define k_match k_match_runs
#define launch_match launch_match_runs
#define launch_match_listed launch_match_runs_listed
#define launch_match_direct launch_match_runs_direct
#define k_match_rest k_match_rest_runs
#define launch_match_rest launch_match_rest_runs
#endif
// FCX_LISTED (fcx_match_<unit>_listed.hip): the unit's listed kernel instance alone (routed calls,
// fcx_route.hip), in its own translation unit: next to it the direct instance's code moved
#ifndef FCX_LISTED
#define FCX_LISTED 0
#endif
// FCX_DIRECT (fcx_match_<unit>_direct.hip): the unit's checked direct instance alone (a routed call
// whose estimate gives the unit most but not nearly all tiles).  Beside the unrouted instances it
// moved their code: the helpers the kernels share are inlined differently with a third caller (the
// runs unit went from 54 VGPRs / 12 B of stack to 62 / 40).
#ifndef FCX_DIRECT
#define FCX_DIRECT 0
#endif
#define FCX_UNIT (FCX_KEY4 || FCX_NOFILTER || FCX_SPARSE || FCX_RUNS)
#if FCX_RUNS
#define FCX_RMODE_CALL __forceinline__
#else
#define FCX_RMODE_CALL __noinline__
#endif

namespace fcx {

#if FCX_REST
// k_match_rest loops over tiles: the thread index is re-read per use through an opaque asm, so
// nothing derived from it is hoisted out of the loop and kept live across a whole tile body
__device__ inline uint32_t rest_tid() {
    uint32_t t = threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
}
#define FCX_TID rest_tid()
#else
#define FCX_TID threadIdx.x
#endif

constexpr uint32_t kWinPos = kHalo + 1 + kTile;      // 6144 window positions per tile
constexpr uint32_t kMT = kMatchThreads;              // 512
constexpr uint32_t kSeg = kTile / kMT;               // 8 positions per lane in the parse
constexpr uint32_t kQPL = kTile / kMT;               // 8 queries per lane
#if defined(FCX_UNIT_ILP)
constexpr uint32_t kIlp = FCX_UNIT_ILP;   // a unit's own width (fcx_match_nf.hip, fcx_match_k4.hip)
#else
constexpr uint32_t kIlp = 4;                         // interleaved chain walks per lane
#endif
constexpr uint32_t kWaves = kMT / 64;
constexpr uint32_t kHeadWords = (1u << kHashBits) / 2 + 4;                 // u16 counters + sentinel
constexpr uint32_t kEntWords = kWinPos / 2;                                 // u16 entries
constexpr uint32_t kIns = kWinPos / kMT;              // 12 window positions per lane (insert / filter)
static_assert(kIns * kMT == kWinPos && kIns == 12, "12 consecutive window positions per lane");
// repeat filter: "seen" and "dup" bitmaps of 17-bit key hashes (2 x 16 KiB)
constexpr uint32_t kFilterBits = 17;
constexpr uint32_t kFilterWords = 2 * (1u << kFilterBits) / 32;
constexpr uint32_t kSparseEvents = 448;              // repeats up to which the sparse search runs
constexpr uint32_t kSampleWords = 128;               // repeat sample: 2^12-bit bitmap of 512 sampled keys
constexpr uint32_t kSampleEvents = 96;               // sampled repeats above which the filter is skipped
constexpr uint32_t kSparseBuckets = 1024;            // buckets of the sparse search's counting sort
// sparse-search layout inside the region (words): step (u16 x 4096) | P | counters | sorted | mbits
constexpr uint32_t kSpP = kTile / 2, kSpCnt = kSpP + 2 * kSparseEvents, kSpSrt = kSpCnt + kSparseBuckets / 2 + 2,
                   kSpMb = kSpSrt + kSparseEvents;   // P: u32 x 2 kSparseEvents; srt: u16 x 2 kSparseEvents
static_assert(kSpMb % 2 == 0 && kSpMb + 128 <= kFilterWords - kTile, "sparse layout below the results");
constexpr uint32_t kBucketWords = kHeadWords + kEntWords > kTile / 2 + 3 * kMT + 1
                                      ? kHeadWords + kEntWords : kTile / 2 + 3 * kMT + 1;
constexpr uint32_t kRegionWords = kBucketWords > kFilterWords ? kBucketWords : kFilterWords;
constexpr uint32_t kResLds = kRegionWords - kTile;   // search results (m) per tile position, kept for the
                                                     // compact match list; clear of step and the parse scratch
static_assert(kResLds >= kTile / 2 + 3 * kMT + 1, "results clear of step and the parse scratch");
// bucket scan pass B (bucket search only): each wave's hot-query slots and owner marks, in the
// region words the counters and entries leave free
constexpr uint32_t kHotCap = 32;                                   // hot queries per wave and group
constexpr uint32_t kHotWords = 3 * kHotCap + 16;                   // x, base, best per slot + 64 u8 marks
constexpr uint32_t kScanHot = kHeadWords + kEntWords;
static_assert(kScanHot + kHotWords * kWaves <= kRegionWords, "hot-query scratch inside the region");
// dense-window phase (run table) inside the same region
constexpr uint32_t kRunBmWords = 208;                // 6656 bitmap positions >= kTileBytes + 1, 13 x kMT
constexpr uint32_t kRunListWords = 2 * 64 * kWaves;   // per-wave candidate lists (se, ext)
constexpr uint32_t kRunTableCap = kRegionWords - (kTile / 2 + kRunBmWords + kRunBmWords / 2 + 2 + kRunListWords) - 4;  // 4 spare
static_assert(32 * kRunBmWords >= kTileBytes + 1 && (32 * kRunBmWords) % kMT == 0, "run bitmap");
static_assert(kRunBmWords <= 4 * 64, "prefix scan spans four waves");
static_assert(kRunTableCap >= 1536, "run table");

__device__ inline uint32_t key_mix(uint32_t key) { return (key * 0x9E3779B1u) & 0xFFFFFFu; }  // bijective mod 2^24
#if FCX_KEY4
__device__ inline uint32_t key_mix4(uint32_t key) { return (key * 0x9E3779B1u) >> 8; }   // 24 mixed bits of 4 bytes
constexpr uint32_t kNeed3 = 0xFFFFFFFEu;   // query result: no 4-byte candidate, take the leftmost 3-byte match
#endif

// lanes below this one with their bit set in a wave mask
__device__ inline uint32_t lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// ---- 3b. dense windows (zeros, runs): the positions the bucket search left
// "unknown" get their exact match from the run table (run_match, fcx_device.h).
// Kept out of line so its registers do not weigh on the search loop; it runs
// only in tiles that have unknown positions.  mx = m of image position 0, ilen =
// block length - image base, w0 = image base in the block.  mbx (whole-tile mode,
// no bucket search ran): mbits of image position 0, written here per 64 positions.
template <bool kDev>
__device__ __attribute__((always_inline)) inline void dense_phase_body(const uint32_t *sdw, uint32_t *region, uint16_t *step,
                                                                      uint32_t *s_red, uint32_t *s_unknown, uint32_t *mx,
                                                                      uint64_t *mbx, uint32_t q0, uint32_t npos, uint32_t nload,
                                                                      uint32_t ilen, uint32_t w0, uint32_t dbg_in,
                                                                      uint16_t *dist, uint32_t rt_cap) {
    const uint32_t dbg = kDev ? uni(dbg_in) : 0u;   // development bits exist only in k_match<true>
    q0 = uni(q0); npos = uni(npos); nload = uni(nload); ilen = uni(ilen); w0 = uni(w0);   // (arguments arrive
    rt_cap = uni(rt_cap);                                                                 //  in VGPRs)
    const uint32_t tid = FCX_TID;
    uint32_t *rbm = region + kTile / 2;                       // boundary bitmap, kRunBmWords
    uint16_t *prc = (uint16_t *)(rbm + kRunBmWords);          // prefix counts per bitmap word
    uint32_t *rt = rbm + kRunBmWords + kRunBmWords / 2 + 2 + kRunListWords;   // run table
    // bitmap by ballot: a wave's 64 lanes cover 64 consecutive image positions
    for (uint32_t y0 = 0; y0 < 32 * kRunBmWords; y0 += kMT) {
        const uint32_t y = y0 + tid;
        const bool bit = y == nload || (y < nload && (y == 0 || lds_ld1(sdw, y) != lds_ld1(sdw, y - 1)));
        const uint64_t bal = __ballot(bit);
        if ((tid & 63) == 0) { rbm[y >> 5] = (uint32_t)bal; rbm[(y >> 5) + 1] = (uint32_t)(bal >> 32); }
    }
    __syncthreads();
    // exclusive prefix counts (kRunBmWords <= 4 waves of lanes)
    const uint32_t pc = tid < kRunBmWords ? (uint32_t)__builtin_popcount(rbm[tid]) : 0u;
    const uint32_t inc = wave_incl_scan(pc);
    if ((tid & 63) == 63) s_red[tid >> 6] = inc;
    __syncthreads();
    uint32_t pre = inc - pc;
    for (uint32_t w = 0; w < (tid >> 6); w++) pre += s_red[w];
    const uint32_t nruns = s_red[0] + s_red[1] + s_red[2] + s_red[3];
    if (tid < kRunBmWords) prc[tid] = (uint16_t)pre;
    if (nruns <= rt_cap && tid < kRunBmWords)
        for (uint32_t v = rbm[tid], o = pre; v; v &= v - 1, o++) {
            const uint32_t y = 32 * tid + __builtin_ctz(v);
            rt[o] = y | (y < nload ? lds_ld1(sdw, y) << 16 : 0x1000000u);
        }
    if (tid == 0) *s_unknown = 0;
    __syncthreads();
    if (dbg & 8192u) return;   // timing: run table only
    // Evaluation, one chunk of 64 consecutive positions per wave step.  The chunk's
    // positions fall into a few own runs; for each, the wave scans the window's
    // runs one per lane, keeps those of the own run's byte (with ext, the run-level
    // common prefix after them, precomputed up to kMaxL) in a per-wave list by
    // ballot compaction, and every position of that own run walks the list.  The
    // list keeps run order, so the strict > keeps the leftmost maximum.
    const uint32_t lane = tid & 63, wv = tid >> 6;
    uint2 *wl2 = (uint2 *)(rt - kRunListWords) + 64 * wv;    // per-wave candidate list (se, ext)
    bool left = false;
    for (uint32_t c0 = q0 + 64 * wv; c0 < npos; c0 += kMT) {
        const uint32_t x = c0 + lane;
        const bool need = x < npos && step[x - q0] == 0;
        if (__ballot(need) == 0ull) continue;
        const uint32_t xv = min(x, npos - 1);
        const uint32_t cap = min(kMaxL, ilen - xv) - 1;
        const uint32_t xlo = max(w0 + xv, kWin) - kWin - w0;
        const uint32_t ko = run_rank(rbm, prc, xv) - 1;
        const uint32_t kfirst = __shfl(ko, 0, 64), klast = __shfl(ko, 63, 64);
        uint32_t res = 0;
        bool lost = need && nruns > rt_cap;
        const bool table = nruns <= rt_cap;
        // this lane's own run: r bytes left from xv, own run start / byte
        const uint32_t own = table ? rt[ko] : 0u;
        const uint32_t r = (table ? rt[ko + 1] & 0xFFFFu : xv) - xv;
        const bool big = r > cap;
        uint32_t best = 0;   // packed L << 13 | (8191 - j): max = longest, then leftmost
        // The candidate lists of the chunk's own runs go side by side into the wave's list
        // (as long as they fit) and are folded in one pass, each lane over its own run's
        // list: the fold loop runs max(n) times instead of once per own run.
        uint32_t lst = 0, ln = 0, used = 0;   // lane's pending list wl2[lst, lst + ln); used: wave-uniform
        auto fold = [&](uint32_t base, uint32_t n) {
            if (dbg & 32768u) n = 0;   // timing: no fold
            // four entries per step, loaded unconditionally (clamped index) and folded by
            // selects: no branch, so the four 8-B LDS reads are in flight together
            for (uint32_t t = 0; t < n; t += 4) {
                uint2 w[4];
#pragma unroll
                for (uint32_t u = 0; u < 4; u++) w[u] = wl2[base + min(t + u, n - 1)];
#pragma unroll
                for (uint32_t u = 0; u < 4; u++) {
                    const uint32_t ep = w[u].x >> 16;
                    const uint32_t sp = max(w[u].x & 0xFFFFu, xlo);
                    const uint32_t A = ep - sp;
                    const uint32_t Lr = min(r + w[u].y, cap);
                    const bool ge = !big & (A >= r);
                    const uint32_t Lc = ge ? Lr : min(A, cap);
                    const uint32_t j = (ge & (w[u].y != 0) & (r < cap)) ? ep - r : sp;
                    const uint32_t key = (Lc << 13) | (8191u - j);
                    best = max(best, ((ep > xlo) & (t + u < n)) ? key : 0u);
                }
            }
        };
        auto flush = [&]() {   // fold the pending lists and free the list (wave-uniform call)
            __builtin_amdgcn_wave_barrier();
            fold(lst, ln);
            ln = 0;
            used = 0;
            __builtin_amdgcn_wave_barrier();
        };
        // the window runs kc in [k0, min(k0 + 64, kr)) of the own run's byte, with ext
        // (equal (byte, length) runs extend it; the first run that differs in length adds
        // the shorter length and ends it; the query side meets the image end (sentinel)
        // only past the cap), compacted into wl2 from `at`; returns their count
        auto collect = [&](uint32_t k0, uint32_t kr, uint32_t cb, uint32_t vb0, uint32_t at) -> uint32_t {
            const uint32_t kc = k0 + lane;
            bool cand = false;
            uint32_t se = 0, ext = 0;
            if (kc < kr) {
                const uint32_t v = rt[kc], nv = rt[kc + 1];
                if ((v >> 16) == cb) {
                    cand = true;
                    se = (v & 0xFFFFu) | (nv << 16);
                    uint32_t ka = kc + 1, kb = kr + 1, va = nv, vb = vb0;
                    while ((va >> 16) == (vb >> 16)) {
                        const uint32_t na = rt[ka + 1], nb = rt[kb + 1];
                        const uint32_t la = (na & 0xFFFFu) - (va & 0xFFFFu), lb = (nb & 0xFFFFu) - (vb & 0xFFFFu);
                        if (la != lb) { ext += min(la, lb); break; }
                        ext += la;
                        if (ext >= kMaxL) break;
                        ka++; kb++; va = na; vb = nb;
                    }
                }
            }
            const uint64_t cm = __ballot(cand);
            if (cand) wl2[at + (uint32_t)__builtin_popcountll(cm & ((1ull << lane) - 1ull))] = make_uint2(se, ext);
            return (uint32_t)__builtin_popcountll(cm);
        };
        for (uint32_t kr = kfirst; kr <= klast && table && !(dbg & 16384u); kr++) {
            const bool mine = need && ko == kr;
            const uint64_t in_run = __ballot(mine);
            if (in_run == 0ull) continue;
            const uint32_t cb = rt[kr] >> 16;
            const uint32_t xf = c0 + (uint32_t)__builtin_ctzll(in_run);     // first position of the run here
            const uint32_t klo = run_rank(rbm, prc, max(w0 + xf, kWin) - kWin - w0) - 1;
            if (kr - klo > kRunBudget) { lost = lost || mine; continue; }
            const uint32_t vb0 = rt[kr + 1];
            if (kr - klo <= 64) {   // one pass of lanes over the window runs: a pending list
                if (used + (kr - klo) > 64) flush();
                const uint32_t n = collect(klo, kr, cb, vb0, used);
                if (mine) { lst = used; ln = n; }
                used += n;
            } else {                // a long window: fold each pass of 64 runs at once
                if (used) flush();
                for (uint32_t k0 = klo; k0 < kr; k0 += 64) {
                    const uint32_t n = collect(k0, kr, cb, vb0, 0);
                    __builtin_amdgcn_wave_barrier();
                    if (mine) fold(0, n);
                    __builtin_amdgcn_wave_barrier();
                }
            }
        }
        if (used) flush();
        if (need && !lost) {
            const uint32_t sp = max(own & 0xFFFFu, xlo);
            if (sp < xv) best = max(best, ((big ? cap : r) << 13) | (8191u - sp));
            const uint32_t bL = best >> 13, bj = 8191u - (best & 0x1FFFu);
            res = bL >= kMinL ? m_pack(bL, xv - bj) : 0u;
        }
        if (mbx) {   // whole-tile mode: this wave writes the positions' mbits word and m row
            const uint64_t mb = __ballot(need && !lost && res != 0), lb = __ballot(lost);
            if (lane == 0) mbx[c0 >> 6] = mb | lb;
            if (lost) mx[x] = kUnknown;
            else if (mb && need) mx[x] = res;
        } else if (need && !lost) {
            mx[x] = res;
        }
        if (need && !lost) {
            step[x - q0] = (uint16_t)(res ? m_len(res) + 1 : 1);
            if (dist) dist[x - q0] = (uint16_t)m_dist(res);
        }
        left = left || lost;
    }
    if (left) *s_unknown = 1;
    __syncthreads();
}
// the search kernel's copy (tiles the bucket search left unknown positions in): out of line, so its
// registers do not weigh on the search; the run-mode kernel inlines the body
template <bool kDev>
__device__ __noinline__ void dense_phase(const uint32_t *sdw, uint32_t *region, uint16_t *step, uint32_t *s_red,
                                         uint32_t *s_unknown, uint32_t *mx, uint64_t *mbx, uint32_t q0, uint32_t npos,
                                         uint32_t nload, uint32_t ilen, uint32_t w0, uint32_t dbg_in, uint16_t *dist,
                                         uint32_t rt_cap) {
    dense_phase_body<kDev>(sdw, region, step, s_red, s_unknown, mx, mbx, q0, npos, nload, ilen, w0, dbg_in, dist, rt_cap);
}

// ---- 3c. run-mode tiles (whole-tile run table: zeros-free low-entropy data, e.g. runs).
// Only the resolve span [t0, t0 + kResolveSpan) is evaluated at every position (dense_phase:
// k_resolve reads those m rows); past it, m is evaluated at the chain positions only (about
// one position in 66 on runs data), by one wave per position over the run table.
constexpr uint32_t kRunTableOff = kTile / 2 + kRunBmWords + kRunBmWords / 2 + 2 + kRunListWords;   // rt in region
constexpr uint32_t kRmDist = kRegionWords - kTile / 2;           // u16 x kTile: distance of every evaluated position
constexpr uint32_t kRmOnA = kRmDist - kTile / 16;                // kTile bits: the sub-tile walks' A1 chains
constexpr uint32_t kRmOnB = kRmOnA + kTile / 32;                 // kTile bits: the fix-up walks' positions
constexpr uint32_t kRmRunCap = kRmOnA - kRunTableOff - 4;        // run table entries kept clear of both
constexpr uint32_t kRmSub = kTile / kWaves;                      // 512 positions per wave's sub-tile walk
static_assert(kRmRunCap >= kRunTile + 8, "run-mode table");

// step (L + 1) of tile position x, evaluated over the run table when dense_phase / an earlier
// walk did not (then stored with its distance); wave-uniform; 0 = unknown
__device__ inline uint32_t rm_stepat(FCX_LDS uint32_t *region, uint32_t x, uint32_t q0, uint32_t ilen, uint32_t w0) {
    FCX_LDS uint16_t *step = (FCX_LDS uint16_t *)region;
    // below the span dense_phase stored every position; past it a walk meets only positions
    // no walk has evaluated (A1 walks its own sub-tile forward, A2 stops at the A1 chain), so
    // the lookup would only add a round trip: evaluate directly
    uint32_t sv = x < kRmSpan ? uni(step[x]) : 0u;
    if (sv == 0) {
        const FCX_LDS uint32_t *rbm = region + kTile / 2;
        const uint32_t mm = run_match_wave(rbm, (const FCX_LDS uint16_t *)(rbm + kRunBmWords), region + kRunTableOff,
                                           q0 + x, ilen, w0);
        if (mm == kUnknown) return 0u;
        sv = m_len(mm) + 1;
        if (lane_id() == 0) {
            step[x] = (uint16_t)sv;
            ((FCX_LDS uint16_t *)(region + kRmDist))[x] = (uint16_t)m_dist(mm);
        }
    }
    return sv;
}

__device__ FCX_RMODE_CALL void rmode_walk(FCX_LDS uint32_t *region, FCX_LDS uint32_t *s_ex, FCX_LDS uint32_t *s_unknown,
                                        uint32_t q0, uint32_t nt, uint32_t ilen, uint32_t w0, uint32_t t0, uint64_t *mbw,
                                        uint64_t *cw, uint64_t *pfx, uint32_t *ti, uint32_t *mt, uint32_t dbg) {
    const uint32_t tid = FCX_TID, lane = tid & 63, wv = uni(tid >> 6);   // walks: wave-uniform, scalar
    q0 = uni(q0); nt = uni(nt); ilen = uni(ilen); w0 = uni(w0); t0 = uni(t0);   // (arguments arrive in VGPRs)
    FCX_LDS uint16_t *step = (FCX_LDS uint16_t *)region;
    FCX_LDS uint16_t *dist = (FCX_LDS uint16_t *)(region + kRmDist);
    FCX_LDS uint32_t *onA = region + kRmOnA, *onB = region + kRmOnB;
    for (uint32_t w = tid; w < 2 * (kTile / 32); w += kMT) onA[w] = 0;   // onA and onB (adjacent)
    __syncthreads();
    const uint32_t a = kRmSub * wv, bnd = min(a + kRmSub, nt);
    bool lost = false;
    uint32_t X1 = a;
    {   // A1
        uint32_t x = a;
        while (x < bnd) {
            const uint32_t sv = rm_stepat(region, x, q0, ilen, w0);
            if (sv == 0) { lost = true; break; }
            if (lane == 0) onA[x >> 5] |= 1u << (x & 31);   // (the sub-tile's words are this wave's alone)
            x += sv;
        }
        X1 = x;
        if (lane == 0) s_ex[wv] = x;
        if (lost && lane == 0) *s_unknown = 1;
    }
    __syncthreads();
    if (uni(*s_unknown) || (dbg & (1u << 18))) return;   // (timing: A1 only)
    uint32_t curE = a, meet = a;   // this sub-tile's entry and where its chain joins the A1 chain
    for (uint32_t round = 0; round < kWaves; round++) {   // A2
        const uint32_t E = wv == 0 ? 0u : uni(s_ex[wv - 1]);
        __syncthreads();
        bool changed = false;
        if (a < nt && E != curE) {
            curE = E;
            if (lane < kRmSub / 32) onB[a / 32 + lane] = 0;
            __builtin_amdgcn_wave_barrier();
            uint32_t x = E;
            while (x < bnd && !((uni(onA[x >> 5]) >> (x & 31)) & 1u)) {
                const uint32_t sv = rm_stepat(region, x, q0, ilen, w0);
                if (sv == 0) { lost = true; break; }
                if (lane == 0) onB[x >> 5] |= 1u << (x & 31);
                x += sv;
            }
            meet = x < bnd ? x : bnd;
            const uint32_t ex = x < bnd ? X1 : x;
            changed = ex != uni(s_ex[wv]);
            if (lane == 0) {
                s_ex[wv] = ex;
                if (lost) *s_unknown = 1;
            }
        }
        if (__syncthreads_or(changed ? 1 : 0) == 0 || uni(*s_unknown)) break;
    }
    if (uni(*s_unknown) || (dbg & (1u << 19))) return;   // (timing: A1 + A2)
    // C: lanes 0..7 of wave w take the sub-tile's eight chain words
    const uint32_t gw = a / 64 + lane;                 // tile word of this lane
    const bool own = lane < kRmSub / 64 && 64 * gw < nt;
    uint64_t word = 0, mword = 0;
    uint32_t cnt[3] = {0, 0, 0};
    if (own) {
        const uint32_t lo = 64 * gw;
        const uint64_t A = (uint64_t)onA[2 * gw] | ((uint64_t)onA[2 * gw + 1] << 32);
        const uint64_t B = (uint64_t)onB[2 * gw] | ((uint64_t)onB[2 * gw + 1] << 32);
        const uint64_t keep = meet <= lo ? ~0ull : meet >= lo + 64 ? 0ull : ~0ull << (meet - lo);
        word = curE == a ? A : (B | (A & keep));
        for (uint64_t bb = word; bb; bb &= bb - 1) {
            const uint32_t x = lo + (uint32_t)__builtin_ctzll(bb);
            const uint32_t sv = step[x];
            cnt[0]++;
            if (sv > 1) { mword |= 1ull << (x - lo); cnt[1]++; cnt[2] += ((sv - 1) >> 2) + 3; }
        }
    }
    uint32_t inc[3];
#pragma unroll
    for (int q = 0; q < 3; q++) inc[q] = wave_incl_scan(cnt[q]);
    if (lane == 63)
        for (int q = 0; q < 3; q++) s_ex[kWaves + q * kWaves + wv] = inc[q];   // (s_ex holds >= 4 kWaves words)
    __syncthreads();
    uint32_t pre[3], tot[3];
#pragma unroll
    for (int q = 0; q < 3; q++) {
        uint32_t p = 0, t = 0;
        for (uint32_t w = 0; w < kWaves; w++) {
            const uint32_t v = s_ex[kWaves + q * kWaves + w];
            if (w < wv) p += v;
            t += v;
        }
        pre[q] = p + inc[q] - cnt[q];
        tot[q] = t;
    }
    if (own) {
        cw[gw] = word;
        pfx[gw] = (uint64_t)pre[0] | ((uint64_t)pre[1] << 13) | ((uint64_t)pre[2] << 24);
        if (gw >= kRmSpan / 64) mbw[gw] = ~word | mword;
        uint32_t o = pre[1];
        for (uint64_t bb = mword; bb; bb &= bb - 1) {
            const uint32_t x = 64 * gw + (uint32_t)__builtin_ctzll(bb);
            mt[o++] = m_pack((uint32_t)step[x] - 1u, dist[x]);
        }
    }
    const uint32_t lastw = (nt - 1) / kRmSub;   // the wave whose sub-tile holds the tile end
    if (tid == 0) {
        ti[0] = kTileSpan2;
        ti[1] = t0 + s_ex[lastw];
        ti[2] = tot[0];
        ti[3] = tot[1];
        ti[4] = tot[2];
    }
}

// one candidate xe (image position, already known to lie in the window left of x) of
// query x with preloaded bytes qa/qb/qc: key check and match length from four aligned
// dwords; >= 12 bytes extend byte-exactly, under a per-query extension budget (periodic
// data: every same-phase candidate runs to the cap), past which the query is unknown.
// A candidate right of the best (>= 12) can only win by being longer: skipped at the cap
// or when its byte at the best length differs.  best = L << 13 | (8191 - position):
// its maximum is the longest, then leftmost match.
__device__ inline void scan_candidate(const uint32_t *sdw, uint32_t xe, uint32_t x, uint32_t qa, uint32_t qb,
                                      uint32_t qc, uint32_t cap, uint32_t &best, uint32_t &next, bool &unk,
                                      uint32_t dbg) {
    const uint32_t wb = xe >> 2, sb = xe & 3;
    const uint32_t w_0 = sdw[wb], w_1 = sdw[wb + 1], w_2 = sdw[wb + 2], w_3 = sdw[wb + 3];
    const uint32_t d0 = __builtin_amdgcn_alignbyte(w_1, w_0, sb) ^ qa;
    if (d0 & 0xFFFFFFu) return;   // other key (hash collision)
    uint32_t Lc;
    if (d0) Lc = 3;
    else {
        const uint32_t d1 = __builtin_amdgcn_alignbyte(w_2, w_1, sb) ^ qb;
        if (d1) Lc = 4 + (__builtin_ctz(d1) >> 3);
        else {
            const uint32_t d2 = __builtin_amdgcn_alignbyte(w_3, w_2, sb) ^ qc;
            if (d2) Lc = 8 + (__builtin_ctz(d2) >> 3);
            else {
                const uint32_t bL = best >> 13, bxe = 8191u - (best & 0x1FFFu);
                if (cap <= 12 || (dbg & 2u) ||
                    (bL >= 12 && xe > bxe && (bL >= cap || lds_ld1(sdw, xe + bL) != lds_ld1(sdw, x + bL))))
                    Lc = 12;
                else {
                    if (++next > kExtBudget) { unk = true; return; }
                    Lc = lds_match_len(sdw, xe, x, 12, cap);
                }
            }
        }
    }
    Lc = min(Lc, cap);
    best = max(best, (Lc << 13) | (8191u - xe));
}

// ---- 2b. sparse search (few repeated keys: random data).  P = the window positions whose
// 17-bit hash repeats (<= 2 x repeats), counting-sorted by 10 hash bits; each P position
// inside the tile scans its bucket exactly like the bucket search (key check by dword
// compare, leftmost maximum, extension budget); every other position is a literal.
// Writes step (LDS), m and the tile's mbits words.  Kept out of line: its registers do
// not weigh on the bucket search.
template <bool kDev>
__device__ FCX_SPARSE_CALL void sparse_search(const uint32_t *sdw, uint32_t *region, uint32_t kw0, uint32_t kw1,
                                           uint32_t kw2, uint32_t kw3, uint32_t *s_red,
                                           uint32_t *s_np, uint32_t *s_unknown, uint32_t *s_match, uint32_t *mrow,
                                           uint64_t *mbw, uint32_t q0, uint32_t npos, uint32_t ins_end, uint32_t w0,
                                           uint32_t blen, uint32_t ntile, uint32_t dbg_in) {
    const uint32_t dbg = kDev ? uni(dbg_in) : 0u;
    q0 = uni(q0); npos = uni(npos); ins_end = uni(ins_end); w0 = uni(w0); blen = uni(blen); ntile = uni(ntile);
    const uint32_t tid = FCX_TID;
    const uint32_t kw[4] = {kw0, kw1, kw2, kw3};
    auto hash_of = [&](uint32_t r) -> uint32_t {
        return key_mix(__builtin_amdgcn_alignbyte(kw[(r >> 2) + 1], kw[r >> 2], r & 3) & 0xFFFFFFu);
    };
    const uint32_t *dupm = region + kFilterWords / 2;
    uint16_t *step = (uint16_t *)region;
    {
        uint32_t *P = region + kSpP;
        uint32_t *cnt = region + kSpCnt;
        const uint16_t *c16 = (const uint16_t *)cnt;
        uint16_t *srt = (uint16_t *)(region + kSpSrt);
        uint64_t *mbl = (uint64_t *)(region + kSpMb);
        for (uint32_t x = tid; x < kTile / 2; x += kMT) region[x] = 0x00010001u;   // step = 1 (literal)
        for (uint32_t x = tid; x <= kSparseBuckets / 2; x += kMT) cnt[x] = 0;
        // the 12 dup tests (independent LDS reads), then one slot reservation per wave
        uint32_t fm = 0;   // bit r: key r's hash repeats
#pragma unroll
        for (uint32_t r = 0; r < kIns; r++) {
            const uint32_t hf = hash_of(r) >> (24 - kFilterBits);
            if (kIns * tid + r < ins_end && ((dupm[hf >> 5] >> (hf & 31)) & 1u)) fm |= 1u << r;
        }
        const uint32_t nf = (uint32_t)__builtin_popcount(fm);
        const uint32_t incf = wave_incl_scan(nf);
        uint32_t base = 0;
        if ((tid & 63) == 63 && incf) base = atomicAdd(s_np, incf);
        base = (uint32_t)__builtin_amdgcn_readlane((int)base, 63) + incf - nf;
        for (uint32_t bits = fm; bits; bits &= bits - 1) {
            const uint32_t r = __builtin_ctz(bits);
            const uint32_t x = kIns * tid + r;
            const uint32_t key = lds_key3(sdw, x);
            const uint32_t hf = key_mix(key) >> (24 - kFilterBits);
            P[base++] = x | (hf << 13);
        }
        __syncthreads();
        const uint32_t np = *s_np;
        uint32_t pe[2], prk[2];
#pragma unroll
        for (uint32_t r = 0; r < 2; r++) {
            const uint32_t idx = tid + kMT * r;
            pe[r] = 0xFFFFFFFFu;
            prk[r] = 0;
            if (idx < np) {
                pe[r] = P[idx];
                const uint32_t bk = (pe[r] >> 13) & (kSparseBuckets - 1), sh = 16 * (bk & 1);
                prk[r] = (atomicAdd(&cnt[bk >> 1], 1u << sh) >> sh) & 0xFFFFu;
            }
        }
        __syncthreads();
        {   // exclusive scan of the counters, one dword (two buckets) per lane
            static_assert(kSparseBuckets / 2 == kMT, "one counter dword per lane");
            const uint32_t c = cnt[tid], sum = (c & 0xFFFFu) + (c >> 16);
            const uint32_t inc = wave_incl_scan(sum);
            if ((tid & 63) == 63) s_red[tid >> 6] = inc;
            __syncthreads();
            uint32_t pre = inc - sum;
            for (uint32_t w = 0; w < (tid >> 6); w++) pre += s_red[w];
            cnt[tid] = pre | ((pre + (c & 0xFFFFu)) << 16);
            if (tid == 0) cnt[kSparseBuckets / 2] = np;   // start[kSparseBuckets]
        }
        if (tid < 64) mbl[tid] = 0;   // (the results array is read only where step marks a match)
        __syncthreads();
#pragma unroll
        for (uint32_t r = 0; r < 2; r++)
            if (pe[r] != 0xFFFFFFFFu) srt[c16[(pe[r] >> 13) & (kSparseBuckets - 1)] + prk[r]] = (uint16_t)(pe[r] & 0x1FFFu);
        __syncthreads();
        if (dbg & 32u) return;   // timing: + filter and sparse sort
#pragma unroll
        for (uint32_t r = 0; r < 2; r++) {
            if (pe[r] == 0xFFFFFFFFu) continue;
            const uint32_t x = pe[r] & 0x1FFFu;
            const uint32_t i = w0 + x;
            if (x < q0 || x >= npos || i == 0 || blen - i < 4 || (dbg & 1u)) continue;
            const uint32_t cap = min(kMaxL, blen - i) - 1;
            const uint32_t qa = lds_ld4(sdw, x), qb = lds_ld4(sdw, x + 4), qc = lds_ld4(sdw, x + 8);
            const uint32_t bk = (pe[r] >> 13) & (kSparseBuckets - 1);
            const uint32_t xlo = max(i, kWin) - kWin - w0;
            uint32_t best = 0, next = 0;
            bool unk = false;
            for (uint32_t e = c16[bk], e1 = c16[bk + 1]; e < e1 && !unk; e++) {
                const uint32_t xe = srt[e];
                if (xe < x && xe >= xlo) scan_candidate(sdw, xe, x, qa, qb, qc, cap, best, next, unk, dbg);
            }
            const uint32_t Lb = best >> 13;
            if (unk || Lb >= kMinL) {
                const uint32_t res = unk ? kUnknown : m_pack(Lb, x - (8191u - (best & 0x1FFFu)));
                mrow[x] = res;
                region[kResLds + x - q0] = res;
                step[x - q0] = (uint16_t)(unk ? 0u : Lb + 1);
                atomicOr(&mbl[(x - q0) >> 6], 1ull << ((x - q0) & 63));
                if (unk) *s_unknown = 1;
                else *s_match = 1;
            }
        }
        __syncthreads();
        if (tid < (ntile + 63) / 64) mbw[tid] = mbl[tid];
    }
}

// ---- sparse tiles with a few matches (random data) ----
// Every position is a literal except the handful of match positions the sparse search found,
// so the greedy chain from t0 follows from the ordered match list: a match is taken when the
// chain reaches it (no earlier taken match covers it), everything else is a literal token.
// Wave 0 publishes what the Jacobi parse publishes (chain words, prefix counts, compact match
// list, tile totals).  mbl: the search's per-64-position match words (tile-relative), step:
// L + 1 per position, res: m per position, list: 64 words of scratch.  Returns false (nothing
// written) above 64 match positions; every wave returns the same verdict.
__device__ inline bool sparse_parse(const uint64_t *mbl, const uint16_t *step, const uint32_t *res, uint32_t *list,
                                    uint32_t nt, uint32_t t0, uint64_t *cw, uint64_t *pfx, uint32_t *ti, uint32_t *mt) {
    const uint32_t lane = FCX_TID & 63;
    const uint32_t nwords = (nt + 63) / 64;
    const uint64_t wm = lane < nwords ? mbl[lane] : 0ull;
    const uint32_t cntw = (uint32_t)__popcll(wm);
    const uint32_t inc = wave_incl_scan(cntw);
    const uint32_t nm = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
    if (nm > 64) return false;
    if (FCX_TID >= 64) return true;
    uint32_t k = inc - cntw;
    for (uint64_t bits = wm; bits; bits &= bits - 1, k++) list[k] = 64 * lane + (uint32_t)__builtin_ctzll(bits);
    __builtin_amdgcn_wave_barrier();
    const uint32_t pos = lane < nm ? list[lane] : 0u;
    const uint32_t Lv = lane < nm ? (uint32_t)step[pos] - 1u : 0u;
    // the chain takes a match when it reaches it (uniform walk over the ordered list)
    uint64_t tk = 0;
    uint32_t cur = 0;
    for (uint32_t i = 0; i < nm; i++) {
        const uint32_t p = (uint32_t)__builtin_amdgcn_readlane((int)pos, (int)i);
        if (p >= cur) {
            tk |= 1ull << i;
            cur = p + (uint32_t)__builtin_amdgcn_readlane((int)Lv, (int)i) + 1;
        }
    }
    // lane w: chain word w (literal tokens minus the taken matches' covered positions) and the
    // counts of the chain positions before it
    const uint32_t lo = 64 * lane;
    uint64_t cov = 0;
    uint32_t cov_before = 0, cov_tile = 0, mat_before = 0, gb_before = 0, gb_all = 0;
    for (uint64_t bits = tk; bits; bits &= bits - 1) {
        const uint32_t i = (uint32_t)__builtin_ctzll(bits);
        const uint32_t p = (uint32_t)__builtin_amdgcn_readlane((int)pos, (int)i);
        const uint32_t Lm = (uint32_t)__builtin_amdgcn_readlane((int)Lv, (int)i);
        const uint32_t c0 = p + 1, c1 = p + Lm + 1;   // covered positions [c0, c1)
        const uint32_t a = max(c0, lo), z = min(c1, lo + 64);
        if (a < z) cov |= (z - a == 64 ? ~0ull : ((1ull << (z - a)) - 1ull)) << (a - lo);
        cov_before += c1 <= lo ? c1 - c0 : (c0 < lo ? lo - c0 : 0u);
        cov_tile += min(c1, nt) - c0;
        const uint32_t g = (Lm >> 2) + 3;
        if (p < lo) { mat_before++; gb_before += g; }
        gb_all += g;
    }
    const uint32_t ntk = (uint32_t)__popcll(tk);
    if (lane < nwords) {
        const uint32_t nb = min(64u, nt - lo);
        const uint64_t valid = nb == 64 ? ~0ull : ((1ull << nb) - 1ull);
        cw[lane] = valid & ~cov;
        pfx[lane] = (uint64_t)(lo - cov_before) | ((uint64_t)mat_before << 13) | ((uint64_t)gb_before << 24);
    }
    if (lane < nm && ((tk >> lane) & 1ull)) mt[__popcll(tk & ((1ull << lane) - 1ull))] = res[pos];
    if (lane == 0) {
        ti[0] = 0u;
        ti[1] = t0 + max(cur, nt);
        ti[2] = nt - cov_tile;
        ti[3] = ntk;
        ti[4] = gb_all;
    }
    return true;
}

// ---- uniform tiles (one byte value over the whole image: zeros) ----
// m is m_uniform everywhere: no search, no run table, no m[] rows.  The speculative chain
// from t0 follows directly; this publishes what the parse below publishes for other tiles
// (mbits, chain words, per-word prefix counts, tile info with kTileUniform).
__device__ inline void uniform_tile_out(uint32_t *sc /* >= kMT + 1 words */, uint32_t *s_red, uint64_t *mbw,
                                        uint64_t *cw, uint64_t *pfx, uint32_t *ti, uint32_t t0, uint32_t t1,
                                        uint32_t blen) {
    const uint32_t tid = FCX_TID, lane = tid & 63, wv = tid >> 6;
    auto ustep = [&](uint32_t p) -> uint32_t { return m_len(m_uniform(p, blen)) + 1; };
#if FCX_RUNS
    // (the runs unit's shards are mostly uniform tiles, zeros: the closed forms)  m_uniform is a match
    // except at the block's first position and where fewer than 4 bytes remain: lane w writes mbits
    // word w directly; a step is min(258, blen - p), so a lane's walk to its segment jumps the
    // full-length steps at once
    if (tid < (t1 - t0 + 63) / 64) {
        const uint32_t a = t0 + 64 * tid, lo = blen >= 3 ? blen - 3 : 0u;   // literal from lo on
        uint64_t word = t1 - a < 64 ? (1ull << (t1 - a)) - 1 : ~0ull;
        if (a == 0) word &= ~1ull;
        if (lo < a + 64) word &= lo <= a ? 0ull : (1ull << (lo - a)) - 1;
        mbw[a >> 6] = word;
    }
    const uint32_t s = t0 + tid * kSeg, se = min(s + kSeg, t1);
    uint32_t T = 0, p = t0;
    if (p == 0 && s > 0) p = 1;   // position 0: a literal
    if (p < s && blen - p >= kMaxL) {
        const uint32_t kmax = (blen - p - kMaxL) / kMaxL + 1, ks = (s - p + kMaxL - 1) / kMaxL;
        p += kMaxL * min(kmax, ks);
    }
    while (p < s) p += ustep(p);
#else
#pragma unroll
    for (uint32_t r = 0; r < kQPL; r++) {   // a wave's 64 lanes: 64 consecutive positions
        const uint32_t i = t0 + tid + kMT * r;
        const uint64_t mb = __ballot(i < t1 && m_uniform(i, blen) != 0);
        if (lane == 0 && i < t1) mbw[i >> 6] = mb;
    }
    const uint32_t s = t0 + tid * kSeg, se = min(s + kSeg, t1);
    uint32_t T = 0, p = t0;
    while (p < s) p += ustep(p);
#endif
    uint32_t cnt[3] = {0, 0, 0};
    while (p < se) {
        T |= 1u << (p - s);
        const uint32_t Lm = ustep(p) - 1;
        cnt[0]++;
        if (Lm) { cnt[1]++; cnt[2] += (Lm >> 2) + 3; }
        p += Lm + 1;
    }
    if (s < t1 && se == t1) sc[kMT] = p;   // the tile's exit
    uint32_t inc[3];
#pragma unroll
    for (int q = 0; q < 3; q++) inc[q] = wave_incl_scan(cnt[q]);
    if (lane == 63)
        for (int q = 0; q < 3; q++) s_red[q * kWaves + wv] = inc[q];
    sc[tid] = T;
    __syncthreads();
    uint32_t pre[3], tot[3];
#pragma unroll
    for (int q = 0; q < 3; q++) {
        uint32_t a = 0, b = 0;
        for (uint32_t w = 0; w < kWaves; w++) {
            const uint32_t v = s_red[q * kWaves + w];
            if (w < wv) a += v;
            b += v;
        }
        pre[q] = a + inc[q] - cnt[q];
        tot[q] = b;
    }
    constexpr uint32_t kLanesPerWord = 64 / kSeg;
    const uint32_t nwords = (t1 - t0 + 63) / 64;
    if ((tid % kLanesPerWord) == 0 && tid / kLanesPerWord < nwords) {
        const uint32_t w = tid / kLanesPerWord;
        uint64_t word = 0;
#pragma unroll
        for (uint32_t q = 0; q < kLanesPerWord; q++) word |= (uint64_t)sc[tid + q] << (kSeg * q);
        cw[w] = word;
        pfx[w] = (uint64_t)pre[0] | ((uint64_t)pre[1] << 13) | ((uint64_t)pre[2] << 24);
    }
    if (tid == 0) {
        ti[0] = kTileUniform | kTileMFull;
        ti[1] = sc[kMT];
        ti[2] = tot[0];
        ti[3] = tot[1];
        ti[4] = tot[2];
    }
}

// Workgroups are dealt round-robin over the 8 XCDs (workgroups w and w + 8 share one L2).  Each
// XCD takes a contiguous run of tiles instead, so the neighbouring tiles that re-read a tile's
// bytes as their 2 KiB left halo run on the same XCD at about the same time and find them in
// its L2 (a bijection of [0, n); any placement stays correct, only the re-reads move).
__device__ inline uint32_t xcd_tile(uint32_t w, uint32_t n) {
    const uint32_t x = w & 7u, j = w >> 3, q = n >> 3, r = n & 7u;
    return x * q + min(x, r) + j;
}

// One tile bx of the shard, by the whole workgroup (every return is workgroup-uniform).
// kDev = false is the product kernel: every development / test-mode bit is compiled out.
// k_match<true> carries them (phase exits for tools/matchphase.py through fcx_debug_match, and
// the forced tile modes of fcx_ctx_set_match_mode, which the parity tests use).  kRt = false: the
// unrouted code, the route's lines never emitted (a constant empty route folds them only after
// optimisations that already moved the kernel's code generation -- 2 % on random data).
template <bool kDev, bool kRt>
__device__ __forceinline__ void match_tile(const uint8_t *__restrict__ in, const Layout L, uint32_t *__restrict__ m,
                                           uint64_t *__restrict__ mbits, uint64_t *__restrict__ chain,
                                           uint64_t *__restrict__ chain_pfx, uint32_t *__restrict__ tinfo,
                                           uint32_t *__restrict__ mtok, uint32_t dbg_in, const uint32_t bx,
                                           const MatchRoute &rt) {
    const uint32_t dbg = kDev ? dbg_in : (uint32_t)FCX_MATCH_EXIT;   // (FCX_MATCH_EXIT: phase-timing builds only)
    __shared__ __attribute__((aligned(16))) uint32_t sdw[kTileBytes / 4 + 4];   // byte image of the window
    // one region, two lives: [bucket counters/starts (u16 x 4104) | entries (u16 x 6144)] during the
    // search, [step (u16 x 4096) | parse scratch] after it
    __shared__ __attribute__((aligned(16))) uint32_t region[kRegionWords];
#if !FCX_NOBUCKET
    uint32_t *hw = region;                                  // packed u16 bucket counters, then starts
    uint16_t *h16 = (uint16_t *)region;
    uint16_t *ent = (uint16_t *)(region + kHeadWords);     // window entries, bucket-sorted
#endif
    __shared__ uint32_t s_unknown;
    __shared__ uint32_t s_match;    // some position of the tile has a match (else the chain is every position)
#if !FCX_SPARSE && !FCX_NOFILTER
    __shared__ uint32_t s_nruns;    // image runs counted in the first 2 KiB (pass 1)
    __shared__ uint32_t s_nruns2;   // ... and in the rest (pass 2, only when pass 1 allows run mode)
#endif
#if FCX_SAMPLE
    __shared__ uint32_t s_smp[kSampleWords];   // repeat sample bitmap
    __shared__ uint32_t s_sample;   // repeat sample: sampled keys whose hash was seen before
#endif
    __shared__ uint32_t s_events;   // repeat filter: window keys whose hash was seen before
    __shared__ uint32_t s_np;       // sparse search: positions whose hash repeats
    __shared__ uint32_t s_chg[2];
    __shared__ uint32_t s_red[4 * kWaves];   // cross-wave scan partials (rmode_walk: exits + 3 scans)

    const uint32_t tid = FCX_TID;
    const uint32_t b = bx / L.tpb, k = bx % L.tpb;
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
    static_assert((kTileBytes / 4 + 4) % 4 == 0 && (kTileBytes / 4 + 4) / 4 <= kMT, "one 16-B load per lane");
    if ((((uintptr_t)src) & 15) == 0) {
        // one 16-B load per lane, all in flight at once
        if (tid < (kTileBytes / 4 + 4) / 4) {
            uint4 v = make_uint4(0u, 0u, 0u, 0u);
            if (16 * tid + 16 <= nload) v = ((const uint4 *)src)[tid];
            else if (16 * tid < nload) {
                uint32_t w[4];
#pragma unroll
                for (uint32_t q = 0; q < 4; q++) {
                    w[q] = 0;
#pragma unroll
                    for (uint32_t j = 0; j < 4; j++)
                        if (16 * tid + 4 * q + j < nload) w[q] |= (uint32_t)src[16 * tid + 4 * q + j] << (8 * j);
                }
                v = make_uint4(w[0], w[1], w[2], w[3]);
            }
            ((uint4 *)sdw)[tid] = v;
        }
    } else {
        for (uint32_t x = tid; x < kTileBytes / 4 + 4; x += kMT) {
            uint32_t v = 0;
            for (uint32_t q = 0; q < 4; q++)
                if (4 * x + q < nload) v |= (uint32_t)src[4 * x + q] << (8 * q);
            sdw[x] = v;
        }
    }
    if (tid == 0) {
#if FCX_SPARSE || FCX_NOFILTER
        s_unknown = 0; s_match = 0; s_chg[0] = 0; s_chg[1] = 0;
#elif !FCX_SAMPLE
        s_unknown = 0; s_match = 0; s_nruns = 0; s_nruns2 = 0; s_chg[0] = 0; s_chg[1] = 0;
#else
        s_unknown = 0; s_match = 0; s_nruns = 0; s_nruns2 = 0; s_sample = 0; s_chg[0] = 0; s_chg[1] = 0;
#endif
        s_events = 0; s_np = 0;
    }
#if FCX_SAMPLE
    if (tid < kSampleWords) s_smp[tid] = 0;
#endif
#if !FCX_NOFILTER
    {   // the repeat filter's bitmaps are zeroed here, under the staging loads' latency
        uint4 *r4 = (uint4 *)region;
        for (uint32_t x = tid; x < kFilterWords / 4; x += kMT) r4[x] = make_uint4(0u, 0u, 0u, 0u);
    }
#endif
    // a direct routed launch (every tile in the grid): another unit's tile ends here, its kind read
    // while the staging loads were in flight; nothing but this workgroup's LDS was written
    if (kRt && !rt.list && rt.kind && rt.kind[bx] != rt.mine) return;
    __syncthreads();
    const uint32_t npos = t1 - w0;
    const uint32_t q0 = t0 - w0;
    uint16_t *step = (uint16_t *)region;               // after the search: L + 1 per position, 0 = unknown

    // ---- 1b. run count of the image: a tile of long runs (zeros, runs) skips the
    // bucket search and takes every match from the run table (dense_phase) ----
#if FCX_SPARSE || FCX_NOFILTER
    // (no run count: run mode is the sparse unit's path for non-sparse tiles; the no-filter unit
    // takes the bucket search for every tile, exact for any tile through the run table / stitch)
    const uint32_t nruns_img = kRunTile + 1;
#else
    {
        // per dword: bytes differing from their predecessor (byte 0 of the image counts
        // once).  The first 2 KiB decide most tiles: more than kRunTile runs there
        // already rules the run mode out (random data, text), so the rest is skipped.
        auto runs_in = [&](uint32_t w) -> uint32_t {
            if (4 * w >= nload) return 0u;
            const uint32_t v = sdw[w], pv = w ? sdw[w - 1] : v << 24;
            uint32_t x = v ^ ((v << 8) | (pv >> 24));
            x |= x >> 4; x |= x >> 2; x |= x >> 1;
            uint32_t msk = x & 0x01010101u;
            const uint32_t nb = nload - 4 * w;
            if (nb < 4) msk &= (1u << (8 * nb)) - 1u;
            return (uint32_t)__builtin_popcount(msk);
        };
        uint32_t cnt = (tid == 0 && nload > 0 ? 1u : 0u) + runs_in(tid);
        cnt = wave_sum_u32(cnt);
        if ((tid & 63) == 0) atomicAdd(&s_nruns, cnt);
#if FCX_SAMPLE
        {   // repeat sample: the key of every 12th window position into a 2^12-bit bitmap;
            // random data repeats ~32 times in 512 samples, text far more often
            const uint32_t x = kIns * tid;
            bool rep = false;
            if (x + 3 <= nload) {
                const uint32_t hs = key_mix(lds_key3(sdw, x)) >> 12;
                const uint32_t bit = 1u << (hs & 31);
                rep = (atomicOr(&s_smp[hs >> 5], bit) & bit) != 0;
            }
            const uint64_t bal = __ballot(rep);
            if ((tid & 63) == 0 && bal) atomicAdd(&s_sample, (uint32_t)__popcll(bal));
        }
#endif
        __syncthreads();
        if (s_nruns <= kRunTile) {   // (s_nruns is final here: the decision is uniform)
            cnt = 0;
            for (uint32_t w = tid + kMT; 4 * w < nload; w += kMT) cnt += runs_in(w);
            cnt = wave_sum_u32(cnt);
            if ((tid & 63) == 0 && cnt) atomicAdd(&s_nruns2, cnt);
            __syncthreads();
        }
    }
    const uint32_t nruns_img = s_nruns + s_nruns2;   // s_nruns2 = 0 unless pass 2 ran (then after its barrier)
#endif
#if FCX_NOBUCKET
    bool rmode = (nruns_img <= kRunTile && !(dbg & 4u)) || (dbg & 8u);   // (set below for non-sparse tiles)
#else
    const bool rmode = (nruns_img <= kRunTile && !(dbg & 4u)) || (dbg & 8u);
#endif
    if (dbg & 16u) return;   // timing: staging + run count only

    // this lane's 12 consecutive window positions 12 tid .. 12 tid + 11 take their keys from
    // bytes [12 tid, 12 tid + 16) of the image, held in registers (stride-3 dword reads:
    // conflict-free)
    const uint32_t ins_end = min(npos, blen >= 3 ? blen - 2 - w0 : 0);  // j + 3 <= blen
    uint32_t kw[4];
#pragma unroll
    for (uint32_t q = 0; q < 4; q++) kw[q] = sdw[kIns / 4 * tid + q];
    auto hash_of = [&](uint32_t r) -> uint32_t {   // r: compile-time after unrolling
        return key_mix(__builtin_amdgcn_alignbyte(kw[(r >> 2) + 1], kw[r >> 2], r & 3) & 0xFFFFFFu);
    };

    bool sparse = false;   // the sparse search ran (few repeated keys: random data)
    if (rmode) {
        if (nruns_img == 1 && !(dbg & 12u)) {   // one byte value over the whole image (zeros)
            uniform_tile_out(region, s_red, mbits + (uint64_t)b * L.wpb,
                             chain + (uint64_t)b * L.wpb + (uint64_t)k * (kTile / 64),
                             chain_pfx + (uint64_t)bx * (kTile / 64), tinfo + 8ull * bx, t0, t1, blen);
            return;
        }
        for (uint32_t x = tid; x < kTile; x += kMT) step[x] = 0;
        if (tid == 0) s_unknown = 1;
        __syncthreads();
    } else {
    // ---- 2a. repeat filter (tiles whose sample repeats little): every window key's
    // 17-bit hash goes into "seen"; a hash seen before goes into "dup" and counts as a
    // repeat.  Random data has a few hundred repeats per tile (almost all hash
    // collisions), so the search below visits only the positions whose hash repeats
    // (sparse search); above kSparseEvents repeats the tile takes the bucket search. ----
#if FCX_NOFILTER
    if (false) {
#elif !FCX_SAMPLE
    if (!(dbg & 128u)) {
#else
    if (s_sample <= kSampleEvents && !(dbg & 128u)) {
#endif
    uint32_t *seen = region, *dupm = region + kFilterWords / 2;   // (zeroed with the staging)
    {
        // all 12 "seen" atomics in flight at once (program order keeps a lane's own
        // repeats visible to it), then the "dup" marks without return values
        uint32_t old[kIns];
#pragma unroll
        for (uint32_t r = 0; r < kIns; r++) {
            old[r] = 0;
            if (kIns * tid + r < ins_end) {
                const uint32_t hf = hash_of(r) >> (24 - kFilterBits);
                old[r] = atomicOr(&seen[hf >> 5], 1u << (hf & 31));
            }
        }
        uint32_t ev = 0;
#pragma unroll
        for (uint32_t r = 0; r < kIns; r++) {
            const uint32_t hf = hash_of(r) >> (24 - kFilterBits);
            const uint32_t bit = 1u << (hf & 31);
            if (kIns * tid + r < ins_end && (old[r] & bit)) {
                atomicOr(&dupm[hf >> 5], bit);
                ev++;
            }
        }
        ev = wave_sum_u32(ev);
        if ((tid & 63) == 0 && ev) atomicAdd(&s_events, ev);
    }
    __syncthreads();
    if (dbg & 4096u) return;   // timing: + repeat filter
    sparse = s_events <= kSparseEvents;
    }   // repeat filter

    if (sparse) {
        sparse_search<kDev>(sdw, region, kw[0], kw[1], kw[2], kw[3], s_red, &s_np, &s_unknown, &s_match, m + bstart + w0,
                      mbits + (uint64_t)b * L.wpb + (t0 >> 6), q0, npos, ins_end, w0, blen, t1 - t0, dbg);
        __syncthreads();
        if (dbg & 32u) return;
#if FCX_NOBUCKET
    } else if (kRt && rt.defer_list) {
        // not sparse, in a routed call: the tile goes on to the no-filter unit's list (launched after
        // this one), which searches it by buckets.  Nothing of it has been written yet.  (The run
        // table below overflows on match-dense tiles and leaves them to the stitch's serial walk.)
        // Not in the direct kernel (k_match<kDev, false> passes a null list: the branch is compiled
        // out there, where it cost the sparse unit ~4 % on random data): a misfiled tile in the unit
        // that has most of the call's tiles takes the run table below.
        if (tid == 0) {
            rt.defer_list[atomicAdd(rt.defer_cnt, 1u)] = bx;
            rt.kind[bx] = (uint8_t)kRouteNoFilter;   // (a direct no-filter launch finds it by its kind)
        }
        return;
    } else {   // not sparse: the whole-tile run-table mode, as for run-mode tiles
        rmode = true;
        for (uint32_t x = tid; x < kTile; x += kMT) step[x] = 0;
        if (tid == 0) s_unknown = 1;
        __syncthreads();
    }
#else
    } else {
    for (uint32_t x = tid; x < kHeadWords; x += kMT) hw[x] = 0;
    __syncthreads();

    // ---- 2. counting sort of the window positions by bucket ----
    // 16-bit counters, two per dword (a bucket never exceeds 6144 entries).  Pass p inserts
    // the slab [512 p, 512 p + 512) of window positions (x = tid + kMT p), one barrier per
    // pass, so a bucket lists its entries slab by slab in position order.  A query at x
    // (slab s = x / 512) needs only the entries in [x - 2047, x): slabs s - 4 .. s.  Its
    // bucket counter read during pass s - 5 (before that pass's barrier: every slab <= s - 6
    // is in, slab s - 5 partly) bounds from below the entries left of slab s - 4 (all out of
    // the window); read during pass s + 1 (after the barrier of pass s) it bounds from above
    // the entries of slabs <= s (every later entry lies right of x).  The query scans only
    // between the two snapshots: about half of its bucket.
    uint32_t ins_hr[kIns];                                             // bucket << 16 | tag << 13 | rank
    // query r: lo rank | hi rank << 16 (hi 0xFFFF = bucket end)
    uint32_t snap[kQPL];
    const uint32_t qsl = q0 >> 9;   // slab of query r = r + qsl (q0 = 0 or 2048)
#pragma unroll
    for (uint32_t r = 0; r < kQPL; r++) snap[r] = 0xFFFF0000u;
    auto qbucket = [&](uint32_t r) -> uint32_t {   // bucket of query r (its insertion record)
        return (qsl ? ins_hr[r + 4] : ins_hr[r]) >> 16;
    };
    auto counter = [&](uint32_t bk) -> uint32_t { return (hw[bk >> 1] >> (16 * (bk & 1))) & 0xFFFFu; };
#pragma unroll
    for (uint32_t p = 0; p < kIns; p++) {
        ins_hr[p] = 0xFFFFFFFFu;
#if FCX_KEY4
        if (tid + kMT * p < min(npos, blen >= 4 ? blen - 3 - w0 : 0)) {   // j + 4 <= blen
            const uint32_t h = key_mix4(lds_ld4(sdw, tid + kMT * p));
#else
        if (tid + kMT * p < ins_end) {
            const uint32_t h = key_mix(lds_key3(sdw, tid + kMT * p));
#endif
            const uint32_t bk = h >> (24 - kHashBits), sh = 16 * (bk & 1);
            const uint32_t old = atomicAdd(&hw[bk >> 1], 1u << sh);
            ins_hr[p] = (bk << 16) | ((h & 7u) << 13) | ((old >> sh) & 0x1FFFu);   // rank < 6144
        }
        // snapshots taken in pass p: lo of the query whose slab is p + 5, hi of the query
        // whose slab is p - 1 (queries of slabs qsl .. qsl + 7; unsearched queries have no
        // insertion record and keep the whole bucket, unused)
#pragma unroll
        for (uint32_t r = 0; r < kQPL; r++) {
            // lo: the query is not inserted yet; its bucket comes from its key
            if ((qsl == 4 && p + 1 == r) || (qsl == 0 && p + 5 == r)) {
#if FCX_KEY4
                const uint32_t bk = key_mix4(lds_ld4(sdw, q0 + tid + kMT * r)) >> (24 - kHashBits);
#else
                const uint32_t bk = key_mix(lds_key3(sdw, q0 + tid + kMT * r)) >> (24 - kHashBits);
#endif
                snap[r] = (snap[r] & 0xFFFF0000u) | counter(bk);
            }
            if ((qsl == 4 && p == r + 5) || (qsl == 0 && p == r + 1)) {
                const uint32_t bk = qbucket(r);
                if (bk != 0xFFFFu) snap[r] = (snap[r] & 0xFFFFu) | (counter(bk) << 16);
            }
        }
        __syncthreads();
    }
    {   // exclusive scan of the bucket counts: kBkDw consecutive counter dwords per lane
        constexpr uint32_t kBkDw = (1u << kHashBits) / 2 / kMT;
        uint32_t cw4[kBkDw], sum = 0;
#pragma unroll
        for (uint32_t q = 0; q < kBkDw; q++) { cw4[q] = hw[tid * kBkDw + q]; sum += (cw4[q] & 0xFFFFu) + (cw4[q] >> 16); }
        const uint32_t inc = wave_incl_scan(sum);
        const uint32_t lane = tid & 63, wv = tid >> 6;
        if (lane == 63) s_red[wv] = inc;
        __syncthreads();
        uint32_t run = inc - sum;
        for (uint32_t w = 0; w < wv; w++) run += s_red[w];
#pragma unroll
        for (uint32_t q = 0; q < kBkDw; q++) {
            const uint32_t lo = run, hi = run + (cw4[q] & 0xFFFFu);
            run = hi + (cw4[q] >> 16);
            hw[tid * kBkDw + q] = lo | (hi << 16);
        }
        if (tid == kMT - 1) hw[(1u << kHashBits) / 2] = run;   // start[nbuckets] = total
    }
    __syncthreads();
    // scatter into bucket order: entry = position | 3 more hash bits << 13
#pragma unroll
    for (uint32_t r = 0; r < kIns; r++)
        if (ins_hr[r] != 0xFFFFFFFFu) {
            const uint32_t bk = ins_hr[r] >> 16;
            ent[h16[bk] + (ins_hr[r] & 0x1FFFu)] = (uint16_t)((ins_hr[r] & 0xE000u) | (tid + kMT * r));
        }
    __syncthreads();

    if (dbg & 32u) return;   // timing: + counting sort
    // ---- 3. queries: position i = w0 + q0 + tid + kMT*r, kIlp at a time ----
    // Pass A: every lane walks its kIlp queries' bucket ranges together (independent LDS
    // loads), but only for their first K entries.  K is the smallest count that leaves at most
    // kHotCap queries of the wave with entries beyond it, so a few hot keys (text: " th",
    // "the") no longer hold all 64 lanes for their whole range.  Pass B deals the hot queries'
    // remaining (query, entry) pairs over the wave, 64 at a time, one per lane: a pair finds
    // its query through owner marks (the hot slot whose segment starts in the chunk marks it; a
    // running maximum carries the marks along), and its candidate length goes into the slot by
    // an LDS atomic maximum of L << 13 | (8191 - position) (longest, then leftmost; the slot
    // starts at the query's pass-A best, and a partial best prunes extensions as in pass A).
    // per walk: range (start | len << 16), packed best = L << 13 | (8191 - position),
    // query bytes 0..11, x | cap << 13 | tag3 << 22
    uint32_t rs[kQPL];   // result of query r: m (0 = literal, kUnknown)
    const uint32_t lane = tid & 63, wv = tid >> 6;
    uint32_t *h_x = region + kScanHot + kHotWords * wv;   // hot slot: x | first entry << 13 | ext << 26
    uint32_t *h_base = h_x + kHotCap;                      // first pair index of the slot
    uint32_t *h_best = h_base + kHotCap;                   // packed best (bit 31: unknown)
    uint8_t *h_mk = (uint8_t *)(h_best + kHotCap);         // owner marks of a 64-pair chunk
#pragma unroll
    for (uint32_t g = 0; g < kQPL; g += kIlp) {
        uint32_t rng[kIlp], best[kIlp], xpk[kIlp], qa[kIlp], qb[kIlp], qc[kIlp];   // rng ~0 = unknown
        uint32_t nmax = 0;
#pragma unroll
        for (uint32_t u = 0; u < kIlp; u++) {
            const uint32_t x = q0 + tid + kMT * (g + u);
            rng[u] = 0; best[u] = 0; xpk[u] = x; qa[u] = qb[u] = qc[u] = 0;
            if (x < npos) {
                const uint32_t i = w0 + x;
                if (i != 0 && blen - i >= 4 && !(dbg & 1u)) {
                    const uint32_t cap = min(kMaxL, blen - i) - 1;
                    qa[u] = lds_ld4(sdw, x);
                    qb[u] = lds_ld4(sdw, x + 4);
                    qc[u] = lds_ld4(sdw, x + 8);
#if FCX_KEY4
                    const uint32_t h = key_mix4(qa[u]);
#else
                    const uint32_t h = key_mix(qa[u] & 0xFFFFFFu);
#endif
                    const uint32_t bk = h >> (24 - kHashBits);
                    const uint32_t sn = snap[g + u];
                    const uint32_t b0 = h16[bk], b1 = h16[bk + 1];
                    const uint32_t lo = b0 + (sn & 0xFFFFu);
                    const uint32_t n = ((sn >> 16) == 0xFFFFu ? b1 : min(b1, b0 + (sn >> 16))) - lo;
                    xpk[u] = x | (cap << 13) | ((h & 7u) << 22);   // bits 25..31: extension count
                    if (dbg & (1u << 22)) rng[u] = lo;   // (timing: setup only, no candidates)
                    else if (n > kMaxChainSteps) rng[u] = 0xFFFFFFFFu;
                    else { rng[u] = lo | (n << 16); nmax = max(nmax, n); }
                }
            }
        }
        // K: binary search for the smallest count with at most kHotCap longer ranges
        auto nrange = [&](uint32_t u) -> uint32_t { return rng[u] == 0xFFFFFFFFu ? 0u : rng[u] >> 16; };
        uint32_t klo = 0, khi = wave_max_dpp(nmax);
#if FCX_SHORTK
        // a wave whose longest range is short takes every range whole in pass A: no K search, no
        // pass B (its ballots, scans, slots and read-back cost more than the few extra pass-A steps)
        const uint32_t wmax = khi;
        if (wmax <= FCX_SHORTK) klo = khi;
#endif
        while (klo < khi) {
            const uint32_t mid = (klo + khi) >> 1;
            uint32_t c = 0;
#pragma unroll
            for (uint32_t u = 0; u < kIlp; u++) c += (uint32_t)__popcll(__ballot(nrange(u) > mid));
            if (c <= kHotCap) khi = mid; else klo = mid + 1;
        }
        const uint32_t K = (dbg & (1u << 20)) ? wave_max_dpp(nmax) : (dbg & (1u << 21)) ? 0u : klo;   // (A/B: all pass A / all pass B)
        for (uint32_t j = 0; j < K; j++) {
#pragma unroll
            for (uint32_t u = 0; u < kIlp; u++) {
                if (j >= (rng[u] >> 16) || rng[u] == 0xFFFFFFFFu) continue;
                const uint32_t nd = ent[(rng[u] & 0xFFFFu) + j];
                const uint32_t xe = nd & 0x1FFFu;
                const uint32_t x = xpk[u] & 0x1FFFu;
                const uint32_t xlo = max(w0 + x, kWin) - kWin - w0;
                if (((nd >> 13) & 7u) != ((xpk[u] >> 22) & 7u) || xe >= x || xe < xlo) continue;
                const uint32_t cap = (xpk[u] >> 13) & 0x1FFu;
                // bytes 0..11 of the candidate, from four aligned dwords
                const uint32_t wb = xe >> 2, sb = xe & 3;
                const uint32_t w_0 = sdw[wb], w_1 = sdw[wb + 1], w_2 = sdw[wb + 2], w_3 = sdw[wb + 3];
                const uint32_t d0 = __builtin_amdgcn_alignbyte(w_1, w_0, sb) ^ qa[u];
#if FCX_KEY4
                if (d0) continue;   // 3-tag-bit collision: different key
#else
                if (d0 & 0xFFFFFFu) continue;   // 3-tag-bit collision: different key
#endif
                uint32_t Lc;
                if (d0) Lc = 3;
                else {
                    const uint32_t d1 = __builtin_amdgcn_alignbyte(w_2, w_1, sb) ^ qb[u];
                    if (d1) Lc = 4 + (__builtin_ctz(d1) >> 3);
                    else {
                        const uint32_t d2 = __builtin_amdgcn_alignbyte(w_3, w_2, sb) ^ qc[u];
                        if (d2) Lc = 8 + (__builtin_ctz(d2) >> 3);
                        else {
                            // >= 12 bytes.  A candidate right of the best (>= 12) wins only if
                            // longer: not past the cap, not if its byte at the best length differs
                            const uint32_t bL = best[u] >> 13, bxe = 8191u - (best[u] & 0x1FFFu);
                            if (cap <= 12 || (dbg & 2u) ||
                                (bL >= 12 && xe > bxe && (bL >= cap || lds_ld1(sdw, xe + bL) != lds_ld1(sdw, x + bL))))
                                Lc = 12;
                            else {
                                // extension budget per query (periodic data: every same-phase
                                // candidate runs to the cap); past it the position is left to
                                // the exact lazy evaluation
                                xpk[u] += 1u << 25;
                                if ((xpk[u] >> 25) > kExtBudget) { rng[u] = 0xFFFFFFFFu; continue; }
                                Lc = lds_match_len(sdw, xe, x, 12, cap);
                            }
                        }
                    }
                }
                Lc = min(Lc, cap);
                best[u] = max(best[u], (Lc << 13) | (8191u - xe));
            }
        }
        // pass B: the hot queries' entries from K on, flattened over the wave
#if FCX_SHORTK
        if (K < wmax) {
#endif
        bool hot[kIlp];
        uint32_t slot[kIlp], hbase[kIlp], T = 0, nh = 0;
#pragma unroll
        for (uint32_t u = 0; u < kIlp; u++) {
            hot[u] = rng[u] != 0xFFFFFFFFu && (rng[u] >> 16) > K;
            const uint64_t bal = __ballot(hot[u]);
            slot[u] = nh + lanes_below(bal);
            nh += (uint32_t)__popcll(bal);
            const uint32_t m = hot[u] ? (rng[u] >> 16) - K : 0u;
            const uint32_t inc = wave_incl_scan(m);
            hbase[u] = T + inc - m;
            T += (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
            if (hot[u]) {
                h_x[slot[u]] = (xpk[u] & 0x1FFFu) | (((rng[u] & 0xFFFFu) + K) << 13);
                h_base[slot[u]] = hbase[u];
                h_best[slot[u]] = best[u];
            }
        }
        __builtin_amdgcn_wave_barrier();
        for (uint32_t c0 = 0; c0 < T; c0 += 64) {
            if (lane < 16) ((uint32_t *)h_mk)[lane] = 0u;
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (uint32_t u = 0; u < kIlp; u++)
                if (hot[u] && hbase[u] < c0 + 64 && hbase[u] + (rng[u] >> 16) - K > c0)
                    h_mk[hbase[u] > c0 ? hbase[u] - c0 : 0] = (uint8_t)(slot[u] + 1);
            __builtin_amdgcn_wave_barrier();
            const uint32_t hs = wave_incl_max_dpp(h_mk[lane]) - 1u;
            const uint32_t k = c0 + lane;
            if (k >= T) continue;
            const uint32_t hx = h_x[hs];
            const uint32_t x = hx & 0x1FFFu;
            const uint32_t nd = ent[((hx >> 13) & 0x1FFFu) + k - h_base[hs]];
            const uint32_t xe = nd & 0x1FFFu;
            const uint32_t xlo = max(w0 + x, kWin) - kWin - w0;
            if (xe >= x || xe < xlo) continue;
            const uint32_t wq = x >> 2, sq = x & 3;
            const uint32_t q_0 = sdw[wq], q_1 = sdw[wq + 1];
            const uint32_t qa1 = __builtin_amdgcn_alignbyte(q_1, q_0, sq);
#if FCX_KEY4
            if (((nd >> 13) & 7u) != (key_mix4(qa1) & 7u)) continue;
#else
            if (((nd >> 13) & 7u) != (key_mix(qa1 & 0xFFFFFFu) & 7u)) continue;
#endif
            const uint32_t wb = xe >> 2, sb = xe & 3;
            const uint32_t w_0 = sdw[wb], w_1 = sdw[wb + 1];
            const uint32_t d0 = __builtin_amdgcn_alignbyte(w_1, w_0, sb) ^ qa1;
#if FCX_KEY4
            if (d0) continue;
#else
            if (d0 & 0xFFFFFFu) continue;
#endif
            const uint32_t cap = min(kMaxL, blen - (w0 + x)) - 1;
            uint32_t Lc;
            if (d0) Lc = 3;
            else {
                const uint32_t q_2 = sdw[wq + 2], w_2 = sdw[wb + 2];
                const uint32_t d1 = __builtin_amdgcn_alignbyte(w_2, w_1, sb) ^ __builtin_amdgcn_alignbyte(q_2, q_1, sq);
                if (d1) Lc = 4 + (__builtin_ctz(d1) >> 3);
                else {
                    const uint32_t q_3 = sdw[wq + 3], w_3 = sdw[wb + 3];
                    const uint32_t d2 = __builtin_amdgcn_alignbyte(w_3, w_2, sb) ^ __builtin_amdgcn_alignbyte(q_3, q_2, sq);
                    if (d2) Lc = 8 + (__builtin_ctz(d2) >> 3);
                    else {
                        // >= 12 bytes, against the slot's partial best (it only grows)
                        const uint32_t cur = h_best[hs];
                        if (cur >> 31) continue;   // already unknown
                        const uint32_t bL = cur >> 13, bxe = 8191u - (cur & 0x1FFFu);
                        if (cap <= 12 || (dbg & 2u) ||
                            (bL >= 12 && xe > bxe && (bL >= cap || lds_ld1(sdw, xe + bL) != lds_ld1(sdw, x + bL))))
                            Lc = 12;
                        else {
                            const uint32_t old = atomicAdd(&h_x[hs], 1u << 26);
                            if ((old >> 26) >= kExtBudget) { atomicOr(&h_best[hs], 0x80000000u); continue; }
                            Lc = lds_match_len(sdw, xe, x, 12, cap);
                        }
                    }
                }
            }
            atomicMax(&h_best[hs], (min(Lc, cap) << 13) | (8191u - xe));
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (uint32_t u = 0; u < kIlp; u++)
            if (hot[u]) {
                const uint32_t b = h_best[slot[u]];
                if (b >> 31) rng[u] = 0xFFFFFFFFu;
                else best[u] = b;
            }
#if FCX_SHORTK
        }
#endif
#pragma unroll
        for (uint32_t u = 0; u < kIlp; u++) {
            const uint32_t x = xpk[u] & 0x1FFFu;
            uint32_t res = 0;
            if (x < npos) {
                const uint32_t Lb = best[u] >> 13, xb = 8191u - (best[u] & 0x1FFFu);
                if (rng[u] == 0xFFFFFFFFu) { res = kUnknown; s_unknown = 1; }
#if FCX_KEY4
                else if (Lb >= kMinL + 1) { res = m_pack(Lb, x - xb); s_match = 1; }
                else if (((xpk[u] >> 13) & 0x1FFu) >= kMinL) res = kNeed3;   // (cap >= 3: a 3-byte match may exist)
#else
                else if (Lb >= kMinL) { res = m_pack(Lb, x - xb); s_match = 1; }
#endif
            }
            rs[g + u] = res;
        }
    }
#if FCX_KEY4
    // queries without a 4-byte candidate: their longest match is < 4, so it is the leftmost 3-byte
    // match in the window (the reference's leftmost-longest, capped at 3), found by a wave scan
#pragma unroll
    for (uint32_t r = 0; r < kQPL; r++) {
        for (uint64_t nb = __ballot(rs[r] == kNeed3); nb; nb &= nb - 1) {
            const uint32_t l = (uint32_t)__builtin_ctzll(nb);
            const uint32_t x = q0 + 64 * wv + l + kMT * r;   // (lane l's query r)
            const uint32_t key = lds_key3(sdw, x);
            const uint32_t xlo = max(w0 + x, kWin) - kWin - w0;
            uint32_t res = 0;
            for (uint32_t j0 = xlo; j0 < x; j0 += 64) {
                const uint32_t j = j0 + lane;
                const uint64_t hit = __ballot(j < x && lds_key3(sdw, j) == key);
                if (hit) { res = m_pack(kMinL, x - (j0 + (uint32_t)__builtin_ctzll(hit))); break; }
            }
            if (lane == l) rs[r] = res;
            if (res && lane == 0) s_match = 1;
        }
    }
#endif
    __syncthreads();   // the search region is dead from here on; s_unknown is final
    {
        uint32_t *res_lds = region + kResLds;
        const bool mfull = s_unknown != 0;
#pragma unroll
        for (uint32_t r = 0; r < kQPL; r++) {
            const uint32_t rel = tid + kMT * r, x = q0 + rel;
            const uint32_t res = rs[r];
            step[rel] = (uint16_t)(res == kUnknown ? 0u : m_len(res) + 1);
            res_lds[rel] = res;
            // the wave's 64 lanes hold 64 consecutive positions = one mbits word.  m rows
            // (256 B, zeros included) go to HBM only where k_resolve / the stitch read them
            // (the first kResolveSpan positions) or the tile needs the run table (all);
            // every other match reaches k_emit through the tile's compact match list
            const uint64_t mb = __ballot(res != 0);
            if (mb && x < npos && (mfull || rel < kResolveSpan)) m[bstart + w0 + x] = res;
            if ((tid & 63) == 0 && x < npos) mbits[(uint64_t)b * L.wpb + ((t0 + rel) >> 6)] = mb;
        }
    }
    __syncthreads();
    }   // bucket search
#endif
    }   // filter: sparse or bucket search

    // ---- 3b. dense windows: exact matches of the unknown positions over the run table ----
    const bool dense = s_unknown != 0;   // matches may come from the run table: no fast path below
    if (dense)   // (run mode: the resolve span only; rmode_walk evaluates the chain past it)
        dense_phase<kDev>(sdw, region, step, s_red, &s_unknown, m + bstart + w0,
                    rmode ? mbits + (uint64_t)b * L.wpb + (w0 >> 6) : nullptr, q0,
                    rmode ? min(npos, q0 + kRmSpan) : npos, nload, blen - w0, w0, dbg,
                    rmode ? (uint16_t *)(region + kRmDist) : nullptr, rmode ? kRmRunCap : kRunTableCap);

    if (dbg & 64u) return;   // timing: + queries (no parse)
    uint64_t *cw = chain + (uint64_t)b * L.wpb + (uint64_t)k * (kTile / 64);
    uint32_t *ti = tinfo + 8ull * bx;
    const uint32_t nwords = (t1 - t0 + 63) / 64;
    if (rmode) {
        uint64_t *mbw = mbits + (uint64_t)b * L.wpb + (t0 >> 6);
        if (s_unknown == 0)
            rmode_walk((FCX_LDS uint32_t *)region, (FCX_LDS uint32_t *)s_red, (FCX_LDS uint32_t *)&s_unknown, q0,
                       t1 - t0, blen - w0, w0, t0, mbw, cw,
                       chain_pfx + (uint64_t)bx * (kTile / 64), ti, mtok + (uint64_t)bx * kTileMatches, dbg);
        __syncthreads();
        if (s_unknown != 0) {   // lazy tile: m rows in the span only, "unknown" past it
            for (uint32_t w = tid; w < nwords; w += kMT) {
                cw[w] = 0;
                if (w >= kRmSpan / 64) mbw[w] = ~0ull;
            }
            if (tid == 0) { ti[0] = kTileLazy | kTileSpan2; ti[1] = 0; ti[2] = ti[3] = ti[4] = 0; }
        }
        return;
    }
    if (s_unknown != 0) {
        for (uint32_t w = tid; w < nwords; w += kMT) cw[w] = 0;
        if (tid == 0) { ti[0] = kTileLazy | kTileMFull; ti[1] = 0; ti[2] = ti[3] = ti[4] = 0; }
        return;
    }

    if (s_match == 0 && !dense) {
        // no match anywhere (most tiles of random data): every position is a literal
        // token; the chain words, their prefix counts and the totals follow directly
        if (tid < nwords) {
            const uint32_t nb = min(64u, t1 - t0 - 64 * tid);
            cw[tid] = nb == 64 ? ~0ull : ((1ull << nb) - 1ull);
            chain_pfx[(uint64_t)bx * (kTile / 64) + tid] = 64ull * tid;   // tokens before; no matches
        }
        if (tid == 0) { ti[0] = 0; ti[1] = t1; ti[2] = t1 - t0; ti[3] = 0; ti[4] = 0; }
        return;
    }

    if (sparse && !dense && !(dbg & 65536u) &&
        sparse_parse((const uint64_t *)(region + kSpMb), step, region + kResLds, region + kSpP, t1 - t0, t0, cw,
                     chain_pfx + (uint64_t)bx * (kTile / 64), ti, mtok + (uint64_t)bx * kTileMatches))
        return;

    // ---- 4. tile-local greedy parse ----
    uint32_t *Gs = region + kTile / 2;                 // kMT + 1 entries
    uint32_t *Xs = Gs + kMT + 1;
    uint32_t *Vs = Xs + kMT;
    const uint32_t s = t0 + tid * kSeg;
    const uint32_t se = min(s + kSeg, t1);
    uint32_t V = 0, X = s;
    uint32_t T = 0;
    uint32_t *Ys = Vs;   // exits of a Jacobi round (Vs is free until the counts below)
    if (s < t1) {
        uint32_t t = s;
        while (t < se) { V |= 1u << (t - s); t += step[t - t0]; }
        X = t;
    }
    Xs[tid] = X;
    Gs[tid + 1] = X;
    if (tid == 0) Gs[0] = t0;
    __syncthreads();
    if (dbg & 512u) return;   // timing: + sub-segment walks
    // Jacobi rounds.  A segment is active when its entry lies inside it; the next
    // entry of segment k + 1 is the exit of the nearest active segment <= k (a
    // block-wide running max of active indices), so a long token passes over any
    // number of segments in one round.
    for (uint32_t r = 0;; r++) {
        const uint32_t e = Gs[tid];
        uint32_t ex;
        bool act = false;
        if (s >= t1 || e >= se) {
            ex = e; T = 0;
        } else if ((V >> (e - s)) & 1u) {
            act = true; ex = X; T = V & (~0u << (e - s));
        } else {
            act = true; T = 0;
            uint32_t t = e;
            while (t < se && !((V >> (t - s)) & 1u)) { T |= 1u << (t - s); t += step[t - t0]; }
            if (t < se) { ex = X; T |= V & (~0u << (t - s)); }
            else ex = t;
        }
        Ys[tid] = ex;
        // nearest active segment <= tid: highest set bit of the wave's ballot at or
        // below this lane, else the last active segment of an earlier wave
        const uint64_t am = __ballot(act);
        const uint32_t lane = tid & 63;
        if (lane == 0) s_red[tid >> 6] = am ? (tid & ~63u) + 64 - (uint32_t)__clzll(am) : 0u;
        __syncthreads();
        const uint64_t le = am & (lane == 63 ? ~0ull : ((2ull << lane) - 1));
        uint32_t li = le ? (tid & ~63u) + 64 - (uint32_t)__clzll(le) : 0u;
        for (int w = (int)(tid >> 6) - 1; w >= 0 && !li; w--) li = s_red[w];
        const uint32_t ne = li ? Ys[li - 1] : Gs[tid + 1];
        if (ne != Gs[tid + 1]) { Gs[tid + 1] = ne; s_chg[r & 1] = 1; }
        if (tid == 0) s_chg[(r + 1) & 1] = 0;
        __syncthreads();
        if (!s_chg[r & 1]) break;
    }
    if (dbg & 256u) return;   // timing: + Jacobi rounds
    // counts of this lane's chain positions, prefix over lanes.  The lane's 8 steps come
    // in one 16-B LDS read (no serial read per chain position)
    static_assert(kSeg == 8, "one uint4 of u16 steps per lane");
    uint32_t stp[kSeg];
    {
        const uint4 st4 = ((const uint4 *)step)[tid];
        const uint32_t w4[4] = {st4.x, st4.y, st4.z, st4.w};
#pragma unroll
        for (uint32_t q = 0; q < kSeg; q++) stp[q] = (w4[q >> 1] >> (16 * (q & 1))) & 0xFFFFu;
    }
    uint32_t cnt[3] = {(uint32_t)__builtin_popcount(T), 0, 0};
#pragma unroll
    for (uint32_t q = 0; q < kSeg; q++) {
        const uint32_t Lm = stp[q] - 1u;
        if (((T >> q) & 1u) && Lm) { cnt[1]++; cnt[2] += (Lm >> 2) + 3; }
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
    if (dbg & 1024u) return;   // timing: + counts and their scan
    if (!dense) {
        // compact match list: the speculative chain's match tokens in order (m values
        // from the search results); with m rows only in the first kResolveSpan
        // positions, k_emit takes the rest of the tile's matches from here
        const uint32_t *res_lds = region + kResLds;
        uint32_t *mt = mtok + (uint64_t)bx * kTileMatches + pre[1];
#pragma unroll
        for (uint32_t q = 0; q < kSeg; q++)
            if (((T >> q) & 1u) && stp[q] > 1) *mt++ = res_lds[s - t0 + q];
    }
    if (dbg & 2048u) return;   // timing: + compact list
    constexpr uint32_t kLanesPerWord = 64 / kSeg;   // 8
    if ((tid % kLanesPerWord) == 0 && tid / kLanesPerWord < nwords) {
        const uint32_t w = tid / kLanesPerWord;
        uint64_t word = 0;
#pragma unroll
        for (uint32_t q = 0; q < kLanesPerWord; q++) word |= (uint64_t)Vs[tid + q] << (kSeg * q);
        cw[w] = word;
        chain_pfx[(uint64_t)bx * (kTile / 64) + w] =
            (uint64_t)pre[0] | ((uint64_t)pre[1] << 13) | ((uint64_t)pre[2] << 24);
    }
    if (tid == 0) {
        const uint32_t nsub = (t1 - t0 + kSeg - 1) / kSeg;
        ti[0] = dense ? kTileMFull : 0u;   // dense: the run table wrote m for every position
        ti[1] = Gs[nsub];
        ti[2] = tot[0];
        ti[3] = tot[1];
        ti[4] = tot[2];
    }
}

// The unit's kernel: one workgroup per tile.  Unrouted (rt.list null: forced units, development)
// the grid is every tile of the shard; routed (fcx_route.hip) the grid is a host estimate of the
// unit's list and workgroup i takes list entry i, if there is one (the entries past the grid go to
// k_match_rest).  Either way each XCD takes a contiguous run of entries (xcd_tile).
#if !FCX_REST
// kRouted = false: the route is a constant empty one (unrouted calls, and a direct launch over a call
// whose tiles the estimate gives all to this unit): the list read, the kind check and the hand-on
// branch fold away, and the kernel is the unrouted unit's code exactly.  Every unit is exact for any
// tile, and each tile's outputs are complete from whichever kernel wrote them last, so a tile of
// another kind searched here is searched again by its own unit (launched after this one).
template <bool kDev, bool kListed, bool kRouted>
__global__ __launch_bounds__(kMT, 8) void k_match(const uint8_t *__restrict__ in, Layout L, uint32_t *__restrict__ m,
                                              uint64_t *__restrict__ mbits, uint64_t *__restrict__ chain,
                                              uint64_t *__restrict__ chain_pfx,
                                              uint32_t *__restrict__ tinfo, uint32_t *__restrict__ mtok, uint32_t dbg_in,
                                              MatchRoute rt) {
    uint32_t bx = xcd_tile(blockIdx.x, gridDim.x);
    if constexpr (kListed) {   // (its own instance: the list read moves the unlisted kernel's code)
        // both loads in flight together (the grid never exceeds the list's storage, so list[bx] is
        // always readable); the empty asm keeps the compiler from sinking the second below the test
        const uint32_t c = *rt.cnt, t = rt.list[bx];
        asm volatile("" ::"v"(c), "v"(t));
        if (bx >= c) return;
        bx = uni(t);
    }
    if constexpr (kListed) {
        match_tile<kDev, true>(in, L, m, mbits, chain, chain_pfx, tinfo, mtok, dbg_in, bx, rt);
    } else if constexpr (kRouted) {
        MatchRoute rd = rt;
        rd.defer_list = nullptr;   // (a constant: the hand-on branch folds away)
        match_tile<kDev, true>(in, L, m, mbits, chain, chain_pfx, tinfo, mtok, dbg_in, bx, rd);
    } else {
        const MatchRoute none{};   // (constant: list, kind check and hand-on all fold away)
        match_tile<kDev, false>(in, L, m, mbits, chain, chain_pfx, tinfo, mtok, dbg_in, bx, none);
    }
}

#endif

#if FCX_REST
// The routed call's remainder for this unit: the entries of its list from rest.start on (past its
// launch's grid; every entry when it was not launched; past a direct launch's cover) -- tiles of a
// kind the host's estimate did not foresee, and the no-filter list's late hand-ons.  A fixed grid of
// workgroups loops over them (the count is only known on the device); with none left every
// workgroup exits at once.  Looped, the body needs up to 128 VGPRs, so FCX_REST_WAVES is 4.
__global__ __launch_bounds__(kMT, FCX_REST_WAVES) void k_match_rest(const uint8_t *__restrict__ in, Layout L, uint32_t *__restrict__ m,
                                                   uint64_t *__restrict__ mbits, uint64_t *__restrict__ chain,
                                                   uint64_t *__restrict__ chain_pfx, uint32_t *__restrict__ tinfo,
                                                   uint32_t *__restrict__ mtok, RouteRest rest, MatchRoute rt) {
    const uint32_t c = *rest.cnt, s0 = rest.start_dev ? min(rest.start, *rest.start_dev) : rest.start;
    rt.list = nullptr;   // (the tiles come from the loop; kind bytes and hand-ons as in the routed launch)
    for (uint32_t p = s0 + blockIdx.x; p < c; p += gridDim.x) {
        const uint32_t bx = rest.list[p];
        match_tile<false, true>(in, L, m, mbits, chain, chain_pfx, tinfo, mtok, 0u, bx, rt);
        __syncthreads();   // the next tile's staging overwrites the LDS this one read
    }
}

void launch_match_rest(const uint8_t *in, const Layout &L, uint32_t *m, uint64_t *mbits, uint64_t *chain,
                       uint64_t *chain_pfx, uint32_t *tinfo, uint32_t *mtok, const RouteRest &rest, const MatchRoute &rt,
                       uint32_t grid, hipStream_t st) {
    hipLaunchKernelGGL(k_match_rest, dim3(grid), dim3(kMT), 0, st, in, L, m, mbits, chain, chain_pfx, tinfo, mtok, rest,
                       rt);
}
#endif

#if FCX_LISTED
void launch_match_listed(const uint8_t *in, const Layout &L, uint32_t *m, uint64_t *mbits, uint64_t *chain,
                         uint64_t *chain_pfx, uint32_t *tinfo, uint32_t *mtok, hipStream_t st, const MatchRoute &rt,
                         uint32_t grid) {
    hipLaunchKernelGGL((k_match<false, true, true>), dim3(grid), dim3(kMT), 0, st, in, L, m, mbits, chain, chain_pfx,
                       tinfo, mtok, 0u, rt);
}
#elif FCX_DIRECT
void launch_match_direct(const uint8_t *in, const Layout &L, uint32_t *m, uint64_t *mbits, uint64_t *chain,
                         uint64_t *chain_pfx, uint32_t *tinfo, uint32_t *mtok, hipStream_t st, const MatchRoute &rt,
                         uint32_t grid) {
    hipLaunchKernelGGL((k_match<false, false, true>), dim3(grid), dim3(kMT), 0, st, in, L, m, mbits, chain, chain_pfx,
                       tinfo, mtok, 0u, rt);
}
#elif !FCX_REST
#if FCX_UNIT
void launch_match_listed(const uint8_t *in, const Layout &L, uint32_t *m, uint64_t *mbits, uint64_t *chain,
                         uint64_t *chain_pfx, uint32_t *tinfo, uint32_t *mtok, hipStream_t st, const MatchRoute &rt,
                         uint32_t grid);   // (fcx_match_<unit>_listed.hip)
void launch_match_direct(const uint8_t *in, const Layout &L, uint32_t *m, uint64_t *mbits, uint64_t *chain,
                         uint64_t *chain_pfx, uint32_t *tinfo, uint32_t *mtok, hipStream_t st, const MatchRoute &rt,
                         uint32_t grid);   // (fcx_match_<unit>_direct.hip)
#endif
void launch_match(const uint8_t *in, const Layout &L, uint32_t *m, uint64_t *mbits, uint64_t *chain, uint64_t *chain_pfx,
                  uint32_t *tinfo, uint32_t *mtok, hipStream_t st, uint32_t dbg_override, const MatchRoute *route,
                  uint32_t grid_override) {
    // dbg bits (k_match<true> only): fcx_debug_match's phase exits and experiment bits
    // (development; the kernel alone on scratch the caller discards) and the forced tile modes
    // of fcx_ctx_set_match_mode (bit2 never / bit3 always the whole-tile run mode, bit7 no
    // repeat filter; output unchanged).  The default path launches k_match<false>, compiled
    // without any of them; nothing is read from the environment.
    const uint32_t dbg = dbg_override != ~0u ? dbg_override : 0u;
    const MatchRoute rt = route ? *route : MatchRoute{};
    const uint32_t grid = rt.list ? grid_override : L.nblocks * L.tpb;
    if (grid == 0) return;
    if (rt.list) {
#if FCX_UNIT
        launch_match_listed(in, L, m, mbits, chain, chain_pfx, tinfo, mtok, st, rt, grid);
#endif
#if FCX_UNIT
    } else if (rt.kind) {   // direct, checked: tiles of other kinds end at their kind byte
        launch_match_direct(in, L, m, mbits, chain, chain_pfx, tinfo, mtok, st, rt, grid);
#endif
    } else if (dbg == 0)   // unrouted, or direct over every tile
        hipLaunchKernelGGL((k_match<false, false, false>), dim3(grid), dim3(kMT), 0, st, in, L, m, mbits, chain, chain_pfx,
                           tinfo, mtok, 0u, rt);
    else
        hipLaunchKernelGGL((k_match<true, false, false>), dim3(grid), dim3(kMT), 0, st, in, L, m, mbits, chain, chain_pfx,
                           tinfo, mtok, dbg, rt);
}
#endif

}  // namespace fcx

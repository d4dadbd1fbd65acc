// routebench.hip — what does routing tiles to per-kind match kernels cost by itself?
// (1) a k_match-shaped launch (512 lanes, ~39 KB LDS, one workgroup per 4096-byte tile of
// 1 GiB) in which every workgroup reads its tile's kind byte and exits: the price of
// launching a unit that owns no tile; (2) the same launch where 1/4 of the tiles do the
// launchbench staging work, against a grid of just those tiles; (3) the stream bubble of a
// host read-back between two kernels.  Development measurement only.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <chrono>
#include <vector>

constexpr int kT = 512, kTile = 4096, kWinW = 6464 / 4 + 4, kRegion = 8192;

__device__ inline uint32_t body(const uint32_t *sdw, uint32_t *region, uint32_t tid) {
    uint32_t acc = 0;
    for (uint32_t w = tid; w < kWinW - 1; w += kT) {
        const uint32_t v = sdw[w], p = w ? sdw[w - 1] : 0u;
        uint32_t x = v ^ ((v << 8) | (p >> 24));
        x |= x >> 4; x |= x >> 2; x |= x >> 1;
        acc += __builtin_popcount(x & 0x01010101u);
    }
    region[tid] = acc;
    __syncthreads();
    return region[(tid + 1) & (kT - 1)] + acc;
}

__device__ inline void tile_work(const uint8_t *in, uint64_t n, uint32_t *out, uint32_t t) {
    __shared__ __attribute__((aligned(16))) uint32_t sdw[kWinW];
    __shared__ uint32_t region[kRegion];
    const uint32_t tid = threadIdx.x;
    const uint64_t t0 = (uint64_t)t * kTile, w0 = t0 >= 2048 ? t0 - 2048 : 0;
    if (tid < kWinW / 4) {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (w0 + 16 * tid + 16 <= n) v = ((const uint4 *)(in + w0))[tid];
        ((uint4 *)sdw)[tid] = v;
    }
    __syncthreads();
    const uint32_t r = body(sdw, region, tid);
    if (tid == 0) out[t] = r;
}

// every workgroup: its tile's kind; work only on tiles of kind `mine`
__global__ __launch_bounds__(kT, 8) void k_routed(const uint8_t *in, uint64_t n, uint32_t *out, const uint8_t *kind,
                                               uint32_t mine) {
    const uint32_t t = blockIdx.x;
    if (kind[t] != mine) return;
    tile_work(in, n, out, t);
}

// a grid of only the listed tiles
__global__ __launch_bounds__(kT, 8) void k_listed(const uint8_t *in, uint64_t n, uint32_t *out, const uint32_t *list) {
    tile_work(in, n, out, list[blockIdx.x]);
}

__global__ void k_tiny(uint32_t *x) {
    if (threadIdx.x == 0) x[0] += 1;
}

__global__ __launch_bounds__(256) void k_busy(uint32_t *x, uint32_t iters) {
    uint32_t v = threadIdx.x;
    for (uint32_t i = 0; i < iters; i++) v = v * 1664525u + 1013904223u;
    if (v == 0x12345678u) x[1] = v;
}

int main() {
    const uint64_t n = 1ull << 30;
    const uint32_t ntiles = (uint32_t)(n / kTile);
    uint8_t *in, *kind;
    uint32_t *out, *list;
    (void)hipMalloc(&in, n + 64);
    (void)hipMalloc(&out, ntiles * 4ull);
    (void)hipMalloc(&kind, ntiles);
    (void)hipMalloc(&list, ntiles * 4ull);
    (void)hipMemset(in, 0x5a, n);
    std::vector<uint8_t> hk(ntiles);
    std::vector<uint32_t> hl;
    for (uint32_t t = 0; t < ntiles; t++) {   // kinds cycle per 1 MiB block (256 tiles)
        hk[t] = (uint8_t)((t / 256) & 3);
        if (hk[t] == 1) hl.push_back(t);
    }
    (void)hipMemcpy(kind, hk.data(), ntiles, hipMemcpyHostToDevice);
    (void)hipMemcpy(list, hl.data(), hl.size() * 4, hipMemcpyHostToDevice);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    auto timeit = [&](const char *name, auto launch) {
        launch();
        (void)hipDeviceSynchronize();
        float best = 1e9, sum = 0;
        for (int it = 0; it < 10; it++) {
            (void)hipEventRecord(a);
            launch();
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, a, b);
            best = ms < best ? ms : best;
            sum += ms;
        }
        printf("%-52s best %.4f ms  mean %.4f ms (%s)\n", name, best, sum / 10, hipGetErrorString(hipGetLastError()));
    };
    for (uint32_t tiles : {ntiles, ntiles / 4, ntiles / 16}) {
        char nm[96];
        snprintf(nm, sizeof nm, "all-exit grid, %u tiles", tiles);
        timeit(nm, [&] { hipLaunchKernelGGL(k_routed, dim3(tiles), dim3(kT), 0, 0, in, n, out, kind, 7u); });
    }
    timeit("all tiles work (kind array all match)", [&] {
        (void)hipMemsetAsync(kind, 1, ntiles, 0);
        hipLaunchKernelGGL(k_routed, dim3(ntiles), dim3(kT), 0, 0, in, n, out, kind, 1u); });
    timeit("memset of the kind array alone", [&] { (void)hipMemsetAsync(kind, 1, ntiles, 0); });
    (void)hipMemcpy(kind, hk.data(), ntiles, hipMemcpyHostToDevice);
    timeit("1/4 of tiles work, routed over full grid", [&] {
        hipLaunchKernelGGL(k_routed, dim3(ntiles), dim3(kT), 0, 0, in, n, out, kind, 1u); });
    timeit("1/4 of tiles work, grid of the listed tiles", [&] {
        hipLaunchKernelGGL(k_listed, dim3((uint32_t)hl.size()), dim3(kT), 0, 0, in, n, out, list); });
    timeit("4 routed launches (every tile works once)", [&] {
        for (uint32_t k = 0; k < 4; k++)
            hipLaunchKernelGGL(k_routed, dim3(ntiles), dim3(kT), 0, 0, in, n, out, kind, k); });

    // stream bubble of a host read-back: busy; tiny; [sync]; busy, 50 times
    uint64_t *hw;
    (void)hipHostMalloc((void **)&hw, 64, hipHostMallocDefault);
    const uint32_t iters = 200000;
    auto loop = [&](int mode) {
        (void)hipDeviceSynchronize();
        auto c0 = std::chrono::steady_clock::now();
        (void)hipEventRecord(a);
        for (int i = 0; i < 50; i++) {
            hipLaunchKernelGGL(k_busy, dim3(1024), dim3(256), 0, 0, out, iters);
            hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, 0, out);
            if (mode >= 1) (void)hipMemcpyAsync(hw, out, 24, hipMemcpyDeviceToHost, 0);
            if (mode == 2) (void)hipStreamSynchronize(0);
            for (int q = 0; q < 12; q++) hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, 0, out);
        }
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        auto c1 = std::chrono::steady_clock::now();
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        printf("loop mode %d (%s): %.4f ms per iteration (host %.4f)\n", mode,
               mode == 0 ? "no read-back" : mode == 1 ? "async 24-B copy" : "copy + stream sync", ms / 50,
               std::chrono::duration<double, std::milli>(c1 - c0).count() / 50);
    };
    for (int rep = 0; rep < 2; rep++)
        for (int mode = 0; mode < 3; mode++) loop(mode);
    return 0;
}

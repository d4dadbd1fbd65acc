// launchbench.hip — what does k_match's grid shape cost by itself?  One 512-lane workgroup per
// 4096-byte tile (262144 tiles per GiB) staging its 6464-byte window into LDS, vs a persistent
// grid that loops over the same tiles, vs the persistent grid with the next tile's loads issued
// before the current tile's work (double-buffered staging).  Same LDS footprint as k_match
// (~39 KB, 4 workgroups per CU).  Development measurement only (not part of the library).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int kT = 512, kTile = 4096, kWinW = 6464 / 4 + 4, kRegion = 8192;

__device__ inline uint32_t body(const uint32_t *sdw, uint32_t *region, uint32_t tid) {
    // a little LDS work per tile (runs of the image, as k_match's first phase)
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

__global__ __launch_bounds__(kT, 8) void k_grid(const uint8_t *in, uint64_t n, uint32_t *out) {
    __shared__ __attribute__((aligned(16))) uint32_t sdw[kWinW];
    __shared__ uint32_t region[kRegion];
    const uint32_t tid = threadIdx.x, t = blockIdx.x;
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

__global__ __launch_bounds__(kT, 8) void k_persist(const uint8_t *in, uint64_t n, uint32_t *out, uint32_t ntiles) {
    __shared__ __attribute__((aligned(16))) uint32_t sdw[kWinW];
    __shared__ uint32_t region[kRegion];
    const uint32_t tid = threadIdx.x;
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const uint64_t t0 = (uint64_t)t * kTile, w0 = t0 >= 2048 ? t0 - 2048 : 0;
        __syncthreads();
        if (tid < kWinW / 4) {
            uint4 v = make_uint4(0, 0, 0, 0);
            if (w0 + 16 * tid + 16 <= n) v = ((const uint4 *)(in + w0))[tid];
            ((uint4 *)sdw)[tid] = v;
        }
        __syncthreads();
        const uint32_t r = body(sdw, region, tid);
        if (tid == 0) out[t] = r;
    }
}

// the next tile's 16 B per lane are loaded into registers before this tile's work
__global__ __launch_bounds__(kT, 8) void k_persist_pf(const uint8_t *in, uint64_t n, uint32_t *out, uint32_t ntiles) {
    __shared__ __attribute__((aligned(16))) uint32_t sdw[kWinW];
    __shared__ uint32_t region[kRegion];
    const uint32_t tid = threadIdx.x;
    auto load = [&](uint32_t t) -> uint4 {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (t < ntiles && tid < kWinW / 4) {
            const uint64_t t0 = (uint64_t)t * kTile, w0 = t0 >= 2048 ? t0 - 2048 : 0;
            if (w0 + 16 * tid + 16 <= n) v = ((const uint4 *)(in + w0))[tid];
        }
        return v;
    };
    uint4 nxt = load(blockIdx.x);
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        __syncthreads();
        if (tid < kWinW / 4) ((uint4 *)sdw)[tid] = nxt;
        __syncthreads();
        nxt = load(t + gridDim.x);
        const uint32_t r = body(sdw, region, tid);
        if (tid == 0) out[t] = r;
    }
}

// k_encode's shape: a 128-lane workgroup per 8192-byte chunk, 64 bytes per lane (4 x 16 B in, 4 x 16 B out)
template <int kLanes, int kPer>
__global__ __launch_bounds__(kLanes) void k_copy_grid(const uint4 *in, uint4 *out, uint64_t n16) {
    const uint64_t base = (uint64_t)blockIdx.x * kLanes * kPer;
    uint4 v[kPer];
#pragma unroll
    for (int q = 0; q < kPer; q++) {
        const uint64_t i = base + (uint64_t)q * kLanes + threadIdx.x;
        v[q] = i < n16 ? in[i] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < kPer; q++) {
        const uint64_t i = base + (uint64_t)q * kLanes + threadIdx.x;
        if (i < n16) out[i] = make_uint4(v[q].y, v[q].x, v[q].w, v[q].z);
    }
}
template <int kLanes, int kPer>
__global__ __launch_bounds__(kLanes) void k_copy_persist(const uint4 *in, uint4 *out, uint64_t n16) {
    for (uint64_t base = (uint64_t)blockIdx.x * kLanes * kPer; base < n16; base += (uint64_t)gridDim.x * kLanes * kPer) {
        uint4 v[kPer];
#pragma unroll
        for (int q = 0; q < kPer; q++) {
            const uint64_t i = base + (uint64_t)q * kLanes + threadIdx.x;
            v[q] = i < n16 ? in[i] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int q = 0; q < kPer; q++) {
            const uint64_t i = base + (uint64_t)q * kLanes + threadIdx.x;
            if (i < n16) out[i] = make_uint4(v[q].y, v[q].x, v[q].w, v[q].z);
        }
    }
}

int main(int argc, char **argv) {
    const uint64_t n = 1ull << 30;
    const uint32_t ntiles = (uint32_t)(n / kTile);
    uint8_t *in;
    uint32_t *out;
    (void)hipMalloc(&in, n + 64);
    (void)hipMalloc(&out, ntiles * 4ull);
    (void)hipMemset(in, 0x5a, n);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    auto timeit = [&](const char *name, auto launch) {
        launch();
        (void)hipDeviceSynchronize();
        float best = 1e9;
        for (int it = 0; it < 5; it++) {
            (void)hipEventRecord(a);
            launch();
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, a, b);
            best = ms < best ? ms : best;
        }
        printf("%-28s %.3f ms per GiB (%s)\n", name, best, hipGetErrorString(hipGetLastError()));
    };
    timeit("grid (k_match shape)", [&] { hipLaunchKernelGGL(k_grid, dim3(ntiles), dim3(kT), 0, 0, in, n, out); });
    for (int per : {4, 8, 16}) {
        const uint32_t g = (uint32_t)cus * (uint32_t)per / 4;
        char nm[64];
        snprintf(nm, sizeof nm, "persistent %u WGs", g);
        timeit(nm, [&] { hipLaunchKernelGGL(k_persist, dim3(g), dim3(kT), 0, 0, in, n, out, ntiles); });
        snprintf(nm, sizeof nm, "persistent+prefetch %u WGs", g);
        timeit(nm, [&] { hipLaunchKernelGGL(k_persist_pf, dim3(g), dim3(kT), 0, 0, in, n, out, ntiles); });
    }
    uint8_t *o2;
    (void)hipMalloc(&o2, n + 64);
    const uint64_t n16 = n / 16;
    timeit("hipMemcpy D2D 1 GiB", [&] { (void)hipMemcpyAsync(o2, in, n, hipMemcpyDeviceToDevice, 0); });
    timeit("copy grid 128x(4x16B)", [&] {
        hipLaunchKernelGGL((k_copy_grid<128, 4>), dim3((uint32_t)(n16 / 512)), dim3(128), 0, 0, (const uint4 *)in, (uint4 *)o2, n16); });
    timeit("copy grid 256x(4x16B)", [&] {
        hipLaunchKernelGGL((k_copy_grid<256, 4>), dim3((uint32_t)(n16 / 1024)), dim3(256), 0, 0, (const uint4 *)in, (uint4 *)o2, n16); });
    timeit("copy grid 256x(8x16B)", [&] {
        hipLaunchKernelGGL((k_copy_grid<256, 8>), dim3((uint32_t)(n16 / 2048)), dim3(256), 0, 0, (const uint4 *)in, (uint4 *)o2, n16); });
    for (int per : {8, 16, 32}) {
        char nm[64];
        snprintf(nm, sizeof nm, "copy persistent 256x4 x%d/CU", per);
        timeit(nm, [&] { hipLaunchKernelGGL((k_copy_persist<256, 4>), dim3((uint32_t)(cus * per)), dim3(256), 0, 0,
                                            (const uint4 *)in, (uint4 *)o2, n16); });
    }
    printf("(copy: 2 GiB of traffic per GiB)\n");
    return 0;
}

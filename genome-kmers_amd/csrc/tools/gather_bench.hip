// Random-row gather rate vs table size (tuning probe for the C5 key materialisation):
// out[i] = xor of the 32-B row hash(i) mod rows, for tables of 0.4 .. 99 GB (or the sizes in GB given
// as arguments, down to cache-resident ones: round 5); then the same rows SCATTERED: tab[hash(i) mod
// rows] = i (random row writes).  One launch per size; prints ms and random rows per second.
// Build: hipcc --offload-arch=gfx950 -O3 gather_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x;
}

template <int ROWB>
__global__ __launch_bounds__(256) void gather(const uint4 *__restrict__ tab, uint64_t rows, uint64_t n,
                                              uint64_t *__restrict__ out) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const uint64_t r = mix(i) % rows;
        uint64_t acc = 0;
#pragma unroll
        for (int q = 0; q < ROWB / 16; ++q) {
            const uint4 v = tab[r * (ROWB / 16) + q];
            acc ^= ((uint64_t)v.y << 32 | v.x) ^ ((uint64_t)v.w << 32 | v.z);
        }
        out[i] = acc;
    }
}

template <int ROWB>
__global__ __launch_bounds__(256) void scatter(uint4 *__restrict__ tab, uint64_t rows, uint64_t n) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const uint64_t r = mix(i) % rows;
#pragma unroll
        for (int q = 0; q < ROWB / 16; ++q) tab[r * (ROWB / 16) + q] = make_uint4((uint32_t)i, q, 1, 2);
    }
}

__global__ void fill(uint4 *t, uint64_t n) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
        t[i] = make_uint4((uint32_t)i, (uint32_t)(i >> 32), 1, 2);
}

#include <cstdlib>
#include <vector>
int main(int argc, char **argv) {
    const uint64_t n = 1000000000ull;
    uint64_t *out;
    if (hipMalloc(&out, 8 * n) != hipSuccess) return 1;
    std::vector<double> gbs = {0.4, 3.1, 25.0, 99.0};
    if (argc > 1) {
        gbs.clear();
        for (int a = 1; a < argc; ++a) gbs.push_back(std::atof(argv[a]));
    }
    for (double gb : gbs) {
        const uint64_t bytes = (uint64_t)(gb * 1e9) & ~63ull;
        uint4 *tab;
        if (hipMalloc(&tab, bytes) != hipSuccess) { printf("alloc %.1f GB failed\n", gb); return 1; }
        hipLaunchKernelGGL(fill, dim3(65536), dim3(256), 0, 0, tab, bytes / 16);
        hipEvent_t a, b;
        hipEventCreate(&a); hipEventCreate(&b);
        for (int rowb : {16, 32}) {
            const uint64_t rows = bytes / rowb;
            for (int rep = 0; rep < 2; ++rep) {
                hipEventRecord(a);
                if (rowb == 16) hipLaunchKernelGGL(gather<16>, dim3(65536), dim3(256), 0, 0, tab, rows, n, out);
                else hipLaunchKernelGGL(gather<32>, dim3(65536), dim3(256), 0, 0, tab, rows, n, out);
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms = 0;
                hipEventElapsedTime(&ms, a, b);
                if (rep) printf("table %7.3f GB, %2d-B rows: %8.2f ms for %llu gathers = %.1f G rows/s\n", gb, rowb, ms,
                                (unsigned long long)n, n / (ms * 1e6));
            }
            for (int rep = 0; rep < 2; ++rep) {
                hipEventRecord(a);
                if (rowb == 16) hipLaunchKernelGGL(scatter<16>, dim3(65536), dim3(256), 0, 0, tab, rows, n);
                else hipLaunchKernelGGL(scatter<32>, dim3(65536), dim3(256), 0, 0, tab, rows, n);
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms = 0;
                hipEventElapsedTime(&ms, a, b);
                if (rep) printf("table %7.3f GB, %2d-B rows: %8.2f ms for %llu scatters = %.1f G rows/s\n", gb, rowb, ms,
                                (unsigned long long)n, n / (ms * 1e6));
            }
        }
        hipFree(tab);
    }
    return 0;
}

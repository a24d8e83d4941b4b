// radix_bench.hip -- A/B timing of radix-pass variants on one MI355X (development tool).
//
// Build: hipcc -O3 --offload-arch=gfx950 -I.. -I../../../include radix_bench.hip -o radix_bench
// Run:   ./radix_bench [n]        (default n = 3.1e9 keys: 62-bit random, uint32 payload)
// Every variant sorts digit 0 of the same input; variants with look-back are checked (digit
// order, stability of the payload inside a digit, key checksum).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../gkm_onesweep.h"

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            std::exit(1);                                                                       \
        }                                                                                       \
    } while (0)

using namespace gkm;

__global__ void init_kernel(uint64_t *k, uint32_t *v, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t x = i * 0x9E3779B97F4A7C15ull + 0x1234567ull;
        x ^= x >> 31;
        x *= 0xBF58476D1CE4E5B9ull;
        x ^= x >> 29;
        k[i] = x >> 2;
        v[i] = (uint32_t)i;
    }
}

__global__ void hist_kernel(const uint64_t *k, uint64_t n, int shift, uint32_t *h) {
    __shared__ uint32_t s[256];
    s[threadIdx.x] = 0;
    __syncthreads();
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        atomicAdd(&s[(k[i] >> shift) & 255], 1u);
    __syncthreads();
    atomicAdd(&h[threadIdx.x], s[threadIdx.x]);
}

// violations: digit decreasing, or equal digit with decreasing payload (input payload = index)
__global__ void check_kernel(const uint64_t *k, const uint32_t *v, uint64_t n, int shift, unsigned long long *bad,
                             unsigned long long *sum) {
    unsigned long long b = 0, s = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        s += k[i];
        if (i) {
            uint32_t d0 = (k[i - 1] >> shift) & 255, d1 = (k[i] >> shift) & 255;
            if (d1 < d0 || (d1 == d0 && v[i] <= v[i - 1])) ++b;
        }
    }
    atomicAdd(bad, b);
    atomicAdd(sum, s);
}

__global__ void copy_kernel(const uint4 *a, uint4 *b, uint64_t n16) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x)
        b[i] = a[i];
}

struct Bufs {
    uint64_t *k[2];
    uint32_t *v[2];
    uint64_t *status;
    uint32_t *counter;
    uint32_t *doff;
    uint64_t n;
    uint32_t epoch = 0;
};

template <int T, int I, bool LB>
float run_variant(Bufs &b, const char *name, hipStream_t st, int reps, unsigned long long ref_sum) {
    const uint64_t tile = (uint64_t)T * I;
    const uint64_t tiles = (b.n + tile - 1) / tile;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float best = 1e30f, total = 0.f;
    for (int r = 0; r < reps + 1; ++r) {
        CK(hipMemsetAsync(b.counter, 0, 4, st));
        b.epoch = (b.epoch + 1) & kEpochMask;
        CK(hipEventRecord(e0, st));
        hipLaunchKernelGGL((onesweep_kernel<1, T, I, LB>), dim3((unsigned)tiles), dim3(T), 0, st, b.k[0], b.v[0],
                           b.k[1], b.v[1], b.n, 0, 0, b.doff, b.status, b.counter, b.epoch);
        CK(hipGetLastError());
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r > 0) {
            total += ms;
            if (ms < best) best = ms;
        }
    }
    const char *ok = "-";
    if (LB) {
        unsigned long long *d;
        CK(hipMalloc(&d, 16));
        CK(hipMemset(d, 0, 16));
        hipLaunchKernelGGL(check_kernel, dim3(2048), dim3(256), 0, st, b.k[1], b.v[1], b.n, 0, d, d + 1);
        unsigned long long h[2];
        CK(hipMemcpy(h, d, 16, hipMemcpyDeviceToHost));
        CK(hipFree(d));
        ok = (h[0] == 0 && h[1] == ref_sum) ? "sorted" : "BROKEN";
    }
    const float avg = total / reps;
    std::printf("%-34s tile %6llu  avg %8.3f ms  best %8.3f ms  %7.1f GB/s (24 B/key)  %s\n", name,
                (unsigned long long)tile, avg, best, b.n * 24.0 / (avg * 1e-3) / 1e9, ok);
    return avg;
}

int main(int argc, char **argv) {
    uint64_t n = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 3100000000ull;
    Bufs b;
    b.n = n;
    for (int i = 0; i < 2; ++i) {
        CK(hipMalloc(&b.k[i], 8 * n));
        CK(hipMalloc(&b.v[i], 4 * n));
    }
    const uint64_t max_tiles = n / 1024 + 2;
    CK(hipMalloc(&b.status, 8 * 256 * max_tiles));
    CK(hipMemset(b.status, 0, 8 * 256 * max_tiles));
    CK(hipMalloc(&b.counter, 64));
    CK(hipMalloc(&b.doff, 4 * 256));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipLaunchKernelGGL(init_kernel, dim3(8192), dim3(256), 0, st, b.k[0], b.v[0], n);
    uint32_t *dh;
    CK(hipMalloc(&dh, 4 * 256));
    CK(hipMemset(dh, 0, 4 * 256));
    hipLaunchKernelGGL(hist_kernel, dim3(2048), dim3(256), 0, st, b.k[0], n, 0, dh);
    std::vector<uint32_t> h(256), off(256);
    CK(hipMemcpy(h.data(), dh, 4 * 256, hipMemcpyDeviceToHost));
    uint64_t run = 0;
    for (int i = 0; i < 256; ++i) {
        off[i] = (uint32_t)run;
        run += h[i];
    }
    CK(hipMemcpy(b.doff, off.data(), 4 * 256, hipMemcpyHostToDevice));
    unsigned long long ref_sum = 0;
    {
        unsigned long long *d;
        CK(hipMalloc(&d, 16));
        CK(hipMemset(d, 0, 16));
        hipLaunchKernelGGL(check_kernel, dim3(2048), dim3(256), 0, st, b.k[0], b.v[0], n, 0, d, d + 1);
        unsigned long long hh[2];
        CK(hipMemcpy(hh, d, 16, hipMemcpyDeviceToHost));
        ref_sum = hh[1];
        CK(hipFree(d));
    }
    std::printf("n = %llu keys\n", (unsigned long long)n);
    // copy baseline: 12 B read + 12 B write per key, as 16-B vector copies of both arrays
    {
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        float tot = 0;
        for (int r = 0; r < 4; ++r) {
            CK(hipEventRecord(e0, st));
            hipLaunchKernelGGL(copy_kernel, dim3(256 * 8), dim3(256), 0, st, (const uint4 *)b.k[0], (uint4 *)b.k[1],
                               n / 2);
            hipLaunchKernelGGL(copy_kernel, dim3(256 * 8), dim3(256), 0, st, (const uint4 *)b.v[0], (uint4 *)b.v[1],
                               n / 4);
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r) tot += ms;
        }
        std::printf("%-34s                avg %8.3f ms                  %7.1f GB/s\n", "copy keys+vals (uint4)", tot / 3,
                    n * 24.0 / (tot / 3 * 1e-3) / 1e9);
    }
    const int R = 4;
    run_variant<256, 16, true>(b, "onesweep T256 I16 (current)", st, R, ref_sum);
    run_variant<256, 16, false>(b, "onesweep T256 I16 no-lookback", st, R, ref_sum);
    run_variant<512, 16, true>(b, "onesweep T512 I16", st, R, ref_sum);
    run_variant<256, 24, true>(b, "onesweep T256 I24", st, R, ref_sum);
    run_variant<256, 12, true>(b, "onesweep T256 I12", st, R, ref_sum);
    run_variant<512, 8, true>(b, "onesweep T512 I8", st, R, ref_sum);
    run_variant<1024, 8, true>(b, "onesweep T1024 I8", st, R, ref_sum);
    run_variant<1024, 12, true>(b, "onesweep T1024 I12", st, R, ref_sum);
    return 0;
}

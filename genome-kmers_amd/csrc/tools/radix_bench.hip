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
#include "../gkm_partition.h"

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

// ideal uniform partition: tile t sends R = TILE/256 consecutive elements to each digit region,
// landing next to tile t-1's run -- the memory-side ceiling of a partition pass with runs of R
// one MSD partition pass (production msd_scatter_kernel) over the whole array as one bucket
struct MsdTables {
    uint32_t *t_start = nullptr, *t_count = nullptr, *tile_off = nullptr;
    uint64_t tiles = 0;
    int tile = 0, rbits = 8;
};

static void msd_tables_for(Bufs &b, hipStream_t st, int tile, MsdTables &m, int rbits = 8) {
    if (m.tile == tile && m.rbits == rbits) return;
    m.rbits = rbits;
    const int RADIX = 1 << rbits;
    if (m.t_start) {
        CK(hipFree(m.t_start));
        CK(hipFree(m.t_count));
        CK(hipFree(m.tile_off));
    }
    m.tile = tile;
    m.tiles = (b.n + tile - 1) / tile;
    std::vector<uint32_t> ts(m.tiles), tc(m.tiles);
    for (uint64_t j = 0; j < m.tiles; ++j) {
        ts[j] = (uint32_t)(j * tile);
        tc[j] = (uint32_t)std::min<uint64_t>(tile, b.n - j * tile);
    }
    CK(hipMalloc(&m.t_start, 4 * m.tiles));
    CK(hipMalloc(&m.t_count, 4 * m.tiles));
    CK(hipMalloc(&m.tile_off, 4 * RADIX * m.tiles));
    CK(hipMemcpy(m.t_start, ts.data(), 4 * m.tiles, hipMemcpyHostToDevice));
    CK(hipMemcpy(m.t_count, tc.data(), 4 * m.tiles, hipMemcpyHostToDevice));
    if (rbits == 8)
        hipLaunchKernelGGL(msd_count_kernel<8>, dim3((unsigned)m.tiles), dim3(256), 0, st, m.t_start, m.t_count,
                           Dig{54, 255u}, b.k[0], m.tile_off);
    else
        hipLaunchKernelGGL(msd_count_kernel<7>, dim3((unsigned)m.tiles), dim3(256), 0, st, m.t_start, m.t_count,
                           Dig{55, 127u}, b.k[0], m.tile_off);
    CK(hipStreamSynchronize(st));
    std::vector<uint32_t> h((size_t)RADIX * m.tiles);
    CK(hipMemcpy(h.data(), m.tile_off, 4 * RADIX * m.tiles, hipMemcpyDeviceToHost));
    std::vector<uint64_t> tot(RADIX, 0);
    for (uint64_t j = 0; j < m.tiles; ++j)
        for (int d = 0; d < RADIX; ++d) tot[d] += h[j * RADIX + d];
    std::vector<uint64_t> run(RADIX);
    uint64_t r = 0;
    for (int d = 0; d < RADIX; ++d) {
        run[d] = r;
        r += tot[d];
    }
    for (uint64_t j = 0; j < m.tiles; ++j)
        for (int d = 0; d < RADIX; ++d) {
            const uint32_t c = h[j * RADIX + d];
            h[j * RADIX + d] = (uint32_t)run[d];
            run[d] += c;
        }
    CK(hipMemcpy(m.tile_off, h.data(), 4 * (size_t)RADIX * m.tiles, hipMemcpyHostToDevice));
}

template <int T, int I, int MODE>
static void run_msd(Bufs &b, MsdTables &m, const char *name, hipStream_t st, unsigned long long ref_sum,
                    unsigned grid = 256, int stagger = 0) {
    msd_tables_for(b, st, T * I, m);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float tot = 0, best = 1e30f;
    const int R = 4;
    for (int r = 0; r <= R; ++r) {
        CK(hipEventRecord(e0, st));
        hipLaunchKernelGGL((msd_scatter_kernel<T, I, 8, MODE, false>), dim3(grid), dim3(T), 0, st, m.t_start, m.t_count,
                           Dig{54, 255u}, m.tile_off, b.k[0], b.v[0], b.k[1], b.v[1], (uint32_t)m.tiles, b.n,
                           nullptr, stagger);
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r) {
            tot += ms;
            best = std::min(best, ms);
        }
    }
    const char *verdict = "-";
    if (MODE == 0) {
        unsigned long long *d;
        CK(hipMalloc(&d, 16));
        CK(hipMemset(d, 0, 16));
        hipLaunchKernelGGL(check_kernel, dim3(2048), dim3(256), 0, st, b.k[1], b.v[1], b.n, 62 - R, d, d + 1);
        unsigned long long hh[2];
        CK(hipMemcpy(hh, d, 16, hipMemcpyDeviceToHost));
        CK(hipFree(d));
        verdict = (hh[0] == 0 && hh[1] == ref_sum) ? "sorted" : "WRONG";
    }
    std::printf("%-34s tile %6d  avg %8.3f ms  best %8.3f ms  %7.1f GB/s (24 B/key)  %s\n", name, T * I, tot / R, best,
                b.n * 24.0 / (best * 1e-3) / 1e9, verdict);
}

// phase profile of the production partition kernel (timing build): clock ticks per tile
template <int T, int I>
static void profile_msd(Bufs &b, MsdTables &m, hipStream_t st, unsigned grid) {
    msd_tables_for(b, st, T * I, m);
    unsigned long long *prof;
    CK(hipMalloc(&prof, 8 * 8));
    CK(hipMemset(prof, 0, 64));
    hipLaunchKernelGGL((msd_scatter_kernel<T, I, 8, 0, true>), dim3(grid), dim3(T), 0, st, m.t_start, m.t_count,
                       Dig{54, 255u}, m.tile_off, b.k[0], b.v[0], b.k[1], b.v[1], (uint32_t)m.tiles, b.n, prof);
    CK(hipStreamSynchronize(st));
    unsigned long long h[8];
    CK(hipMemcpy(h, prof, 64, hipMemcpyDeviceToHost));
    const char *names[6] = {"rank", "scan", "slots", "stage", "reset", "store+top"};
    unsigned long long tot = 0;
    for (int i = 0; i < 6; ++i) tot += h[i];
    std::printf("phase profile T%d I%d grid %u (clock ticks per tile, thread 0):", T, I, grid);
    for (int i = 0; i < 6; ++i) std::printf("  %s %.0f (%.0f%%)", names[i], (double)h[i] / m.tiles, 100.0 * h[i] / tot);
    std::printf("\n");
    CK(hipFree(prof));
}

template <int T, int I, int R, int MODE, int PRE = 0>
static void run_pipe(Bufs &b, MsdTables &m, const char *name, hipStream_t st, unsigned long long ref_sum,
                     unsigned grid) {
    msd_tables_for(b, st, T * I, m, R);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float tot = 0, best = 1e30f;
    const int RR = 4;
    for (int r = 0; r <= RR; ++r) {
        CK(hipEventRecord(e0, st));
        hipLaunchKernelGGL((msd_pipe_kernel<T, I, R, MODE, false, PRE>), dim3(grid), dim3(T), 0, st, m.t_start, m.t_count,
                           Dig{62 - R, (1u << R) - 1}, m.tile_off, b.k[0], b.v[0], b.k[1], b.v[1], (uint32_t)m.tiles, b.n);
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r) {
            tot += ms;
            best = std::min(best, ms);
        }
    }
    const char *verdict = "-";
    if (MODE == 0) {
        unsigned long long *d;
        CK(hipMalloc(&d, 16));
        CK(hipMemset(d, 0, 16));
        hipLaunchKernelGGL(check_kernel, dim3(2048), dim3(256), 0, st, b.k[1], b.v[1], b.n, 62 - R, d, d + 1);
        unsigned long long hh[2];
        CK(hipMemcpy(hh, d, 16, hipMemcpyDeviceToHost));
        CK(hipFree(d));
        verdict = (hh[0] == 0 && hh[1] == ref_sum) ? "sorted" : "WRONG";
    }
    std::printf("%-34s tile %6d  avg %8.3f ms  best %8.3f ms  %7.1f GB/s (24 B/key)  %s\n", name, T * I, tot / RR, best,
                b.n * 24.0 / (best * 1e-3) / 1e9, verdict);
}

template <int TILE>
__global__ __launch_bounds__(256) void runscatter_kernel(const uint64_t *__restrict__ k, const uint32_t *__restrict__ v,
                                                         uint64_t *__restrict__ ko, uint32_t *__restrict__ vo,
                                                         uint64_t n, uint64_t stride) {
    constexpr int R = TILE / 256;
    const uint64_t t = blockIdx.x;
    for (int s = threadIdx.x; s < TILE; s += 256) {
        const uint64_t e = t * TILE + s;
        const uint64_t o = (uint64_t)(s / R) * stride + t * R + (s % R);
        if (e < n && o < n) {
            ko[o] = k[e];
            vo[o] = v[e];
        }
    }
}

template <int TILE>
static void run_scatter(Bufs &b, hipStream_t st) {
    const uint64_t nt = (b.n + TILE - 1) / TILE;
    const uint64_t stride = nt * (TILE / 256);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float tot = 0;
    for (int r = 0; r < 4; ++r) {
        CK(hipEventRecord(e0, st));
        hipLaunchKernelGGL(runscatter_kernel<TILE>, dim3((unsigned)nt), dim3(256), 0, st, b.k[0], b.v[0], b.k[1], b.v[1],
                           b.n, stride);
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r) tot += ms;
    }
    std::printf("ideal run scatter, run %4d keys   tile %6d  avg %8.3f ms                  %7.1f GB/s\n", TILE / 256,
                TILE, tot / 3, b.n * 24.0 / (tot / 3 * 1e-3) / 1e9);
}


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
    run_scatter<4096>(b, st);
    run_scatter<12288>(b, st);
    run_scatter<24576>(b, st);
    run_scatter<49152>(b, st);
    run_scatter<98304>(b, st);
    MsdTables m;
    run_pipe<1024, 11, 8, 0>(b, m, "pipe T1024 I11 R8 grid 1024", st, ref_sum, 1024);
    run_pipe<1024, 11, 7, 0>(b, m, "pipe T1024 I11 R7 grid 1024", st, ref_sum, 1024);
    if (argc > 2) return 0;
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

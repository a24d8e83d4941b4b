// lds_rank_probe.hip -- does a returning LDS atomic add give lane-ordered results on gfx950?
// (development probe, not product code)
//
// When several lanes of ONE wave instruction `ds_add_rtn_u32` the same LDS word, each lane gets
// the word's value before its own add.  If the LDS applies same-address lanes in increasing lane
// order, a lane's return value is (value before the instruction) + (lanes below it with the same
// address): exactly the stable rank a radix partition needs, in one LDS instruction instead of a
// ballot-match or a mask round trip.  This probe checks that property against a ballot-match
// ground truth over many random address patterns, with every CU busy, and times both rankings.
//
// Build: hipcc -O3 --offload-arch=gfx950 lds_rank_probe.hip -o lds_rank_probe
// Run:   ./lds_rank_probe [iters]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            std::exit(1);                                                                       \
        }                                                                                       \
    } while (0)

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
    const uint32_t lane = threadIdx.x & 63;
    return (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
}

// ground truth: lanes below with the same 8-bit digit (8 ballots)
__device__ __forceinline__ uint64_t match8(uint32_t d) {
    uint64_t m = ~0ull;
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        const uint64_t x = __ballot((d >> b) & 1);
        m &= ((d >> b) & 1) ? x : ~x;
    }
    return m;
}

// mode: digit mask (0xff random 256, 0x0f 16 digits, 0x3 4 digits, 0 all the same); items per
// trial: successive instructions accumulate in the same counters
template <int ITEMS>
__global__ __launch_bounds__(256) void order_kernel(uint32_t iters, uint32_t dmask, uint32_t seed,
                                                    unsigned long long *bad, unsigned long long *checked) {
    __shared__ uint32_t s_cnt[4][256];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint32_t *cnt = s_cnt[wave];
    unsigned long long nb = 0, nc = 0;
    for (uint32_t t = 0; t < iters; ++t) {
#pragma unroll
        for (int u = 0; u < 4; ++u) cnt[u * 64 + lane] = 0;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        uint32_t dd[ITEMS], got[ITEMS];
#pragma unroll
        for (int i = 0; i < ITEMS; ++i) {
            dd[i] = mix(seed ^ (blockIdx.x * 7919u + t * 131u + i * 17u) * 64u + lane * 2654435761u) & dmask;
            got[i] = atomicAdd(&cnt[dd[i]], 1u);
        }
        // exact expected value: count over all earlier items by shuffles (64 lanes x j < i)
#pragma unroll
        for (int i = 0; i < ITEMS; ++i) {
            uint32_t exp = lanes_below(match8(dd[i]));
            for (int j = 0; j < i; ++j) {
                for (int l = 0; l < 64; ++l) exp += __shfl(dd[j], l) == dd[i];
            }
            nb += got[i] != exp;
            nc += 1;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    }
    atomicAdd(bad, nb);
    atomicAdd(checked, nc);
}

// throughput: rank ITEMS items per trial by (a) one returning atomic per item, (b) the mask
// round trip (or, read, zero) + leader add + broadcast
template <int MODE>
__global__ __launch_bounds__(256) void rank_time_kernel(uint32_t iters, uint32_t seed, uint32_t *sink) {
    __shared__ uint32_t s_cnt[4][256];
    __shared__ uint64_t s_mask[4][256];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint32_t *cnt = s_cnt[wave];
    uint64_t *msk = s_mask[wave];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        cnt[u * 64 + lane] = 0;
        msk[u * 64 + lane] = 0;
    }
    uint32_t acc = 0;
    for (uint32_t t = 0; t < iters; ++t) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t d = mix(seed + t * 8 + i + lane * 977u) & 255;
            uint32_t r;
            if (MODE == 0) {
                r = atomicAdd(&cnt[d], 1u);
            } else {
                atomicOr((unsigned long long *)&msk[d], 1ull << lane);
                const uint64_t peers = msk[d];
                msk[d] = 0;
                const uint32_t below = lanes_below(peers);
                uint32_t old = 0;
                if (below == 0) old = atomicAdd(&cnt[d], (uint32_t)__popcll(peers));
                old = __shfl(old, __ffsll((unsigned long long)peers) - 1);
                r = old + below;
            }
            acc += r;
        }
    }
    sink[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main(int argc, char **argv) {
    const uint32_t iters = argc > 1 ? (uint32_t)atoi(argv[1]) : 2000;
    unsigned long long *d;
    CK(hipMalloc(&d, 16));
    const int blocks = 256 * 8;  // every CU, 8 workgroups each
    const uint32_t masks[] = {0xff, 0x0f, 0x3, 0x1, 0x0};
    unsigned long long tot_bad = 0, tot = 0;
    for (uint32_t m : masks) {
        for (int rep = 0; rep < 2; ++rep) {
            CK(hipMemset(d, 0, 16));
            hipLaunchKernelGGL((order_kernel<4>), dim3(blocks), dim3(256), 0, 0, iters, m, 1234u + rep * 99u, d, d + 1);
            CK(hipGetLastError());
            CK(hipDeviceSynchronize());
            unsigned long long h[2];
            CK(hipMemcpy(h, d, 16, hipMemcpyDeviceToHost));
            std::printf("order: digit mask 0x%02x rep %d: %llu of %llu lane-items out of lane order\n", m, rep, h[0],
                        h[1] * 64);
            tot_bad += h[0];
            tot += h[1] * 64;
        }
    }
    uint32_t *sink;
    CK(hipMalloc(&sink, (size_t)blocks * 256 * 4));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int mode = 0; mode < 2; ++mode) {
        for (int rep = 0; rep < 2; ++rep) {
            CK(hipEventRecord(a));
            if (mode == 0)
                hipLaunchKernelGGL((rank_time_kernel<0>), dim3(blocks), dim3(256), 0, 0, iters * 10, 7u, sink);
            else
                hipLaunchKernelGGL((rank_time_kernel<1>), dim3(blocks), dim3(256), 0, 0, iters * 10, 7u, sink);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            const double items = (double)blocks * 256 * iters * 10 * 8;
            std::printf("rank %s: %.3f ms, %.2f G items/s\n", mode == 0 ? "atomic-return" : "mask round trip", ms,
                        items / (ms * 1e-3) / 1e9);
        }
    }
    std::printf("TOTAL: %llu of %llu out of lane order\n", tot_bad, tot);
    return tot_bad ? 2 : 0;
}

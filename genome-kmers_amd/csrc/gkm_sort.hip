// gkm_sort.hip -- stable LSD radix sort of (W-word key, uint32 start) pairs on gfx950.
//
// Replaces the reference's serial numba quicksort (kmers.py:1624-1731 -> numba misc/quicksort.py)
// with a one-sweep-per-digit radix sort:
//   * one upfront histogram of every 8-bit digit (fused into the encoder on the enumerate path);
//   * per digit ONE kernel: tile = 256 threads x 16 keys; per-wave 64-lane match via 8 ballots
//     gives each key its stable rank inside the tile; the tile's digit counts are combined with
//     its predecessors' by decoupled look-back over epoch-tagged 64-bit status words (agent-scope
//     relaxed atomics: the status word is its own flag, no fences); keys are then staged in LDS
//     in digit order and written out so each digit's run is a coalesced burst.
//   * digits whose histogram has a single non-empty bin are skipped.
// Stability + ascending-start input => equal k-mers end up ordered by start index, i.e. the
// reference's get_is_less_than_func(break_ties=True) order (kmers.py:1710-1711).
#include <algorithm>

#include "gkm_internal.h"

namespace gkm {

constexpr uint64_t kFlagAgg = 1ull << 62;
constexpr uint64_t kFlagIncl = 2ull << 62;
constexpr uint64_t kValueMask = (1ull << 40) - 1;
constexpr uint32_t kEpochMask = (1u << 22) - 1;

__device__ __forceinline__ uint64_t pack_status(uint64_t flag, uint32_t epoch, uint64_t v) {
    return flag | ((uint64_t)(epoch & kEpochMask) << 40) | (v & kValueMask);
}

// ---------------------------------------------------------------------------------------------
// histogram of all digits of materialised keys
// ---------------------------------------------------------------------------------------------
template <int W>
__global__ __launch_bounds__(256) void histogram_kernel(const uint64_t *__restrict__ keys, uint64_t n, int digits,
                                                        uint32_t *__restrict__ ghist) {
    __shared__ uint32_t s_hist[kMaxWords * 8 * 256];
    for (int i = threadIdx.x; i < digits * 256; i += 256) s_hist[i] = 0;
    __syncthreads();
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        for (int w = 0; w < W; ++w) {
            const uint64_t k = keys[(uint64_t)w * n + i];
            const int dbase = (W - 1 - w) * 8;
            for (int b = 0; b < 8; ++b) {
                const int d = dbase + b;
                if (d < digits) atomicAdd(&s_hist[d * 256 + ((k >> (8 * b)) & 0xFF)], 1u);
            }
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < digits * 256; i += 256) {
        uint32_t v = s_hist[i];
        if (v) atomicAdd(&ghist[i], v);
    }
}

hipError_t launch_histogram(gk_ctx *c, const uint64_t *keys, uint64_t n, int words, int digits, uint32_t *hist) {
    hipError_t e = hipMemsetAsync(hist, 0, sizeof(uint32_t) * 256 * digits, c->stream);
    if (e != hipSuccess) return e;
    int grid = (int)std::min<uint64_t>((n + 255) / 256, 256 * 4);
    if (grid < 1) grid = 1;
    switch (words) {
    case 1: hipLaunchKernelGGL(histogram_kernel<1>, dim3(grid), dim3(256), 0, c->stream, keys, n, digits, hist); break;
    case 2: hipLaunchKernelGGL(histogram_kernel<2>, dim3(grid), dim3(256), 0, c->stream, keys, n, digits, hist); break;
    case 3: hipLaunchKernelGGL(histogram_kernel<3>, dim3(grid), dim3(256), 0, c->stream, keys, n, digits, hist); break;
    case 4: hipLaunchKernelGGL(histogram_kernel<4>, dim3(grid), dim3(256), 0, c->stream, keys, n, digits, hist); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// one radix pass
// ---------------------------------------------------------------------------------------------
template <int W>
struct PassSmem {
    static constexpr int kStage = W * kSortTile * 8 + kSortTile * 4;  // keys + vals staging
    static constexpr int kCounters = 4 * 256 * 4;                      // per-wave digit counters
    static constexpr int kUnion = kStage > kCounters ? kStage : kCounters;
};

template <int W>
__global__ __launch_bounds__(kSortThreads) void onesweep_kernel(
    const uint64_t *__restrict__ kin, const uint32_t *__restrict__ vin, uint64_t *__restrict__ kout,
    uint32_t *__restrict__ vout, uint64_t n, int word, int shift, const uint32_t *__restrict__ doff,
    uint64_t *__restrict__ status, uint32_t *__restrict__ tile_counter, uint32_t epoch) {
    constexpr int I = kSortItems;
    constexpr int TILE = kSortTile;
    __shared__ __attribute__((aligned(16))) unsigned char s_raw[PassSmem<W>::kUnion];
    __shared__ uint32_t s_tile_start[256];
    __shared__ uint32_t s_gbase[256];
    __shared__ uint32_t s_wsum[4];
    __shared__ uint32_t s_tile;

    uint32_t *s_wc = reinterpret_cast<uint32_t *>(s_raw);  // [4][256], alias of the staging area
    uint64_t *s_keys = reinterpret_cast<uint64_t *>(s_raw);
    uint32_t *s_vals = reinterpret_cast<uint32_t *>(s_raw + W * TILE * 8);

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;

    if (tid == 0) s_tile = atomicAdd(tile_counter, 1u);
    for (int i = tid; i < 4 * 256; i += kSortThreads) s_wc[i] = 0;
    __syncthreads();
    const uint64_t tile = s_tile;
    const uint64_t base = tile * TILE;

    // ---- load (wave-striped: item i of this lane is element wave*I*64 + i*64 + lane) ----
    uint64_t key[I][W];
    uint32_t val[I];
    uint32_t rank[I];
#pragma unroll
    for (int i = 0; i < I; ++i) {
        const uint64_t e = base + (uint64_t)wave * I * 64 + i * 64 + lane;
        if (e < n) {
#pragma unroll
            for (int w = 0; w < W; ++w) key[i][w] = kin[(uint64_t)w * n + e];
            val[i] = vin[e];
        } else {
#pragma unroll
            for (int w = 0; w < W; ++w) key[i][w] = 0;
            val[i] = 0;
        }
    }

    // ---- stable in-tile ranking: 64-lane match by 8 ballots, per-wave LDS counters ----
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
#pragma unroll
    for (int i = 0; i < I; ++i) {
        const uint64_t e = base + (uint64_t)wave * I * 64 + i * 64 + lane;
        const bool valid = e < n;
        uint32_t kw = 0;
#pragma unroll
        for (int w = 0; w < W; ++w)
            if (w == word) kw = (uint32_t)(key[i][w] >> shift) & 0xFFu;
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const bool bit = (kw >> b) & 1u;
            const uint64_t bb = __ballot(bit);
            peers &= bit ? bb : ~bb;
        }
        const int leader = valid ? (__ffsll((unsigned long long)peers) - 1) : lane;
        const uint32_t rank_in = __popcll(peers & lt_mask);
        uint32_t old = 0;
        if (valid && lane == leader) {
            old = s_wc[wave * 256 + kw];
            s_wc[wave * 256 + kw] = old + (uint32_t)__popcll(peers);
        }
        old = __shfl(old, leader);
        rank[i] = old + rank_in;
    }
    __syncthreads();

    // ---- per-digit tile totals, wave prefixes, tile-local digit starts ----
    const int d = tid;  // one thread per digit
    uint32_t total = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const uint32_t v = s_wc[w * 256 + d];
        s_wc[w * 256 + d] = total;
        total += v;
    }
    // block exclusive scan of totals over digits
    uint32_t incl = total;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(incl, off);
        if (lane >= off) incl += y;
    }
    if (lane == 63) s_wsum[wave] = incl;
    __syncthreads();
    uint32_t wpre = 0;
    for (int w = 0; w < wave; ++w) wpre += s_wsum[w];
    s_tile_start[d] = wpre + incl - total;

    // ---- decoupled look-back over predecessor tiles (one digit per thread) ----
    {
        uint64_t *st = status + tile * 256 + d;
        uint64_t excl = 0;
        if (tile == 0) {
            __hip_atomic_store(st, pack_status(kFlagIncl, epoch, total), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            __hip_atomic_store(st, pack_status(kFlagAgg, epoch, total), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            int64_t t = (int64_t)tile - 1;
            while (true) {
                const uint64_t s = __hip_atomic_load(status + (uint64_t)t * 256 + d, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
                const uint64_t flag = s & (3ull << 62);
                const uint32_t ep = (uint32_t)(s >> 40) & kEpochMask;
                if (flag == 0 || ep != (epoch & kEpochMask)) {
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                excl += s & kValueMask;
                if (flag == kFlagIncl) break;
                --t;
            }
            __hip_atomic_store(st, pack_status(kFlagIncl, epoch, excl + total), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        s_gbase[d] = doff[d] + (uint32_t)excl;
    }
    __syncthreads();

    // ---- destination slot inside the tile, then stage keys in digit order ----
    uint32_t slot[I];
#pragma unroll
    for (int i = 0; i < I; ++i) {
        uint32_t kw = 0;
#pragma unroll
        for (int w = 0; w < W; ++w)
            if (w == word) kw = (uint32_t)(key[i][w] >> shift) & 0xFFu;
        slot[i] = s_tile_start[kw] + s_wc[wave * 256 + kw] + rank[i];
    }
    __syncthreads();  // s_wc (aliased) fully read
    const uint32_t tile_n = (uint32_t)std::min<uint64_t>(TILE, n - base);
#pragma unroll
    for (int i = 0; i < I; ++i) {
        const uint64_t e = base + (uint64_t)wave * I * 64 + i * 64 + lane;
        if (e < n) {
#pragma unroll
            for (int w = 0; w < W; ++w) s_keys[w * TILE + slot[i]] = key[i][w];
            s_vals[slot[i]] = val[i];
        }
    }
    __syncthreads();

    // ---- coalesced write-out: consecutive slots of one digit go to consecutive addresses ----
    for (uint32_t s = tid; s < tile_n; s += kSortThreads) {
        uint64_t kk[W];
#pragma unroll
        for (int w = 0; w < W; ++w) kk[w] = s_keys[w * TILE + s];
        uint32_t kw = 0;
#pragma unroll
        for (int w = 0; w < W; ++w)
            if (w == word) kw = (uint32_t)(kk[w] >> shift) & 0xFFu;
        const uint64_t o = (uint64_t)s_gbase[kw] + (s - s_tile_start[kw]);
#pragma unroll
        for (int w = 0; w < W; ++w) kout[(uint64_t)w * n + o] = kk[w];
        vout[o] = s_vals[s];
    }
}

template <int W>
static hipError_t launch_pass(gk_ctx *c, int word, int shift, const uint32_t *doff, uint32_t *counter, uint32_t epoch) {
    const uint64_t tiles = (c->n + kSortTile - 1) / kSortTile;
    const int src = c->cur, dst = c->cur ^ 1;
    hipLaunchKernelGGL(onesweep_kernel<W>, dim3((unsigned)tiles), dim3(kSortThreads), 0, c->stream, c->keys[src],
                       c->vals[src], c->keys[dst], c->vals[dst], c->n, word, shift, doff, c->status, counter, epoch);
    return hipGetLastError();
}

// Sort (keys[cur], vals[cur]) by the low total_bits of the W-word keys; result in keys/vals[cur].
int radix_sort(gk_ctx *c, int words, int total_bits, bool hist_ready) {
    const int D = (total_bits + 7) / 8;
    if (c->n < 2 || D == 0) return GK_OK;
    if (!hist_ready) {
        int slot;
        timer_begin(c, "histogram", &slot);
        GK_TRY_HIP(c, launch_histogram(c, c->keys[c->cur], c->n, words, D, c->hist));
        timer_end(c, slot);
    }
    std::vector<uint32_t> h((size_t)D * 256);
    GK_TRY_HIP(c, hipMemcpyAsync(h.data(), c->hist, 4 * h.size(), hipMemcpyDeviceToHost, c->stream));
    GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
    std::vector<uint32_t> off((size_t)D * 256);
    std::vector<int> todo;
    for (int d = 0; d < D; ++d) {
        uint64_t run = 0;
        bool trivial = false;
        for (int b = 0; b < 256; ++b) {
            off[(size_t)d * 256 + b] = (uint32_t)run;
            run += h[(size_t)d * 256 + b];
            if (h[(size_t)d * 256 + b] == c->n) trivial = true;
        }
        if (run != c->n) return fail(c, GK_E_HIP, "radix histogram does not add up to the key count");
        if (!trivial) todo.push_back(d);
    }
    if (todo.empty()) return GK_OK;
    GK_TRY_HIP(c, hipMemcpyAsync(c->offsets, off.data(), 4 * off.size(), hipMemcpyHostToDevice, c->stream));
    GK_TRY_HIP(c, hipMemsetAsync(c->counters, 0, 4 * 64, c->stream));
    const uint64_t tiles = (c->n + kSortTile - 1) / kSortTile;
    if (tiles * 256 > c->status_cap) return fail(c, GK_E_HIP, "radix status buffer too small");
    int pass = 0;
    for (int d : todo) {
        c->epoch = (c->epoch + 1) & kEpochMask;
        if (c->epoch == 0) {  // wrapped: stale tags could alias, clear once
            GK_TRY_HIP(c, hipMemsetAsync(c->status, 0, 8 * c->status_cap, c->stream));
            c->epoch = 1;
        }
        const int word = words - 1 - d / 8, shift = 8 * (d % 8);
        uint32_t *counter = c->counters + (pass % 64);
        if (pass > 0 && pass % 64 == 0) GK_TRY_HIP(c, hipMemsetAsync(c->counters, 0, 4 * 64, c->stream));
        int slot;
        timer_begin(c, "radix_pass", &slot);
        hipError_t e;
        switch (words) {
        case 1: e = launch_pass<1>(c, word, shift, c->offsets + (size_t)d * 256, counter, c->epoch); break;
        case 2: e = launch_pass<2>(c, word, shift, c->offsets + (size_t)d * 256, counter, c->epoch); break;
        case 3: e = launch_pass<3>(c, word, shift, c->offsets + (size_t)d * 256, counter, c->epoch); break;
        case 4: e = launch_pass<4>(c, word, shift, c->offsets + (size_t)d * 256, counter, c->epoch); break;
        default: return fail(c, GK_E_ARG, "unsupported key width");
        }
        GK_TRY_HIP(c, e);
        timer_end(c, slot);
        c->cur ^= 1;
        ++pass;
    }
    return GK_OK;
}

}  // namespace gkm

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
#include <cstdlib>

#include "gkm_internal.h"
#include "gkm_onesweep.h"

namespace gkm {

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

// tile shape per key width: one-word keys use 1024 x 12 (12288 keys, 150 KB LDS, one workgroup per
// CU: fewest tiles and look-back hops, longest digit runs per write burst -- profiles/r1/
// radix_bench_variants.log); wider keys fall back to 256 x 16 to fit LDS.
template <int W>
struct PassShape {
    static constexpr int kThreads = 256, kItems = 16;
};
template <>
struct PassShape<1> {
    static constexpr int kThreads = 1024, kItems = 12;
};

template <int W>
static hipError_t launch_pass(gk_ctx *c, int word, int shift, const uint32_t *doff, uint32_t *counter, uint32_t epoch) {
    constexpr int T = PassShape<W>::kThreads, I = PassShape<W>::kItems;
    const uint64_t tiles = (c->n + (uint64_t)T * I - 1) / ((uint64_t)T * I);
    const int src = c->cur, dst = c->cur ^ 1;
    hipLaunchKernelGGL((onesweep_kernel<W, T, I, true>), dim3((unsigned)tiles), dim3(T), 0, c->stream, c->keys[src],
                       c->vals[src], c->keys[dst], c->vals[dst], c->n, word, shift, doff, c->status, counter, epoch);
    return hipGetLastError();
}

// Sort (keys[cur], vals[cur]) by the low total_bits of the W-word keys; result in keys/vals[cur].
hipError_t rank_mode_sort(int ballot) { return set_rank_ballot_here(ballot); }

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
        timer_units(c, slot, c->n);
        c->cur ^= 1;
        ++pass;
    }
    return GK_OK;
}

// The sorts of whole key arrays (the variable-length encodings, the prefix-doubling seeds and
// rank pairs): large one-word ones by MSD levels over the keys (msd_sort_keys: two global passes
// and the local rounds for 1e8 keys, where the LSD passes are one per 8 bits), the rest by
// radix_sort.  GKM_SORT_KEYS_LSD=1 keeps the LSD passes (A/B, tests).  Result in keys / vals[cur]
// either way; the MSD path also writes the group heads.
bool sort_keys_msd(const gk_ctx *c, uint64_t n, int words, int total_bits) {
    const bool lsd = opt("GKM_SORT_KEYS_LSD") != nullptr;  // (read per call: tests flip it)
    const char *tm = opt("GKM_MSD_KEYS_MIN");                // (tests: the MSD path at small n)
    const uint64_t nmin = tm ? std::strtoull(tm, nullptr, 10) : kMsdKeysMin;
    if (!(words == 1 && n >= nmin && n <= 0xFFFFFFFFull && !lsd)) return false;
    // the MSD levels pay off where the LSD passes (one per 8 bits) outnumber them by two or more:
    // msd_sort_keys takes L levels to ~400-key buckets, plus a count pass and the finishing round
    // (1e8 keys: L = 3; 24-bit keys (max 10) ran 3.67 ms against 2.90 by LSD, 45-bit ones 3.51
    // against 5.30, profiles/r4/keys_ab.txt)
    int b = 0;
    while (b < total_bits && (n >> b) > 400) ++b;
    const int L = std::max(1, (b + 7) / 8);
    return tm != nullptr || (total_bits + 7) / 8 >= L + 2;
}

int sort_keys(gk_ctx *c, int words, int total_bits, bool hist_ready) {
    if (sort_keys_msd(c, c->n, words, total_bits)) return msd_sort_keys(c, total_bits);
    return radix_sort(c, words, total_bits, hist_ready);
}

}  // namespace gkm

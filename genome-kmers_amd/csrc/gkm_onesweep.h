// gkm_onesweep.h -- one LSD radix pass over (W-word key, uint32 start) pairs, gfx950.
//
// Tile = THREADS x ITEMS keys, loaded wave-striped (item i of lane l in wave w is element
// w*ITEMS*64 + i*64 + l, so every load instruction is one contiguous 64-lane burst).
//   1. stable in-tile rank: per item one returning LDS atomic on the wave's counter of the digit
//      (rank_atomic, gkm_partition.h; waves own disjoint counters);
//   2. per-digit tile totals -> wave prefixes and tile-local digit starts (block scan);
//   3. decoupled look-back: the tile publishes its per-digit counts as epoch-tagged 64-bit words
//      (flag | epoch | value) with agent-scope relaxed atomics -- the word is its own flag, so no
//      fences are needed -- and sums predecessors' words until it meets an inclusive prefix;
//   4. keys are placed in LDS in digit order, then written so each digit run is a coalesced burst.
// LOOKBACK=false replaces step 3 by a fixed offset (timing experiments only: output is wrong).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gkm_partition.h"

namespace gkm {

constexpr uint64_t kFlagAgg = 1ull << 62;
constexpr uint64_t kFlagIncl = 2ull << 62;
constexpr uint64_t kValueMask = (1ull << 40) - 1;
constexpr uint32_t kEpochMask = (1u << 22) - 1;

__device__ __forceinline__ uint64_t pack_status(uint64_t flag, uint32_t epoch, uint64_t v) {
    return flag | ((uint64_t)(epoch & kEpochMask) << 40) | (v & kValueMask);
}

template <int W, int THREADS, int ITEMS>
struct OnesweepSmem {
    static constexpr int kTile = THREADS * ITEMS;
    static constexpr int kWaves = THREADS / 64;
    static constexpr int kStage = W * kTile * 8 + kTile * 4;
    static constexpr int kCounters = kWaves * 256 * 4;
    static constexpr int kUnion = kStage > kCounters ? kStage : kCounters;
};

template <int W>
__device__ __forceinline__ uint32_t digit_of(const uint64_t (&k)[W], int word, int shift) {
    uint32_t kw = 0;
#pragma unroll
    for (int w = 0; w < W; ++w)
        if (w == word) kw = (uint32_t)(k[w] >> shift) & 0xFFu;
    return kw;
}

template <int W, int THREADS, int ITEMS, bool LOOKBACK>
__global__ __launch_bounds__(THREADS) void onesweep_kernel(
    const uint64_t *__restrict__ kin, const uint32_t *__restrict__ vin, uint64_t *__restrict__ kout,
    uint32_t *__restrict__ vout, uint64_t n, int word, int shift, const uint32_t *__restrict__ doff,
    uint64_t *__restrict__ status, uint32_t *__restrict__ tile_counter, uint32_t epoch) {
    using SM = OnesweepSmem<W, THREADS, ITEMS>;
    constexpr int I = ITEMS;
    constexpr int TILE = SM::kTile;
    constexpr int NW = SM::kWaves;
    static_assert(THREADS >= 256, "one thread per digit");
    __shared__ __attribute__((aligned(16))) unsigned char s_raw[SM::kUnion];
    __shared__ uint32_t s_tile_start[256];
    __shared__ uint32_t s_gbase[256];
    __shared__ uint32_t s_wsum[4];
    __shared__ uint32_t s_tile;

    uint32_t *s_wc = reinterpret_cast<uint32_t *>(s_raw);  // [NW][256], alias of the staging area
    uint64_t *s_keys = reinterpret_cast<uint64_t *>(s_raw);
    uint32_t *s_vals = reinterpret_cast<uint32_t *>(s_raw + W * TILE * 8);

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;

    if (tid == 0) s_tile = atomicAdd(tile_counter, 1u);
    for (int i = tid; i < NW * 256; i += THREADS) s_wc[i] = 0;
    __syncthreads();
    const uint64_t tile = s_tile;
    const uint64_t base = tile * TILE;
    const uint64_t wbase = base + (uint64_t)wave * I * 64 + lane;

    uint64_t key[I][W];
    uint32_t val[I];
    uint32_t rank[I];
#pragma unroll
    for (int i = 0; i < I; ++i) {
        const uint64_t e = wbase + i * 64;
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

#pragma unroll
    for (int i = 0; i < I; ++i)  // stable rank: one returning LDS atomic (rank_atomic, gkm_partition.h)
        rank[i] = rank_atomic(s_wc + wave * 256, digit_of<W>(key[i], word, shift), wbase + i * 64 < n);
    __syncthreads();

    uint32_t total = 0;
    if (tid < 256) {
        const int d = tid;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            const uint32_t v = s_wc[w * 256 + d];
            s_wc[w * 256 + d] = total;
            total += v;
        }
        const uint32_t incl = wave_incl_scan(total);
        if (lane == 63) s_wsum[wave] = incl;
        s_tile_start[d] = incl - total;  // wave-local for now
    }
    __syncthreads();
    if (tid < 256) {
        const int d = tid;
        uint32_t wpre = 0;
        for (int w = 0; w < wave; ++w) wpre += s_wsum[w];
        s_tile_start[d] += wpre;

        uint64_t excl = 0;
        if (LOOKBACK) {
            uint64_t *st = status + tile * 256 + d;
            if (tile == 0) {
                __hip_atomic_store(st, pack_status(kFlagIncl, epoch, total), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            } else {
                __hip_atomic_store(st, pack_status(kFlagAgg, epoch, total), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
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
        } else {
            excl = (tile * TILE) / 256;  // timing only
        }
        s_gbase[d] = doff[d] + (uint32_t)excl;
    }
    __syncthreads();

    uint32_t slot[I];
#pragma unroll
    for (int i = 0; i < I; ++i) {
        const uint32_t kw = digit_of<W>(key[i], word, shift);
        slot[i] = s_tile_start[kw] + s_wc[wave * 256 + kw] + rank[i];
    }
    __syncthreads();
    const uint32_t tile_n = (uint32_t)((n - base) < (uint64_t)TILE ? (n - base) : (uint64_t)TILE);
#pragma unroll
    for (int i = 0; i < I; ++i) {
        if (wbase + i * 64 < n) {
#pragma unroll
            for (int w = 0; w < W; ++w) s_keys[w * TILE + slot[i]] = key[i][w];
            s_vals[slot[i]] = val[i];
        }
    }
    __syncthreads();

    for (uint32_t s = tid; s < tile_n; s += THREADS) {
        uint64_t kk[W];
#pragma unroll
        for (int w = 0; w < W; ++w) kk[w] = s_keys[w * TILE + s];
        const uint32_t kw = digit_of<W>(kk, word, shift);
        uint64_t o = (uint64_t)s_gbase[kw] + (s - s_tile_start[kw]);
        if (!LOOKBACK && o >= n) o -= n;
#pragma unroll
        for (int w = 0; w < W; ++w) kout[(uint64_t)w * n + o] = kk[w];
        vout[o] = s_vals[s];
    }
}

}  // namespace gkm

// gkm_partition.h -- stable one-digit partition of (64-bit key, uint32 start) tiles, gfx950.
//
// Shared by the MSD sort (gkm_msd.hip) and the timing tool (tools/radix_bench.hip), so the tool
// measures the production kernels.  MODE != 0 variants exist for timing experiments only and
// produce wrong output: 1 = no global stores, 2 = scatter straight from registers (no LDS staging).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gkm {

// workgroup barrier that orders LDS only: global stores stay in flight across it (__syncthreads
// would wait for every outstanding store of the wave before the barrier)
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// s_waitcnt immediate (gfx9 encoding) for vmcnt(0) with expcnt/lgkmcnt left at their maximum
constexpr int kVmcnt0 = 0x0F70;

// A digit is `w` bits of a B-bit key below its top `hi` bits (the bits already sorted).
struct Dig {
    int shift;
    uint32_t mask;
};

__host__ __device__ inline Dig dig_at(int B, int hi, int w) {
    int lo = B - hi - w;
    if (lo < 0) lo = 0;
    return Dig{lo, (uint32_t)((1ull << (B - hi - lo)) - 1)};
}

__device__ __forceinline__ uint32_t dg_of(uint64_t k, Dig d) { return (uint32_t)(k >> d.shift) & d.mask; }

// bucket-list entry: x = bucket start, y = len << 8 | hi << 1 | parity (hi = key bits already
// sorted, parity = the key/start buffer holding the bucket)
__host__ __device__ inline uint2 local_entry(uint32_t start, uint32_t len, int hi, int parity) {
    return make_uint2(start, (len << 8) | ((uint32_t)hi << 1) | (uint32_t)parity);
}

// ---------------------------------------------------------------------------------------------
// shared building blocks
// ---------------------------------------------------------------------------------------------
// lanes of the wave holding the same R-bit digit (and valid): R ballots; per bit the lane keeps
// the ballot or its complement via a sign-extended bit (one 3-input bitop per half)
template <int R>
__device__ __forceinline__ uint64_t match_peers(uint32_t d, bool valid) {
    const uint64_t v = __ballot(valid);
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
#pragma unroll
    for (int b = 0; b < R; ++b) {
        const uint32_t m = (uint32_t)(((int32_t)(d << (31 - b))) >> 31);  // 0 or ~0
        const uint64_t bb = __ballot(m != 0);
        lo &= ~((uint32_t)bb ^ m);
        hi &= ~((uint32_t)(bb >> 32) ^ m);
    }
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// stable 64-lane ranking of I wave-striped items by an R-bit digit (per-wave LDS counters):
// every lane reads its digit's counter, the first lane of each peer group bumps it.  LDS ops of
// one wave complete in order, so item i+1 reads item i's update.
template <int I, int R>
__device__ __forceinline__ void rank_items(const uint32_t (&dig)[I], const bool (&valid)[I], uint32_t *s_wc_wave,
                                           uint32_t (&rank)[I]) {
#pragma unroll
    for (int i = 0; i < I; ++i) {
        const uint64_t peers = match_peers<R>(dig[i], valid[i]);
        const uint32_t rank_in = lanes_below(peers);
        const uint32_t old = s_wc_wave[dig[i]];
        if (valid[i] && rank_in == 0) s_wc_wave[dig[i]] = old + (uint32_t)__popcll(peers);
        rank[i] = old + rank_in;
    }
}

template <int T, int I, int R>
struct PartSmem {
    static constexpr int kTile = T * I;
    static constexpr int kWaves = T / 64;
    static constexpr int kRadix = 1 << R;
    static constexpr int kValOff = (kTile + 2) * 8;           // keys [kTile + 1], then starts [kTile + 1]
    static constexpr int kStage = kValOff + (kTile + 1) * 4;  // (slot kTile: sink for invalid items)
    static constexpr int kCounters = kWaves * kRadix * 4;     // per-wave digit counters (aliased)
    static constexpr int kUnion = kStage > kCounters ? kStage : kCounters;
    static constexpr int kDPT = kRadix > T ? kRadix / T : 1;  // digits per thread in the scan
    static_assert(kRadix <= T || kRadix % T == 0, "digits split evenly over threads");
};

// Stable partition of one tile (item i of lane l in wave w = tile element w*I*64 + i*64 + l) by
// an R-bit digit d, in two halves so the caller can issue the next tile's loads in between:
//   partition_stage  rank in registers, tile digit starts, keys and starts into LDS in digit order
//   partition_store  coalesced runs from LDS to tile_off[digit] (global digit offsets of the tile)
// s_wc (= s_raw) must be zero on entry; s_toff holds the tile's global digit offsets.
// Barriers inside: all T threads must call.
// s_start[RADIX + 1] receives the tile-local digit starts (s_start[RADIX] = item count) and
// slot[] each item's staging slot (invalid items: the sink slot kTile); s_toff may be null.
template <int T, int I, int R>
__device__ __forceinline__ void partition_stage(const uint64_t (&key)[I], const uint32_t (&val)[I],
                                                const bool (&valid)[I], Dig d, unsigned char *s_raw,
                                                uint32_t *s_toff, uint32_t *s_wsum, uint32_t *s_start,
                                                uint32_t (&slot)[I]) {
    using SM = PartSmem<T, I, R>;
    constexpr int NW = SM::kWaves;
    constexpr int TILE = SM::kTile;
    constexpr int RADIX = SM::kRadix;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t *s_wc = reinterpret_cast<uint32_t *>(s_raw);
    uint64_t *s_keys = reinterpret_cast<uint64_t *>(s_raw);
    uint32_t *s_vals = reinterpret_cast<uint32_t *>(s_raw + SM::kValOff);

    uint32_t dig[I], rank[I];
#pragma unroll
    for (int i = 0; i < I; ++i) dig[i] = dg_of(key[i], d);
    rank_items<I, R>(dig, valid, s_wc + wave * RADIX, rank);
    lds_barrier();
    // per-digit totals over the waves -> per-wave exclusive prefixes; block scan over digits
    // (thread t owns digits t*K .. t*K+K-1, K = kDPT)
    constexpr int K = SM::kDPT;
    constexpr int ACT = RADIX / K;  // threads taking part
    uint32_t total[K], sum = 0, incl = 0;
    if (tid < ACT) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int dgt = tid * K + k;
            total[k] = 0;
#pragma unroll
            for (int w = 0; w < NW; ++w) {
                const uint32_t v = s_wc[w * RADIX + dgt];
                s_wc[w * RADIX + dgt] = total[k];
                total[k] += v;
            }
            sum += total[k];
        }
        incl = sum;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(incl, off);
            if (lane >= off) incl += y;
        }
        if (lane == 63) s_wsum[wave] = incl;
    }
    lds_barrier();
    if (tid < ACT) {
        uint32_t pre = 0;
        for (int w = 0; w < wave; ++w) pre += s_wsum[w];
        uint32_t run = pre + incl - sum;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int dgt = tid * K + k;
            s_start[dgt] = run;
            if (s_toff) s_toff[dgt] -= run;  // global offset of tile slot s = s_toff[digit] + s
            run += total[k];
        }
        if (tid == ACT - 1) s_start[RADIX] = run;
    }
    lds_barrier();
#pragma unroll
    for (int i = 0; i < I; ++i)
        slot[i] = valid[i] ? s_start[dig[i]] + s_wc[wave * RADIX + dig[i]] + rank[i] : (uint32_t)TILE;
    lds_barrier();  // counters consumed: the staging area is reused
#pragma unroll
    for (int i = 0; i < I; ++i) {  // branch-free: invalid items go to the sink slot
        s_keys[slot[i]] = key[i];
        s_vals[slot[i]] = val[i];
    }
    lds_barrier();
}

// Branch-free and fully unrolled, so the compiler's count of stores in flight is static (it can
// then wait for the next tile's loads without draining these stores): slots past cnt repeat the
// last valid element (an identical rewrite); an empty tile writes only to the sink element.
template <int T, int I, int R, int MODE>
__device__ __forceinline__ void partition_store(Dig d, const unsigned char *s_raw, const uint32_t *s_toff,
                                                uint32_t cnt, uint64_t sink, uint64_t *__restrict__ kout,
                                                uint32_t *__restrict__ vout, uint64_t seq_base = 0) {
    const uint64_t *s_keys = reinterpret_cast<const uint64_t *>(s_raw);
    const uint32_t *s_vals = reinterpret_cast<const uint32_t *>(s_raw + PartSmem<T, I, R>::kValOff);
#pragma unroll
    for (int j = 0; j < I; ++j) {
        const uint32_t s = min(threadIdx.x + j * T, cnt - 1);  // cnt == 0: s stays in the tile
        const uint64_t k = s_keys[s];
        const uint32_t v = s_vals[s];
        uint64_t o = cnt ? (uint64_t)(s_toff[dg_of(k, d)] + s) : sink;
        if (MODE == 3) o = seq_base + s;  // timing only: perfectly sequential runs
        if (MODE != 1 || o == 0xFFFFFFFFu) {
            kout[o] = k;
            vout[o] = v;
        }
    }
}

// persistent-grid tile order: XCD x (= block % 8) takes the x-th eighth of the tiles, so runs of
// neighbouring tiles meet in the same L2
struct TileWalk {
    uint32_t first, end, step;
    __device__ TileWalk(uint32_t ntiles) {
        const uint32_t x = blockIdx.x & 7, per = gridDim.x >> 3;
        first = (uint32_t)((uint64_t)ntiles * x / 8) + (blockIdx.x >> 3);
        end = (uint32_t)((uint64_t)ntiles * (x + 1) / 8);
        step = per;
    }
};

// ---------------------------------------------------------------------------------------------
// L>=1: partition big buckets; tiles never cross bucket boundaries
// ---------------------------------------------------------------------------------------------
template <int R>
__global__ __launch_bounds__(256) void msd_count_kernel(const uint32_t *__restrict__ t_start,
                                                        const uint32_t *__restrict__ t_count, Dig dl,
                                                        const uint64_t *__restrict__ kin,
                                                        uint32_t *__restrict__ tile_hist) {
    constexpr int RADIX = 1 << R;
    __shared__ uint32_t s_hist[RADIX];
    const int t = threadIdx.x;
    for (int i = t; i < RADIX; i += 256) s_hist[i] = 0;
    lds_barrier();
    const uint64_t b = t_start[blockIdx.x];
    const uint32_t m = t_count[blockIdx.x];
    for (uint32_t i = t; i < m; i += 256) atomicAdd(&s_hist[dg_of(kin[b + i], dl)], 1u);
    lds_barrier();
    for (int i = t; i < RADIX; i += 256) tile_hist[(uint64_t)blockIdx.x * RADIX + i] = s_hist[i];
}

// persistent: grid = a multiple of 8 blocks, each walks its XCD's tiles; the next tile's keys
// and starts are loaded while the current tile's runs are stored
template <int T, int I, int R, int MODE = 0>
__global__ __launch_bounds__(T) void msd_scatter_kernel(const uint32_t *__restrict__ t_start,
                                                        const uint32_t *__restrict__ t_count, Dig dl,
                                                        const uint32_t *__restrict__ tile_off,
                                                        const uint64_t *__restrict__ kin,
                                                        const uint32_t *__restrict__ vin, uint64_t *__restrict__ kout,
                                                        uint32_t *__restrict__ vout, uint32_t ntiles,
                                                        uint64_t sink) {
    using SM = PartSmem<T, I, R>;
    constexpr int RADIX = SM::kRadix;
    __shared__ __attribute__((aligned(16))) unsigned char s_raw[SM::kUnion];
    __shared__ uint32_t s_toff[RADIX];
    __shared__ uint32_t s_wsum[SM::kWaves];
    __shared__ uint32_t s_start[RADIX + 1];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t *s_wc = reinterpret_cast<uint32_t *>(s_raw);
    const TileWalk walk(ntiles);
    uint64_t key[I];
    uint32_t val[I], m = 0, toff = 0;
    auto load = [&](uint32_t t) {
        const uint64_t b = t_start[t];
        m = t_count[t];  // >= 1
        toff = tile_off[(uint64_t)t * RADIX + (tid & (RADIX - 1))];  // every lane loads: no branch
        uint32_t q0 = wave * (I * 64) + lane;
        asm volatile("" : "+v"(q0));  // keep the per-item offsets inside the loop (no hoisting)
#pragma unroll
        for (int i = 0; i < I; ++i) {
            const uint64_t e = b + min(q0 + i * 64, m - 1);  // clamped: loads stay branch-free
            key[i] = kin[e];
            val[i] = vin[e];
        }
    };
    if (walk.first < walk.end) load(walk.first);
    // drain the prologue loads so the loop-entry wait state equals the back-edge one (loads done,
    // stores of the previous tile in flight): the compiler then never waits for stores in the loop
    __builtin_amdgcn_s_waitcnt(kVmcnt0);
    for (uint32_t t = walk.first; t < walk.end; t += walk.step) {
        lds_barrier();  // the previous tile's runs have been read out of LDS
        for (int i = tid; i < SM::kWaves * RADIX; i += T) s_wc[i] = 0;
        if (tid < RADIX) s_toff[tid] = toff;
        lds_barrier();
        bool valid[I];
#pragma unroll
        for (int i = 0; i < I; ++i) valid[i] = (uint32_t)(wave * (I * 64) + i * 64 + lane) < m;
        uint32_t slot[I];
        partition_stage<T, I, R>(key, val, valid, dl, s_raw, s_toff, s_wsum, s_start, slot);
        const uint32_t cnt = s_start[RADIX];
        const uint64_t seq = (uint64_t)t * (T * I);
        if (t + walk.step < walk.end) load(t + walk.step);
        partition_store<T, I, R, MODE>(dl, s_raw, s_toff, cnt, sink, kout, vout, seq);
    }
}

}  // namespace gkm

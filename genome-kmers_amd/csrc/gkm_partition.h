// gkm_partition.h -- stable one-digit partition of (64-bit key, uint32 start) tiles, gfx950.
//
// Shared by the MSD sort (gkm_msd.hip) and the timing tool (tools/radix_bench.hip), so the tool
// measures the production kernels.  MODE != 0 variants exist for timing experiments only and
// produce wrong output: 1 = no global stores, 2 = scatter straight from registers (no LDS staging).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gkm {

// global-memory views of device pointers: the kernels' arguments are generic pointers, and
// where the compiler cannot infer that one stays global (a pointer chosen at run time, a
// reinterpretation) it emits flat loads / stores, which wait for LDS and memory counters together
template <class T>
__device__ __forceinline__ __attribute__((address_space(1))) T *gmem(T *p) {
    return (__attribute__((address_space(1))) T *)p;
}
typedef __attribute__((address_space(1))) const uint64_t gu64;
typedef __attribute__((address_space(1))) const uint8_t gu8;
typedef __attribute__((address_space(1))) const uint32_t __attribute__((aligned(1))) gu32u;  // unaligned

// workgroup barrier that orders LDS only: global stores stay in flight across it (__syncthreads
// would wait for every outstanding store of the wave before the barrier)
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// s_waitcnt immediate (gfx9 encoding) for vmcnt(0) with expcnt/lgkmcnt left at their maximum
constexpr int kVmcnt0 = 0x0F70;
// ... and for vmcnt(v), v < 64 (vmcnt bits [3:0] and [15:14])
constexpr int vmcnt_imm(int v) { return kVmcnt0 | (v & 15) | ((v >> 4) << 14); }

// A digit is `w` bits of a B-bit key below its top `hi` bits (the bits already sorted).
struct Dig {
    int shift;
    uint32_t mask;
};

__host__ __device__ inline Dig dig_at(int B, int hi, int w) {
    if (hi >= B) return Dig{0, 0u};  // no bits left: every key has digit 0
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
__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Stable rank of a wave-striped item by its digit, ONE LDS instruction: every valid lane adds 1 to
// its digit's counter with a returning atomic and gets the counter's value before its add.  The
// LDS of gfx950 applies the same-address lanes of one wave instruction in increasing lane order, so
// that value is the count before the instruction plus the lanes below with the same digit -- the
// stable rank.  Successive items of a wave accumulate in order (one wave's LDS operations complete
// in order).  A ballot-match takes R + 1 ballots per item and the LDS-mask round trip five LDS
// instructions (tools/lds_rank_probe.hip: 3.9 vs 0.88 T items/s chip-wide).  The lane order is a
// hardware property, not an ISA guarantee: gk_create checks it once per device and process
// (gkm_capi.hip, lds_rank_check) over every digit width the partitions use, and where it does not
// hold switches every partition to the ballot-match ranking below (g_rank_ballot), which relies
// on nothing but ballots: the same ranks, slower.
//
// g_rank_ballot: one copy per code object (every .hip file that ranks sets its own, gk_create ->
// rank_mode_*); read once per kernel into an SGPR, the test is one scalar branch per item.
static __constant__ int g_rank_ballot = 0;

// Ballot-match rank: the valid lanes with this lane's digit (digits of up to DB bits) by DB
// ballots, the rank among them by mbcnt, and one returning atomic per distinct digit, from the
// lowest such lane (distinct addresses: lane order cannot matter), whose pre-add count is then
// broadcast to its peers.  P16: the counters are u16 halves of u32 words (rank_atomic16).
template <int DB = 10, bool P16 = false>
__device__ __forceinline__ uint32_t rank_ballot(uint32_t *wc, uint32_t d, bool valid) {
    uint64_t m = __ballot(valid);
#pragma unroll
    for (int b = 0; b < DB; ++b) {
        const uint64_t x = __ballot((d >> b) & 1u);
        m &= ((d >> b) & 1u) ? x : ~x;
    }
    const uint32_t below = lanes_below(m);
    uint32_t old = 0;
    if (valid && below == 0) {
        if (P16) {
            const uint32_t sh = (d & 1u) << 4;
            old = (atomicAdd(&wc[d >> 1], (uint32_t)__popcll(m) << sh) >> sh) & 0xFFFFu;
        } else {
            old = atomicAdd(&wc[d], (uint32_t)__popcll(m));
        }
    }
    const int leader = m ? __builtin_ctzll(m) : 0;
    old = (uint32_t)__builtin_amdgcn_ds_bpermute(leader << 2, (int)old);
    return valid ? old + below : 0u;
}

__device__ __forceinline__ uint32_t rank_atomic(uint32_t *wc, uint32_t d, bool valid) {
    if (__builtin_expect(g_rank_ballot != 0, 0)) return rank_ballot(wc, d, valid);
    return valid ? atomicAdd(&wc[d], 1u) : 0u;
}

// The same rank with 16-bit counters, two digits per u32 word (digit d: half d & 1 of word d >> 1),
// for digit spaces whose per-wave u32 counters would not fit the LDS (2^11 digits x 16 waves).
// Counts stay below 2^16 (a wave ranks at most 64 I items), so an add never carries into the
// other half; the lane-order property is the same one (same-address lanes of one instruction,
// whatever they add), checked by lds_rank_check in this form too.
template <int DB = 11>
__device__ __forceinline__ uint32_t rank_atomic16(uint32_t *wc, uint32_t d, bool valid) {
    if (__builtin_expect(g_rank_ballot != 0, 0)) return rank_ballot<DB, true>(wc, d, valid);
    const uint32_t sh = (d & 1u) << 4;
    return valid ? (atomicAdd(&wc[d >> 1], 1u << sh) >> sh) & 0xFFFFu : 0u;
}

// host: switch this code object's partitions to the ballot-match ranking (or back)
static inline hipError_t set_rank_ballot_here(int on) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_rank_ballot), &on, sizeof(int));
}

// ranks of I items (items >= live hold no valid element: skipped, wave-uniform)
template <int I>
__device__ __forceinline__ void rank_items(const uint32_t (&dig)[I], const bool (&valid)[I], uint32_t *s_wc_wave,
                                           uint32_t (&rank)[I], int live = I) {
#pragma unroll
    for (int i = 0; i < I; ++i) {
        rank[i] = 0;
        if (i >= live) continue;
        rank[i] = rank_atomic(s_wc_wave, dig[i], valid[i]);
    }
}

// inclusive scan of one u32 per lane over the wave, VALU only: row_shr 1/2/4/8 inside rows of 16
// lanes, then the gfx9 DPP row broadcasts row_bcast:15 and row_bcast:31 (rocPRIM's gfx9 warp scan)
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    const int lane = threadIdx.x & 63, rl = lane & 15;
    uint32_t t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);
    if (rl >= 1) v += t;
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);
    if (rl >= 2) v += t;
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);
    if (rl >= 4) v += t;
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);
    if (rl >= 8) v += t;
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xf, 0xf, false);  // row_bcast:15
    if (lane & 16) v += t;
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xf, 0xf, false);  // row_bcast:31
    if (lane >= 32) v += t;
    return v;
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
// live (wave-uniform): items >= live of this wave hold no valid element and are skipped.
// PROF (timing builds of tools/radix_bench only): thread 0 adds the clock ticks of each phase to
// prof[0..3] (rank, scan, slots, staging).
template <int T, int I, int R, bool PROF = false>
__device__ __forceinline__ void partition_stage(const uint64_t (&key)[I], const uint32_t (&val)[I],
                                                const bool (&valid)[I], Dig d, unsigned char *s_raw,
                                                uint32_t *s_toff, uint32_t *s_wsum, uint32_t *s_start,
                                                uint32_t (&slot)[I], unsigned long long *prof = nullptr,
                                                int live = I) {
    using SM = PartSmem<T, I, R>;
    constexpr int NW = SM::kWaves;
    constexpr int TILE = SM::kTile;
    constexpr int RADIX = SM::kRadix;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t *s_wc = reinterpret_cast<uint32_t *>(s_raw);
    uint64_t *s_keys = reinterpret_cast<uint64_t *>(s_raw);
    uint32_t *s_vals = reinterpret_cast<uint32_t *>(s_raw + SM::kValOff);

    uint64_t t0 = PROF ? clock64() : 0;
    auto mark = [&](int ph) {
        if (PROF && tid == 0) {
            const uint64_t t1 = clock64();
            atomicAdd(&prof[ph], (unsigned long long)(t1 - t0));
            t0 = t1;
        }
    };
    uint32_t dig[I], rank[I];
#pragma unroll
    for (int i = 0; i < I; ++i) dig[i] = dg_of(key[i], d);
    rank_items<I>(dig, valid, s_wc + wave * RADIX, rank, live);
    lds_barrier();
    mark(0);
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
        incl = wave_incl_scan(sum);
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
    mark(1);
#pragma unroll
    for (int i = 0; i < I; ++i)
        slot[i] = valid[i] ? s_start[dig[i]] + s_wc[wave * RADIX + dig[i]] + rank[i] : (uint32_t)TILE;
    lds_barrier();  // counters consumed: the staging area is reused
    mark(2);
#pragma unroll
    for (int i = 0; i < I; ++i) {  // invalid items go to the sink slot
        if (i >= live) continue;
        s_keys[slot[i]] = key[i];
        s_vals[slot[i]] = val[i];
    }
    lds_barrier();
    mark(3);
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
    // in groups of G slots: all key / start reads, then all digit-offset reads, then the stores,
    // so each group pays the LDS latency twice instead of every slot
    constexpr int G = (I % 6 == 0) ? 6 : ((I % 4 == 0) ? 4 : 1);
#pragma unroll
    for (int j0 = 0; j0 < I; j0 += G) {
        uint32_t s[G], v[G], o[G];
        uint64_t k[G];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            s[g] = min(threadIdx.x + (j0 + g) * T, cnt - 1);  // cnt == 0: s stays in the tile
            k[g] = s_keys[s[g]];
            v[g] = s_vals[s[g]];
        }
#pragma unroll
        for (int g = 0; g < G; ++g) o[g] = s_toff[dg_of(k[g], d)] + s[g];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            uint64_t oo = cnt ? (uint64_t)o[g] : sink;
            if (MODE == 3) oo = seq_base + s[g];  // timing only: perfectly sequential runs
            if (MODE != 1 || oo == 0xFFFFFFFFu) {
                kout[oo] = k[g];
                vout[oo] = v[g];
            }
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

// the count pass when the previous pass wrote the digits (NextDigits): 1 byte per key
template <int R>
__global__ __launch_bounds__(256) void msd_count_nd_kernel(const uint32_t *__restrict__ t_start,
                                                           const uint32_t *__restrict__ t_count,
                                                           const uint8_t *__restrict__ nd,
                                                           uint32_t *__restrict__ tile_hist) {
    constexpr int RADIX = 1 << R;
#ifndef GKM_COUNT_COPIES
#define GKM_COUNT_COPIES 1
#endif
    // NC interleaved histogram copies (digit d, copy c at NC d + c; copy = thread % NC): lanes of
    // one atomic that share a digit land on NC different words in NC banks
    constexpr int NC = GKM_COUNT_COPIES;
    __shared__ uint32_t s_hist[RADIX * NC];
    const int t = threadIdx.x;
    for (int i = t; i < RADIX * NC; i += 256) s_hist[i] = 0;
    lds_barrier();
    uint32_t *hc = s_hist + (t & (NC - 1));
    const uint64_t b = t_start[blockIdx.x];
    const uint32_t m = t_count[blockIdx.x];
    // 16 digits per load where the run is 16-byte aligned (a tile's ~11 K digits: <= 3 loads per
    // thread, all in flight together), bytes at the ragged ends
    const uint32_t head = min<uint32_t>((uint32_t)((16 - ((uintptr_t)(nd + b) & 15)) & 15), m);
    const uint32_t quads = (m - head) >> 4;
    const uint4 *w = reinterpret_cast<const uint4 *>(nd + b + head);
    if (t < (int)head) atomicAdd(&hc[NC * nd[b + t]], 1u);
    for (uint32_t i0 = 0; i0 < quads; i0 += 3 * 256) {
        uint4 x4[3];
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            const uint32_t i = i0 + r * 256 + t;
            x4[r] = i < quads ? w[i] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            if (i0 + r * 256 + t >= quads) continue;
            const uint32_t xs[4] = {x4[r].x, x4[r].y, x4[r].z, x4[r].w};
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                atomicAdd(&hc[NC * (xs[u] & 0xFF)], 1u);
                atomicAdd(&hc[NC * ((xs[u] >> 8) & 0xFF)], 1u);
                atomicAdd(&hc[NC * ((xs[u] >> 16) & 0xFF)], 1u);
                atomicAdd(&hc[NC * (xs[u] >> 24)], 1u);
            }
        }
    }
    const uint32_t tail0 = head + 16 * quads;  // < 16 bytes left
    if (tail0 + t < m) atomicAdd(&hc[NC * nd[b + tail0 + t]], 1u);
    lds_barrier();
    for (int i = t; i < RADIX; i += 256) {
        uint32_t v = 0;
#pragma unroll
        for (int c = 0; c < NC; ++c) v += s_hist[NC * i + c];
        tile_hist[(uint64_t)blockIdx.x * RADIX + i] = v;
    }
}

// persistent: grid = a multiple of 8 blocks, each walks its XCD's tiles; the next tile's keys
// and starts are loaded while the current tile's runs are stored
template <int T, int I, int R, int MODE = 0, bool PROF = false>
__global__ __launch_bounds__(T) void msd_scatter_kernel(const uint32_t *__restrict__ t_start,
                                                        const uint32_t *__restrict__ t_count, Dig dl,
                                                        const uint32_t *__restrict__ tile_off,
                                                        const uint64_t *__restrict__ kin,
                                                        const uint32_t *__restrict__ vin, uint64_t *__restrict__ kout,
                                                        uint32_t *__restrict__ vout, uint32_t ntiles,
                                                        uint64_t sink, unsigned long long *prof = nullptr,
                                                        int stagger = 0) {
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
    // stagger (experiments): the second half of the grid starts later, so workgroups sharing a CU
    // run their compute and memory phases out of step
    if (stagger && blockIdx.x >= gridDim.x / 2)
        for (int i = 0; i < stagger; ++i) __builtin_amdgcn_s_sleep(127);
    if (walk.first < walk.end) load(walk.first);
    // drain the prologue loads so the loop-entry wait state equals the back-edge one (loads done,
    // stores of the previous tile in flight): the compiler then never waits for stores in the loop
    __builtin_amdgcn_s_waitcnt(kVmcnt0);
    uint64_t tp = PROF ? clock64() : 0;
    for (uint32_t t = walk.first; t < walk.end; t += walk.step) {
        lds_barrier();  // the previous tile's runs have been read out of LDS
        if (PROF && tid == 0) {  // phase 5: previous store loop issue + this top barrier
            const uint64_t t1 = clock64();
            atomicAdd(&prof[5], (unsigned long long)(t1 - tp));
            tp = t1;
        }
        for (int i = tid; i < SM::kWaves * RADIX; i += T) s_wc[i] = 0;
        if (tid < RADIX) s_toff[tid] = toff;
        lds_barrier();
        if (PROF && tid == 0) {  // phase 4: counter reset (+ the wait for this tile's loads)
            const uint64_t t1 = clock64();
            atomicAdd(&prof[4], (unsigned long long)(t1 - tp));
            tp = t1;
        }
        bool valid[I];
#pragma unroll
        for (int i = 0; i < I; ++i) valid[i] = (uint32_t)(wave * (I * 64) + i * 64 + lane) < m;
        uint32_t slot[I];
        partition_stage<T, I, R, PROF>(key, val, valid, dl, s_raw, s_toff, s_wsum, s_start, slot, prof);
        if (PROF) tp = clock64();
        const uint32_t cnt = s_start[RADIX];
        const uint64_t seq = (uint64_t)t * (T * I);
        if (t + walk.step < walk.end) load(t + walk.step);
        partition_store<T, I, R, MODE>(dl, s_raw, s_toff, cnt, sink, kout, vout, seq);
    }
}

// ---------------------------------------------------------------------------------------------
// Software-pipelined partition: the previous tile's stores overlap this tile's load wait and its
// ranking.  Digit counters have their own LDS (not aliased with the staging area), so the staged
// previous tile can be stored while this tile is ranked:
//   top    zero this wave's counters; digit offsets of this tile into s_toff[cur]
//   B      PRE store groups of the previous tile (this tile's loads are still in flight), then
//          rank item i interleaved with store group PRE + i
//   C      scan -> tile digit starts, s_toff[cur] -= start          (barrier before and after)
//   D      slots, staging of this tile (its count kept for the next iteration), barrier
//   E      loads of the next tile
// The last tile's stores follow the loop.  R-bit digits, one thread per digit (T >= 2^R).
// ---------------------------------------------------------------------------------------------
template <int T, int I>
struct PipeSmem {
    static constexpr int kTile = T * I;
    static constexpr int kWaves = T / 64;
    static constexpr int kValOff = (kTile + 2) * 8;
    static constexpr int kStage = kValOff + (kTile + 1) * 4;
};

// the next level's digit of every stored key, one byte per element at the key's output index, so
// that level's count pass reads 1 byte per key instead of 8 (ND = false: not written)
struct NextDigits {
    Dig d;
    uint8_t *out;
    // MODE 4 (a compact level, gkm_msd.hip): kout[] gets the key bits below the next digit
    // (lowmask) in the high half and the start in the low half; vout[] is not written
    uint32_t lowmask = 0;
    // MODE 5 (a packed-pair level, gkm_msd.hip): the rem = 64 - pshi key bits below the sorted ones
    // and the start in 80 bits -- kout[] = low key bits << pshi | start >> (32 - pshi), out16[] =
    // the start's low 32 - pshi bits; vout[] is not written
    uint16_t *out16 = nullptr;
    int pshi = 0;
    // INP == 2 (a level behind the packed L0, gkm_msd.hip): the input's top key byte, one per element
    const uint8_t *in8 = nullptr;
};

// a packed-pair element (MODE 5's output) -> (key bits below the sorted ones, start)
__device__ __forceinline__ void unpack_pair(uint64_t a, uint32_t b16, int shi, uint64_t &key, uint32_t &val) {
    key = a >> shi;
    val = ((uint32_t)(a & ((1ull << shi) - 1)) << (32 - shi)) | b16;
}

template <int T, int I, int R, int MODE, bool ND>
__device__ __forceinline__ void pipe_store(int g, Dig d, const uint64_t *s_keys, const uint32_t *s_vals,
                                           const uint32_t *toff, uint32_t cnt, uint64_t sink,
                                           uint64_t *__restrict__ kout, uint32_t *__restrict__ vout,
                                           NextDigits nd, uint32_t base = 0) {
    const uint32_t s = min((uint32_t)(threadIdx.x + g * T), cnt - 1);  // cnt == 0: stays in the tile
    const uint64_t k = s_keys[s];
    const uint32_t v = s_vals[s];
    const uint64_t o = cnt ? (uint64_t)(toff[dg_of(k, d)] + base + s) : sink;
    if (MODE == 4) {  // compact: (low key bits << 32 | start) in the key array, the next digit byte
        kout[o] = ((uint64_t)((uint32_t)k & nd.lowmask) << 32) | v;
        nd.out[o] = (uint8_t)dg_of(k, nd.d);
    } else if (MODE == 5) {  // packed pair: 10 bytes (+ the next digit byte) instead of 12
        const int shi = nd.pshi;
        kout[o] = ((k & ((1ull << (64 - shi)) - 1)) << shi) | (v >> (32 - shi));
        nd.out16[o] = (uint16_t)(v & ((1u << (32 - shi)) - 1));
        nd.out[o] = (uint8_t)dg_of(k, nd.d);
    } else if (MODE != 1 || o == 0xFFFFFFFFu) {
        kout[o] = k;
        vout[o] = v;
        if (ND) nd.out[o] = (uint8_t)dg_of(k, nd.d);
    }
}

// INP (input format): 0 = (key, start); 1 = packed pairs (a MODE 5 level's output: kin[] + in16[],
// key bits below the sorted ones); 2 = packed pairs below a digit byte (the packed L0's output,
// gkm_msd.hip: nd.in8[] holds the top 8 of the unsorted key bits, kin[] the rest above the start's
// high bits, in16[] the start's low bits).  Only a compact (MODE 4) or packed-pair output, which
// never store the sorted bits, may read packed input.
template <int T, int I, int R = 8, int MODE = 0, bool ND = false, int PRE_ = 0, int INP = 0>
__global__ __launch_bounds__(T) void msd_pipe_kernel(const uint32_t *__restrict__ t_start,
                                                     const uint32_t *__restrict__ t_count, Dig dl,
                                                     const uint32_t *__restrict__ tile_off,
                                                     const uint64_t *__restrict__ kin, const uint32_t *__restrict__ vin,
                                                     uint64_t *__restrict__ kout, uint32_t *__restrict__ vout,
                                                     uint32_t ntiles, uint64_t sink, NextDigits nd = {},
                                                     const uint16_t *__restrict__ in16 = nullptr, int in_shi = 0) {
    static_assert(INP == 0 || MODE == 4 || MODE == 5, "packed-pair input keeps only the unsorted key bits");
    using SM = PipeSmem<T, I>;
    constexpr int NW = SM::kWaves;
    constexpr int TILE = SM::kTile;
    constexpr int PRE = PRE_ ? PRE_ : (I + 2) / 3;  // store groups issued before the ranking starts
    constexpr int RADIX = 1 << R;
    static_assert(T >= RADIX, "one thread per digit");
    __shared__ __attribute__((aligned(16))) unsigned char s_stage[SM::kStage];
    __shared__ uint32_t s_wc[NW * RADIX];
    __shared__ uint32_t s_toff[2][RADIX];
    __shared__ uint32_t s_start[RADIX + 1];
    __shared__ uint32_t s_wsum[RADIX / 64 > 0 ? RADIX / 64 : 1];
    uint64_t *s_keys = reinterpret_cast<uint64_t *>(s_stage);
    uint32_t *s_vals = reinterpret_cast<uint32_t *>(s_stage + SM::kValOff);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const TileWalk walk(ntiles);
    uint64_t key[I];
    uint32_t val[I], m = 0, toff = 0;
    auto load = [&](uint32_t t) {
        toff = tile_off[(uint64_t)t * RADIX + (tid & (RADIX - 1))];  // first: waiting for it leaves the keys in flight
        const uint64_t b = t_start[t];
        m = t_count[t];  // >= 1
        uint32_t q0 = wave * (I * 64) + lane;
        asm volatile("" : "+v"(q0));
#pragma unroll
        for (int i = 0; i < I; ++i) {
            const uint64_t e = b + min(q0 + i * 64, m - 1);
            if (INP == 1) {
                key[i] = kin[e];  // packed pair: unpacked at the item's first use (the rank loop)
                val[i] = in16[e];
            } else if (INP == 2) {  // + the digit byte above it, kept in val's high half until then
                key[i] = kin[e];
                val[i] = in16[e] | ((uint32_t)nd.in8[e] << 16);
            } else {
                key[i] = kin[e];
                val[i] = vin[e];
            }
        }
    };
    uint32_t pcnt = 0;  // staged elements of the previous tile (0: none -> stores go to the sink)
    int cur = 0;
    if (walk.first < walk.end) load(walk.first);
    __builtin_amdgcn_s_waitcnt(kVmcnt0);
    for (uint32_t t = walk.first; t < walk.end; t += walk.step) {
        uint32_t *wc = s_wc + wave * RADIX;
#pragma unroll
        for (int u = 0; u < (RADIX + 63) / 64; ++u)
            if (u * 64 + lane < RADIX) wc[u * 64 + lane] = 0;
        if (tid < RADIX) s_toff[cur][tid] = toff;
        const uint32_t *ptoff = s_toff[cur ^ 1];
#pragma unroll
        for (int g = 0; g < PRE; ++g) pipe_store<T, I, R, MODE, ND>(g, dl, s_keys, s_vals, ptoff, pcnt, sink, kout, vout, nd);
        bool valid[I];
        uint32_t dig[I], rank[I];
#pragma unroll
        for (int i = 0; i < I; ++i) {
            valid[i] = (uint32_t)(wave * (I * 64) + i * 64 + lane) < m;
            if (INP == 1) unpack_pair(key[i], val[i], in_shi, key[i], val[i]);  // (at the item's first use)
            if (INP == 2) {
                const uint64_t top = (uint64_t)(val[i] >> 16) << (64 - in_shi);
                unpack_pair(key[i], val[i] & 0xFFFFu, in_shi, key[i], val[i]);
                key[i] |= top;
            }
            dig[i] = dg_of(key[i], dl);
            rank[i] = rank_atomic(wc, dig[i], valid[i]);
            if (PRE + i < I) pipe_store<T, I, R, MODE, ND>(PRE + i, dl, s_keys, s_vals, ptoff, pcnt, sink, kout, vout, nd);
        }
        lds_barrier();  // ranks final; the previous tile's staging has been read out
        uint32_t total = 0, incl = 0;
        if (tid < RADIX) {
#pragma unroll
            for (int w = 0; w < NW; ++w) {
                const uint32_t v = s_wc[w * RADIX + tid];
                s_wc[w * RADIX + tid] = total;
                total += v;
            }
            incl = wave_incl_scan(total);
            if (lane == 63) s_wsum[wave] = incl;
        }
        lds_barrier();
        if (tid < RADIX) {
            uint32_t pre = 0;
            for (int w = 0; w < wave; ++w) pre += s_wsum[w];
            const uint32_t st = pre + incl - total;
            s_start[tid] = st;
            s_toff[cur][tid] -= st;
            if (tid == RADIX - 1) s_start[RADIX] = pre + incl;
        }
        lds_barrier();
#pragma unroll
        for (int i = 0; i < I; ++i) {
            const uint32_t sl = valid[i] ? s_start[dig[i]] + wc[dig[i]] + rank[i] : (uint32_t)TILE;
            s_keys[sl] = key[i];
            s_vals[sl] = val[i];
        }
        pcnt = s_start[RADIX];
        lds_barrier();  // staging complete; counters read
        if (t + walk.step < walk.end) load(t + walk.step);
        cur ^= 1;
    }
    if (walk.first < walk.end) {
        const uint32_t *ptoff = s_toff[cur ^ 1];
#pragma unroll
        for (int g = 0; g < I; ++g) pipe_store<T, I, R, MODE, ND>(g, dl, s_keys, s_vals, ptoff, pcnt, sink, kout, vout, nd);
    }
}

}  // namespace gkm

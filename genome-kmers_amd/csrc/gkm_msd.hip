// gkm_msd.hip -- MSD radix sort of one-word k-mer keys (the C3 hot path), gfx950.
//
// An LSD sort of 62-bit keys moves every (key, start) pair 8 times.  Here each pass partitions
// only what is still unsorted, and buckets small enough for LDS are finished there:
//   L0     encode + partition by the top 8 bits, straight from the sequence byte array
//   L1..   partition every bucket larger than kBlockMax by the next 8 bits
//   local  buckets of kWaveMax+1..kBlockMax elements: one 256-thread workgroup each; buckets of
//          1..kWaveMax: one wave each.  The bucket is partitioned by its next digit in LDS,
//          sub-buckets of <= kSmall are finished by rank-by-count, and the bucket is written
//          back once, with its group-head flags; larger sub-buckets go to another round.
// For 3.1e9 random 31-mers: L0, L1, L2 and one wave-local round -- 4 movements of the data.
//
// Order contract: equal keys come out by ascending start index, the reference's break_ties=True
// order (kmers.py:1710-1711).  Every partition here is STABLE (64-lane ballot-match ranking,
// tiles and workgroups in input order) and the L0 input is in ascending start order, so equal
// keys stay in start order without ever comparing starts; a sub-bucket whose key bits are
// exhausted is final as it stands.  Every global partition offset is known before its scatter
// starts (count pass + column scan of per-tile digit histograms): no look-back chain.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "gkm_canon.h"
#include "gkm_internal.h"
#include "gkm_partition.h"
#include "gkm_swar.h"

namespace gkm {

constexpr int kGR = 8;                  // global digit bits
constexpr int kGRadix = 1 << kGR;
// global partition tile: 1024 threads x 11 keys (tuning overrides GKM_PT / GKM_PI: tools/build_variant.sh)
#ifndef GKM_PT
#define GKM_PT 1024
#endif
#ifndef GKM_PI
#define GKM_PI 11
#endif
constexpr int kPT = GKM_PT, kPI = GKM_PI;
// wide L0 (msd0_wide_kernel): 11-bit digits over 18,432-position tiles of its own, 512 threads x 36
constexpr int kWideL0 = 11, kWT = 512, kWI = 36;
constexpr int kPTile = kPT * kPI;
constexpr int kChunkTiles = 256;        // tiles per scan chunk (GKM_TEST_CHUNK_TILES overrides: tests only)
constexpr int kBT = 512, kBI = 8, kBR = 8;    // block-local: 512 threads x 8 keys, 8-bit digit
constexpr int kBT2 = 1024, kBR2 = 10;         // big block-local: 1024 threads x 8 keys, 10-bit digit
                                              // (~5.9 K keys over 1024 digits: sub-buckets of ~6,
                                              // finished by rank-by-count, few re-listed)
constexpr int kBlockMax = kBT2 * kBI;   // 8192: larger buckets take another global level
// local finishing classes by bucket size: one wave x 4, 8 or 16 keys (msd_wave_kernel), 512
// threads x 8 keys (msd_local_kernel, <= 4096), 4 = tiny (<= kTiny elements: one thread per
// bucket), 5 = 1024 threads x 8 keys (<= 8192: the buckets an 11-bit L0 + one level leave at C3)
constexpr int kLocal = 6;
constexpr int kTiny = 8;
constexpr int kSmall = 24;
// waves per SIMD the wave-local kernels' registers are capped for (msd_wave_kernel<I, W, .>); the
// LDS (7.2 KB per wave at I = 8) admits 5 per SIMD
#ifndef GKM_WAVE_OCC8
#define GKM_WAVE_OCC8 4
#endif
constexpr int kWaveOcc4 = 6, kWaveOcc8 = GKM_WAVE_OCC8, kWaveOcc16 = 3;
// digit bits of the wave-local kernels' in-LDS partition: buckets of ~370 keys (C3) over 512
// digits leave sub-buckets of ~0.7 keys (rank-by-count reads half of what 256 digits need)
#ifndef GKM_WAVE_R8
#define GKM_WAVE_R8 9
#endif
constexpr int kWaveR4 = 8, kWaveR8 = GKM_WAVE_R8, kWaveR16 = 10;
// later local rounds (buckets re-listed because a sub-bucket outgrew kSmall: repeat families) and
// later phases finish sub-buckets of up to kSmallLate by rank-by-count instead of re-listing them
// for another round -- a round costs a bucket load, ranking and write-back per bucket
constexpr int kSmallLate = 96;
// The local rounds write back the keys of a bucket only when some of its elements are re-listed
// (rare): the sort's product is the start order (+ group heads), and keys are re-encoded from the
// sorted starts when an API call needs them (gk_ctx::keys_stale).
constexpr int kMaxLevels = 16;              // sub-buckets <= this: rank-by-count

__constant__ uint8_t c_code4_msd[256];
static bool g_msd_tables = false;

static hipError_t msd_tables() {
    if (g_msd_tables) return hipSuccess;
    uint8_t code4[256] = {0};
    const char *order = "ABCDGHKMNRSTVWY";
    for (int i = 0; order[i]; ++i) code4[(uint8_t)order[i]] = (uint8_t)(i + 1);
    hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(c_code4_msd), code4, 256);
    if (e == hipSuccess) g_msd_tables = true;
    return e;
}

// ---------------------------------------------------------------------------------------------
// L0: keys straight from the sequence byte array
// ---------------------------------------------------------------------------------------------
// A tile's bases are first packed into LDS: symbol codes MSB-first (64/BITS per word) and a '$'
// bitmask (32 positions per word).  The key of position p is then one funnel shift of two code
// words, and p is a valid start iff the S mask bits from p are all zero ('$' ends a contig; the
// pad after the array is '$').
struct L0Args {
    const uint8_t *sba;
    uint64_t lo, hi;  // k-mer starts in [lo, hi) (lo a multiple of 32: 16-B aligned tiles)
    int symbols, total_bits;
    int acgt_only;    // 2-bit keys of a mixed sba: k-mers holding a non-ACGT byte are not started
    // key-range shard: only k-mers whose ownership digit o (the top own_bits key bits) has
    // o - own_lo < own_span are kept (all: 0, ~0)
    uint32_t own_lo = 0, own_span = 0xFFFFFFFFu;
    int own_bits = 7;
    // 2-bit packed copy of an ACGT sba (pack2_kernel, 32 positions per word; null: pack bytes)
    const uint64_t *pk_code = nullptr;
    const uint32_t *pk_dol = nullptr;
    // timing builds only (GKM_L0_PROF): per-phase clock sums of the L0 partition's first and last
    // wave of every workgroup
    unsigned long long *prof = nullptr;
};

__device__ __forceinline__ bool l0_owned(uint32_t d, const L0Args &a) { return d - a.own_lo < a.own_span; }
// the ownership digit of a total_bits-bit key (own_bits <= total_bits)
__device__ __forceinline__ bool l0_owned_key(uint64_t key, const L0Args &a) {
    return l0_owned((uint32_t)(key >> (a.total_bits - a.own_bits)), a);
}

template <int BITS, int TILE>
struct L0Pack {
    static constexpr int kGroups = TILE / 32 + 3;             // 32-position groups packed (k <= 64)
    static constexpr int kCodeWords = kGroups * BITS / 2 + 1;  // u64 words (+1 for the funnel)
};

// The tile's bytes (kGroups * 32, incl. the halo) in 8-byte units, spread over all T threads:
// thread t holds units t, t + T, ... (kPer registers; index clamped so the loads stay branch-free)
template <int BITS, int TILE, int T>
struct L0Units {
    static constexpr int kUnits = L0Pack<BITS, TILE>::kGroups * 4;
    static constexpr int kPer = (kUnits + T - 1) / T;
};

template <int BITS, int TILE, int T>
__device__ __forceinline__ void l0_load(const L0Args &a, uint64_t P0, uint64_t (&r)[L0Units<BITS, TILE, T>::kPer]) {
    using U = L0Units<BITS, TILE, T>;
    static_assert(U::kPer >= 2, "the packed path keeps a code word and a stop word");
    // every element of r is written on both paths (a path that leaves some unwritten made the
    // compiler keep r in scratch memory at kPer = 3)
    if (BITS == 2 && a.pk_code) {  // pre-packed: thread t holds the words of groups t, t + T, ...
        constexpr int kPairs = U::kPer / 2;
        static_assert(kPairs * T >= L0Pack<BITS, TILE>::kGroups, "every packed group has a register pair");
#pragma unroll
        for (int j = 0; j < kPairs; ++j) {
            const uint64_t g = (P0 >> 5) + min((uint32_t)(threadIdx.x + j * T), (uint32_t)L0Pack<BITS, TILE>::kGroups - 1);
            r[2 * j] = a.pk_code[g];
            r[2 * j + 1] = a.pk_dol[g];
        }
#pragma unroll
        for (int j = 2 * kPairs; j < U::kPer; ++j) r[j] = 0;
    } else {
        const uint64_t *s8 = reinterpret_cast<const uint64_t *>(a.sba + P0);
#pragma unroll
        for (int j = 0; j < U::kPer; ++j) r[j] = s8[min((uint32_t)(threadIdx.x + j * T), (uint32_t)U::kUnits - 1)];
    }
}

// 2-bit codes (A0 C1 G2 T3) of 8 bytes as 16 bits, position 0 in the most significant pair
__device__ __forceinline__ uint32_t pack2_8(uint64_t x) {
    uint64_t t = __builtin_bswap64(((x >> 1) ^ (x >> 2)) & 0x0303030303030303ull);
    t = (t | (t >> 6)) & 0x000F000F000F000Full;
    t = (t | (t >> 12)) & 0x000000FF000000FFull;
    return (uint32_t)((t | (t >> 24)) & 0xFFFFu);
}

// s_dol bit = the position ends k-mers: '$' (or, acgt_only, any byte outside ACGT).  Every thread
// packs its 8-byte units: 2-bit codes into 16-bit (4-bit: 32-bit) pieces of the MSB-first code
// words, stop flags into bytes of the 32-position mask words.
template <int BITS, int TILE, int T>
__device__ __forceinline__ void l0_pack(const uint64_t (&r)[L0Units<BITS, TILE, T>::kPer], uint64_t *s_code,
                                        uint32_t *s_dol, const uint8_t *lut4, int acgt_only, bool packed) {
    using U = L0Units<BITS, TILE, T>;
    using P = L0Pack<BITS, TILE>;
    constexpr uint64_t kOnes = 0x0101010101010101ull;
    if (BITS == 2 && packed) {
#pragma unroll
        for (int j = 0; j < U::kPer / 2; ++j) {
            const uint32_t g = threadIdx.x + j * T;
            if (g < (uint32_t)P::kGroups) {
                s_code[g] = r[2 * j];
                s_dol[g] = (uint32_t)r[2 * j + 1];
            }
        }
        if (threadIdx.x == 0) s_code[P::kCodeWords - 1] = 0;
        return;
    }
#pragma unroll
    for (int j = 0; j < U::kPer; ++j) {
        const uint32_t u = threadIdx.x + j * T;
        if (u < (uint32_t)U::kUnits) {
            const uint64_t x = r[j];
            uint64_t z;
            if (acgt_only)
                z = non_acgt_bytes(x);
            else
                z = zero_bytes(x ^ (kOnes * GK_DOLLAR));
            reinterpret_cast<uint8_t *>(s_dol)[(u & ~3u) + 3 - (u & 3u)] = (uint8_t)gather_flags8(z);
            if (BITS == 2) {
                reinterpret_cast<uint16_t *>(s_code)[(u & ~3u) + 3 - (u & 3u)] = (uint16_t)pack2_8(x);
            } else {
                uint32_t v = 0;
#pragma unroll
                for (int b = 0; b < 8; ++b) v = (v << 4) | lut4[(x >> (8 * b)) & 0xFFu];
                reinterpret_cast<uint32_t *>(s_code)[(u & ~1u) + 1 - (u & 1u)] = v;
            }
        }
    }
    if (threadIdx.x == 0) s_code[P::kCodeWords - 1] = 0;
}

template <int BITS>
__device__ __forceinline__ uint64_t l0_key(const uint64_t *s_code, uint32_t p, int B) {
    const uint32_t o = p * BITS, w = o >> 6, s = o & 63;
    uint64_t x = s_code[w] << s;
    if (s) x |= s_code[w + 1] >> (64 - s);
    return x >> (64 - B);
}

// CANON: the first key word of the canonical k-mer (gkm_canon.h) is the smaller of the first word
// of the k-mer and the first word of its reverse complement -- the reverse complement of the
// k-mer's last B / BITS symbols.  (If the two are equal the whole-k-mer choice does not change the
// first word; later words are decided in tie_encode_kernel.)
template <int BITS, bool CANON>
__device__ __forceinline__ uint64_t l0_key_of(const uint64_t *s_code, uint32_t p, int B, int k) {
    const uint64_t f = l0_key<BITS>(s_code, p, B);
    if (!CANON) return f;
    const int n = B / BITS;
    const uint64_t r = revcomp_word<BITS>(l0_key<BITS>(s_code, p + k - n, B), n);
    return r < f ? r : f;
}

__device__ __forceinline__ bool l0_valid(const uint32_t *s_dol, uint32_t p, int S) {
    const uint32_t w = p >> 5, s = p & 31;
    const uint64_t x = (((uint64_t)s_dol[w] << 32) | s_dol[w + 1]) << s;
    if (S <= 32) return (x >> (64 - S)) == 0;
    // multi-word keys (33 <= S <= 64): the first 32 positions, then the rest from p + 32
    const uint64_t y = (((uint64_t)s_dol[w + 1] << 32) | s_dol[w + 2]) << s;
    return (x >> 32) == 0 && (y >> (96 - S)) == 0;
}

// Eight consecutive positions q0 .. q0 + 7 (q0 % 8 == 0) of a packed 2-bit tile from one 128-bit
// code window and one 64-position stop window: keep mask (valid, before a.hi, owned) and the keys
// (only if `keys`) or the L0 digits.  When no lane of the wave sees a stop or the sequence end and
// the L0 digit is the top 7 bits of a key of >= 8 bits, the digits come straight from the window's
// high half (bits [25 - 2i, 32 - 2i)) -- a shift, a mask and a compare per position.
struct Win8 {
    uint64_t T, T2;  // symbols q0 .., q0 + 32 ..
    uint64_t D;      // stops q0 .. q0 + 63, MSB first
};

__device__ __forceinline__ Win8 win8_load(const uint64_t *s_code, const uint32_t *s_dol, uint32_t q0) {
    const uint32_t w0 = q0 >> 5, s0 = (q0 & 31) * 2;  // s0 in {0, 16, 32, 48}
    const uint64_t A0 = s_code[w0], A1 = s_code[w0 + 1], A2 = s_code[w0 + 2];
    Win8 w;
    w.T = s0 ? (A0 << s0) | (A1 >> (64 - s0)) : A0;
    w.T2 = s0 ? (A1 << s0) | (A2 >> (64 - s0)) : A1;
    const uint32_t ds = q0 & 31;  // in {0, 8, 16, 24}
    const uint64_t D0 = ((uint64_t)s_dol[w0] << 32) | s_dol[w0 + 1];
    w.D = ds ? (D0 << ds) | (s_dol[w0 + 2] >> (32 - ds)) : D0;
    return w;
}

__device__ __forceinline__ uint64_t win8_key(const Win8 &w, int i, int B) {
    const uint64_t Ti = i ? (w.T << (2 * i)) | (w.T2 >> (64 - 2 * i)) : w.T;
    return B >= 64 ? Ti : Ti >> (64 - B);
}

// the 32 symbols from position q of a packed 2-bit tile, MSB first (any q)
__device__ __forceinline__ uint64_t win32_at(const uint64_t *s_code, uint32_t q) {
    const uint32_t w = q >> 5, s = (q & 31) * 2;
    return s ? (s_code[w] << s) | (s_code[w + 1] >> (64 - s)) : s_code[w];
}

// wave-uniform call (a ballot inside)
__device__ __forceinline__ uint32_t win8_keep(const Win8 &w, const L0Args &a, Dig d0, int64_t left,
                                              const uint32_t *s_dol, uint32_t q0, uint32_t (&dig)[8]) {
    const uint32_t Th = (uint32_t)(w.T >> 32);
    const bool top7 = d0.mask == 0x7Fu && (int)d0.shift == a.total_bits - 7 && a.symbols <= 56;
    uint32_t keepm = 0;
    // ownership digits of up to 18 bits come from the same 32-bit window (2 i + own_bits <= 32)
    const uint32_t omask = (1u << a.own_bits) - 1;
    if (top7 && a.own_bits <= a.total_bits && a.own_bits <= 18 && __ballot(w.D != 0 || left < 8) == 0) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            dig[i] = (Th >> (25 - 2 * i)) & 0x7Fu;
            keepm |= (l0_owned((Th >> (32 - 2 * i - a.own_bits)) & omask, a) ? 1u : 0u) << i;
        }
        return keepm;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint64_t key = win8_key(w, i, a.total_bits);
        dig[i] = dg_of(key, d0);
        const uint64_t Di = w.D << i;
        const bool valid = a.symbols <= 56 ? (Di == 0 || (int)__clzll((long long)Di) >= a.symbols)
                                           : l0_valid(s_dol, q0 + i, a.symbols);
        keepm |= ((valid && i < left && l0_owned_key(key, a)) ? 1u : 0u) << i;
    }
    return keepm;
}

template <int BITS, int T, int I, int R, bool CANON = false>
__global__ __launch_bounds__(T) void msd0_count_kernel(L0Args a, Dig d0, uint32_t *__restrict__ tile_hist,
                                                       uint32_t ntiles) {
    constexpr int TILE = T * I;
    constexpr int RADIX = 1 << R;
    using P = L0Pack<BITS, TILE>;
    __shared__ uint64_t s_code[P::kCodeWords];
    __shared__ uint32_t s_dol[P::kGroups];
    // 4 interleaved histogram copies (digit d, copy c at 4 d + c; copy = thread & 3): the lanes of
    // one atomic that share a digit land on 4 different words in 4 banks (C3: 1.845 -> 1.797 ms, A/B)
    constexpr int NC = 4;
    __shared__ uint32_t s_hist[RADIX * NC];
    __shared__ uint8_t s_lut4[256];
    const int t = threadIdx.x;
    if (t < 256) s_lut4[t] = c_code4_msd[t];
    // persistent: the next tile's bytes are loaded while this one is counted
    uint64_t rr[L0Units<BITS, TILE, T>::kPer];
    if (blockIdx.x < ntiles) l0_load<BITS, TILE, T>(a, a.lo + (uint64_t)blockIdx.x * TILE, rr);
    for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const uint64_t P0 = a.lo + (uint64_t)tile * TILE;
        // each thread zeroes the copies it summed for the previous tile (no barrier between)
        for (int i = t; i < RADIX; i += T)
#pragma unroll
            for (int c = 0; c < NC; ++c) s_hist[i * NC + c] = 0;
        lds_barrier();  // the LUT; the previous tile's histogram and codes have been read
        l0_pack<BITS, TILE, T>(rr, s_code, s_dol, s_lut4, a.acgt_only, a.pk_code != nullptr);
        lds_barrier();
        if (tile + gridDim.x < ntiles) l0_load<BITS, TILE, T>(a, P0 + (uint64_t)gridDim.x * TILE, rr);
        if constexpr (BITS == 2 && !CANON) {  // 8 consecutive positions per thread (Win8)
            static_assert(TILE % 8 == 0 && (TILE / 8) % 64 == 0, "whole waves per round");
            for (uint32_t g = t; g < TILE / 8; g += T) {
                const uint32_t q0 = g * 8;
                const Win8 w = win8_load(s_code, s_dol, q0);
                uint32_t dig[8];
                const uint32_t keepm = win8_keep(w, a, d0, (int64_t)a.hi - (int64_t)(P0 + q0), s_dol, q0, dig);
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    if ((keepm >> i) & 1u) atomicAdd(&s_hist[dig[i] * NC + (t & (NC - 1))], 1u);
            }
        } else {
            // canonical 2-bit keys in a tile without stops: the digit is the smaller of the forward
            // and the reverse-complement top 7 bits, 8 consecutive positions per thread from two
            // 32-symbol windows (at q0 and at q0 + k - 4)
            bool fast = false;
            if constexpr (BITS == 2 && CANON && (R == 7 || R == 8)) {
                uint32_t anystop = 0;
                for (int j = t; j < P::kGroups; j += T) anystop |= s_dol[j];
                // (ownership digits other than the L0 digit -- the key-range ranks' 12 bits -- take the
                // per-position path below)
                fast = __syncthreads_or(anystop != 0) == 0 && P0 + TILE <= a.hi &&
                       (d0.mask == 0x7Fu || d0.mask == 0xFFu) && (int)d0.shift == a.total_bits - R &&
                       a.symbols >= 4 && (a.own_span == 0xFFFFFFFFu || a.own_bits == R);
                if (fast) {
                    for (uint32_t g = t; g < TILE / 8; g += T) {
                        const uint32_t q0 = g * 8;
                        // only the top 32 bits of each window are read (16 symbols: positions q0 .. q0 + 10,
                        // q0 + k - 4 .. q0 + k + 6): 32-bit shifts per position instead of 64-bit ones
                        // (the 64-bit form ran this pass VALU-bound at 5.0 ms for C5)
                        const uint32_t tf = (uint32_t)(win32_at(s_code, q0) >> 32);
                        const uint32_t tr = (uint32_t)(win32_at(s_code, q0 + a.symbols - 4) >> 32);
#pragma unroll
                        for (int i = 0; i < 8; ++i) {
                            // (R = 8: the top 8 bits of both words; the smaller digit is the top of the smaller word)
                            const uint32_t f7 = (tf >> (32 - R - 2 * i)) & ((1u << R) - 1);
                            const uint32_t v = (tr >> (24 - 2 * i)) & 0xFFu;  // symbols q0+k-4+i ..
                            const uint32_t rv = ((v & 3u) << 6) | ((v & 0xCu) << 2) | ((v >> 2) & 0xCu) | (v >> 6);
                            const uint32_t d = min(f7, (~rv & 0xFFu) >> (8 - R));
                            if (l0_owned(d, a)) atomicAdd(&s_hist[d * NC], 1u);
                        }
                    }
                }
            }
            if (!fast) {
                // (tiles with stops, or the sequence end).  Canonical keys: two windows and a
                // reverse complement per position -- a loop, not unrolled, so the fast path above
                // keeps its registers (unrolled over the 96 positions it took 256 VGPRs, spilled
                // to scratch and ran the whole kernel at one wave per SIMD).  4-bit forward keys
                // (every tile takes this path): unrolled by 4 (fully unrolled: 256 VGPRs + 206
                // AGPRs, one wave per SIMD)
                constexpr int UNR = CANON ? 1 : 4;
#pragma unroll UNR
                for (int i = 0; i < I; ++i) {
                    const uint32_t p = i * T + t;
                    const uint64_t key = l0_key_of<BITS, CANON>(s_code, p, a.total_bits, a.symbols);
                    const uint32_t d = dg_of(key, d0);
                    if (l0_valid(s_dol, p, a.symbols) && P0 + p < a.hi && l0_owned_key(key, a))
                        atomicAdd(&s_hist[d * NC], 1u);
                }
            }
        }
        lds_barrier();
        for (int i = t; i < RADIX; i += T) {
            uint32_t h = 0;
#pragma unroll
            for (int c = 0; c < NC; ++c) h += s_hist[i * NC + c];
            tile_hist[(uint64_t)tile * RADIX + i] = h;
        }
    }
}

// L0 partition, software-pipelined with position staging.  The L0 input is the packed tile
// itself, so a staged element needs only its tile position (u16): its key is re-derived from the
// tile's codes when it is stored, and its start is the tile base + position.  Positions and codes
// are double-buffered (2 x (48 + 6) KB at 24,576 positions), so the previous tile's stores are
// spread over EVERY phase of this tile -- packing, ranking, scan, staging -- and the memory pipe
// never idles (staged as (key, start) in one 135 KB buffer, the stores had to finish before the
// staging: a phase profile (GKM_L0_PROF) showed them issued in 45 % of the tile time, backed up,
// and the pipe idle for the rest).  Twice the tile of the level passes: runs of ~192 per digit.
// PROF (timing builds, GKM_L0_PROF): the first and the last wave of each workgroup add the clock
// ticks of every phase of the tile loop to a.prof[wave != 0][phase]
constexpr int kL0Phases = 9;
#ifndef GKM_L0_T
#define GKM_L0_T 1024
#endif
#ifndef GKM_L0_I
#define GKM_L0_I 24
#endif
// (tuning overrides, tools/build_variant.sh: GKM_L0_T threads x GKM_L0_I positions per tile)
constexpr int kP0T = GKM_L0_T;           // L0 tile: kP0T threads x kP0I positions
constexpr int kP0I = GKM_L0_I;
constexpr int kP0Tile = kP0T * kP0I;     // 24,576 (< 65,536: positions staged as u16)

// P88 (the packed L0, round 5): each element leaves as the level-1 digit byte (nd), the key bits below
// it above the start's high bits (u64: key << shi | start >> (32 - shi)) and the start's low bits
// (u16 in nd.out16) -- 11 B instead of 13 (key, start, digit); the level behind reads it (INP = 2)
// OWN (the key-range ranks' fused select, round 5): only k-mers whose ownership digit (the top
// a.own_bits key bits) is in the rank's range are partitioned -- the select pass and its 13-byte
// round trip per kept k-mer fall away
template <int BITS, int T, int I, int R, bool ND, bool CANON = false, bool PROF = false, bool P88 = false,
          bool OWN = false>
__global__ __launch_bounds__(T) void msd0_pipe_kernel(L0Args a, Dig d0, const uint32_t *__restrict__ tile_off,
                                                      uint64_t *__restrict__ kout, uint32_t *__restrict__ vout,
                                                      uint32_t ntiles, uint64_t sink, NextDigits nd) {
    constexpr int TILE = T * I;
    static_assert(TILE < 65536, "tile positions are staged as u16");
    constexpr int RADIX = 1 << R;
    constexpr int NW = T / 64;
    // store groups of the previous tile: G_TOP after the packing, one per ranked item, G_SCAN
    // during the scan, the rest after the staging
#ifndef GKM_L0_GTOP
#define GKM_L0_GTOP 1
#endif
#ifndef GKM_L0_GSCAN
#define GKM_L0_GSCAN 2
#endif
    // (tuning overrides, tools/gpu_ab_l0_groups.sh: G_TOP 1 beat 0, 2 and 4 by 0.2-0.6 ms at C3)
    constexpr int G_TOP = GKM_L0_GTOP, G_SCAN = GKM_L0_GSCAN;
    constexpr int G_RANK = I - G_TOP - G_SCAN - 2 > 0 ? I - G_TOP - G_SCAN - 2 : 0;
    using P = L0Pack<BITS, TILE>;
    static_assert(T >= RADIX, "one thread per digit");
    __shared__ uint16_t s_pos[2][TILE + 2];          // positions in digit order (slot TILE: sink)
    __shared__ uint64_t s_code[2][P::kCodeWords];   // this tile's and the staged tile's codes
    __shared__ uint32_t s_dol[P::kGroups];
    __shared__ uint32_t s_wc[NW * RADIX];
    __shared__ uint32_t s_toff[2][RADIX];
    __shared__ uint32_t s_start[RADIX + 1];
    __shared__ uint32_t s_wsum[RADIX / 64 > 0 ? RADIX / 64 : 1];
    __shared__ uint8_t s_lut4[256];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid < 256) s_lut4[tid] = c_code4_msd[tid];
    // the first iteration's stores read buffer 1 before anything was staged (they go to the
    // sink): keep their positions inside the tile
    for (int i = tid; i < TILE + 2; i += T) s_pos[1][i] = 0;
    lds_barrier();  // the LUT, read by every thread's pack
    const TileWalk walk(ntiles);
    uint64_t rr[L0Units<BITS, TILE, T>::kPer];
    uint32_t toff = 0;
    auto load = [&](uint32_t t) {
        toff = tile_off[(uint64_t)t * RADIX + (tid & (RADIX - 1))];
        l0_load<BITS, TILE, T>(a, a.lo + (uint64_t)t * TILE, rr);
    };
    uint32_t pcnt = 0;  // staged elements of the previous tile (0: none -> its stores go to the sink)
    uint64_t pP0 = 0;   // the previous tile's first position
    int b = 0;          // this tile's buffers; b ^ 1: the staged previous tile
    // one store group of the previous tile: slot s -> position -> key (from the staged codes)
    auto store_group = [&](int g) {
        const uint32_t s = min((uint32_t)(tid + g * T), pcnt - 1);  // pcnt == 0: stays in the tile
        const uint32_t p = s_pos[b ^ 1][s];
        const uint64_t key = l0_key_of<BITS, CANON>(s_code[b ^ 1], p, a.total_bits, a.symbols);
        const uint64_t o = pcnt ? (uint64_t)(s_toff[b ^ 1][dg_of(key, d0)] + s) : sink;
        if (P88) {
            const uint32_t st = (uint32_t)(pP0 + p);
            const int shi = nd.pshi;
            kout[o] = (key << shi) | (st >> (32 - shi));  // (the sorted and digit bits shift out)
            nd.out16[o] = (uint16_t)(st & ((1u << (32 - shi)) - 1));
            nd.out[o] = (uint8_t)dg_of(key, nd.d);
        } else {
            if (kout) kout[o] = key;  // (none: a starts-only shard send, GK_SHARD_STARTS_ONLY)
            vout[o] = (uint32_t)(pP0 + p);
            if (ND) nd.out[o] = (uint8_t)dg_of(key, nd.d);
        }
        // keep each group's loads and stores in place: hoisting the groups' LDS reads ahead (the
        // scheduler's choice) keeps 22 groups' positions and keys live and spills them to scratch,
        // whose vmcnt waits then drain every store in flight
        __builtin_amdgcn_sched_barrier(0);
    };
    if (walk.first < walk.end) load(walk.first);
    __builtin_amdgcn_s_waitcnt(kVmcnt0);
    const bool pw = PROF && lane == 0 && (wave == 0 || wave == NW - 1);
    unsigned long long ph[kL0Phases] = {0}, tp = PROF ? clock64() : 0;
    auto mark = [&](int k) {
        if constexpr (PROF) {
            if (pw) {
                const unsigned long long t1 = clock64();
                ph[k] += t1 - tp;
                tp = t1;
            }
        }
    };
    for (uint32_t t = walk.first; t < walk.end; t += walk.step) {
        uint32_t *wc = s_wc + wave * RADIX;
#pragma unroll
        for (int u = 0; u < (RADIX + 63) / 64; ++u)
            if (u * 64 + lane < RADIX) wc[u * 64 + lane] = 0;
        if (tid < RADIX) s_toff[b][tid] = toff;
        l0_pack<BITS, TILE, T>(rr, s_code[b], s_dol, s_lut4, a.acgt_only, a.pk_code != nullptr);
        // rr and toff are consumed: the next tile's bytes fly during this whole tile (the last
        // tile re-loads itself, so every iteration issues the same loads: static wait counts)
        load(min(t + walk.step, walk.end - 1));
        mark(0);
#pragma unroll
        for (int g = 0; g < G_TOP; ++g) store_group(g);
        mark(1);
        lds_barrier();  // packed codes visible
        mark(2);
        const uint64_t P0 = a.lo + (uint64_t)t * TILE;
        // a tile without stops that ends before a.hi: every position starts a k-mer (wave-uniform)
        uint32_t anystop = 0;
#pragma unroll
        for (int j = 0; j < (P::kGroups + 63) / 64; ++j)
            anystop |= s_dol[min((uint32_t)(j * 64 + lane), (uint32_t)P::kGroups - 1)];
        const bool clean = __ballot(anystop != 0) == 0 && P0 + TILE <= a.hi;
        uint32_t dr[I], validm = 0;  // per item: digit | rank << 8 (rank < I * 64)
        uint32_t p0 = wave * (I * 64) + lane;
        asm volatile("" : "+v"(p0));
        mark(3);
#pragma unroll
        for (int i = 0; i < I; ++i) {
            const uint32_t p = p0 + i * 64;
            const uint64_t key = l0_key_of<BITS, CANON>(s_code[b], p, a.total_bits, a.symbols);
            bool valid = clean || (l0_valid(s_dol, p, a.symbols) && P0 + p < a.hi);
            if (OWN) valid = valid && l0_owned_key(key, a);
            validm |= (valid ? 1u : 0u) << i;
            const uint32_t dig = dg_of(key, d0);
            // stable rank by one returning LDS atomic (rank_atomic, gkm_partition.h); the LDS-mask
            // round trip it replaces took C3 L0 14.0 -> 12.9 ms against R + 1 ballots per item
            dr[i] = dig | (rank_atomic(wc, dig, valid) << 8);
            if (i < G_RANK) store_group(G_TOP + i);
            __builtin_amdgcn_sched_barrier(0);  // one item at a time (register pressure, see above)
        }
        mark(4);
        lds_barrier();  // ranks final
        mark(5);
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
#pragma unroll
        for (int g = 0; g < G_SCAN; ++g) store_group(G_TOP + G_RANK + g);
        lds_barrier();
        if (tid < RADIX) {
            uint32_t pre = 0;
            for (int w = 0; w < wave; ++w) pre += s_wsum[w];
            const uint32_t st = pre + incl - total;
            s_start[tid] = st;
            s_toff[b][tid] -= st;
            if (tid == RADIX - 1) s_start[RADIX] = pre + incl;
        }
        lds_barrier();
        mark(6);
#pragma unroll
        for (int i = 0; i < I; ++i) {
            const bool valid = (validm >> i) & 1u;
            const uint32_t dg = dr[i] & 0xFFu;
            const uint32_t sl = valid ? s_start[dg] + wc[dg] + (dr[i] >> 8) : (uint32_t)TILE;
            s_pos[b][sl] = (uint16_t)(p0 + i * 64);
        }
        const uint32_t cnt = s_start[RADIX];
#pragma unroll
        for (int g = G_TOP + G_RANK + G_SCAN; g < I; ++g) store_group(g);
        mark(7);
        pcnt = cnt;
        pP0 = P0;
        lds_barrier();  // staging complete; counters, codes and the previous staging read
        mark(8);
        b ^= 1;
    }
    if (walk.first < walk.end) {
#pragma unroll
        for (int g = 0; g < I; ++g) store_group(g);
    }
    if constexpr (PROF) {
        if (pw)
            for (int k = 0; k < kL0Phases; ++k) atomicAdd(&a.prof[(wave != 0) * kL0Phases + k], ph[k]);
    }
}

// TIMING EXPERIMENTS ONLY (GKM_EXP_L0=1, wrong output): the L0 partition's memory traffic with no
// encoding or ranking -- each persistent workgroup walks the same tiles (XCD-aware), reads the
// tile's sequence bytes, and writes (key, start, digit byte) for every position to 2^R runs of
// TILE / 2^R consecutive slots per tile, run d of tile t at d * (n / 2^R) + t * (TILE / 2^R): the
// real layout of an L0 output over uniform digits.  Its time is the floor of the L0's scatter.
template <int T, int I, int R>
__global__ __launch_bounds__(T) void l0_scatter_floor_kernel(const uint8_t *__restrict__ sba, uint64_t n,
                                                             uint32_t ntiles, uint64_t *__restrict__ kout,
                                                             uint32_t *__restrict__ vout, uint8_t *__restrict__ nd) {
    constexpr int TILE = T * I, RUN = TILE >> R;
    const TileWalk walk(ntiles);
    const uint64_t bsz = n >> R;
    for (uint32_t t = walk.first; t < walk.end; t += walk.step) {
        const uint64_t P0 = (uint64_t)t * TILE;
        const uint32_t x = reinterpret_cast<const uint32_t *>(sba + P0)[threadIdx.x];  // (the tile's bytes)
#pragma unroll 4
        for (int g = 0; g < I; ++g) {
            const uint32_t s = threadIdx.x + g * T, d = s / RUN, j = s - d * RUN;
            const uint64_t o = min((uint64_t)d * bsz + (uint64_t)t * RUN + j, n - 1);
            const uint64_t h = (P0 + s + (x & 1u)) * 0x9E3779B97F4A7C15ull;  // distinct keys, uniform digits
            kout[o] = h;
            vout[o] = (uint32_t)(P0 + s);
            nd[o] = (uint8_t)(h >> 49);
        }
    }
}

// TIMING EXPERIMENTS ONLY (GKM_EXP_L0=v, wrong output): the scatter floor above with each lane
// writing 4 consecutive slots of one run by vector stores (two 16-byte stores of keys, one of starts,
// one 4-byte store of digits) -- how much of the floor is the store width rather than the stream?
template <int T, int I, int R>
__global__ __launch_bounds__(T) void l0_scatter_floor4_kernel(const uint8_t *__restrict__ sba, uint64_t n,
                                                              uint32_t ntiles, uint64_t *__restrict__ kout,
                                                              uint32_t *__restrict__ vout, uint8_t *__restrict__ nd) {
    constexpr int TILE = T * I, RUN = TILE >> R;
    static_assert(RUN % 4 == 0 && I % 4 == 0, "whole 4-slot groups per run");
    const TileWalk walk(ntiles);
    const uint64_t bsz = (n >> R) & ~3ull;
    for (uint32_t t = walk.first; t < walk.end; t += walk.step) {
        const uint64_t P0 = (uint64_t)t * TILE;
        const uint32_t x = reinterpret_cast<const uint32_t *>(sba + P0)[threadIdx.x];
#pragma unroll 2
        for (int g = 0; g < I / 4; ++g) {
            const uint32_t s = 4 * (threadIdx.x + g * T), d = s / RUN, j = s - d * RUN;
            const uint64_t o = min((uint64_t)d * bsz + (uint64_t)t * RUN + j, (n - 4) & ~3ull);
            uint64_t h[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) h[u] = (P0 + s + u + (x & 1u)) * 0x9E3779B97F4A7C15ull;
            uint4 *k4 = reinterpret_cast<uint4 *>(kout + o);
            k4[0] = make_uint4((uint32_t)h[0], (uint32_t)(h[0] >> 32), (uint32_t)h[1], (uint32_t)(h[1] >> 32));
            k4[1] = make_uint4((uint32_t)h[2], (uint32_t)(h[2] >> 32), (uint32_t)h[3], (uint32_t)(h[3] >> 32));
            reinterpret_cast<uint4 *>(vout + o)[0] =
                make_uint4((uint32_t)(P0 + s), (uint32_t)(P0 + s + 1), (uint32_t)(P0 + s + 2), (uint32_t)(P0 + s + 3));
            reinterpret_cast<uint32_t *>(nd + o)[0] = (uint32_t)(h[0] >> 49 & 0xFF) | (uint32_t)(h[1] >> 49 & 0xFF) << 8 |
                                                      (uint32_t)(h[2] >> 49 & 0xFF) << 16 | (uint32_t)(h[3] >> 49 & 0xFF) << 24;
        }
    }
}

// Wide L0 partition (R = 10 or 11 bits; 2-bit keys of one word, forward, no profile): the
// position-staged, software-pipelined scheme of msd0_pipe_kernel with a digit space the 7-bit one
// cannot hold -- per-wave u16 counters, two per word (rank_atomic16), K = RADIX / T digits per
// thread in the scan, K tile offsets per thread.  With the level pass behind it, 11 + 8 bits leave
// the C3 buckets at ~5.9 K keys, finished in one block-local round (three passes instead of
// four global ones plus the wave-local round).
template <int T, int I, int R, bool ND>
__global__ __launch_bounds__(T) void msd0_wide_kernel(L0Args a, Dig d0, const uint32_t *__restrict__ tile_off,
                                                      uint64_t *__restrict__ kout, uint32_t *__restrict__ vout,
                                                      uint32_t ntiles, uint64_t sink, NextDigits nd) {
    constexpr int TILE = T * I;
    static_assert(TILE < 65536, "tile positions are staged as u16");
    constexpr int RADIX = 1 << R;
    constexpr int NW = T / 64;
    constexpr int K = RADIX / T;  // digits per thread in the scan
    static_assert(RADIX % T == 0 && K >= 1, "whole digits per thread");
    static_assert(I * 64 < 65536, "per-wave counts fit 16 bits");
    constexpr int G_TOP = 1, G_SCAN = 2;
    constexpr int G_RANK = I - G_TOP - G_SCAN - 2 > 0 ? I - G_TOP - G_SCAN - 2 : 0;
    using P = L0Pack<2, TILE>;
    __shared__ uint16_t s_pos[2][TILE + 2];          // positions in digit order (slot TILE: sink)
    __shared__ uint64_t s_code[2][P::kCodeWords];   // this tile's and the staged tile's codes
    __shared__ uint32_t s_dol[P::kGroups];
    __shared__ uint32_t s_wc[NW * RADIX / 2];        // per-wave u16 digit counters
    __shared__ uint32_t s_toff[2][RADIX];
    __shared__ uint32_t s_start[RADIX + 1];
    __shared__ uint32_t s_wsum[NW];
    uint16_t *const s_wc16 = reinterpret_cast<uint16_t *>(s_wc);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int i = tid; i < TILE + 2; i += T) s_pos[1][i] = 0;
    lds_barrier();
    const TileWalk walk(ntiles);
    uint64_t rr[L0Units<2, TILE, T>::kPer];
    uint32_t toff[K];
    auto load = [&](uint32_t t) {
#pragma unroll
        for (int k = 0; k < K; ++k) toff[k] = tile_off[(uint64_t)t * RADIX + tid * K + k];
        l0_load<2, TILE, T>(a, a.lo + (uint64_t)t * TILE, rr);
    };
    uint32_t pcnt = 0;
    uint64_t pP0 = 0;
    int b = 0;
    auto store_group = [&](int g) {
        const uint32_t s = min((uint32_t)(tid + g * T), pcnt - 1);
        const uint32_t p = s_pos[b ^ 1][s];
        const uint64_t key = l0_key<2>(s_code[b ^ 1], p, a.total_bits);
        const uint64_t o = pcnt ? (uint64_t)(s_toff[b ^ 1][dg_of(key, d0)] + s) : sink;
        kout[o] = key;
        vout[o] = (uint32_t)(pP0 + p);
        if (ND) nd.out[o] = (uint8_t)dg_of(key, nd.d);
        __builtin_amdgcn_sched_barrier(0);
    };
    if (walk.first < walk.end) load(walk.first);
    __builtin_amdgcn_s_waitcnt(kVmcnt0);
    for (uint32_t t = walk.first; t < walk.end; t += walk.step) {
        uint32_t *wc = s_wc + wave * (RADIX / 2);
#pragma unroll
        for (int u = 0; u < RADIX / 2 / 64; ++u) wc[u * 64 + lane] = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) s_toff[b][tid * K + k] = toff[k];
        l0_pack<2, TILE, T>(rr, s_code[b], s_dol, nullptr, 0, a.pk_code != nullptr);
        load(min(t + walk.step, walk.end - 1));
#pragma unroll
        for (int g = 0; g < G_TOP; ++g) store_group(g);
        lds_barrier();  // packed codes visible
        const uint64_t P0 = a.lo + (uint64_t)t * TILE;
        uint32_t anystop = 0;
#pragma unroll
        for (int j = 0; j < (P::kGroups + 63) / 64; ++j)
            anystop |= s_dol[min((uint32_t)(j * 64 + lane), (uint32_t)P::kGroups - 1)];
        const bool clean = __ballot(anystop != 0) == 0 && P0 + TILE <= a.hi;
        uint32_t dr[I];  // per item: digit | rank << R, all ones when not valid
        uint32_t p0 = wave * (I * 64) + lane;
        asm volatile("" : "+v"(p0));
#pragma unroll
        for (int i = 0; i < I; ++i) {
            const uint32_t p = p0 + i * 64;
            const bool valid = clean || (l0_valid(s_dol, p, a.symbols) && P0 + p < a.hi);
            const uint32_t dig = dg_of(l0_key<2>(s_code[b], p, a.total_bits), d0);
            const uint32_t rk = rank_atomic16<R>(wc, dig, valid);
            dr[i] = valid ? dig | (rk << R) : ~0u;
            if (i < G_RANK) store_group(G_TOP + i);
            __builtin_amdgcn_sched_barrier(0);
        }
        lds_barrier();  // ranks final
        // per-digit totals over the waves -> per-wave exclusive prefixes (u16), block scan of the
        // digit totals (thread tid owns digits tid K .. tid K + K - 1)
        uint32_t tot[K], sum = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int d = tid * K + k;
            uint32_t run = 0;
#pragma unroll
            for (int w = 0; w < NW; ++w) {
                const uint32_t v = s_wc16[w * RADIX + d];
                s_wc16[w * RADIX + d] = (uint16_t)run;
                run += v;
            }
            tot[k] = run;
            sum += run;
        }
        const uint32_t incl = wave_incl_scan(sum);
        if (lane == 63) s_wsum[wave] = incl;
#pragma unroll
        for (int g = 0; g < G_SCAN; ++g) store_group(G_TOP + G_RANK + g);
        lds_barrier();
        {
            uint32_t pre = 0;
            for (int w = 0; w < wave; ++w) pre += s_wsum[w];
            uint32_t run = pre + incl - sum;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int d = tid * K + k;
                s_start[d] = run;
                s_toff[b][d] -= run;
                run += tot[k];
            }
            if (tid == T - 1) s_start[RADIX] = run;
        }
        lds_barrier();
#pragma unroll
        for (int i = 0; i < I; ++i) {
            const bool valid = dr[i] != ~0u;
            const uint32_t dg = dr[i] & (RADIX - 1);
            const uint32_t sl = valid ? s_start[dg] + s_wc16[wave * RADIX + dg] + (dr[i] >> R) : (uint32_t)TILE;
            s_pos[b][sl] = (uint16_t)(p0 + i * 64);
        }
        const uint32_t cnt = s_start[RADIX];
#pragma unroll
        for (int g = G_TOP + G_RANK + G_SCAN; g < I; ++g) store_group(g);
        pcnt = cnt;
        pP0 = P0;
        lds_barrier();  // staging complete; counters, codes and the previous staging read
        b ^= 1;
    }
    if (walk.first < walk.end) {
#pragma unroll
        for (int g = 0; g < I; ++g) store_group(g);
    }
}

// ---------------------------------------------------------------------------------------------
// Key-range shard select (gk_shard_sort_range)
// ---------------------------------------------------------------------------------------------
// A rank scans the WHOLE sequence and keeps the k-mers whose L0 digit lies in its range -- about
// 1/N of them -- writing them contiguously in position order.  Two light streaming passes over
// 4096-position tiles (small LDS and registers, so several workgroups per CU overlap their loads):
//   STORE = false  kept k-mers per tile -> tile_cnt[t]          (then an exclusive scan)
//   STORE = true   each wave compacts its kept k-mers with one ballot per row; the kept lanes of
//                  a row store to consecutive addresses from tile_off[t]
// Stable: tiles, waves, rows and lanes follow positions.  The kept k-mers then go through the
// ordinary MSD levels as one bucket (the store pass writes their L0 digit bytes, so the first
// level counts 1 byte per k-mer).  A tile is kSR rounds of 4096 positions (512 per wave per round):
// one load of the tile's bytes (or packed words) per kSR rounds keeps more bytes in flight per
// workgroup than one 4096-position tile did.
#ifndef GKM_SEL_ROUNDS
#define GKM_SEL_ROUNDS 1
#endif
constexpr int kST = 512, kSI = 8, kSR = GKM_SEL_ROUNDS;  // threads, rows of 64 positions per wave per round, rounds
constexpr int kSRound = kST * kSI;                       // 4096 positions per round
constexpr int kSTile = kSRound * kSR;                    // positions per tile
constexpr int kSW = kST / 64;                            // waves per tile

// MODE 0 / 1 are the two passes above.  MODE 2 is a single pass: workgroup w walks its own chunk of
// tpw consecutive tiles and appends its kept k-mers at a running offset into its own region of
// the output, [t0 * kSTile, (t0 + tpw) * kSTile) (room for every position of the chunk, so no
// count pass is needed); wave_cnt[w] receives the chunk's kept count.  The regions, in workgroup
// order, are the pieces of one bucket in position order (first_level_from_pieces).
template <int BITS, bool CANON, int MODE>
#ifndef GKM_SEL_MINW
#define GKM_SEL_MINW 1
#endif
// (tuning override: GKM_SEL_MINW = the waves per SIMD the forward kernels' registers are capped
// for; the canonical ones would spill to scratch)
__global__ __launch_bounds__(kST, CANON ? 1 : GKM_SEL_MINW) void msd0_select_kernel(L0Args a, Dig d0, uint32_t ntiles, uint32_t tpw,
                                                          uint32_t *__restrict__ wave_cnt,
                                                          const uint32_t *__restrict__ wave_off,
                                                          uint64_t *__restrict__ kout, uint32_t *__restrict__ vout,
                                                          uint8_t *__restrict__ nd_out) {
    constexpr bool STORE = MODE != 0;
    using P = L0Pack<BITS, kSTile>;
    // per-wave staging of the kept positions (tile-relative u16; the key is re-derived from the
    // tile's codes when it is stored): 512 slots + one dump slot per lane for the positions not
    // kept, so the staging writes need no branch.  (Staged as (key, start), 48 KB, the kernel fit
    // 3 workgroups per CU and its divergent staging loop cost more scalar than vector work.)
    constexpr int kSlots = 512 + 64;
    constexpr int kStage = STORE ? kSW * kSlots : 1;
    __shared__ uint64_t s_code[P::kCodeWords];
    __shared__ uint32_t s_dol[P::kGroups];
    __shared__ uint8_t s_lut4[256];
    __shared__ uint16_t s_spos[kStage];
    __shared__ uint32_t s_wtot[2][kSW];  // per round parity (a round's barrier orders the reuse)
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid < 256) s_lut4[tid] = c_code4_msd[tid];
    // tiles of this workgroup: a strided walk (MODE 0 / 1) or a chunk (MODE 2)
    const uint32_t tfirst = MODE == 2 ? blockIdx.x * tpw : blockIdx.x;
    const uint32_t tend = MODE == 2 ? min(tfirst + tpw, ntiles) : ntiles;
    const uint32_t tstep = MODE == 2 ? 1u : gridDim.x;
    const uint64_t region = (uint64_t)tfirst * kSTile;  // MODE 2: this chunk's output region
    uint64_t run = 0;                                   // MODE 2: kept so far in the chunk
    uint64_t rr[L0Units<BITS, kSTile, kST>::kPer];
    if (tfirst < tend) l0_load<BITS, kSTile, kST>(a, a.lo + (uint64_t)tfirst * kSTile, rr);
    for (uint32_t t = tfirst; t < tend; t += tstep) {
        const uint64_t P0 = a.lo + (uint64_t)t * kSTile;
        __syncthreads();  // the LUT; the previous tile's codes and wave totals have been read
        l0_pack<BITS, kSTile, kST>(rr, s_code, s_dol, s_lut4, a.acgt_only, a.pk_code != nullptr);
        __syncthreads();
        // the next tile's bytes fly while this one is processed
        if (t + tstep < tend) l0_load<BITS, kSTile, kST>(a, P0 + (uint64_t)tstep * kSTile, rr);
        // MODE 2: the wave's output offset from the kept counts of the tile's waves (block-uniform
        // call: both paths below reach it)
        auto chunk_offset = [&](uint32_t wcount, int r) -> uint64_t {
            if (lane == 0) s_wtot[r & 1][wave] = wcount;
            __syncthreads();
            uint32_t pre = 0, tot = 0;
#pragma unroll
            for (int w = 0; w < kSW; ++w) {
                const uint32_t v = s_wtot[r & 1][w];
                pre += w < wave ? v : 0u;
                tot += v;
            }
            const uint64_t o = region + run + pre;
            run += tot;
            return o;
        };
        bool win = BITS == 2;
        // canonical: the count pass takes the digits from windows in a tile without stops; the store
        // passes keep the row layout below (a per-lane loop over the kept positions' canonical keys
        // was slower: 11.9 against 8.3 ms per C5 rank at N = 8).  Both visit a wave's 512 positions
        // in position order, so their per-wave counts and offsets agree.
        if constexpr (BITS == 2 && CANON) {
            if (STORE) win = false;
            uint32_t anystop = 0;
            for (int j = tid; j < P::kGroups; j += kST) anystop |= s_dol[j];
            win = win && __syncthreads_or(anystop != 0) == 0 && P0 + kSTile <= a.hi && d0.mask == 0x7Fu &&
                  (int)d0.shift == a.total_bits - 7 && a.symbols >= (a.own_bits + 1) / 2 && a.own_bits <= a.total_bits;
        }
        for (int r = 0; r < kSR; ++r) {
            const uint32_t R0 = r * kSRound;                       // the round's first tile position
            const uint64_t wslot = ((uint64_t)t * kSR + r) * kSW + wave;
            if (BITS == 2 && win) {
                // 8 consecutive positions per thread (Win8)
                const uint32_t q0 = R0 + tid * 8;
                Win8 win8{};
                uint32_t keepm = 0;
                if constexpr (!CANON) {
                    win8 = win8_load(s_code, s_dol, q0);
                    uint32_t dig[8];
                    keepm = win8_keep(win8, a, d0, (int64_t)a.hi - (int64_t)(P0 + q0), s_dol, q0, dig);
                } else {  // the smaller of the forward and reverse-complement top own_bits bits
                    // (msd0_count_kernel): the reverse complement's first ns symbols are the complement
                    // of the k-mer's last ns symbols, reversed
                    const int ob = a.own_bits, ns = (ob + 1) >> 1;
                    const uint64_t tf = win32_at(s_code, q0), tr = win32_at(s_code, q0 + a.symbols - ns);
                    const uint32_t om = (1u << ob) - 1;
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        const uint32_t f = (uint32_t)(tf >> (64 - ob - 2 * i)) & om;
                        const uint32_t v = (uint32_t)(tr >> (64 - 2 * ns - 2 * i)) & ((1u << (2 * ns)) - 1);
                        const uint32_t r = (uint32_t)(__builtin_bitreverse64(~(uint64_t)v) >> (64 - 2 * ns));
                        // bitreverse flips each pair's bit order too: swap the bits of every pair back
                        const uint32_t rr = ((r >> 1) & 0x55555555u) | ((r & 0x55555555u) << 1);
                        keepm |= (l0_owned(min(f, rr >> (2 * ns - ob)), a) ? 1u : 0u) << i;
                    }
                }
                const uint32_t cnt = (uint32_t)__popc(keepm);
                const uint32_t incl = wave_incl_scan(cnt);
                const uint32_t total = __builtin_amdgcn_readlane(incl, 63);
                if (!STORE) {
                    if (lane == 63) wave_cnt[wslot] = incl;
                    continue;
                }
                const uint64_t o = MODE == 2 ? chunk_offset(total, r) : (uint64_t)wave_off[wslot];
                // stage the wave's kept positions in position order, then store the k-mers as one
                // coalesced run
                uint16_t *sp = s_spos + wave * kSlots;
                uint32_t j = incl - cnt;
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const uint32_t kp = (keepm >> i) & 1u;
                    sp[kp ? j : 512u + (uint32_t)lane] = (uint16_t)(q0 + i);  // (tile positions < 65,536)
                    j += kp;
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
                for (uint32_t e = lane; e < total; e += 64) {
                    const uint32_t p = sp[e];
                    const uint64_t k = CANON ? l0_key_of<2, true>(s_code, p, a.total_bits, a.symbols)
                                             : l0_key<2>(s_code, p, a.total_bits);
                    kout[o + e] = k;
                    vout[o + e] = (uint32_t)(P0 + p);
                    nd_out[o + e] = (uint8_t)dg_of(k, d0);
                }
                continue;
            }
            {
                // one ballot per row of 64 positions
                const uint32_t wbase = R0 + wave * (kSI * 64);
                uint64_t key[kSI];
                uint32_t at[kSI];
                uint32_t keepm = 0, kept = 0;
#pragma unroll
                for (int i = 0; i < kSI; ++i) {
                    const uint32_t p = wbase + i * 64 + lane;
                    key[i] = l0_key_of<BITS, CANON>(s_code, p, a.total_bits, a.symbols);
                    const bool keep = l0_valid(s_dol, p, a.symbols) && P0 + p < a.hi && l0_owned_key(key[i], a);
                    const uint64_t m = __ballot(keep);
                    at[i] = kept + lanes_below(m);
                    kept += (uint32_t)__popcll(m);
                    keepm |= (keep ? 1u : 0u) << i;
                }
                if (!STORE) {
                    if (lane == 0) wave_cnt[wslot] = kept;
                    continue;
                }
                const uint64_t base = MODE == 2 ? chunk_offset(kept, r) : (uint64_t)wave_off[wslot];
#pragma unroll
                for (int i = 0; i < kSI; ++i) {
                    if ((keepm >> i) & 1u) {
                        const uint64_t o = base + at[i];
                        kout[o] = key[i];
                        vout[o] = (uint32_t)(P0 + wbase + i * 64 + lane);
                        nd_out[o] = (uint8_t)dg_of(key[i], d0);
                    }
                }
            }
        }  // rounds
    }
    if (MODE == 2 && tid == 0 && blockIdx.x * tpw < ntiles) wave_cnt[blockIdx.x] = (uint32_t)run;
}

// Key-range select from the packed copy, SWAR (round 6): forward 2-bit keys of <= 32 symbols whose
// sequence has a 2-bit packed copy (a.pk_code / a.pk_dol: 32 positions per u64 of codes and u32 of
// stops).  No LDS tile, no barrier: each WAVE walks its own chunk of gpw consecutive 32-position
// groups, 64 groups (2,048 positions) per step, one group per lane, and appends its kept k-mers at
// a running offset into its own region of the output, [first group * 32, + gpw * 32) -- the pieces
// of one bucket in position order, as the workgroup chunks of msd0_select_kernel<..., 2> are.
// Per lane and group (w = the group's codes, x2 = the top half of the next group's codes):
//   ownership digit of position j = the top own_bits bits of the 32-bit window at bit 2 j of
//   w:x2 (one funnel shift); the range test is one subtract and one compare against the range
//   shifted to the window's top, so the digit is never extracted (~4 VALU per position; the tile
//   select spent ~20 per position, VALU-bound at 2.8 ms per C3 rank);
//   stops: a lane with a stop in its 64-position window smears them over S positions in 5
//   doubling steps (all 32 positions at once).
// The kept positions are staged per wave as group-relative u16 in position order (a loop over the
// set bits of the keep mask), the step's 65 code words beside them, and the k-mers leave as one
// coalesced run: key (re-derived from the staged words), start, L0 digit byte.
constexpr int kRselW = 4;  // waves per workgroup (independent: no barrier)
__global__ __launch_bounds__(kRselW * 64) void msd0_rsel_kernel(L0Args a, Dig d0, uint64_t ngroups, uint64_t gpw,
                                                                 uint32_t lo_w, uint32_t spm1_w,
                                                                 uint32_t *__restrict__ wave_cnt,
                                                                 uint64_t *__restrict__ kout,
                                                                 uint32_t *__restrict__ vout,
                                                                 uint8_t *__restrict__ nd_out) {
    __shared__ uint16_t s_pos[kRselW][2048];
    __shared__ uint64_t s_w[kRselW][65];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t gw = (uint64_t)blockIdx.x * kRselW + wave;
    const uint64_t g0 = gw * gpw, g1 = min(g0 + gpw, ngroups);
    uint16_t *sp = s_pos[wave];
    uint64_t *sw = s_w[wave];
    const int S = a.symbols, B = a.total_bits;
    uint64_t run = 0;
    const uint64_t out0 = g0 * 32;
    // software pipeline: the next step's words fly while this one is processed
    uint64_t w = 0, w1 = 0;
    uint32_t d = 0, d1 = 0;
    auto load = [&](uint64_t base) {
        const uint64_t g = min(base + (uint64_t)lane, ngroups - 1);
        w = a.pk_code[g];
        w1 = a.pk_code[g + 1];
        d = a.pk_dol[g];
        d1 = a.pk_dol[g + 1];
    };
    if (g0 < g1) load(g0);
    for (uint64_t base = g0; base < g1; base += 64) {
        const uint64_t W0 = w, W1 = w1;
        const uint32_t D0 = d, D1 = d1;
        const bool live = base + (uint64_t)lane < g1;
        if (base + 64 < g1) load(base + 64);
        // ownership: position j <-> bit 31 - j of m (MSB first, the order of the staging loop)
        const uint32_t x0 = (uint32_t)(W0 >> 32), x1 = (uint32_t)W0, x2 = (uint32_t)(W1 >> 32);
        uint32_t m = 0;
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            const int r = (2 * j) & 31;
            const uint32_t hi = j < 16 ? x0 : x1, lo = j < 16 ? x1 : x2;
            const uint32_t win = r ? __builtin_amdgcn_alignbit(hi, lo, 32 - r) : hi;
            m = (m << 1) | (uint32_t)(win - lo_w <= spm1_w);
        }
        // stops: invalid where a stop lies in [j, j + S); D0 / D1 bit 31 - i = position i
        if (__ballot((D0 | D1) != 0)) {
            uint64_t x = ((uint64_t)D0 << 32) | D1;
            uint64_t sm = x;  // sm: a stop in [j, j + len)
            int len = 1;
#pragma unroll
            for (int s = 1; s < 32; s <<= 1) {
                if (2 * len <= S) {
                    sm |= sm << len;
                    len *= 2;
                }
            }
            if (len < S) sm |= sm << (S - len);
            m &= ~(uint32_t)(sm >> 32);
        }
        if (!live) m = 0;
        const uint32_t cnt = (uint32_t)__popc(m);
        const uint32_t incl = wave_incl_scan(cnt);
        const uint32_t total = __builtin_amdgcn_readlane(incl, 63);
        if (total == 0) continue;
        // stage: the group-relative positions of the kept k-mers in position order, the words
        uint32_t j = incl - cnt;
        while (m) {
            const uint32_t b = __clz(m);
            sp[j++] = (uint16_t)(lane * 32 + b);
            m ^= 0x80000000u >> b;
        }
        sw[lane] = W0;
        if (lane == 63) sw[64] = W1;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
        const uint64_t o = out0 + run, P0 = base * 32;
        for (uint32_t e = lane; e < total; e += 64) {
            const uint32_t p = sp[e], q = p >> 5, s = (p & 31) * 2;
            const uint64_t A = sw[q];
            const uint64_t T = s ? (A << s) | (sw[q + 1] >> (64 - s)) : A;
            const uint64_t k = T >> (64 - B);
            kout[o + e] = k;
            vout[o + e] = (uint32_t)(P0 + p);
            nd_out[o + e] = (uint8_t)dg_of(k, d0);
        }
        run += total;
        // the next step's staging overwrites these slots: every lane has read them
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
    }
    if (lane == 0 && g0 < ngroups) wave_cnt[gw] = (uint32_t)run;
}

// ---------------------------------------------------------------------------------------------
// Key-range ranks' L0, compaction first (round 6): the fused select of msd0_pipe_kernel<..., OWN>
// ranked, staged and keyed EVERY position of the sequence to store the ~1/N it keeps (7.7 ms over
// C3 at any N).  These two kernels test the positions with the SWAR range test of msd0_rsel_kernel
// (forward 2-bit keys of <= 32 symbols, packed copy), compact the kept ones per tile in position
// order, and only then rank, stage and store them -- the L0 partition of the rank's k-mers
// straight from the sequence: no select pass, no 13-byte round trip, no level from pieces.
// Tiles are the L0's (kP0Tile = 768 groups of 32 positions, l0_count's tables); threads < 768
// take one group each in the test, the kept elements then spread over all 1,024 threads in the
// partition's wave-major item order (stable: items of a wave in order, waves in order).
// ---------------------------------------------------------------------------------------------
constexpr int kOwnT = 1024, kOwnG = kP0Tile / 32;  // threads, groups per tile
constexpr int kOwnI = kP0Tile / kOwnT;             // items per thread (capacity: every position)
static_assert(kOwnG <= kOwnT && kOwnI * kOwnT == kP0Tile, "one group per thread; every position fits");

struct OwnTest {
    uint32_t lo_w, spm1_w;  // the range shifted to the top of a 32-bit window (msd0_rsel_kernel)
};

// keep mask of the group at position P (bit 31 - j = position P + j): in [a.lo, a.hi), no stop in
// [j, j + S), ownership digit in range; W0 / W1 / D0 / D1 the group's and the next group's words.
// Wave-uniform call (a ballot inside).
__device__ __forceinline__ uint32_t own_keep(const L0Args &a, OwnTest ot, uint64_t P, uint64_t W0, uint64_t W1,
                                             uint32_t D0, uint32_t D1, bool live) {
    const uint32_t x0 = (uint32_t)(W0 >> 32), x1 = (uint32_t)W0, x2 = (uint32_t)(W1 >> 32);
    uint32_t m = 0;
#pragma unroll
    for (int j = 0; j < 32; ++j) {
        const int r = (2 * j) & 31;
        const uint32_t hi = j < 16 ? x0 : x1, lo = j < 16 ? x1 : x2;
        const uint32_t win = r ? __builtin_amdgcn_alignbit(hi, lo, 32 - r) : hi;
        m = (m << 1) | (uint32_t)(win - ot.lo_w <= ot.spm1_w);
    }
    if (__ballot(live && (D0 | D1) != 0)) {
        uint64_t sm = ((uint64_t)D0 << 32) | D1;
        int len = 1;
#pragma unroll
        for (int s = 1; s < 32; s <<= 1) {
            if (2 * len <= a.symbols) {
                sm |= sm << len;
                len *= 2;
            }
        }
        if (len < a.symbols) sm |= sm << (a.symbols - len);
        m &= ~(uint32_t)(sm >> 32);
    }
    const uint64_t jb = a.lo > P ? a.lo - P : 0, je = a.hi > P ? min(a.hi - P, (uint64_t)32) : 0;
    m &= jb < je ? (uint32_t)((0xFFFFFFFFull >> jb) & ~(0xFFFFFFFFull >> je)) : 0u;
    return live ? m : 0u;
}

// the B-bit key of position j of a group (j in [0, 32))
__device__ __forceinline__ uint64_t group_key(uint64_t W0, uint64_t W1, uint32_t j, int B) {
    const uint32_t s = 2 * j;
    const uint64_t T = s ? (W0 << s) | (W1 >> (64 - s)) : W0;
    return T >> (64 - B);
}

// count pass: per-tile histograms of the kept k-mers' L0 digits (R bits)
template <int R>
__global__ __launch_bounds__(kOwnT) void own_count_kernel(L0Args a, Dig d0, OwnTest ot, uint32_t *__restrict__ tile_hist,
                                                           uint32_t ntiles) {
    constexpr int RADIX = 1 << R, NC = 4;
    __shared__ uint32_t s_hist[RADIX * NC];
    const int t = threadIdx.x;
    const uint64_t g_end = (a.hi + 31) / 32;
    for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        for (int i = t; i < RADIX * NC; i += kOwnT) s_hist[i] = 0;
        __syncthreads();
        if (t < kOwnG) {
            const uint64_t g = a.lo / 32 + (uint64_t)tile * kOwnG + t;
            const bool live = g < g_end;
            const uint64_t gc = live ? g : g_end - 1;
            const uint64_t W0 = a.pk_code[gc], W1 = a.pk_code[gc + 1];
            uint32_t m = own_keep(a, ot, gc * 32, W0, W1, a.pk_dol[gc], a.pk_dol[gc + 1], live);
            while (m) {
                const uint32_t j = __clz(m);
                m ^= 0x80000000u >> j;
                atomicAdd(&s_hist[dg_of(group_key(W0, W1, j, a.total_bits), d0) * NC + (t & (NC - 1))], 1u);
            }
        }
        __syncthreads();
        for (int i = t; i < RADIX; i += kOwnT) {
            uint32_t h = 0;
#pragma unroll
            for (int c = 0; c < NC; ++c) h += s_hist[i * NC + c];
            tile_hist[(uint64_t)tile * RADIX + i] = h;
        }
    }
}

// partition pass: the kept k-mers of each tile compacted, ranked by their L0 digit (R bits), staged
// and stored at the tile's digit offsets -- (key, start, next digit) or the packed L0 form (P88)
template <int R, bool P88>
__global__ __launch_bounds__(kOwnT) void own_part_kernel(L0Args a, Dig d0, OwnTest ot,
                                                          const uint32_t *__restrict__ tile_off,
                                                          uint64_t *__restrict__ kout, uint32_t *__restrict__ vout,
                                                          uint32_t ntiles, NextDigits nd) {
    constexpr int RADIX = 1 << R, NW = kOwnT / 64;
    __shared__ uint16_t s_pos[kP0Tile];             // kept positions in order, then in digit order
    __shared__ uint64_t s_code[kOwnG + 1];
    __shared__ uint32_t s_wc[NW * RADIX];
    __shared__ uint32_t s_wsum[NW];
    __shared__ uint32_t s_start[RADIX + 1];
    __shared__ uint32_t s_toff[RADIX];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const uint64_t g_end = (a.hi + 31) / 32;
    for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const uint64_t g0 = a.lo / 32 + (uint64_t)tile * kOwnG;
        if (t < RADIX) s_toff[t] = tile_off[(uint64_t)tile * RADIX + t];
        uint32_t *wc = s_wc + wave * RADIX;
#pragma unroll
        for (int u = 0; u < (RADIX + 63) / 64; ++u)
            if (u * 64 + lane < RADIX) wc[u * 64 + lane] = 0;
        // 1. test: keep mask and count of this thread's group; its code words into LDS
        uint32_t m = 0;
        if (t < kOwnG) {
            const uint64_t g = g0 + t;
            const bool live = g < g_end;
            const uint64_t gc = live ? g : g_end - 1;
            const uint64_t W0 = a.pk_code[gc], W1 = a.pk_code[gc + 1];
            m = own_keep(a, ot, gc * 32, W0, W1, a.pk_dol[gc], a.pk_dol[gc + 1], live);
            s_code[t] = W0;
            if (t == kOwnG - 1) s_code[kOwnG] = W1;
        }
        const uint32_t cnt = (uint32_t)__popc(m);
        const uint32_t incl = wave_incl_scan(cnt);
        if (lane == 63) s_wsum[wave] = incl;
        __syncthreads();
        uint32_t pre = 0, total = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            const uint32_t v = s_wsum[w];
            pre += w < wave ? v : 0u;
            total += v;
        }
        // 2. compaction: the kept positions (tile-relative) in position order
        {
            uint32_t j = pre + incl - cnt;
            while (m) {
                const uint32_t b = __clz(m);
                m ^= 0x80000000u >> b;
                s_pos[j++] = (uint16_t)(t * 32 + b);
            }
        }
        __syncthreads();
        // 3. rank: element e = wave * kOwnI * 64 + i * 64 + lane (wave-major, position order)
        uint32_t dr[kOwnI];
        uint16_t pp[kOwnI];
        const uint32_t e0 = wave * (kOwnI * 64);
#pragma unroll
        for (int i = 0; i < kOwnI; ++i) {
            dr[i] = ~0u;
            pp[i] = 0;
            if (e0 + i * 64 < total) {  // (wave-uniform)
                const uint32_t e = e0 + i * 64 + lane;
                const bool valid = e < total;
                const uint32_t p = s_pos[valid ? e : 0];
                const uint32_t dig = dg_of(l0_key<2>(s_code, p, a.total_bits), d0);
                const uint32_t rk = rank_atomic(wc, dig, valid);
                dr[i] = valid ? dig | (rk << 8) : ~0u;
                pp[i] = (uint16_t)p;
            }
        }
        __syncthreads();  // ranks final; every compacted position read
        // 4. digit starts: per-digit totals over the waves, their scan
        uint32_t dtot = 0, dincl = 0;
        if (t < RADIX) {
#pragma unroll
            for (int w = 0; w < NW; ++w) {
                const uint32_t v = s_wc[w * RADIX + t];
                s_wc[w * RADIX + t] = dtot;
                dtot += v;
            }
            dincl = wave_incl_scan(dtot);
            if (lane == 63) s_wsum[wave] = dincl;
        }
        __syncthreads();
        if (t < RADIX) {
            uint32_t p2 = 0;
            for (int w = 0; w < wave; ++w) p2 += s_wsum[w];
            const uint32_t st = p2 + dincl - dtot;
            s_start[t] = st;
            s_toff[t] -= st;
        }
        __syncthreads();
        // 5. stage in digit order (over the compacted positions: all were read in 3)
#pragma unroll
        for (int i = 0; i < kOwnI; ++i) {
            if (dr[i] != ~0u) {
                const uint32_t dg = dr[i] & 0xFFu;
                s_pos[s_start[dg] + wc[dg] + (dr[i] >> 8)] = pp[i];
            }
        }
        __syncthreads();
        // 6. store: runs of each digit at the tile's offsets
        const uint64_t P0 = g0 * 32;
        for (uint32_t s = t; s < total; s += kOwnT) {
            const uint32_t p = s_pos[s];
            const uint64_t key = l0_key<2>(s_code, p, a.total_bits);
            const uint64_t o = (uint64_t)s_toff[dg_of(key, d0)] + s;
            const uint32_t st = (uint32_t)(P0 + p);
            if (P88) {
                const int shi = nd.pshi;
                kout[o] = (key << shi) | (st >> (32 - shi));
                nd.out16[o] = (uint16_t)(st & ((1u << (32 - shi)) - 1));
            } else {
                kout[o] = key;
                vout[o] = st;
            }
            nd.out[o] = (uint8_t)dg_of(key, nd.d);
        }
        __syncthreads();  // the staging and the codes are read before the next tile's
    }
}

// The same histogram from the packed copy, SWAR (round 6; forward 2-bit keys of <= 32 symbols, as
// msd0_rsel_kernel): one 32-position group per lane, the digit of position j the top own_bits bits
// of the 32-bit window at bit 2 j of the group's codes; positions that start no k-mer (a stop in
// [j, j + S), or outside [lo, hi)) count into junk bins (4096 + 64 j + lane: conflict-free) instead
// of being branched around.  One LDS table per workgroup, its waves walking the chunk together.
__global__ __launch_bounds__(kRselW * 64) void own_hist_rsel_kernel(L0Args a, uint64_t gpb,
                                                                     uint32_t *__restrict__ ghist) {
    __shared__ uint32_t s_hist[4096 + 64 * 32];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < 4096 + 64 * 32; i += kRselW * 64) s_hist[i] = 0;
    __syncthreads();
    const uint64_t G0 = a.lo / 32, G1 = (a.hi + 31) / 32;
    const uint64_t g0 = G0 + blockIdx.x * gpb, g1 = min(g0 + gpb, G1);
    const int S = a.symbols, osh = 32 - a.own_bits;
    for (uint64_t base = g0 + wave * 64; base < g1; base += kRselW * 64) {
        const uint64_t g = base + lane;
        const bool live = g < g1;
        const uint64_t gc = live ? g : g1 - 1;
        const uint64_t W0 = a.pk_code[gc], W1 = a.pk_code[gc + 1];
        const uint32_t D0 = a.pk_dol[gc], D1 = a.pk_dol[gc + 1];
        // valid positions, bit 31 - j = position j: inside [lo, hi) ...
        const uint64_t P0 = gc * 32;
        const uint64_t jb = a.lo > P0 ? a.lo - P0 : 0, je = a.hi - P0 < 32 ? a.hi - P0 : 32;
        uint32_t m = live && jb < je ? (uint32_t)((0xFFFFFFFFull >> jb) & ~(0xFFFFFFFFull >> je)) : 0u;
        // ... and no stop in [j, j + S)
        if (__ballot((D0 | D1) != 0)) {
            uint64_t sm = ((uint64_t)D0 << 32) | D1;
            int len = 1;
#pragma unroll
            for (int s = 1; s < 32; s <<= 1) {
                if (2 * len <= S) {
                    sm |= sm << len;
                    len *= 2;
                }
            }
            if (len < S) sm |= sm << (S - len);
            m &= ~(uint32_t)(sm >> 32);
        }
        const uint32_t x0 = (uint32_t)(W0 >> 32), x1 = (uint32_t)W0, x2 = (uint32_t)(W1 >> 32), inv = ~m;
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            const int r = (2 * j) & 31;
            const uint32_t hi = j < 16 ? x0 : x1, lo = j < 16 ? x1 : x2;
            const uint32_t win = r ? __builtin_amdgcn_alignbit(hi, lo, 32 - r) : hi;
            // (an invalid position's bin depends on the lane only: the N runs of a mixed sba would
            // otherwise send a whole wave to one address, serialising the atomic)
            const uint32_t bin = ((inv >> (31 - j)) & 1u) ? 4096u + 64u * j + (uint32_t)lane : win >> osh;
            atomicAdd(&s_hist[bin], 1u);
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < (1 << a.own_bits); i += kRselW * 64)
        if (s_hist[i]) atomicAdd(&ghist[i], s_hist[i]);
}

// Ownership-digit histogram of a key-range shard's position share: the top own_bits (<= 12) bits
// of every k-mer starting in [a.lo, a.hi), one LDS table per workgroup flushed into ghist.
template <int BITS, bool CANON>
__global__ __launch_bounds__(kST) void own_hist_kernel(L0Args a, uint32_t ntiles, uint32_t *__restrict__ ghist) {
    using P = L0Pack<BITS, kSTile>;
    __shared__ uint64_t s_code[P::kCodeWords];
    __shared__ uint32_t s_dol[P::kGroups];
    __shared__ uint8_t s_lut4[256];
    __shared__ uint32_t s_hist[4096];
    const int tid = threadIdx.x;
    if (tid < 256) s_lut4[tid] = c_code4_msd[tid];
    for (int i = tid; i < 4096; i += kST) s_hist[i] = 0;
    const int osh = a.total_bits - a.own_bits;
    uint64_t rr[L0Units<BITS, kSTile, kST>::kPer];
    if (blockIdx.x < ntiles) l0_load<BITS, kSTile, kST>(a, a.lo + (uint64_t)blockIdx.x * kSTile, rr);
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const uint64_t P0 = a.lo + (uint64_t)t * kSTile;
        __syncthreads();  // the LUT and the zeroed table; the previous tile's codes have been read
        l0_pack<BITS, kSTile, kST>(rr, s_code, s_dol, s_lut4, a.acgt_only, a.pk_code != nullptr);
        __syncthreads();
        if (t + gridDim.x < ntiles) l0_load<BITS, kSTile, kST>(a, P0 + (uint64_t)gridDim.x * kSTile, rr);
#pragma unroll
        for (int i = 0; i < kSI * kSR; ++i) {
            const uint32_t p = i * kST + tid;
            const uint64_t key = l0_key_of<BITS, CANON>(s_code, p, a.total_bits, a.symbols);
            if (l0_valid(s_dol, p, a.symbols) && P0 + p < a.hi) atomicAdd(&s_hist[(uint32_t)(key >> osh)], 1u);
        }
    }
    __syncthreads();
    for (int i = tid; i < (1 << a.own_bits); i += kST)
        if (s_hist[i]) atomicAdd(&ghist[i], s_hist[i]);
}

// ---------------------------------------------------------------------------------------------
// 2-bit packed copy of an ACGT sba: one u64 of codes (A0 C1 G2 T3, MSB first) and one u32 stop
// mask ('$') per 32 positions -- the layout the L0 kernels build in LDS.  Packed once per sort and
// read by every full-sequence pass (L0 count and partition; histogram, select count and store of
// the key-range shards) instead of each pass re-packing the bytes: 0.28 B per position.
// ---------------------------------------------------------------------------------------------
template <bool NONACGT = false>
__global__ __launch_bounds__(256) void pack2_kernel(const uint8_t *__restrict__ sba, uint64_t nwords,
                                                    uint64_t *__restrict__ code, uint32_t *__restrict__ dol) {
    for (uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x; g < nwords; g += (uint64_t)gridDim.x * 256) {
        uint64_t cw;
        uint32_t dw;
        pack2_word<NONACGT>(sba + 32 * g, cw, dw);
        code[g] = cw;
        dol[g] = dw;
    }
}

// (the transfer's resident copy: stops at every non-ACGT byte, pack2_word<true>)
hipError_t launch_pack2(const uint8_t *from, uint64_t nwords, uint64_t *code, uint32_t *dol, hipStream_t s) {
    if (nwords == 0) return hipSuccess;
    hipLaunchKernelGGL(pack2_kernel<true>, dim3((unsigned)std::min<uint64_t>((nwords + 255) / 256, 65536)), dim3(256),
                       0, s, from, nwords, code, dol);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// column-wise segmented exclusive scan of per-tile digit histograms -> per-tile digit offsets
// (one thread per digit: blockDim = RADIX)
// ---------------------------------------------------------------------------------------------
// Column scans of per-tile digit histograms.  Threads per block: min(RADIX, 1024); wider digit
// spaces (the wide L0's 2048) take blockIdx.y for the digit block (chunk sums, tile apply) or
// several consecutive digits per thread (the bucket scan).
template <int RADIX>
constexpr int scan_threads() { return RADIX < 1024 ? RADIX : 1024; }

template <int RADIX>
__global__ __launch_bounds__(scan_threads<RADIX>()) void chunk_sum_kernel(const uint32_t *__restrict__ tile_hist,
                                                          const uint32_t *__restrict__ c_first,
                                                          const uint32_t *__restrict__ c_ntiles,
                                                          uint32_t *__restrict__ chunk_hist) {
    const int d = blockIdx.y * scan_threads<RADIX>() + threadIdx.x;
    const uint64_t f = c_first[blockIdx.x];
    const uint32_t nt = c_ntiles[blockIdx.x];
    uint32_t acc = 0;
    uint32_t i = 0;
    for (; i + 8 <= nt; i += 8) {
        uint32_t v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = tile_hist[(f + i + u) * RADIX + d];
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; i < nt; ++i) acc += tile_hist[(f + i) * RADIX + d];
    chunk_hist[(uint64_t)blockIdx.x * RADIX + d] = acc;
}

// one block per bucket: chunk bases within the bucket, digit bases, digit counts
template <int RADIX>
__global__ __launch_bounds__(scan_threads<RADIX>()) void seg_scan_kernel(uint32_t *__restrict__ chunk_hist,
                                                         const uint32_t *__restrict__ s_cfirst,
                                                         const uint32_t *__restrict__ s_nchunks,
                                                         const uint32_t *__restrict__ s_start,
                                                         uint32_t *__restrict__ seg_base, uint32_t *__restrict__ seg_cnt) {
    constexpr int TH = scan_threads<RADIX>(), DPT = RADIX / TH;  // DPT consecutive digits per thread
    __shared__ uint32_t s_wsum[TH / 64];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const uint64_t cf = s_cfirst[blockIdx.x];
    const uint32_t nc = s_nchunks[blockIdx.x];
    uint32_t run[DPT], sum = 0;
#pragma unroll
    for (int k = 0; k < DPT; ++k) {
        const int d = t * DPT + k;
        run[k] = 0;
        for (uint32_t i = 0; i < nc; ++i) {
            const uint32_t v = chunk_hist[(cf + i) * RADIX + d];
            chunk_hist[(cf + i) * RADIX + d] = run[k];
            run[k] += v;
        }
        sum += run[k];
    }
    uint32_t incl = sum;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(incl, off);
        if (lane >= off) incl += y;
    }
    if (lane == 63) s_wsum[wave] = incl;
    __syncthreads();
    uint32_t pre = 0;
    for (int w = 0; w < wave; ++w) pre += s_wsum[w];
    uint32_t base = s_start[blockIdx.x] + pre + incl - sum;
#pragma unroll
    for (int k = 0; k < DPT; ++k) {
        const int d = t * DPT + k;
        seg_base[(uint64_t)blockIdx.x * RADIX + d] = base;
        seg_cnt[(uint64_t)blockIdx.x * RADIX + d] = run[k];
        for (uint32_t c = 0; c < nc; ++c) chunk_hist[(cf + c) * RADIX + d] += base;
        base += run[k];
    }
}

template <int RADIX>
__global__ __launch_bounds__(scan_threads<RADIX>()) void tile_apply_kernel(uint32_t *__restrict__ tile_hist,
                                                           const uint32_t *__restrict__ c_first,
                                                           const uint32_t *__restrict__ c_ntiles,
                                                           const uint32_t *__restrict__ chunk_base) {
    const int d = blockIdx.y * scan_threads<RADIX>() + threadIdx.x;
    const uint64_t f = c_first[blockIdx.x];
    const uint32_t nt = c_ntiles[blockIdx.x];
    uint32_t run = chunk_base[(uint64_t)blockIdx.x * RADIX + d];
    uint32_t i = 0;
    for (; i + 8 <= nt; i += 8) {
        uint32_t v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = tile_hist[(f + i + u) * RADIX + d];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            tile_hist[(f + i + u) * RADIX + d] = run;
            run += v[u];
        }
    }
    for (; i < nt; ++i) {
        const uint32_t v = tile_hist[(f + i) * RADIX + d];
        tile_hist[(f + i) * RADIX + d] = run;
        run += v;
    }
}

// wave-aggregated append of one entry per flagged lane; returns the entry index
__device__ __forceinline__ uint32_t wave_append(bool flag, uint32_t *counter, int lane) {
    const uint64_t m = __ballot(flag);
    if (!m) return 0;
    const int leader = __ffsll((unsigned long long)m) - 1;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(counter, (uint32_t)__popcll(m));
    base = __shfl(base, leader);
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    return base + (uint32_t)__popcll(m & lt_mask);
}

// list counters (device, one array): next global level, done, then the local classes
enum { kCtrBig = 0, kCtrDone = 1, kCtrLoc = 2, kLists = kCtrLoc + kLocal, kCtrNbCopy = kLists, kCtrN = 8 + 2 };
// (kCtrNbCopy: the big list's count kept while its counter restarts, MsdDriver::drop_uniform_dev)
// element sums per list, then the next global level's tile and chunk totals (its tile tables'
// sizes, known with the list counts so that planning the level needs no read-back of its own)
enum { kSumTiles = kLists, kSumChunks = kLists + 1, kSumN = kLists + 2 };

__host__ __device__ inline uint32_t tiles_of(uint32_t len, uint32_t tile) { return (len + tile - 1) / tile; }
__host__ __device__ inline uint32_t chunks_of(uint32_t len, uint32_t tile, uint32_t ctiles) {
    return (tiles_of(len, tile) + ctiles - 1) / ctiles;
}

struct Lists {
    uint32_t *nb_start, *nb_len;                 // buckets for the next global level
    uint32_t *dn_start, *dn_len;                 // key bits exhausted: final as they stand
    uint8_t *dn_par;
    uint2 *loc[kLocal];                          // local entries by class
    // per entry: the bucket's sorted key bits (its prefix), | kCompact when its elements are
    // stored compact (a compact level's output, see level_pass); null: not recorded
    uint64_t *nb_pref;
    uint64_t *loc_pref[kLocal];
};

// A compact level writes per element, in the key array, the key bits below the next 8-bit digit
// (high half) and the start (low half), and that digit in the digit bytes: 9 B instead of 12 (and
// two stores instead of three); the bucket's prefix completes the key.
constexpr uint64_t kCompact = 1ull << 63;

__device__ __forceinline__ uint64_t compact_key(uint64_t pref, int hi, int B, uint32_t dig, uint32_t low) {
    const int rem = B - hi;  // 9..40
    return ((pref & ~kCompact) << rem) | ((uint64_t)dig << (rem - 8)) | (uint64_t)low;
}

// local class of a bucket of <= kBlockMax elements
__host__ __device__ constexpr uint32_t local_cap(int cls) {
    return cls == 0 ? 256 : cls == 1 ? 512 : cls == 2 ? 1024 : cls == 3 ? 4096 : cls == 5 ? 8192 : kTiny;
}

// list of a live sub-bucket of `size` elements (kCtr* index)
__device__ __forceinline__ int list_of(uint32_t size, int hi, int B, bool allow_big) {
    if (hi >= B) return kCtrDone;
    if (size > (uint32_t)kBlockMax && allow_big) return kCtrBig;
    if (size <= (uint32_t)kTiny) return kCtrLoc + 4;
    return kCtrLoc + (size <= local_cap(0) ? 0 : size <= local_cap(1) ? 1 : size <= local_cap(2) ? 2
                      : size <= local_cap(3) ? 3 : 5);
}

// entry `at` of list l for a sub-bucket
__device__ __forceinline__ void put_entry(const Lists &L, int l, uint32_t at, uint32_t st, uint32_t size, int hi,
                                          int parity, uint64_t pref = 0) {
    // (global stores: flat ones, through pointers read from memory, would make every later
    // memory wait of the kernel a full drain)
    if (l == kCtrBig) {
        gmem(L.nb_start)[at] = st;
        gmem(L.nb_len)[at] = size;
        if (L.nb_pref) gmem(L.nb_pref)[at] = pref;
    } else if (l == kCtrDone) {
        gmem(L.dn_start)[at] = st;
        gmem(L.dn_len)[at] = size;
        gmem(L.dn_par)[at] = (uint8_t)parity;
    } else {
        const uint2 le = local_entry(st, size, hi, parity);
        gmem(reinterpret_cast<uint64_t *>(L.loc[l - kCtrLoc]))[at] = ((uint64_t)le.y << 32) | le.x;
        if (L.loc_pref[l - kCtrLoc]) gmem(L.loc_pref[l - kCtrLoc])[at] = pref;
    }
}

// route one sub-bucket (size >= 1) by size; hi = key bits sorted once it is cut out
__device__ __forceinline__ void route(uint32_t st, uint32_t size, int hi, int B, int parity, bool allow_big,
                                      const Lists &L, uint32_t *ctr, int lane) {
    const int li = size >= 1 ? list_of(size, hi, B, allow_big) : -1;
#pragma unroll
    for (int l = 0; l < kLists; ++l) {
        const uint32_t at = wave_append(li == l, &ctr[l], lane);
        if (li == l) put_entry(L, l, at, st, size, hi, parity);
    }
}

// The sub-buckets of one global level, one per thread: a workgroup-aggregated append (one
// atomic per list per workgroup) into the next-level / done / block-local / wave-local lists;
// sums[l] += elements routed to list l (for the profile's work counts).
constexpr int kClassT = 1024;

// Prefixes: sub-bucket i of a partition by pw-bit digits has parent i >> pw (prefix ppref[i >> pw],
// 0 when null) and digit i & (2^pw - 1); with pw = 0 the entries are whole buckets (prefix ppref[i]).
// compact: the level wrote compact elements (the entries get kCompact).
__global__ __launch_bounds__(kClassT) void classify_kernel(const uint32_t *__restrict__ seg_base,
                                                           const uint32_t *__restrict__ seg_cnt, uint64_t nsub, int hi,
                                                           int B, int parity, Lists L, uint32_t *__restrict__ ctr,
                                                           unsigned long long *__restrict__ sums, uint32_t min_size,
                                                           const uint64_t *__restrict__ ppref, int pw, int compact,
                                                           uint32_t tile, uint32_t ctiles) {
    constexpr int NW = kClassT / 64;
    __shared__ uint32_t s_cnt[kLists][NW];
    __shared__ uint32_t s_elems[kLists][NW];
    __shared__ uint32_t s_base[kLists];
    __shared__ uint32_t s_tc[2][NW];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t i = (uint64_t)blockIdx.x * kClassT + tid;
    const uint32_t size = i < nsub ? seg_cnt[i] : 0, st = i < nsub ? seg_base[i] : 0;
    const int li = size >= min_size ? list_of(size, hi, B, true) : -1;
    bool f[kLists];
#pragma unroll
    for (int l = 0; l < kLists; ++l) f[l] = li == l;
    uint32_t below[kLists];
#pragma unroll
    for (int l = 0; l < kLists; ++l) {
        const uint64_t m = __ballot(f[l]);
        below[l] = lanes_below(m);
        uint32_t e = f[l] ? size : 0;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) e += __shfl_xor(e, off);
        if (lane == 0) {
            s_cnt[l][wave] = (uint32_t)__popcll(m);
            s_elems[l][wave] = e;
        }
    }
    {
        uint32_t tl = li == kCtrBig ? tiles_of(size, tile) : 0, ch = li == kCtrBig ? chunks_of(size, tile, ctiles) : 0;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            tl += __shfl_xor(tl, off);
            ch += __shfl_xor(ch, off);
        }
        if (lane == 0) {
            s_tc[0][wave] = tl;
            s_tc[1][wave] = ch;
        }
    }
    __syncthreads();
    if (tid >= 64 && tid < 66) {  // (another wave than the list totals below)
        unsigned long long t = 0;
        for (int w = 0; w < NW; ++w) t += s_tc[tid - 64][w];
        if (t) atomicAdd(&sums[kSumTiles + tid - 64], t);
    }
    if (tid < kLists) {
        uint32_t tot = 0;
        unsigned long long el = 0;
        for (int w = 0; w < NW; ++w) {
            tot += s_cnt[tid][w];
            el += s_elems[tid][w];
        }
        s_base[tid] = tot ? atomicAdd(&ctr[tid], tot) : 0;
        if (el) atomicAdd(&sums[tid], el);
    }
    __syncthreads();
    uint32_t at[kLists];
#pragma unroll
    for (int l = 0; l < kLists; ++l) {
        uint32_t pre = s_base[l];
        for (int w = 0; w < wave; ++w) pre += s_cnt[l][w];
        at[l] = pre + below[l];
    }
    uint64_t pref = 0;
    if (li >= 0) {
        if (pw > 0) pref = ((ppref ? ppref[i >> pw] & ~kCompact : 0ull) << pw) | (i & ((1ull << pw) - 1));
        else pref = ppref ? ppref[i] & ~kCompact : 0ull;
        if (compact) pref |= kCompact;
    }
#pragma unroll
    for (int l = 0; l < kLists; ++l)
        if (li == l) put_entry(L, l, at[l], st, size, hi, parity, pref);
}

// workgroups per bucket (grid.y) of the per-bucket copy kernels below: the buckets they see are
// few but can be huge (a repeat's group of identical k-mers: 250 K elements at C4), and one
// workgroup walking such a bucket alone took 3 ms per C4 rank
static unsigned bucket_split(uint64_t nbuckets) { return nbuckets <= 4096 ? 32u : nbuckets <= 65536 ? 4u : 1u; }

// (key, start) of packed-pair elements (a MODE 5 level's output, gkm_partition.h) in place, for
// the buckets a packed-pair level's output goes to that do not read pairs: the next level when it
// is not compact, and the local finishing classes.  Bucket j: start bst[j], length blen[j], sorted
// key bits bpref[j] (the top hi of B); gridDim.y workgroups per bucket.
__global__ __launch_bounds__(256) void expand_pair_kernel(const uint32_t *__restrict__ bst,
                                                          const uint32_t *__restrict__ blen,
                                                          const uint64_t *__restrict__ bpref, int hi, int B, int shi,
                                                          uint64_t *__restrict__ kio, const uint16_t *__restrict__ in16,
                                                          uint32_t *__restrict__ vout) {
    const uint64_t st = bst[blockIdx.x];
    const uint32_t len = blen[blockIdx.x];
    const uint64_t top = (bpref[blockIdx.x] & ~kCompact) << (B - hi);
    for (uint32_t e = blockIdx.y * 256 + threadIdx.x; e < len; e += gridDim.y * 256) {
        uint64_t key;
        uint32_t val;
        unpack_pair(kio[st + e], in16[st + e], shi, key, val);
        kio[st + e] = top | key;
        vout[st + e] = val;
    }
}

// the same over local-list entries [first, first + count) (entry: start, len << 8 | hi << 1 | parity;
// prefixes in pref[]) -- the local buckets a packed-pair level's classify listed
__global__ __launch_bounds__(256) void expand_pair_list_kernel(const uint2 *__restrict__ list,
                                                               const uint64_t *__restrict__ pref, uint32_t first,
                                                               int B, int shi, uint64_t *__restrict__ kio,
                                                               const uint16_t *__restrict__ in16,
                                                               uint32_t *__restrict__ vout) {
    const uint2 en = list[first + blockIdx.x];
    const uint64_t st = en.x;
    const uint32_t len = en.y >> 8;
    const int hi = (en.y >> 1) & 127;
    const uint64_t top = (pref[first + blockIdx.x] & ~kCompact) << (B - hi);
    for (uint32_t e = threadIdx.x; e < len; e += 256) {
        uint64_t key;
        uint32_t val;
        unpack_pair(kio[st + e], in16[st + e], shi, key, val);
        kio[st + e] = top | key;
        vout[st + e] = val;
    }
}

// packed-L0 elements (P88: the digit byte above a packed pair) -> (key bits below the sorted ones,
// start)
__device__ __forceinline__ void unpack_p88(uint64_t a, uint32_t lo, uint32_t dg, int shi, uint64_t &rel, uint32_t &val) {
    unpack_pair(a, lo, shi, rel, val);
    rel |= (uint64_t)dg << (64 - shi);
}

// (key, start) of packed-L0 elements in place, for the buckets whose next reader does not take the
// packed form: the big buckets when the level behind the L0 writes no packed pairs itself (gridDim.y
// workgroups per bucket), and the local classes' entries (expand_p88_list_kernel)
__global__ __launch_bounds__(256) void expand_p88_kernel(const uint32_t *__restrict__ bst,
                                                         const uint32_t *__restrict__ blen,
                                                         const uint64_t *__restrict__ bpref, int hi, int B, int shi,
                                                         uint64_t *__restrict__ kio, const uint16_t *__restrict__ in16,
                                                         const uint8_t *__restrict__ in8, uint32_t *__restrict__ vout) {
    const uint64_t st = bst[blockIdx.x];
    const uint32_t len = blen[blockIdx.x];
    const uint64_t top = (bpref[blockIdx.x] & ~kCompact) << (B - hi);
    for (uint32_t e = blockIdx.y * 256 + threadIdx.x; e < len; e += gridDim.y * 256) {
        uint64_t rel;
        uint32_t val;
        unpack_p88(kio[st + e], in16[st + e], in8[st + e], shi, rel, val);
        kio[st + e] = top | rel;
        vout[st + e] = val;
    }
}

__global__ __launch_bounds__(256) void expand_p88_list_kernel(const uint2 *__restrict__ list,
                                                              const uint64_t *__restrict__ pref, int B, int shi,
                                                              uint64_t *__restrict__ kio, const uint16_t *__restrict__ in16,
                                                              const uint8_t *__restrict__ in8,
                                                              uint32_t *__restrict__ vout) {
    const uint2 en = list[blockIdx.x];
    const uint64_t st = en.x;
    const uint32_t len = en.y >> 8;
    const int hi = (en.y >> 1) & 127;
    const uint64_t top = (pref[blockIdx.x] & ~kCompact) << (B - hi);
    for (uint32_t e = threadIdx.x; e < len; e += 256) {
        uint64_t rel;
        uint32_t val;
        unpack_p88(kio[st + e], in16[st + e], in8[st + e], shi, rel, val);
        kio[st + e] = top | rel;
        vout[st + e] = val;
    }
}

// the same over pieces (first_level_from_pieces: the prefetched L0's region buckets): piece j at
// pp[j], pp[np + j] elements, its bucket (the top hi key bits) pp[2 np + j]
__global__ __launch_bounds__(256) void expand_p88_pieces_kernel(const uint64_t *__restrict__ pp, uint32_t np, int hi,
                                                                int B, int shi, uint64_t *__restrict__ kio,
                                                                const uint16_t *__restrict__ in16,
                                                                const uint8_t *__restrict__ in8,
                                                                uint32_t *__restrict__ vout) {
    const uint64_t st = pp[blockIdx.x], len = pp[np + blockIdx.x];
    const uint64_t top = pp[2 * (uint64_t)np + blockIdx.x] << (B - hi);
    for (uint64_t e = blockIdx.y * 256 + threadIdx.x; e < len; e += gridDim.y * 256) {
        uint64_t rel;
        uint32_t val;
        unpack_p88(kio[st + e], in16[st + e], in8[st + e], shi, rel, val);
        kio[st + e] = top | rel;
        vout[st + e] = val;
    }
}

// keys of compact elements (gridDim.y workgroups per bucket): prefix | digit | low bits
__global__ __launch_bounds__(256) void expand_compact_kernel(const uint32_t *__restrict__ bst,
                                                             const uint32_t *__restrict__ blen,
                                                             const uint64_t *__restrict__ bpref, int hi, int B,
                                                             const uint8_t *__restrict__ nd,
                                                             uint64_t *__restrict__ kio, uint32_t *__restrict__ vout,
                                                             const uint32_t *__restrict__ nb_dev = nullptr) {
    if (nb_dev && blockIdx.x >= *nb_dev) return;  // (a grid sized by a bound: the count is on the device)
    const uint64_t st = bst[blockIdx.x];
    const uint32_t len = blen[blockIdx.x];
    const uint64_t pf = bpref[blockIdx.x];
    for (uint32_t e = blockIdx.y * 256 + threadIdx.x; e < len; e += gridDim.y * 256) {
        const uint64_t x = kio[st + e];
        kio[st + e] = compact_key(pf, hi, B, nd[st + e], (uint32_t)(x >> 32));
        vout[st + e] = (uint32_t)x;
    }
}

// tile + chunk tables of a bucket list (one thread per bucket)
// per-tile (start, count) and per-chunk (first tile, tiles) tables of the nseg buckets of a level:
// one thread per tile (j < T) and per chunk (j < C), each finding its bucket by a binary search over
// the buckets' first tile / first chunk (one thread per bucket wrote a whole bucket's tiles
// serially: 0.6 ms for the one 387 M-key bucket of a key-range rank at N = 8)
__device__ __forceinline__ uint32_t owner_of(const uint32_t *__restrict__ first, uint32_t n, uint32_t j) {
    uint32_t lo = 0, hi = n;  // the last bucket with first <= j
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (first[mid] <= j) lo = mid;
        else hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(256) void tile_table_kernel(const uint32_t *__restrict__ s_start,
                                                         const uint32_t *__restrict__ s_len,
                                                         const uint32_t *__restrict__ s_tfirst,
                                                         const uint32_t *__restrict__ s_cfirst, uint32_t nseg,
                                                         uint32_t tile, uint32_t T, uint32_t C, uint32_t ctiles,
                                                         uint32_t *__restrict__ t_start,
                                                         uint32_t *__restrict__ t_count, uint32_t *__restrict__ c_first,
                                                         uint32_t *__restrict__ c_ntiles) {
    const uint32_t j = blockIdx.x * 256 + threadIdx.x;
    if (j < T) {
        const uint32_t s = owner_of(s_tfirst, nseg, j);
        const uint32_t r = j - s_tfirst[s], len = s_len[s];
        t_start[j] = s_start[s] + r * tile;
        t_count[j] = std::min<uint32_t>(tile, len - r * tile);
    }
    if (j < C) {
        const uint32_t s = owner_of(s_cfirst, nseg, j);
        const uint32_t r = j - s_cfirst[s], nt = (s_len[s] + tile - 1) / tile;
        c_first[j] = s_tfirst[s] + r * ctiles;
        c_ntiles[j] = std::min<uint32_t>(ctiles, nt - r * ctiles);
    }
}

__global__ __launch_bounds__(256) void seg_counts_kernel(const uint32_t *__restrict__ s_len, uint32_t nseg,
                                                         uint32_t tile, uint32_t ctiles, uint32_t *__restrict__ ntiles,
                                                         uint32_t *__restrict__ nchunks) {
    const uint32_t s = blockIdx.x * 256 + threadIdx.x;
    if (s >= nseg) return;
    const uint32_t nt = (s_len[s] + tile - 1) / tile;
    ntiles[s] = nt;
    nchunks[s] = (nt + ctiles - 1) / ctiles;
}

// seg_counts_kernel and the exclusive scans of both counts in ONE workgroup, for the level's
// bucket list of up to kSegScanMax entries (C3: 128 / 32 K buckets; the deep levels of a repeat-rich
// genome: tens): one launch instead of seven, the totals already known from the list counters
constexpr uint32_t kSegScanMax = 1u << 16;
__global__ __launch_bounds__(1024) void seg_tiles_scan_kernel(const uint32_t *__restrict__ s_len, uint32_t nseg,
                                                              uint32_t tile, uint32_t ctiles,
                                                              uint32_t *__restrict__ tfirst,
                                                              uint32_t *__restrict__ cfirst,
                                                              uint32_t *__restrict__ nchunks) {
    __shared__ uint32_t s_w[2][16];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t carry_t = 0, carry_c = 0;
    for (uint32_t b0 = 0; b0 < nseg; b0 += 1024) {  // (block-uniform)
        const uint32_t s = b0 + tid;
        const uint32_t nt = s < nseg ? tiles_of(s_len[s], tile) : 0, nc = (nt + ctiles - 1) / ctiles;
        const uint32_t it = wave_incl_scan(nt), ic = wave_incl_scan(nc);
        if (lane == 63) {
            s_w[0][wave] = it;
            s_w[1][wave] = ic;
        }
        __syncthreads();
        uint32_t pt = carry_t, pc = carry_c;
        for (int w = 0; w < 16; ++w) {
            const uint32_t a = s_w[0][w], d = s_w[1][w];
            if (w < wave) {
                pt += a;
                pc += d;
            }
            carry_t += a;
            carry_c += d;
        }
        if (s < nseg) {
            tfirst[s] = pt + it - nt;
            cfirst[s] = pc + ic - nc;
            nchunks[s] = nc;
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------------------------
// local rounds: a bucket of <= T*I elements per workgroup, persistent over a list
// ---------------------------------------------------------------------------------------------
// Per bucket (entry = start, len, hi, parity):
//   1. stable partition by the R-bit digit below the top `hi` bits into LDS (partition_stage);
//   2. each sub-bucket: singleton, or no key bits left after this digit (equal keys, already in
//      start order) -> final; <= kSmall -> rank-by-count on the key (ties: staging order =
//      start order); larger -> left in stable order and re-listed for the next round (its head
//      flags are provisional: that round rewrites them);
//   3. keys, starts and head flags (key differs from its predecessor) are written back in order.
// Output always goes to buffer 0; the bucket is read fully before any write, so in place is safe.
// Loads and stores are branch-free with static counts (clamped to the bucket), so the next
// bucket's loads -- issued once the current one is final in LDS -- overlap its stores.
// Common-prefix skip: x_or = OR over a bucket's keys of (key ^ first key).  The bits of the key
// below the hi sorted ones that are equal in every element need no partition pass: the bucket's
// next digit starts at its highest differing bit.  All keys equal: one last digit (one sub-bucket,
// final).  Repeats make such buckets common (a 30-copy repeat k-mer would otherwise take one round
// per 8 bits).
__device__ __forceinline__ int skip_hi(uint64_t x_or, int B, int hi) {
    const int rem = B - hi;
    if (rem <= 0) return hi;
    x_or &= rem >= 64 ? ~0ull : ((1ull << rem) - 1);
    if (x_or == 0) return max(hi, B - 8);
    return B - 1 - (63 - __clzll(x_or));
}

__device__ __forceinline__ uint64_t wave_or64(uint64_t x) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) x |= __shfl_xor(x, off);
    return x;
}

// compact inputs (first local round after a compact level): where to find the elements' low key
// bits and next digits, and the entries' prefixes
struct CompactIn {
    const uint64_t *pref;  // per list entry (null: no entry is compact)
    const uint8_t *nd;
};

template <int T, int I>
__device__ __forceinline__ void local_load(const uint2 e, const uint64_t *k0, const uint32_t *v0, const uint64_t *k1,
                                           const uint32_t *v1, uint64_t (&key)[I], uint32_t (&val)[I],
                                           uint64_t pf = 0, const CompactIn *ci = nullptr, int B = 0) {
    const uint64_t st = e.x;
    const uint32_t len = e.y >> 8;
    const uint64_t *sk = (e.y & 1) ? k1 : k0;
    const uint32_t *sv = (e.y & 1) ? v1 : v0;
    uint32_t q0 = (threadIdx.x >> 6) * (I * 64) + (threadIdx.x & 63);
    asm volatile("" : "+v"(q0));
    if (pf & kCompact) {  // (uniform: one bucket per wave / workgroup)
        const int hi = (e.y >> 1) & 127;
#pragma unroll
        for (int i = 0; i < I; ++i) {
            const uint64_t e_ = st + min(q0 + i * 64, len - 1);
            const uint64_t x = sk[e_];
            key[i] = compact_key(pf, hi, B, ci->nd[e_], (uint32_t)(x >> 32));
            val[i] = (uint32_t)x;
        }
        return;
    }
#pragma unroll
    for (int i = 0; i < I; ++i) {
        const uint64_t e_ = st + min(q0 + i * 64, len - 1);
        key[i] = sk[e_];
        val[i] = sv[e_];
    }
}

template <int T, int I, int R>
__global__ __launch_bounds__(T) void msd_local_kernel(const uint2 *__restrict__ list, uint32_t count, int B,
                                                      uint64_t *k0, uint32_t *v0, const uint64_t *k1,
                                                      const uint32_t *v1, uint8_t *__restrict__ heads, Lists L,
                                                      uint32_t *__restrict__ ctr, int skip, uint32_t small, int wkeys,
                                                      CompactIn ci) {
    using SM = PartSmem<T, I, R>;
    constexpr int TILE = SM::kTile;
    constexpr int RADIX = SM::kRadix;
    __shared__ __attribute__((aligned(16))) unsigned char s_raw[SM::kUnion];
    __shared__ uint32_t s_wsum[SM::kWaves];
    __shared__ uint32_t s_start[RADIX + 1];
    __shared__ uint8_t s_hd[TILE + 1];
    __shared__ uint32_t s_any;
    __shared__ uint64_t s_kf, s_or;                  // common-prefix skip: first key, OR of differences
    uint64_t *s_k = reinterpret_cast<uint64_t *>(s_raw);
    uint32_t *s_v = reinterpret_cast<uint32_t *>(s_raw + SM::kValOff);
    uint32_t *s_wc = reinterpret_cast<uint32_t *>(s_raw);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t idx = blockIdx.x;
    if (idx >= count) return;
    uint2 e = list[idx];
    uint64_t pf = ci.pref ? ci.pref[idx] : 0;
    uint64_t key[I];
    uint32_t val[I];
    local_load<T, I>(e, k0, v0, k1, v1, key, val, pf, &ci, B);
    __builtin_amdgcn_s_waitcnt(kVmcnt0);
    for (; idx < count; idx += gridDim.x) {
        const uint2 ce = e;
        const uint64_t st = ce.x;
        const uint32_t len = ce.y >> 8;
        int hi = (ce.y >> 1) & 127;
        if (skip) {
            if (tid == 0) {
                s_kf = key[0];
                s_or = 0;
            }
            lds_barrier();
            uint64_t x = 0;
#pragma unroll
            for (int i = 0; i < I; ++i)
                if ((uint32_t)(wave * (I * 64) + i * 64 + lane) < len) x |= key[i] ^ s_kf;
            x = wave_or64(x);
            if (lane == 0 && x) atomicOr((unsigned long long *)&s_or, (unsigned long long)x);
            lds_barrier();
            hi = skip_hi(s_or, B, hi);
        }
        const Dig dd = dig_at(B, hi, R);
        const int nhi = hi + R;      // key bits sorted within a sub-bucket
        const bool last = nhi >= B;  // sub-bucket keys are equal
        if (idx + gridDim.x < count) {  // else: re-load the current one
            e = list[idx + gridDim.x];
            pf = ci.pref ? ci.pref[idx + gridDim.x] : 0;
        }

        // 1. stable partition into LDS
        for (int i = tid; i < SM::kWaves * RADIX; i += T) s_wc[i] = 0;
        if (tid == 0) s_any = 0;
        lds_barrier();
        bool valid[I];
        uint32_t slot[I];
#pragma unroll
        for (int i = 0; i < I; ++i) valid[i] = (uint32_t)(wave * (I * 64) + i * 64 + lane) < len;
        // items of this wave holding elements (wave-uniform)
        const int wbase = wave * (I * 64);
        const int live = (int)len > wbase ? min(I, ((int)len - wbase + 63) >> 6) : 0;
        partition_stage<T, I, R>(key, val, valid, dd, s_raw, nullptr, s_wsum, s_start, slot, nullptr, live);

        // 2. final position and head flag of every element
        uint32_t out[I];
        uint8_t hd[I];
#pragma unroll
        for (int i = 0; i < I; ++i) {
            out[i] = slot[i];
            hd[i] = 0;
            if (i >= live) continue;  // wave-uniform
            const uint32_t dg = dg_of(key[i], dd);
            const uint32_t sb = s_start[dg], size = s_start[dg + 1] - sb;
            hd[i] = slot[i] == sb;  // singleton or equal keys: the first is the head
            if (valid[i] && size > 1 && !last) {
                if (size <= small) {
                    const uint32_t me = slot[i] - sb;
                    uint32_t lt = 0, eq = 0;
                    for (uint32_t j = 0; j < size; ++j) {
                        const uint64_t kj = s_k[sb + j];
                        lt += kj < key[i];
                        eq += kj == key[i] && j < me;
                    }
                    out[i] = sb + lt + eq;
                    hd[i] = eq == 0;
                } else {
                    hd[i] = 2;  // not final: re-listed, head written by the next round
                }
            }
        }
        // re-list the large sub-buckets (rare): one entry each, from its first element
        bool first[I], any = false;
#pragma unroll
        for (int i = 0; i < I; ++i) {
            first[i] = valid[i] && hd[i] == 2 && slot[i] == s_start[dg_of(key[i], dd)];
            any |= first[i];
        }
        if (any) s_any = 1;
        lds_barrier();  // also: every rank-by-count read is done before the staging is overwritten
        const bool relist = s_any != 0;
        if (relist) {
#pragma unroll
            for (int i = 0; i < I; ++i) {
                const uint32_t dg = dg_of(key[i], dd);
                const uint32_t size = first[i] ? s_start[dg + 1] - s_start[dg] : 0;
                route((uint32_t)st + slot[i], size, nhi, B, 0, false, L, ctr, lane);
            }
        }
#pragma unroll
        for (int i = 0; i < I; ++i) {  // invalid items: out = sink slot
            if (i >= live) continue;
            s_k[out[i]] = key[i];
            s_v[out[i]] = val[i];
            s_hd[out[i]] = hd[i];  // 0 / 1: final (not) a group head; 2: re-listed
        }
        // the next bucket's loads fly while this one is written back
        local_load<T, I>(e, k0, v0, k1, v1, key, val, pf, &ci, B);  // unconditional: static load count
        lds_barrier();

        // 3. in-order write-back with head flags
#pragma unroll
        for (int i = 0; i < I; ++i) {
            const uint32_t p = min((uint32_t)(i * T + tid), len - 1);
            if (relist || wkeys) k0[st + p] = s_k[p];  // keys: final-key sorts, or re-listed elements
            v0[st + p] = s_v[p];
            heads[st + p] = s_hd[p] & 1;
        }
        lds_barrier();  // the write-back has read LDS before the next bucket's staging
    }
}

// list entry j of a wave class (scalar loads) and its prefix (0: not recorded)
__device__ __forceinline__ void wave_entry(const uint2 *__restrict__ list, const uint64_t *__restrict__ cpref,
                                           uint32_t j, uint2 &e, uint64_t &pf) {
    e = list[j];
    pf = cpref ? cpref[j] : 0ull;
}

// raw elements of a wave-class bucket: compact (x = low << 32 | start, next-digit byte) or full
// (key, start).  One global load instruction per word either way (so the compiler's count of
// loads in flight is static); buffers chosen by integer selects (pointer selects between kernel
// arguments went through the stack as flat loads).  Loads clamped to the bucket.
template <int I>
__device__ __forceinline__ void wave_load(const uint2 e, uint64_t pf, int lane, const uint64_t *k0, const uint64_t *k1,
                                          const uint32_t *v0, const uint32_t *v1, const uint8_t *cnd,
                                          uint64_t (&a)[I], uint32_t (&b)[I]) {
    const uint64_t st = e.x;
    const uint32_t len = e.y >> 8;
    const bool p1 = (e.y & 1) != 0, cmp = (pf & kCompact) != 0;
    const uint64_t kb = p1 ? (uint64_t)k1 : (uint64_t)k0;
    const uint64_t bb = cmp ? (uint64_t)cnd : (p1 ? (uint64_t)v1 : (uint64_t)v0);
    const int sh = cmp ? 0 : 2;
    uint32_t q = lane;
    asm volatile("" : "+v"(q));
    if (cmp) {  // byte loads of the digits: 0.1-0.3 ms faster than unaligned 4-byte ones at C3 (A/B)
#pragma unroll
        for (int i = 0; i < I; ++i) {
            const uint64_t at = st + min(q + i * 64, len - 1);
            a[i] = *reinterpret_cast<gu64 *>(kb + 8 * at);
            b[i] = *reinterpret_cast<gu8 *>(bb + at);
        }
        return;
    }
#pragma unroll
    for (int i = 0; i < I; ++i) {
        const uint64_t at = st + min(q + i * 64, len - 1);
        a[i] = *reinterpret_cast<gu64 *>(kb + 8 * at);
        b[i] = *reinterpret_cast<gu32u *>(bb + (at << sh));
    }
}

// Single-wave finishing kernel for buckets of <= 64 I elements (C3: ~370 keys behind the compact
// level, class 1).  Per bucket, one wave:
//   keys   compact entries (a compact level's output): key = prefix | next-digit byte | low bits
//          (compact_key); full entries: (key, start) as stored
//   rank   the next 8-bit digit of every element, ranked by ONE returning LDS atomic per item
//          (rank_atomic: stable); the 256 digit counts are scanned 4 per lane (wave_incl_scan)
//   order  each digit's elements take its slots in stable order; the key bits below the digit are
//          staged at those slots, and a sub-bucket of 2..small elements is ordered by
//          rank-by-count over them (ties: staging order = start order); larger sub-buckets are
//          re-listed for another round; a sub-bucket whose key bits are exhausted is final
//   write  keys (the group-head flag in bit 63 when B < 64) and starts staged at their final slots,
//          then stored contiguously: keys, starts and head flags of the whole bucket
// The next bucket's elements are loaded once the current one is staged in LDS, so they fly during
// its write-back; loads and write-back are branch-free with static counts (slots clamped to the
// bucket), so the next iteration waits for those loads without draining the stores.  The list entries and prefixes are scalar loads two
// buckets ahead.  LDS per wave: staged keys (aliased by the low bits of the ranking: one wave's LDS
// operations complete in order), staged starts, digit counts -- 7.2 KB at I = 8.
// WK: keys are written back (one-word sorts); otherwise only for buckets with re-listed elements.
template <int I, int MINW, bool WK, int R>
__global__ __launch_bounds__(64, MINW) void msd_wave_kernel(const uint2 *__restrict__ list, uint32_t count, int B,
                                                      uint64_t *k0, uint32_t *v0, const uint64_t *k1,
                                                      const uint32_t *v1, uint8_t *__restrict__ heads,
                                                      const Lists *__restrict__ Lp, uint32_t *__restrict__ ctr,
                                                      int skip, uint32_t small, const uint64_t *__restrict__ cpref,
                                                      const uint8_t *__restrict__ cnd) {
    constexpr int CAP = 64 * I;
    // bit budget of the packed per-item words below: sub-bucket start (slot) in 10 bits, size in 11,
    // rank in 11, and the slot in the low 10 bits of a composite rank-by-count value
    static_assert(CAP <= 1024, "slot fields are 10 bits wide");
    constexpr int MINLIVE = I > 4 ? I / 2 + 1 : 1;  // items a bucket of the class always fills
    constexpr int RADIX = 1 << R, CPL = RADIX / 64;  // digits; counters per lane in the scan
    static_assert(CPL % 4 == 0, "16-byte counter groups");
    __shared__ uint64_t s_k[CAP + 4];  // staged keys (slot CAP: sink); rank-by-count values + sentinels
    // digit counts -> starts (s_cnt[RADIX] = len); once the ranks are final, the staged starts
    // (slot CAP: sink) -- one wave's LDS operations complete in order
    constexpr int kUnion = (RADIX + 4) > (CAP + 1) ? (RADIX + 4) : (CAP + 1);
    __shared__ __attribute__((aligned(16))) uint32_t s_cv[kUnion];
    uint32_t *const s_cnt = s_cv;
    uint32_t *const s_v = s_cv;
    const int lane = threadIdx.x;
    // XCD-aware walk (grid a multiple of 8): workgroup b takes the (b % 8)-th eighth of the list,
    // so the list's neighbouring buckets -- neighbours in memory, since classify appends a level's
    // sub-buckets in runs of address order -- are finished at about the same time on one XCD and
    // share the L2 lines at their edges; other grids walk the list with the plain stride
    uint32_t idx = blockIdx.x, lend = count, lstep = gridDim.x;
    if (gridDim.x >= 8 && (gridDim.x & 7) == 0) {
        const uint32_t x = blockIdx.x & 7;
        idx = (uint32_t)((uint64_t)count * x / 8) + (blockIdx.x >> 3);
        lend = (uint32_t)((uint64_t)count * (x + 1) / 8);
        lstep = gridDim.x >> 3;
    }
    if (idx >= lend) return;
    // keys and starts of a bucket from its raw elements
    auto unpack = [B](const uint2 e, uint64_t pf, const uint64_t (&a)[I], const uint32_t (&b)[I], uint64_t (&key)[I],
                      uint32_t (&val)[I]) {
        const int hi0 = (e.y >> 1) & 127;
        const bool cmp = (pf & kCompact) != 0;
#pragma unroll
        for (int i = 0; i < I; ++i) {
            key[i] = cmp ? compact_key(pf, hi0, B, b[i] & 0xFFu, (uint32_t)(a[i] >> 32)) : a[i];
            val[i] = cmp ? (uint32_t)a[i] : b[i];
        }
    };
    uint2 e, en;
    uint64_t pf, pfn;
    uint64_t key[I], a[I];
    uint32_t val[I], b[I];
    wave_entry(list, cpref, idx, e, pf);
    wave_load<I>(e, pf, lane, k0, k1, v0, v1, cnd, a, b);
    en = e;
    pfn = pf;
    if (idx + lstep < lend) wave_entry(list, cpref, idx + lstep, en, pfn);
    __builtin_amdgcn_s_waitcnt(kVmcnt0);
    for (;;) {
        const uint64_t st = e.x;
        const uint32_t len = e.y >> 8;
        const int hi0 = (e.y >> 1) & 127;
        unpack(e, pf, a, b, key, val);
        uint2 enn = en;
        uint64_t pfnn = pfn;
        if (idx + 2 * lstep < lend) wave_entry(list, cpref, idx + 2 * lstep, enn, pfnn);

        int hi = hi0;
        if (skip) {  // common-prefix skip (later rounds and phases: repeats)
            const uint64_t kf = ((uint64_t)__builtin_amdgcn_readlane((int)(uint32_t)(key[0] >> 32), 0) << 32) |
                                (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)key[0], 0);
            uint64_t x = 0;
#pragma unroll
            for (int i = 0; i < I; ++i)
                if ((uint32_t)(i * 64 + lane) < len) x |= key[i] ^ kf;
            hi = skip_hi(wave_or64(x), B, hi);
        }
        const Dig dd = dig_at(B, hi, R);
        const bool last = hi + R >= B;                      // a sub-bucket's keys are equal
        const uint64_t lowm = (1ull << dd.shift) - 1ull;    // key bits below the digit
        const int live = min(I, (int)((len + 63) >> 6));    // items holding elements (wave-uniform)

        // 1. stable rank inside the digit
#pragma unroll
        for (int u = 0; u < CPL / 4; ++u) reinterpret_cast<uint4 *>(s_cnt)[lane * (CPL / 4) + u] = make_uint4(0, 0, 0, 0);
        uint32_t pk[I];  // rank | digit << 16, then rank << 21 | size << 10 | sub-bucket start
#pragma unroll
        for (int i = 0; i < I; ++i) {
            pk[i] = 0;
            if (i >= live) continue;
            const uint32_t d = dg_of(key[i], dd);
            pk[i] = rank_atomic(s_cnt, d, (uint32_t)(i * 64 + lane) < len) | (d << 16);
        }
        // 2. digit starts (exclusive scan of the RADIX counts, CPL per lane); s_cnt[RADIX] = len
        {
            uint4 c[CPL / 4];
            uint32_t sl = 0;
#pragma unroll
            for (int u = 0; u < CPL / 4; ++u) {
                c[u] = reinterpret_cast<const uint4 *>(s_cnt)[lane * (CPL / 4) + u];
                sl += c[u].x + c[u].y + c[u].z + c[u].w;
            }
            const uint32_t incl = wave_incl_scan(sl);
            uint32_t r0 = incl - sl;
#pragma unroll
            for (int u = 0; u < CPL / 4; ++u) {
                const uint4 o = make_uint4(r0, r0 + c[u].x, r0 + c[u].x + c[u].y, r0 + c[u].x + c[u].y + c[u].z);
                reinterpret_cast<uint4 *>(s_cnt)[lane * (CPL / 4) + u] = o;
                r0 = o.w + c[u].w;
            }
            if (lane == 63) s_cnt[RADIX] = incl;
        }
        // 3. slots.  Staged at each element's slot: its key bits below the sorted ones (digit and
        // low bits) with the slot appended -- (x << 10) | slot, unique, and in sub-bucket order
        // exactly the stable order -- when they fit 64 bits; otherwise the low bits alone.  Four
        // sentinels (all ones) follow the bucket, so a rank-by-count may read past its sub-bucket
        // unpredicated: later digits and sentinels are larger than any of its values.
        const bool cmpst = hi + 64 - 10 >= B;  // composite values (C3: 39 + 10 bits)
        const uint64_t xm = B - hi >= 64 ? ~0ull : (1ull << (B - hi)) - 1ull;
#pragma unroll
        for (int i = 0; i < I; ++i) {
            if (i >= live) continue;
            const uint32_t d = pk[i] >> 16, r = pk[i] & 0xFFFFu;
            const uint32_t sb = s_cnt[d], size = s_cnt[d + 1] - sb;
            if ((uint32_t)(i * 64 + lane) < len)
                s_k[sb + r] = cmpst ? ((key[i] & xm) << 10) | (sb + r) : key[i] & lowm;
            pk[i] = (r << 21) | (size << 10) | sb;
        }
        if (lane < 4) s_k[len + lane] = ~0ull;
        // 4. final slot of every element: sub-buckets of 2..small elements by rank-by-count
        bool any = false;
#pragma unroll
        for (int i = 0; i < I; ++i) {
            if (i >= live) continue;
            const uint32_t sb = pk[i] & 0x3FFu, size = (pk[i] >> 10) & 0x7FFu, r = pk[i] >> 21;
            const bool valid = (uint32_t)(i * 64 + lane) < len;
            uint32_t o = valid ? sb + r : (uint32_t)CAP;  // invalid items: the sink
            any |= valid && size > small && !last;        // re-listed: ordered by the next round
            if (valid && size > 1 && size <= small && !last) {
                uint32_t cnt = 0;
                if (cmpst) {
                    const uint64_t me = ((key[i] & xm) << 10) | (sb + r);
                    for (uint32_t j0 = 0; j0 < size; j0 += 4) {
#pragma unroll
                        for (int u = 0; u < 4; ++u) cnt += s_k[sb + j0 + u] < me;
                    }
                } else {  // low bits; ties by slot
                    const uint64_t me = key[i] & lowm;
                    uint32_t lt = 0, eq = 0;
                    for (uint32_t j0 = 0; j0 < size; j0 += 4) {
                        uint64_t x[4];
#pragma unroll
                        for (int u = 0; u < 4; ++u) x[u] = s_k[sb + j0 + u];
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            const uint32_t j = j0 + u;
                            lt += (j < size) & (x[u] < me);
                            eq += (j < r) & (x[u] == me);
                        }
                    }
                    cnt = lt + eq;
                }
                o = sb + cnt;
            }
            pk[i] = o;
        }
        const bool relist = __ballot(any) != 0;
        if (relist) {  // (rare) one entry per re-listed sub-bucket, from its first element
#pragma unroll
            for (int i = 0; i < I; ++i) {
                uint32_t size = 0, at = 0;
                if (i < live && (uint32_t)(i * 64 + lane) < len) {
                    const uint32_t d = dg_of(key[i], dd);
                    const uint32_t sb = s_cnt[d];
                    size = s_cnt[d + 1] - sb;
                    at = pk[i];
                    if (size <= small || last || at != sb) size = 0;
                }
                route((uint32_t)st + at, size, hi + R, B, 0, false, *Lp, ctr, lane);
            }
        }
        // 5. stage at the final slots (after every rank-by-count read of s_k: in order)
#pragma unroll
        for (int i = 0; i < I; ++i) {
            if (i >= live) continue;
            s_k[pk[i]] = key[i];
            s_v[pk[i]] = val[i];
        }
        // the next bucket's raw elements (after the last: this one again -- a static count): its
        // keys and starts are staged, so their registers take the loads, which fly during the
        // write-back (loading at the top of the bucket instead kept two buckets in registers:
        // 4 waves per SIMD, measured 22.2 against 20.3 ms at C3)
        wave_load<I>(en, pfn, lane, k0, k1, v0, v1, cnd, a, b);
        // 6. write-back: contiguous; group-head flag = the key differs from its predecessor (a
        // bucket starts a group; re-listed elements get provisional flags).  Items that may be
        // empty first, skipped when they are; then the MINLIVE items every bucket of the class
        // fills (its buckets hold more than CAP / 2 elements), unconditionally: the compiler then
        // knows at least 3 MINLIVE stores follow the next bucket's loads, and the next iteration
        // waits for those loads without draining them (a branch around every item's stores
        // drained all; stores for empty items cost more than the drain)
        const bool wk = WK || relist;
#pragma unroll
        for (int ii = 0; ii < I; ++ii) {
            const int i = ii < I - MINLIVE ? MINLIVE + ii : ii - (I - MINLIVE);
            if (i >= MINLIVE && i >= live) continue;
            const uint32_t j = min((uint32_t)(i * 64 + lane), len - 1);
            const uint64_t kj = s_k[j], kp = s_k[j > 0 ? j - 1 : 0];
            const uint32_t vj = s_v[j];
            if (wk) gmem(k0)[st + j] = kj;
            gmem(v0)[st + j] = vj;
            gmem(heads)[st + j] = (j == 0 || kj != kp) ? 1 : 0;
        }
        idx += lstep;
        if (idx >= lend) break;
        e = en;
        pf = pfn;
        en = enn;
        pfn = pfnn;
    }
}

// TIMING EXPERIMENTS ONLY (GKM_EXP_WAVECOPY=1, wrong output): the wave kernel's memory traffic
// without its ranking -- the same list walk, loads (compact entries unpacked) and software
// pipelining, then keys, starts and head flags stored straight from registers in load order.
// Its time is the floor of msd_wave_kernel's bucket-granular access pattern.
// HS: head flags stored per element (0), per aligned 4-flag chunk as one dword (1, edge chunks
// per byte), or not at all (2) -- the store pattern's share of the floor
template <int I, int MINW, int HS = 0>
__global__ __launch_bounds__(64, MINW) void msd_wave_copy_kernel(const uint2 *__restrict__ list, uint32_t count, int B,
                                                           uint64_t *k0, uint32_t *v0, const uint64_t *k1,
                                                           const uint32_t *v1, uint8_t *__restrict__ heads,
                                                           const uint64_t *__restrict__ cpref,
                                                           const uint8_t *__restrict__ cnd) {
    const int lane = threadIdx.x;
    uint32_t idx = blockIdx.x, lend = count, lstep = gridDim.x;
    if (gridDim.x >= 8 && (gridDim.x & 7) == 0) {
        const uint32_t x = blockIdx.x & 7;
        idx = (uint32_t)((uint64_t)count * x / 8) + (blockIdx.x >> 3);
        lend = (uint32_t)((uint64_t)count * (x + 1) / 8);
        lstep = gridDim.x >> 3;
    }
    if (idx >= lend) return;
    uint2 e, en;
    uint64_t pf, pfn;
    uint64_t key[I], a[I];
    uint32_t val[I], b[I];
    wave_entry(list, cpref, idx, e, pf);
    wave_load<I>(e, pf, lane, k0, k1, v0, v1, cnd, a, b);
    en = e;
    pfn = pf;
    if (idx + lstep < lend) wave_entry(list, cpref, idx + lstep, en, pfn);
    __builtin_amdgcn_s_waitcnt(kVmcnt0);
    for (;;) {
        const uint64_t st = e.x;
        const uint32_t len = e.y >> 8;
        const int hi0 = (e.y >> 1) & 127;
        const bool cmp = (pf & kCompact) != 0;
#pragma unroll
        for (int i = 0; i < I; ++i) {
            key[i] = cmp ? compact_key(pf, hi0, B, b[i] & 0xFFu, (uint32_t)(a[i] >> 32)) : a[i];
            val[i] = cmp ? (uint32_t)a[i] : b[i];
        }
        uint2 enn = en;
        uint64_t pfnn = pfn;
        if (idx + 2 * lstep < lend) wave_entry(list, cpref, idx + 2 * lstep, enn, pfnn);
        wave_load<I>(en, pfn, lane, k0, k1, v0, v1, cnd, a, b);
#pragma unroll
        for (int i = 0; i < I; ++i) {
            const uint32_t j = min((uint32_t)(i * 64 + lane), len - 1);
            gmem(k0)[st + j] = key[i];
            gmem(v0)[st + j] = val[i];
            if (HS == 0) gmem(heads)[st + j] = 1;
        }
        if (HS == 1) {
            const uint64_t a0 = st & ~3ull, end = st + len;
#pragma unroll
            for (int r = 0; r < (64 * I + 8) / 256 + 1; ++r) {
                const uint64_t p = a0 + 4ull * (r * 64 + lane);
                if (p >= end) continue;
                if (p >= st && p + 4 <= end) {
                    gmem(reinterpret_cast<uint32_t *>(heads + p))[0] = 0x01010101u;
                } else {
                    for (int t = 0; t < 4; ++t)
                        if (p + t >= st && p + t < end) gmem(heads)[p + t] = 1;
                }
            }
        }
        idx += lstep;
        if (idx >= lend) break;
        e = en;
        pf = pfn;
        en = enn;
        pfn = pfnn;
    }
}

// TIMING EXPERIMENTS ONLY (GKM_EXP_WAVECOPY=2): the copy-only variant with the loads issued two
// buckets ahead instead of one -- does more memory in flight per wave move the floor?
template <int I, int MINW>
__global__ __launch_bounds__(64, MINW) void msd_wave_copy2_kernel(const uint2 *__restrict__ list, uint32_t count, int B,
                                                            uint64_t *k0, uint32_t *v0, const uint64_t *k1,
                                                            const uint32_t *v1, uint8_t *__restrict__ heads,
                                                            const uint64_t *__restrict__ cpref,
                                                            const uint8_t *__restrict__ cnd) {
    const int lane = threadIdx.x;
    uint32_t idx = blockIdx.x, lend = count, lstep = gridDim.x;
    if (gridDim.x >= 8 && (gridDim.x & 7) == 0) {
        const uint32_t x = blockIdx.x & 7;
        idx = (uint32_t)((uint64_t)count * x / 8) + (blockIdx.x >> 3);
        lend = (uint32_t)((uint64_t)count * (x + 1) / 8);
        lstep = gridDim.x >> 3;
    }
    if (idx >= lend) return;
    uint2 e0, e1, e2;
    uint64_t p0, p1, p2;
    uint64_t a0[I], a1[I];
    uint32_t b0[I], b1[I];
    wave_entry(list, cpref, idx, e0, p0);
    e1 = e0; p1 = p0;
    if (idx + lstep < lend) wave_entry(list, cpref, idx + lstep, e1, p1);
    wave_load<I>(e0, p0, lane, k0, k1, v0, v1, cnd, a0, b0);
    wave_load<I>(e1, p1, lane, k0, k1, v0, v1, cnd, a1, b1);
    __builtin_amdgcn_s_waitcnt(kVmcnt0);
    for (;;) {
        const uint64_t st = e0.x;
        const uint32_t len = e0.y >> 8;
        const int hi0 = (e0.y >> 1) & 127;
        const bool cmp = (p0 & kCompact) != 0;
        uint64_t key[I];
        uint32_t val[I];
#pragma unroll
        for (int i = 0; i < I; ++i) {
            key[i] = cmp ? compact_key(p0, hi0, B, b0[i] & 0xFFu, (uint32_t)(a0[i] >> 32)) : a0[i];
            val[i] = cmp ? (uint32_t)a0[i] : b0[i];
        }
        e2 = e1; p2 = p1;
        if (idx + 2 * lstep < lend) wave_entry(list, cpref, idx + 2 * lstep, e2, p2);
        wave_load<I>(e2, p2, lane, k0, k1, v0, v1, cnd, a0, b0);  // two buckets ahead
#pragma unroll
        for (int i = 0; i < I; ++i) {
            const uint32_t j = min((uint32_t)(i * 64 + lane), len - 1);
            gmem(k0)[st + j] = key[i];
            gmem(v0)[st + j] = val[i];
            gmem(heads)[st + j] = 1;
        }
        idx += lstep;
        if (idx >= lend) break;
        // rotate: bucket 1 becomes current (its loads were issued a bucket ago)
#pragma unroll
        for (int i = 0; i < I; ++i) {
            const uint64_t ta = a0[i];
            a0[i] = a1[i];
            a1[i] = ta;
            const uint32_t tb = b0[i];
            b0[i] = b1[i];
            b1[i] = tb;
        }
        e0 = e1; p0 = p1;
        e1 = e2; p1 = p2;
    }
}

// TIMING EXPERIMENTS ONLY (GKM_EXP_WAVECOPY=5, wrong output): the wave stage's bytes as one plain
// coalesced stream over the whole array -- 9 B in (compact word + digit byte), 13 B out (key,
// start, head) per element; each wave takes 512 consecutive elements per step, every load and
// store instruction covering one contiguous 512-B or 1-KiB piece -- the streaming floor of the
// stage's traffic, against the bucket-granular floor of msd_wave_copy_kernel
__global__ __launch_bounds__(256) void stream_copy_kernel(uint64_t n, const uint64_t *__restrict__ k1,
                                                          const uint8_t *__restrict__ nd, uint64_t *__restrict__ k0,
                                                          uint32_t *__restrict__ v0, uint8_t *__restrict__ heads) {
    const int lane = threadIdx.x & 63;
    const uint64_t wid = (blockIdx.x * 256ull + threadIdx.x) >> 6, nw = gridDim.x * 4ull;
    for (uint64_t blk = wid; blk < n / 512; blk += nw) {
        const uint64_t e0 = blk * 512;
        const uint4 *ks = reinterpret_cast<const uint4 *>(k1 + e0);
        uint4 kv[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) kv[j] = ks[j * 64 + lane];
        const uint2 d = reinterpret_cast<const uint2 *>(nd + e0)[lane];
        uint4 *ko = reinterpret_cast<uint4 *>(k0 + e0);
#pragma unroll
        for (int j = 0; j < 4; ++j) ko[j * 64 + lane] = make_uint4(kv[j].y ^ d.x, kv[j].x, kv[j].w, kv[j].z);
        uint4 *vo = reinterpret_cast<uint4 *>(v0 + e0);
#pragma unroll
        for (int j = 0; j < 2; ++j)
            vo[j * 64 + lane] = make_uint4(kv[2 * j].x, kv[2 * j].z, kv[2 * j + 1].x, kv[2 * j + 1].z);
        reinterpret_cast<uint2 *>(heads + e0)[lane] = make_uint2(d.y | 0x01010101u, d.x);
    }
}

static bool exp_wave_copy() { return exp_opt("GKM_EXP_WAVECOPY") != nullptr; }

// one round's lists, copied to device memory for the wave kernels
__global__ void lists_store_kernel(Lists L, Lists *__restrict__ dst) { *dst = L; }

// Buckets of <= kTiny elements (mostly from the tie groups of multi-word keys): one thread per
// bucket, stable rank-by-count over the full word (ties: load order = start order), write-back of
// starts and head flags to buffer 0.
__global__ __launch_bounds__(256) void msd_tiny_kernel(const uint2 *__restrict__ list, uint32_t count,
                                                       uint64_t *k0, uint32_t *v0, const uint64_t *k1,
                                                       const uint32_t *v1, uint8_t *__restrict__ heads, int wkeys,
                                                       CompactIn ci, int B) {
    const uint32_t idx = blockIdx.x * 256 + threadIdx.x;
    const bool live = idx < count;
    const uint2 e = live ? list[idx] : make_uint2(0, 1u << 8);
    const uint64_t st = e.x;
    const uint32_t len = e.y >> 8;
    const uint64_t *sk = (e.y & 1) ? k1 : k0;
    const uint32_t *sv = (e.y & 1) ? v1 : v0;
    uint64_t key[kTiny];
    uint32_t val[kTiny];
    const uint64_t pf = live && ci.pref ? ci.pref[idx] : 0;
    const int ehi = (e.y >> 1) & 127;
#pragma unroll
    for (int j = 0; j < kTiny; ++j) {
        const uint64_t at = st + min((uint32_t)j, len - 1);
        const uint64_t x = live ? sk[at] : 0;
        key[j] = (pf & kCompact) ? compact_key(pf, ehi, B, ci.nd[at], (uint32_t)(x >> 32)) : x;
        val[j] = !live ? 0 : (pf & kCompact) ? (uint32_t)x : sv[at];
    }
    uint32_t out[kTiny];
    bool hd[kTiny];
#pragma unroll
    for (int j = 0; j < kTiny; ++j) {
        uint32_t lt = 0, eq = 0;
#pragma unroll
        for (int i = 0; i < kTiny; ++i) {
            lt += (uint32_t)i < len && key[i] < key[j];
            eq += i < j && key[i] == key[j];
        }
        out[j] = lt + eq;
        hd[j] = eq == 0;
    }
    if (!live) return;
#pragma unroll
    for (int j = 0; j < kTiny; ++j) {
        if ((uint32_t)j >= len) break;
        v0[st + out[j]] = val[j];
        if (wkeys) k0[st + out[j]] = key[j];
        heads[st + out[j]] = hd[j] ? 1 : 0;
    }
}

// Multi-word keys: the groups of >= 2 equal earlier words, from the head flags of the order so far.
// The first and last element of every such group, in two light passes over the head flags (no
// flag arrays): COUNT writes per 8192-element tile the numbers of group firsts and lasts; after
// their scans, STORE writes the indices from the tile's offsets (thread t owns elements
// 32 t .. 32 t + 31 of the tile, so thread order = index order).
constexpr int kTieTile = 8192;

template <bool STORE>
__global__ __launch_bounds__(256) void tie_bounds_kernel(const uint8_t *__restrict__ heads, uint64_t n,
                                                         uint32_t *__restrict__ cnt_f, uint32_t *__restrict__ cnt_l,
                                                         const uint32_t *__restrict__ off_f,
                                                         const uint32_t *__restrict__ off_l,
                                                         uint32_t *__restrict__ first, uint32_t *__restrict__ last) {
    __shared__ uint32_t s_w[2][4];
    const uint64_t i0 = (uint64_t)blockIdx.x * kTieTile + threadIdx.x * 32;
    uint32_t mf = 0, ml = 0;
    if (i0 < n) {
        // 33 head flags from i0 (past n reads as a head: the group ends there)
        uint32_t hb = 0;
        if (i0 + 33 <= n) {
            const uint4 *h4 = reinterpret_cast<const uint4 *>(heads + i0);  // i0 % 32 == 0
            const uint4 a = h4[0], b = h4[1];
            const uint32_t wv[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
            for (int q = 0; q < 32; ++q) hb |= (((wv[q >> 2] >> (8 * (q & 3))) & 0xFFu) != 0 ? 1u : 0u) << q;
            const bool h32 = heads[i0 + 32] != 0;
            const uint32_t nxt = (hb >> 1) | ((h32 ? 1u : 0u) << 31);  // bit q: element i0 + q + 1 is a head
            mf = hb & ~nxt;
            ml = ~hb & nxt;
        } else {
            for (int q = 0; q < 32 && i0 + q < n; ++q) {
                const bool h = heads[i0 + q] != 0, hn = i0 + q + 1 >= n || heads[i0 + q + 1] != 0;
                mf |= (h && !hn ? 1u : 0u) << q;
                ml |= (!h && hn ? 1u : 0u) << q;
            }
        }
    }
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t cf = (uint32_t)__popc(mf), cl = (uint32_t)__popc(ml);
    uint32_t inf = cf, inl = cl;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t yf = __shfl_up(inf, o), yl = __shfl_up(inl, o);
        if (lane >= o) {
            inf += yf;
            inl += yl;
        }
    }
    if (lane == 63) {
        s_w[0][wave] = inf;
        s_w[1][wave] = inl;
    }
    __syncthreads();
    if (!STORE) {
        if (threadIdx.x == 0) {
            cnt_f[blockIdx.x] = s_w[0][0] + s_w[0][1] + s_w[0][2] + s_w[0][3];
            cnt_l[blockIdx.x] = s_w[1][0] + s_w[1][1] + s_w[1][2] + s_w[1][3];
        }
        return;
    }
    uint32_t of = off_f[blockIdx.x] + inf - cf, ol = off_l[blockIdx.x] + inl - cl;
    for (uint32_t w = 0; w < wave; ++w) {
        of += s_w[0][w];
        ol += s_w[1][w];
    }
    for (uint32_t m = mf; m; m &= m - 1) first[of++] = (uint32_t)(i0 + __ffs(m) - 1);
    for (uint32_t m = ml; m; m &= m - 1) last[ol++] = (uint32_t)(i0 + __ffs(m) - 1);
}

__global__ __launch_bounds__(256) void tie_run_lengths_kernel(const uint32_t *__restrict__ first,
                                                              uint32_t *__restrict__ last_to_len, uint64_t ng) {
    for (uint64_t g = blockIdx.x * 256ull + threadIdx.x; g < ng; g += (uint64_t)gridDim.x * 256)
        last_to_len[g] = last_to_len[g] - first[g] + 1;
}

// Key word of symbols [sym0, sym0 + nsym) of the (canonical) k-mer at p, 2-bit codes, from 17
// aligned dword loads (issued together) instead of one dependent byte load per symbol: the
// k-mer's codes as a left-aligned 128-bit value F (SWAR per dword), its reverse complement by
// two revcomp_word calls and a 128-bit shift, the smaller of the two, then the word.  k <= 64.
__device__ __forceinline__ uint32_t codes4(uint32_t w) {  // 4 bytes -> 8 bits, byte 0 on top
    uint32_t t = __builtin_bswap32(((w >> 1) ^ (w >> 2)) & 0x03030303u);
    t = (t | (t >> 6)) & 0x000F000Fu;
    return (t | (t >> 12)) & 0xFFu;
}

__device__ __forceinline__ uint64_t tie_word2(const uint8_t *sba, uint32_t p, int k, int sym0, int nsym,
                                              bool canonical) {
    // five 16-byte loads from p & ~15 (80 bytes; 17 dword loads made every k-mer 17 scattered
    // requests: C5's 113 M tie members took 19 ms)
    const uint4 *w4 = reinterpret_cast<const uint4 *>(sba + (p & ~15u));
    uint4 q[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) q[j] = w4[j];
    const uint32_t w[20] = {q[0].x, q[0].y, q[0].z, q[0].w, q[1].x, q[1].y, q[1].z, q[1].w, q[2].x, q[2].y,
                            q[2].z, q[2].w, q[3].x, q[3].y, q[3].z, q[3].w, q[4].x, q[4].y, q[4].z, q[4].w};
    uint64_t c0 = 0, c1 = 0, c2 = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) c0 = (c0 << 8) | codes4(w[j]);
#pragma unroll
    for (int j = 8; j < 16; ++j) c1 = (c1 << 8) | codes4(w[j]);
#pragma unroll
    for (int j = 16; j < 20; ++j) c2 = (c2 << 8) | codes4(w[j]);
    c2 <<= 32;  // symbols 64 .. 79 of the stream, on top
    // symbols 0 .. 63 from p: drop the first `off` (< 16) symbols of the stream
    const int sh = 2 * (int)(p & 15u);
    uint64_t fh = sh ? (c0 << sh) | (c1 >> (64 - sh)) : c0;
    uint64_t fl = sh ? (c1 << sh) | (c2 >> (64 - sh)) : c1;
    if (k < 64) {  // symbols past the k-mer read as 0
        if (k <= 32) {
            fh &= k == 32 ? ~0ull : ~(~0ull >> (2 * k));
            fl = 0;
        } else {
            fl &= ~(~0ull >> (2 * (k - 32)));
        }
    }
    if (canonical) {
        // reverse complement of the 64-symbol value, then shifted left past the (64 - k) pad symbols
        uint64_t rh = revcomp_word<2>(fl, 32), rl = revcomp_word<2>(fh, 32);
        const int ps = 2 * (64 - k);
        if (ps >= 64) {
            rh = rl << (ps - 64);
            rl = 0;
        } else if (ps > 0) {
            rh = (rh << ps) | (rl >> (64 - ps));
            rl <<= ps;
        }
        if (rh < fh || (rh == fh && rl < fl)) {
            fh = rh;
            fl = rl;
        }
    }
    // the word: symbols sym0 .. sym0 + nsym - 1 of (fh, fl)
    const int b0 = 2 * sym0, nb = 2 * nsym;  // bit offset from the top, width
    uint64_t x;
    if (b0 >= 64) x = fl << (b0 - 64);
    else x = b0 ? (fh << b0) | (fl >> (64 - b0)) : fh;
    return nb >= 64 ? x : x >> (64 - nb);
}

// Flat variant of tie_encode_kernel for many groups: tie_members_kernel lists every element in a group
// of >= 2 (a head flag of 0 at it or at its successor) -- 32 consecutive flags per thread from two
// 16-byte loads and one byte; COUNT per 8,192-element tile, scan, STORE at the tile's offset (one
// list append per wave on a global counter serialised 1.5 M atomics at C5: 16 ms) -- and
// tie_encode_list_kernel gives each listed element its next key word, one element per thread.  (One
// thread per element with a byte load per flag kept too few bytes in flight: 9.2 ms for C5's 3.1e9
// flags; 32 flags per thread with the members encoded in place serialised the lanes of the long
// runs of members a repeat leaves in the sorted order: 7.6 ms.)
template <bool STORE>
__global__ __launch_bounds__(256) void tie_members_kernel(const uint8_t *__restrict__ heads, uint64_t n,
                                                          uint32_t *__restrict__ cnt, const uint32_t *__restrict__ off,
                                                          uint32_t *__restrict__ list) {
    __shared__ uint32_t s_m[4][64 * 32];  // per wave: its members, in element order
    __shared__ uint32_t s_w[4];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t i0 = (uint64_t)blockIdx.x * kTieTile + threadIdx.x * 32;  // (as tie_bounds_kernel)
    uint32_t mem = 0;
    if (i0 + 33 <= n) {
        const uint4 *h4 = reinterpret_cast<const uint4 *>(heads + i0);  // i0 % 32 == 0
        const uint4 a = h4[0], b = h4[1];
        const uint32_t wv[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        uint32_t hb = 0;
#pragma unroll
        for (int q = 0; q < 32; ++q) hb |= (((wv[q >> 2] >> (8 * (q & 3))) & 0xFFu) != 0 ? 1u : 0u) << q;
        const uint32_t nxt = (hb >> 1) | ((heads[i0 + 32] != 0 ? 1u : 0u) << 31);  // bit q: i0 + q + 1 is a head
        mem = ~hb | ~nxt;
    } else if (i0 < n) {
        for (int q = 0; q < 32 && i0 + q < n; ++q) {
            const uint64_t i = i0 + q;
            mem |= (heads[i] == 0 || (i + 1 < n && heads[i + 1] == 0) ? 1u : 0u) << q;
        }
    }
    const uint32_t c = (uint32_t)__popc(mem);
    const uint32_t incl = wave_incl_scan(c);
    if (lane == 63) s_w[wave] = incl;
    __syncthreads();
    if (!STORE) {
        if (threadIdx.x == 0) cnt[blockIdx.x] = s_w[0] + s_w[1] + s_w[2] + s_w[3];
        return;
    }
    uint32_t base = off[blockIdx.x];
    for (uint32_t w = 0; w < wave; ++w) base += s_w[w];
    const uint32_t tot = s_w[wave];
    if (tot == 0) return;  // (wave-uniform)
    // the wave's members through LDS, stored by consecutive lanes (stored straight from the lanes,
    // each lane's run of up to 32 made every store instruction 64 scattered partial lines)
    uint32_t *sm = s_m[wave];
    uint32_t at = incl - c;
    for (; mem; mem &= mem - 1) sm[at++] = (uint32_t)(i0 + __ffs(mem) - 1);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
    for (uint32_t j = lane; j < tot; j += 64) list[base + j] = sm[j];
}

template <int BITS>
__global__ __launch_bounds__(256) void tie_encode_list_kernel(const uint8_t *__restrict__ sba,
                                                              const uint32_t *__restrict__ list, uint32_t m,
                                                              const uint32_t *__restrict__ vals,
                                                              uint64_t *__restrict__ keys, int sym0, int nsym, int k,
                                                              int canonical) {
    __shared__ uint8_t s_lut4[256];
    s_lut4[threadIdx.x] = c_code4_msd[threadIdx.x];
    __syncthreads();
    for (uint32_t j = blockIdx.x * 256 + threadIdx.x; j < m; j += gridDim.x * 256) {
        const uint32_t i = list[j];
        if (BITS == 2 && k <= 64) {
            keys[i] = tie_word2(sba, vals[i], k, sym0, nsym, canonical != 0);
            continue;
        }
        const uint8_t *b = sba + vals[i];
        const bool rc = canonical && canon_is_rc<BITS>(b, k, s_lut4);
        uint64_t key = 0;
        for (int t = sym0; t < sym0 + nsym; ++t) key = (key << BITS) | canon_sym<BITS>(b, k, t, rc, s_lut4);
        keys[i] = key;
    }
}

// Next-level buckets whose keys are all equal (a repeat's group of identical k-mers: 250 K
// elements of (CA)n at C4) would go through every remaining global level without splitting, each
// with its host round trips.  uniform_flag_kernel marks the buckets holding two different keys
// (gridDim.y workgroups per bucket); route_uniform_kernel sends the others to the done list.
__global__ __launch_bounds__(256) void uniform_flag_kernel(const uint32_t *__restrict__ bst,
                                                           const uint32_t *__restrict__ blen,
                                                           const uint64_t *__restrict__ keys,
                                                           uint32_t *__restrict__ mixed,
                                                           const uint32_t *__restrict__ nb_dev = nullptr,
                                                           uint32_t *__restrict__ nb_copy = nullptr) {
    if (nb_copy && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) *nb_copy = *nb_dev;
    if (nb_dev && blockIdx.x >= *nb_dev) return;
    const uint64_t st = bst[blockIdx.x];
    const uint32_t len = blen[blockIdx.x];
    const uint64_t k0 = keys[st];
    uint64_t acc = 0;
    for (uint32_t e = blockIdx.y * 256 + threadIdx.x; e < len; e += gridDim.y * 256) acc |= keys[st + e] ^ k0;
    if (__syncthreads_or(acc != 0) && threadIdx.x == 0) atomicOr(&mixed[blockIdx.x], 1u);
}

__global__ __launch_bounds__(256) void route_uniform_kernel(const uint32_t *__restrict__ bst,
                                                            const uint32_t *__restrict__ blen,
                                                            const uint64_t *__restrict__ bpref, uint32_t nb,
                                                            const uint32_t *__restrict__ mixed, Lists L, int parity,
                                                            uint32_t *__restrict__ ctr,
                                                            unsigned long long *__restrict__ sums, uint32_t tile,
                                                            uint32_t ctiles, const uint32_t *__restrict__ nb_dev = nullptr) {
    if (nb_dev) nb = *nb_dev;
    for (uint32_t b = blockIdx.x * 256 + threadIdx.x; b < nb; b += gridDim.x * 256) {
        if (mixed[b]) {
            const uint32_t at = atomicAdd(&ctr[kCtrBig], 1u);
            put_entry(L, kCtrBig, at, bst[b], blen[b], 0, parity, bpref ? bpref[b] : 0);
            atomicAdd(&sums[kCtrBig], (unsigned long long)blen[b]);
            atomicAdd(&sums[kSumTiles], (unsigned long long)tiles_of(blen[b], tile));
            atomicAdd(&sums[kSumChunks], (unsigned long long)chunks_of(blen[b], tile, ctiles));
        } else {
            put_entry(L, kCtrDone, atomicAdd(&ctr[kCtrDone], 1u), bst[b], blen[b], 0, parity);
        }
    }
}

// sub-buckets whose key bits are exhausted: in order already (copied to buffer 0 if needed);
// all keys equal, so the only head is the first element (gridDim.y workgroups per bucket)
__global__ __launch_bounds__(256) void done_copy_kernel(const uint32_t *__restrict__ dn_start,
                                                        const uint32_t *__restrict__ dn_len,
                                                        const uint8_t *__restrict__ dn_par, const uint32_t *__restrict__ v1,
                                                        uint32_t *__restrict__ v0, const uint64_t *__restrict__ k1,
                                                        uint64_t *__restrict__ k0, uint8_t *__restrict__ heads) {
    const uint32_t s = blockIdx.x;
    const uint64_t st = dn_start[s];
    const uint32_t len = dn_len[s];
    const bool copy = dn_par[s];
    for (uint32_t i = blockIdx.y * 256 + threadIdx.x; i < len; i += gridDim.y * 256) {  // keys: final-key sorts
        if (copy) v0[st + i] = v1[st + i];
        if (copy && k1) k0[st + i] = k1[st + i];
        heads[st + i] = i == 0;
    }
}

// Multi-word keys: the next phase's key word of every element of a group of equal earlier words
// (symbols [sym0, sym0 + nsym) of its k-mer, right-aligned).  One wave per group.
template <int BITS>
__global__ __launch_bounds__(256) void tie_encode_kernel(const uint8_t *__restrict__ sba,
                                                         const uint32_t *__restrict__ g_start,
                                                         const uint32_t *__restrict__ g_len, uint32_t ngroups,
                                                         const uint32_t *__restrict__ vals, uint64_t *__restrict__ keys,
                                                         int sym0, int nsym, int k, int canonical) {
    __shared__ uint8_t s_lut4[256];
    s_lut4[threadIdx.x] = c_code4_msd[threadIdx.x];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const uint32_t nw = gridDim.x * 4;
    for (uint32_t g = blockIdx.x * 4 + (threadIdx.x >> 6); g < ngroups; g += nw) {
        const uint64_t st = g_start[g];
        const uint32_t len = g_len[g];
        if (len < 2) continue;
        for (uint32_t i = lane; i < len; i += 64) {
            if (BITS == 2 && k <= 64) {
                keys[st + i] = tie_word2(sba, vals[st + i], k, sym0, nsym, canonical != 0);
                continue;
            }
            const uint8_t *b = sba + vals[st + i];
            const bool rc = canonical && canon_is_rc<BITS>(b, k, s_lut4);
            uint64_t key = 0;
            for (int t = sym0; t < sym0 + nsym; ++t) key = (key << BITS) | canon_sym<BITS>(b, k, t, rc, s_lut4);
            keys[st + i] = key;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// host driver
// ---------------------------------------------------------------------------------------------
static int grid_n(uint64_t n) { return (int)std::max<uint64_t>((n + 255) / 256, 1); }

hipError_t scan_u32_exclusive_pub(gk_ctx *c, const uint32_t *in, uint64_t n, uint32_t *out, uint64_t *total);
hipError_t scan_u32_exclusive_pair(gk_ctx *c, const uint32_t *in1, uint32_t *out1, const uint32_t *in2,
                                   uint32_t *out2, uint64_t n, uint64_t *total1, uint64_t *total2);
hipError_t scan_u32_exclusive_pair_launch(gk_ctx *c, const uint32_t *in1, uint32_t *out1, const uint32_t *in2,
                                          uint32_t *out2, uint64_t n);
hipError_t select_flags(gk_ctx *c, const uint8_t *flags, uint64_t n, uint32_t *out_idx, uint64_t *count);

// grow a device array to hold `need` entries, keeping the first `keep` entries
template <typename T>
static hipError_t grow_keep(gk_ctx *c, const char *name, uint64_t need, uint64_t keep, T **p) {
    auto &e = c->scratch[name];
    if (e.first && e.second >= sizeof(T) * need) {
        *p = static_cast<T *>(e.first);
        return hipSuccess;
    }
    void *np = nullptr;
    const uint64_t bytes = sizeof(T) * (need + need / 2 + 256);
    hipError_t r = dev_alloc(&np, bytes);
    if (r != hipSuccess) return r;
    if (e.first && keep) {
        r = hipMemcpyAsync(np, e.first, sizeof(T) * keep, hipMemcpyDeviceToDevice, c->stream);
        if (r != hipSuccess) return r;
        r = hipStreamSynchronize(c->stream);
        if (r != hipSuccess) return r;
    }
    if (e.first) dev_free(e.first);
    e.first = np;
    e.second = bytes;
    *p = static_cast<T *>(np);
    return hipSuccess;
}

static unsigned cu_count(gk_ctx *c) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess || cus < 8) cus = 256;
    return (unsigned)(cus / 8 * 8);
}

// Packing is opt-in (GKM_PACK=1): measured on MI355X, the L0 partition got slower reading packed
// words (17.8 vs 16.4 ms at C3) and the key-range passes gained less than the 0.8 ms packing costs.
// tuning only (A/B runs): GKM_SELECT_2PASS=1 selects a key-range shard's k-mers by a count pass,
// a scan and a store pass (the single chunked pass is the default)
static bool select_two_pass() {
    static const bool v = opt("GKM_SELECT_2PASS") != nullptr;
    return v;
}

// tuning only (A/B runs): GKM_XCD_WALK_OFF=1 gives the wave kernels a grid that is not a multiple
// of 8 (plain strided walk of the bucket list)
static bool xcd_walk_off() {
    static const bool v = opt("GKM_XCD_WALK_OFF") != nullptr;
    return v;
}

// tuning only (A/B runs): GKM_NO_COMPACT=1 keeps 64-bit keys in every level's output
static bool no_compact() { return opt("GKM_NO_COMPACT") != nullptr; }  // (read per level: tests flip it)

// timing only: GKM_L0_PROF=1 times the phases of the 2-bit L0 partition (tools)
static bool l0_prof() {
    static const bool v = exp_opt("GKM_L0_PROF") != nullptr;
    return v;
}

static bool use_pack() {
    static const bool on = opt("GKM_PACK") != nullptr;
    return on;
}

// the packed copy of c->sba (pack2_kernel) over the whole padded array, for ACGT sequences
static int pack_sequence(gk_ctx *c, const uint64_t **code, const uint32_t **dol) {
    const uint64_t nwords = (c->sba_len + kSbaPad) / 32;  // sba_cap >= sba_len + kSbaPad
    uint64_t *pc;
    uint32_t *pd;
    GK_TRY_HIP(c, scratch(c, "pk_code", nwords, &pc));
    GK_TRY_HIP(c, scratch(c, "pk_dol", nwords, &pd));
    int slot;
    timer_begin(c, "msd_pack", &slot);
    timer_units(c, slot, c->sba_len);
    hipLaunchKernelGGL(pack2_kernel<false>, dim3((unsigned)std::min<uint64_t>((nwords + 255) / 256, 65536)), dim3(256),
                       0, c->stream, c->sba, nwords, pc, pd);
    GK_TRY_HIP(c, hipGetLastError());
    timer_end(c, slot);
    *code = pc;
    *dol = pd;
    c->pk_fresh = true;
    return GK_OK;
}

static const char *kLocPrefName[kLocal] = {"locp0", "locp1", "locp2", "locp3", "locp4", "locp5"};
static const char *kLocName[kLocal][2] = {{"loc0a", "loc0b"}, {"loc1a", "loc1b"}, {"loc2a", "loc2b"},
                                          {"loc3a", "loc3b"}, {"loc4a", "loc4b"}, {"loc5a", "loc5b"}};
static const char *kLocTimer[kLocal][2] = {{"msd_local_wave4", "msd_local_wave4_r"},
                                           {"msd_local_wave8", "msd_local_wave8_r"},
                                           {"msd_local_wave16", "msd_local_wave16_r"},
                                           {"msd_local_block16", "msd_local_block16_r"},
                                           {"msd_local_tiny", "msd_local_tiny_r"},
                                           {"msd_local_block32", "msd_local_block32_r"}};
static const char *kPassNames[] = {"msd_pass_l0", "msd_pass_l1", "msd_pass_l2", "msd_pass_l3",
                                   "msd_pass_l4", "msd_pass_l5", "msd_pass_l6", "msd_pass_l7"};
static const char *kPassNamesP[] = {"msd_pass_l0p", "msd_pass_l1p", "msd_pass_l2p", "msd_pass_l3p",
                                    "msd_pass_l4p", "msd_pass_l5p", "msd_pass_l6p", "msd_pass_l7p"};  // packed pairs
static const char *kPassNamesC[] = {"msd_pass_l0c", "msd_pass_l1c", "msd_pass_l2c", "msd_pass_l3c",
                                    "msd_pass_l4c", "msd_pass_l5c", "msd_pass_l6c", "msd_pass_l7c"};  // compact

// One MSD sort of one-word keys into keys[0] / vals[0] (+ group heads).  The first partition
// comes from the sequence (run_l0) or from received buckets (first_level_from_pieces); the rest
// -- global levels while buckets exceed kBlockMax, local rounds, done copies -- is common.
struct MsdDriver {
    gk_ctx *c;
    KeySpec ks;
    int B;
    uint64_t n = 0;
    unsigned cus, pgrid;
    int slot = -1, total_slot = -1;
    uint32_t *ctr = nullptr, h[kCtrN] = {0};
    unsigned long long *sums = nullptr, hs[kSumN] = {0};  // (one device block: ctr, then sums at byte 64)
    uint32_t *big_start[2], *big_len[2];
    uint64_t *big_pref[2];         // prefixes of the big-list buckets (Lists::nb_pref)
    uint64_t *loc_pref[kLocal];    // prefixes of generation 0's local entries (Lists::loc_pref)
    uint32_t *dn_start, *dn_len;
    uint8_t *dn_par;
    uint2 *loc[kLocal][2];
    int wsched[kMaxLevels];  // digit bits of global level l (L0: 7..8 for 2-bit keys, else 8; l >= 1: 6..8)
    int width(int level) const { return wsched[std::min(level, kMaxLevels - 1)]; }
    uint8_t *heads = nullptr;
    uint8_t *nd = nullptr;  // next-level digit per element of the last pass's output
    // compact level (see classify_kernel): the last pass wrote (low key bits, start) pairs and the
    // next digit instead of keys and starts
    bool compact_now = false;
    int compact_hi = 0;
    bool nd_ready = false, nd_next = true;
    // packed-pair levels (MODE 5): the level before a compact one writes 10-byte (key bits below
    // the sorted ones, start) pairs + the digit byte instead of 12-byte (key, start) + digit; the
    // compact level reads them (IN79).  allow_c79: msd_sort's own levels (GKM_NO_PAIRS=1: off)
    bool allow_c79 = false, c79_in = false, c79_out = false;
    // the packed L0 (P88, msd0_pipe_kernel): its output is (digit byte, packed pair) in nd_l0 /
    // lo16_l0 / keys; p88_in: the next level reads it (p88_wanted: msd_sort's decision)
    bool p88 = false, p88_in = false, pieces_level = false;
    int p88_shi = 0;
    uint16_t *lo16_l0 = nullptr;
    uint8_t *nd_l0 = nullptr;
    int c79_shi = 0;
    uint16_t *lo16 = nullptr;
    uint32_t *tile_hist, *chunk_hist, *c_first, *c_ntiles, *seg_base, *seg_cnt;
    uint64_t nloc[kLocal] = {0}, loc_elems[kLocal] = {0}, ndone = 0, big_elems = 0;
    uint32_t nbig = 0;
    int cur_big = 0;
    int phase = 0;  // key word being sorted (multi-word keys)
    uint32_t ctiles = kChunkTiles;  // tiles per column-scan chunk
    // final keys: the finishing kernels also write every key to keys[0], so a one-word sort ends
    // with sorted keys + starts + heads in HBM (no re-encode by gather afterwards)
    int wkeys = 0;
    const uint64_t *pk_code = nullptr;  // packed sequence for the L0 passes (ACGT, 2-bit keys)
    const uint32_t *pk_dol = nullptr;

    MsdDriver(gk_ctx *c_, const KeySpec &ks_) : c(c_), ks(ks_), B(ks_.total_bits) {
        cus = cu_count(c);
        pgrid = cus * 4;  // 4 workgroups per CU, one resident at a time (LDS); measured faster than 1
        set_widths(opt("GKM_LEVEL_BITS"));
        // test-only: small scan chunks so that parity tests reach the multi-chunk branches of the
        // column scan and tile tables (otherwise only buckets > 2.9 M keys have more than one chunk)
        if (const char *e = opt("GKM_TEST_CHUNK_TILES")) ctiles = (uint32_t)std::max(1, std::atoi(e));
    }

    // the whole sort of forward 2-bit one-word keys (msd_sort's phase 0): an 11-bit L0
    // (msd0_wide_kernel) when GKM_WIDE_L0=1 (A/B), so that 11 + 8 bits leave C3-sized buckets for
    // one block-local round
    void enable_wide_l0() {
        const char *e = opt("GKM_WIDE_L0");  // (read per sort: tests flip it)
        const bool want = e && *e && std::strcmp(e, "0") != 0;
        if (want && ks.bits == 2 && !ks.canonical && !ks.acgt_only && B > kWideL0 + 8) wsched[0] = kWideL0;
    }

    // level digit widths "w0,w1,w2,..." (the last one repeats).  Default 7,8,8,...: for 2-bit
    // keys a 7-bit L0 is ~10% faster than an 8-bit one (longer runs per tile), and after 23 bits
    // the C3 buckets (~370) fit the one-wave finishing kernel; 4-bit keys keep an 8-bit L0.
    void set_widths(const char *spec) {
        for (int l = 0; l < kMaxLevels; ++l) wsched[l] = kGR;
        if (ks.bits == 2) wsched[0] = 7;
        if (!spec) return;
        int l = 0, w = kGR;
        for (const char *p = spec; *p && l < kMaxLevels;) {
            w = std::min(8, std::max(6, std::atoi(p)));
            wsched[l++] = w;
            while (*p && *p != ',') ++p;
            if (*p == ',') ++p;
        }
        for (; l < kMaxLevels; ++l) wsched[l] = w;
        if (ks.bits != 2) wsched[0] = kGR;
        wsched[0] = std::max(wsched[0], ks.canonical ? 7 : 6);  // (6: forward 2-bit L0 only)
    }

    Lists lists(int g, int bigsel) {
        // prefixes are recorded by classify (generation 0); re-listed entries carry full keys
        return Lists{big_start[bigsel], big_len[bigsel], dn_start, dn_len, dn_par,
                     {loc[0][g], loc[1][g], loc[2][g], loc[3][g], loc[4][g], loc[5][g]}, big_pref[bigsel],
                     {g ? nullptr : loc_pref[0], g ? nullptr : loc_pref[1], g ? nullptr : loc_pref[2],
                      g ? nullptr : loc_pref[3], g ? nullptr : loc_pref[4], g ? nullptr : loc_pref[5]}};
    }

    int init(uint64_t n_) {
        n = n_;
        GK_TRY_HIP(c, msd_tables());
        static_assert(4 * kCtrN <= 64 && 64 + 8 * kSumN <= 8 * kHostPinWords, "list counter block");
        uint64_t *cs;
        GK_TRY_HIP(c, scratch(c, "msd_ctr_sums", 8 + kSumN, &cs));
        ctr = reinterpret_cast<uint32_t *>(cs);
        sums = reinterpret_cast<unsigned long long *>(cs + 8);
        GK_TRY_HIP(c, hipMemsetAsync(ctr, 0, 4 * kCtrN, c->stream));
        const uint64_t max_big = n / kBlockMax + 2;
        GK_TRY_HIP(c, scratch(c, "big_start0", max_big, &big_start[0]));
        GK_TRY_HIP(c, scratch(c, "big_len0", max_big, &big_len[0]));
        GK_TRY_HIP(c, scratch(c, "big_start1", max_big, &big_start[1]));
        GK_TRY_HIP(c, scratch(c, "big_len1", max_big, &big_len[1]));
        GK_TRY_HIP(c, scratch(c, "big_pref0", max_big, &big_pref[0]));
        GK_TRY_HIP(c, scratch(c, "big_pref1", max_big, &big_pref[1]));
        GK_TRY_HIP(c, grow_keep(c, "dn_start", 1024, 0, &dn_start));
        GK_TRY_HIP(c, grow_keep(c, "dn_len", 1024, 0, &dn_len));
        GK_TRY_HIP(c, grow_keep(c, "dn_par", 1024, 0, &dn_par));
        for (int k = 0; k < kLocal; ++k) GK_TRY_HIP(c, grow_keep(c, kLocName[k][0], 1024, 0, &loc[k][0]));
        for (int k = 0; k < kLocal; ++k) GK_TRY_HIP(c, grow_keep(c, kLocPrefName[k], 1024, 0, &loc_pref[k]));
        GK_TRY_HIP(c, scratch(c, "msd_heads", n + 64, &heads));
        return GK_OK;
    }

    // the list counters and sums: one copy into pinned host memory
    int read_ctr() {
        uint64_t buf[8 + kSumN];
        GK_TRY_HIP(c, read_back(c, ctr, sizeof(buf), buf));
        std::memcpy(h, buf, 4 * kCtrN);
        std::memcpy(hs, buf + 8, 8 * kSumN);
        return GK_OK;
    }

    // scan per-tile histograms of nseg buckets (C chunks) into per-tile offsets + sub-bucket tables
    template <int RADIX>
    void scan_launch(uint64_t C, const uint32_t *s_cfirst, const uint32_t *s_nchunks, const uint32_t *s_start,
                     uint64_t nseg) {
        constexpr int TH = scan_threads<RADIX>();
        hipLaunchKernelGGL(chunk_sum_kernel<RADIX>, dim3((unsigned)C, RADIX / TH), dim3(TH), 0, c->stream, tile_hist,
                           c_first, c_ntiles, chunk_hist);
        hipLaunchKernelGGL(seg_scan_kernel<RADIX>, dim3((unsigned)nseg), dim3(TH), 0, c->stream, chunk_hist,
                           s_cfirst, s_nchunks, s_start, seg_base, seg_cnt);
        hipLaunchKernelGGL(tile_apply_kernel<RADIX>, dim3((unsigned)C, RADIX / TH), dim3(TH), 0, c->stream, tile_hist,
                           c_first, c_ntiles, chunk_hist);
    }

    int scan_offsets(int R, uint64_t C, const uint32_t *s_cfirst, const uint32_t *s_nchunks, const uint32_t *s_start,
                     uint64_t nseg) {
        timer_begin(c, "msd_scan", &slot);
        if (R == 8) scan_launch<256>(C, s_cfirst, s_nchunks, s_start, nseg);
        else if (R == 7) scan_launch<128>(C, s_cfirst, s_nchunks, s_start, nseg);
        else if (R == kWideL0) scan_launch<1 << kWideL0>(C, s_cfirst, s_nchunks, s_start, nseg);
        else scan_launch<64>(C, s_cfirst, s_nchunks, s_start, nseg);
        GK_TRY_HIP(c, hipGetLastError());
        timer_end(c, slot);
        return GK_OK;
    }

    // tile / chunk tables: device buffers sized for T tiles, C chunks, nseg buckets
    int tables(uint64_t T, uint64_t C, uint64_t nseg) {
        const uint64_t rad = std::max(kGRadix, 1 << wsched[0]);  // the wide L0's digits
        GK_TRY_HIP(c, scratch(c, "tile_hist", T * rad, &tile_hist));
        GK_TRY_HIP(c, scratch(c, "chunk_hist", C * rad, &chunk_hist));
        GK_TRY_HIP(c, scratch(c, "c_first", C, &c_first));
        GK_TRY_HIP(c, scratch(c, "c_ntiles", C, &c_ntiles));
        GK_TRY_HIP(c, scratch(c, "seg_base", nseg * rad, &seg_base));
        GK_TRY_HIP(c, scratch(c, "seg_cnt", nseg * rad, &seg_cnt));
        return GK_OK;
    }

    // L0 kernels: count (per-tile digit histograms) or partition; bits x digit width x next digits
    // x canonical
    template <int BITS, int R, bool ND, bool CANON, bool P88 = false, bool OWN = false>
    void l0_launch(bool count, const L0Args &a, Dig d0, unsigned nt0, uint64_t *kout, uint32_t *vout, uint32_t nt,
                   uint64_t sink, const NextDigits &ndg) {
        // the count pass streams the sequence: 256-thread workgroups, eight per CU, each holding a
        // whole tile of loads in flight (1,024-thread ones, two per CU, kept a quarter as many
        // bytes in flight and measured slower)
        if (count) {
            static int per_cu = 0;  // resident workgroups (the grid is persistent)
            if (!per_cu &&
                (hipOccupancyMaxActiveBlocksPerMultiprocessor(
                     &per_cu, (const void *)msd0_count_kernel<BITS, kP0T / 4, kP0I * 4, R, CANON>, kP0T / 4, 0) !=
                     hipSuccess ||
                 per_cu < 1))
                per_cu = 1;
            hipLaunchKernelGGL((msd0_count_kernel<BITS, kP0T / 4, kP0I * 4, R, CANON>),
                               dim3(std::min<unsigned>(nt0, cus * per_cu)), dim3(kP0T / 4), 0, c->stream, a, d0,
                               tile_hist, nt0);
        }
        else if (BITS == 2 && R == 7 && !CANON && !P88 && l0_prof())
            l0_prof_launch<ND>(a, d0, kout, vout, nt, sink, ndg);
        else
            hipLaunchKernelGGL((msd0_pipe_kernel<BITS, kP0T, kP0I, R, ND, CANON, false, P88, OWN>), dim3(pgrid),
                               dim3(kP0T), 0, c->stream, a, d0, tile_hist, kout, vout, nt, sink, ndg);
    }

    // timing only (GKM_L0_PROF=1): the L0 partition with per-phase clocks, printed to stderr
    template <bool ND>
    void l0_prof_launch(L0Args a, Dig d0, uint64_t *kout, uint32_t *vout, uint32_t nt, uint64_t sink,
                        const NextDigits &ndg) {
#ifndef GKM_EXPERIMENTS
        (void)a, (void)d0, (void)kout, (void)vout, (void)nt, (void)sink, (void)ndg;  // (timing builds only)
#else
        unsigned long long *pr = nullptr;
        if (scratch(c, "l0_prof", 2 * kL0Phases, &pr) != hipSuccess) return;
        hipMemsetAsync(pr, 0, 16 * kL0Phases, c->stream);
        a.prof = pr;
        hipLaunchKernelGGL((msd0_pipe_kernel<2, kP0T, kP0I, 7, ND, false, true>), dim3(pgrid), dim3(kP0T), 0, c->stream,
                           a, d0, tile_hist, kout, vout, nt, sink, ndg);
        unsigned long long h[2 * kL0Phases];
        hipMemcpyAsync(h, pr, 16 * kL0Phases, hipMemcpyDeviceToHost, c->stream);
        hipStreamSynchronize(c->stream);
        static const char *names[kL0Phases] = {"pack+load", "top-stores", "bar1", "clean", "rank+stores",
                                               "bar2", "scan+stores", "staging+stores", "bar5"};
        for (int w = 0; w < 2; ++w) {
            unsigned long long tot = 0;
            for (int k = 0; k < kL0Phases; ++k) tot += h[w * kL0Phases + k];
            std::fprintf(stderr, "[l0prof] wave %s:", w ? "last" : "first");
            for (int k = 0; k < kL0Phases; ++k)
                std::fprintf(stderr, " %s %.1f%%", names[k], tot ? 100.0 * h[w * kL0Phases + k] / tot : 0.0);
            std::fprintf(stderr, " (ticks per tile: %.0f)\n", (double)tot / std::max<uint32_t>(nt, 1));
        }
#endif
    }

    template <bool CANON>
    void l0_dispatch_c(bool count, int w0, bool nd_, const L0Args &a, Dig d0, unsigned nt0, uint64_t *kout,
                       uint32_t *vout, uint32_t nt, uint64_t sink, const NextDigits &ndg) {
        if (ks.bits == 2 && !CANON && w0 == kWideL0) {  // enable_wide_l0: forward 2-bit one-word sorts
            if (count) {
                static int per_cu = 0;
                if (!per_cu &&
                    (hipOccupancyMaxActiveBlocksPerMultiprocessor(
                         &per_cu, (const void *)msd0_count_kernel<2, 256, kWT * kWI / 256, kWideL0, false>, 256,
                         0) != hipSuccess ||
                     per_cu < 1))
                    per_cu = 1;
                hipLaunchKernelGGL((msd0_count_kernel<2, 256, kWT * kWI / 256, kWideL0, false>),
                                   dim3(std::min<unsigned>(nt0, cus * per_cu)), dim3(256), 0, c->stream, a, d0,
                                   tile_hist, nt0);
            } else if (nd_)
                hipLaunchKernelGGL((msd0_wide_kernel<kWT, kWI, kWideL0, true>), dim3(pgrid), dim3(kWT), 0, c->stream,
                                   a, d0, tile_hist, kout, vout, nt, sink, ndg);
            else
                hipLaunchKernelGGL((msd0_wide_kernel<kWT, kWI, kWideL0, false>), dim3(pgrid), dim3(kWT), 0,
                                   c->stream, a, d0, tile_hist, kout, vout, nt, sink, ndg);
            return;
        }
        const bool pk = !count && nd_ && ndg.out16 != nullptr;  // the packed L0 (P88)
        // a key-range rank's L0 over the packed copy: test, compact, then rank only the kept k-mers
        // (GKM_OWN_L0_COMPACT=1, measured slower than the select + level from pieces at N >= 4 and
        // equal to the tile L0 at N = 2: own_part_kernel)
        if (ks.bits == 2 && !CANON && a.own_span != 0xFFFFFFFFu && a.own_span != 0 && a.pk_code &&
            ks.symbols <= 32 && a.own_bits <= 32 && (w0 == 7 || w0 == kGR) && (count || nd_) &&
            opt("GKM_OWN_L0_COMPACT")) {
            const int sh = 32 - a.own_bits;
            const OwnTest ot{(uint32_t)((uint64_t)a.own_lo << sh),
                             (uint32_t)(((uint64_t)std::min<uint64_t>(a.own_span, 1ull << a.own_bits) << sh) - 1)};
            auto grid = [&](const void *k) {
                int per_cu = 0;
                if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, kOwnT, 0) != hipSuccess || per_cu < 1)
                    per_cu = 1;
                return dim3(std::min<unsigned>(nt0, cus * (unsigned)per_cu));
            };
#define GK_OWN(R_)                                                                                             \
    do {                                                                                                       \
        if (count)                                                                                             \
            hipLaunchKernelGGL(own_count_kernel<R_>, grid((const void *)own_count_kernel<R_>), dim3(kOwnT), 0,   \
                               c->stream, a, d0, ot, tile_hist, nt0);                                         \
        else if (pk)                                                                                           \
            hipLaunchKernelGGL((own_part_kernel<R_, true>), grid((const void *)own_part_kernel<R_, true>),       \
                               dim3(kOwnT), 0, c->stream, a, d0, ot, tile_hist, kout, vout, nt, ndg);         \
        else                                                                                                   \
            hipLaunchKernelGGL((own_part_kernel<R_, false>), grid((const void *)own_part_kernel<R_, false>),     \
                               dim3(kOwnT), 0, c->stream, a, d0, ot, tile_hist, kout, vout, nt, ndg);         \
    } while (0)
            if (w0 == 7) GK_OWN(7);
            else GK_OWN(kGR);
#undef GK_OWN
            return;
        }
        if (!count && ks.bits == 2 && nd_ && a.own_span != 0xFFFFFFFFu) {  // a key-range rank's fused select
            if (w0 == 7) {
                if (pk) l0_launch<2, 7, true, CANON, true, true>(count, a, d0, nt0, kout, vout, nt, sink, ndg);
                else l0_launch<2, 7, true, CANON, false, true>(count, a, d0, nt0, kout, vout, nt, sink, ndg);
            } else {
                if (pk) l0_launch<2, kGR, true, CANON, true, true>(count, a, d0, nt0, kout, vout, nt, sink, ndg);
                else l0_launch<2, kGR, true, CANON, false, true>(count, a, d0, nt0, kout, vout, nt, sink, ndg);
            }
            return;
        }
        if (ks.bits == 2 && w0 == 7) {
            if (pk) l0_launch<2, 7, true, CANON, true>(count, a, d0, nt0, kout, vout, nt, sink, ndg);
            else if (nd_) l0_launch<2, 7, true, CANON>(count, a, d0, nt0, kout, vout, nt, sink, ndg);
            else l0_launch<2, 7, false, CANON>(count, a, d0, nt0, kout, vout, nt, sink, ndg);
        } else if (ks.bits == 2 && w0 == 6 && !CANON) {  // (A/B, GKM_LEVEL_BITS=6,...: half the L0's write streams)
            if (pk) l0_launch<2, 6, true, false, true>(count, a, d0, nt0, kout, vout, nt, sink, ndg);
            else if (nd_) l0_launch<2, 6, true, false>(count, a, d0, nt0, kout, vout, nt, sink, ndg);
            else l0_launch<2, 6, false, false>(count, a, d0, nt0, kout, vout, nt, sink, ndg);
        } else if (ks.bits == 2) {
            if (pk) l0_launch<2, kGR, true, CANON, true>(count, a, d0, nt0, kout, vout, nt, sink, ndg);
            else if (nd_) l0_launch<2, kGR, true, CANON>(count, a, d0, nt0, kout, vout, nt, sink, ndg);
            else l0_launch<2, kGR, false, CANON>(count, a, d0, nt0, kout, vout, nt, sink, ndg);
        } else {
            if (nd_) l0_launch<4, kGR, true, CANON>(count, a, d0, nt0, kout, vout, nt, sink, ndg);
            else l0_launch<4, kGR, false, CANON>(count, a, d0, nt0, kout, vout, nt, sink, ndg);
        }
    }

    void l0_dispatch(bool count, int w0, bool nd_, const L0Args &a, Dig d0, unsigned nt0, uint64_t *kout,
                     uint32_t *vout, uint32_t nt, uint64_t sink, const NextDigits &ndg) {
        if (ks.canonical) l0_dispatch_c<true>(count, w0, nd_, a, d0, nt0, kout, vout, nt, sink, ndg);
        else l0_dispatch_c<false>(count, w0, nd_, a, d0, nt0, kout, vout, nt, sink, ndg);
    }

    // L0: encode the k-mers starting in [lo, hi) and partition them by the top kGR key bits into
    // kout / vout (capacity >= n + 1: element n is the scatter's sink).  seg_base / seg_cnt then
    // hold the kGRadix buckets.  *count: k-mers found (checked against cap before the scatter).
    int run_l0(uint64_t lo, uint64_t hi, uint64_t *kout, uint32_t *vout, uint64_t cap, uint64_t *count) {
        int rc = l0_count(lo, hi, 0, 0xFFFFFFFFu, count);
        if (rc != GK_OK) return rc;
        return l0_partition(kout, vout, cap, *count);
    }

    // key-range shards: the L0 digit range [own_lo, own_lo + own_span) is kept (width(0) bits)
    L0Args l0a{};
    uint64_t l0_tiles = 0;

    // L0 count pass: per-tile digit histograms of the kept k-mers starting in [lo, hi), their
    // column scan (seg_base / seg_cnt), *count = k-mers kept
    int l0_count(uint64_t lo, uint64_t hi, uint32_t own_lo, uint32_t own_span, uint64_t *count, int own_bits = 0) {
        const uint64_t span = hi > lo ? hi - lo : 0;
        const uint64_t tile = wsched[0] == kWideL0 ? (uint64_t)kWT * kWI : (uint64_t)kP0Tile;  // (the wide L0's own)
        const uint64_t nt0 = std::max<uint64_t>((span + tile - 1) / tile, 1);
        const uint64_t nc0 = (nt0 + ctiles - 1) / ctiles;
        l0_tiles = nt0;
        int rc = tables(nt0, nc0, 1);
        if (rc != GK_OK) return rc;
        uint32_t *s_misc;
        GK_TRY_HIP(c, scratch(c, "s_misc", 4, &s_misc));
        {
            std::vector<uint32_t> cf(nc0), cn(nc0);
            for (uint64_t j = 0; j < nc0; ++j) {
                cf[j] = (uint32_t)(j * ctiles);
                cn[j] = (uint32_t)std::min<uint64_t>(ctiles, nt0 - j * ctiles);
            }
            const uint32_t misc[3] = {0, (uint32_t)nc0, 0};  // s_cfirst, s_nchunks, s_start
            GK_TRY_HIP(c, hipMemcpyAsync(c_first, cf.data(), 4 * nc0, hipMemcpyHostToDevice, c->stream));
            GK_TRY_HIP(c, hipMemcpyAsync(c_ntiles, cn.data(), 4 * nc0, hipMemcpyHostToDevice, c->stream));
            GK_TRY_HIP(c, hipMemcpyAsync(s_misc, misc, 12, hipMemcpyHostToDevice, c->stream));
            GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
        }
        L0Args a{c->sba, lo, hi, ks.symbols, B, ks.acgt_only};
        a.own_lo = own_lo;
        a.own_span = own_span;
        if (own_bits) a.own_bits = own_bits;
        a.pk_code = pk_code;
        a.pk_dol = pk_dol;
        l0a = a;
        const int w0 = width(0);
        const Dig d0 = dig_at(B, 0, w0);
        timer_begin(c, "msd_l0_count", &slot);
        l0_dispatch(true, w0, false, a, d0, (unsigned)nt0, nullptr, nullptr, 0, 0, NextDigits{});
        GK_TRY_HIP(c, hipGetLastError());
        timer_end(c, slot);
        rc = scan_offsets(w0, nc0, s_misc, s_misc + 1, s_misc + 2, 1);
        if (rc != GK_OK) return rc;
        // the bucket total = k-mers found (the last bucket's base + count)
        uint32_t last[2];
        GK_TRY_HIP(c, hipMemcpyAsync(&last[0], seg_base + (1 << w0) - 1, 4, hipMemcpyDeviceToHost, c->stream));
        GK_TRY_HIP(c, hipMemcpyAsync(&last[1], seg_cnt + (1 << w0) - 1, 4, hipMemcpyDeviceToHost, c->stream));
        GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
        *count = (uint64_t)last[0] + last[1];
        return GK_OK;
    }

    // L0 partition pass after l0_count (same tiles, same range)
    int l0_partition(uint64_t *kout, uint32_t *vout, uint64_t cap, uint64_t count) {
        if (count + 1 > cap) return fail(c, GK_E_ARG, "partition output buffer too small");
        const int w0 = width(0);
        const Dig d0 = dig_at(B, 0, w0);
        timer_begin(c, p88 ? "msd_pass_l0k" : "msd_pass_l0", &slot);  // (l0k: the packed L0 output)
        timer_units(c, slot, count);
        // the sort's own L0 also writes the level-1 digits (shard sends are re-counted after the
        // exchange, so they do not)
        // (a starts-only shard send has no key output: kout == nullptr, which a context whose key
        // buffers are not allocated yet must not mistake for one of them)
        const bool with_nd = kout && (kout == c->keys[0] || kout == c->keys[1]) && !opt("GKM_L0_NO_ND");  // (tuning knob)
        NextDigits ndg{dig_at(B, w0, width(1)), nullptr};
        if (with_nd && p88) {  // the packed L0: digit bytes and low start bits in the free start buffer
            p88_place(vout == c->vals[0] ? 0 : 1);
            nd = nd_l0;
            ndg.out = nd;
            ndg.out16 = lo16_l0;
            ndg.pshi = p88_shi;
        } else if (with_nd) {
            GK_TRY_HIP(c, scratch(c, "msd_nd", n + 64, &nd));
            ndg.out = nd;
        }
        // timing experiments only (wrong output): GKM_EXP_L0=1 the scatter floor at 2^7 runs per tile,
        // =4 / 5 / 6 / 8 at 2^R runs (the same bytes in fewer or more write streams), =v at 2^7 runs
        // with 4-slot vector stores
        static const char *exp_l0 = exp_opt("GKM_EXP_L0");
        const int exp_r = exp_l0 ? (exp_l0[0] == '1' || exp_l0[0] == 'v' ? 7 : exp_l0[0] - '0') : 0;
        if (exp_r && with_nd && w0 == 7) {
            if (exp_r == 4)
                hipLaunchKernelGGL((l0_scatter_floor_kernel<kP0T, kP0I, 4>), dim3(pgrid), dim3(kP0T), 0, c->stream,
                                   c->sba, count, (uint32_t)l0_tiles, kout, vout, nd);
            else if (exp_r == 5)
                hipLaunchKernelGGL((l0_scatter_floor_kernel<kP0T, kP0I, 5>), dim3(pgrid), dim3(kP0T), 0, c->stream,
                                   c->sba, count, (uint32_t)l0_tiles, kout, vout, nd);
            else if (exp_r == 6)
                hipLaunchKernelGGL((l0_scatter_floor_kernel<kP0T, kP0I, 6>), dim3(pgrid), dim3(kP0T), 0, c->stream,
                                   c->sba, count, (uint32_t)l0_tiles, kout, vout, nd);
            else if (exp_l0[0] == 'v')
                hipLaunchKernelGGL((l0_scatter_floor4_kernel<kP0T, kP0I, 7>), dim3(pgrid), dim3(kP0T), 0, c->stream,
                                   c->sba, count, (uint32_t)l0_tiles, kout, vout, nd);
            else if (exp_r == 8)
                hipLaunchKernelGGL((l0_scatter_floor_kernel<kP0T, kP0I, 8>), dim3(pgrid), dim3(kP0T), 0, c->stream,
                                   c->sba, count, (uint32_t)l0_tiles, kout, vout, nd);
            else
                hipLaunchKernelGGL((l0_scatter_floor_kernel<kP0T, kP0I, 7>), dim3(pgrid), dim3(kP0T), 0, c->stream,
                                   c->sba, count, (uint32_t)l0_tiles, kout, vout, nd);
        } else
            l0_dispatch(false, w0, with_nd, l0a, d0, (unsigned)l0_tiles, kout, vout, (uint32_t)l0_tiles, count, ndg);
        GK_TRY_HIP(c, hipGetLastError());
        timer_end(c, slot);
        nd_ready = with_nd;
        p88_in = with_nd && p88;
        return GK_OK;
    }

    // the packed L0 pays when the level behind it writes packed pairs itself (it reads the packed
    // form, INP = 2): the same prediction level_pass makes at L1 from the mean bucket sizes, with the
    // L1 digit being the digit byte (8 bits).  GKM_NO_P88=1: off; GKM_TEST_P88=1 (tests): wherever
    // the bits fit.  C3: 62 - 7 = 55 bits after the L0, 47 of them in the pair (shi 17).
    bool p88_wanted() const {
        if (opt("GKM_NO_P88") || !allow_c79 || ks.bits != 2 || phase != 0 || no_compact()) return false;
        const int w0 = width(0), w1 = width(1), w2 = width(2), rem = B - w0;
        if ((w0 != 6 && w0 != 7 && w0 != kGR) || w1 != 8 || rem - 8 < 33 || rem - 8 > 48) return false;
        if (opt("GKM_TEST_P88")) return true;
        const uint64_t m1 = (n >> w0) >> w1;  // mean L1 sub-bucket
        const int rem2 = rem - w1 - w2;
        return m1 >= (uint64_t)kBlockMax && (m1 >> w2) < (uint64_t)kBlockMax && rem2 >= 9 && rem2 <= 40 && w2 == 8 &&
               width(3) == 8;
    }

    // The packed L0 writes no starts, so its low start bits and digit bytes live in the start buffer
    // of its own output (vals[buf]: 4 B per element; 2 + 1 used) -- no extra memory.  An expansion
    // back to (key, start) writes that buffer, so it first copies them out (p88_detach, rare: skewed
    // genomes and test shapes) and every later reader takes the copy.
    void p88_place(int buf) {
        lo16_l0 = reinterpret_cast<uint16_t *>(c->vals[buf]);
        nd_l0 = reinterpret_cast<uint8_t *>(c->vals[buf]) + ((2 * (c->elem_cap + 64) + 255) & ~255ull);
    }
    int p88_detach() {
        uint8_t *t;
        const uint64_t m = c->elem_cap + 64;
        if (!lo16_l0) return GK_OK;
        GK_TRY_HIP(c, scratch(c, "p88_detached", 3 * m, &t));
        if (reinterpret_cast<uint8_t *>(lo16_l0) == t) return GK_OK;  // (already)
        GK_TRY_HIP(c, hipMemcpyAsync(t, lo16_l0, 2 * m, hipMemcpyDeviceToDevice, c->stream));
        GK_TRY_HIP(c, hipMemcpyAsync(t + 2 * m, nd_l0, m, hipMemcpyDeviceToDevice, c->stream));
        if (nd == nd_l0) nd = t + 2 * m;
        lo16_l0 = reinterpret_cast<uint16_t *>(t);
        nd_l0 = t + 2 * m;
        return GK_OK;
    }

    // after the packed L0's classify: its local entries back to (key, start) for the finishing kernels
    int expand_p88_locals(int buf) {
        bool any = false;
        for (int k = 0; k < kLocal; ++k) any |= nloc[k] > 0;
        if (!any) return GK_OK;
        if (int rc = p88_detach()) return rc;
        for (int k = 0; k < kLocal; ++k) {
            if (!nloc[k]) continue;
            hipLaunchKernelGGL(expand_p88_list_kernel, dim3((unsigned)nloc[k]), dim3(256), 0, c->stream, loc[k][0],
                               loc_pref[k], B, p88_shi, c->keys[buf], lo16_l0, nd_l0, c->vals[buf]);
            GK_TRY_HIP(c, hipGetLastError());
        }
        return GK_OK;
    }

    // one region of the prefetched L0 (L0Prefetch, below): count, column scan and partition of the
    // k-mers starting in [lo, hi) into keys[1] / vals[1] / nd at output indices from lo, then the
    // region's 2^w0 bucket bases and counts into `pieces` -- all on c->stream (the caller points it
    // at the prefetch stream), with the region's chunk tables already in `tab` (c_first[nc],
    // c_ntiles[nc], then s_cfirst, s_nchunks, s_start) and no host round trip
    int l0_region(uint64_t lo, uint64_t hi, uint32_t nt, uint32_t nc, uint32_t nc_max, uint32_t *tab, uint64_t sink,
                  uint32_t *pieces) {
        int rc = tables(nt, nc, 1);  // (allocated by prefetch_plan: no reallocation here)
        if (rc != GK_OK) return rc;
        c_first = tab;  // (the region's table: nc_max entries each, then misc)
        c_ntiles = tab + nc_max;
        const uint32_t *misc = tab + 2 * nc_max;
        // (acgt_only: every byte other than A/C/G/T ends k-mers -- on an ACGT sba exactly the '$'
        // separators, so this is the plain sort's L0 there, and the class-A L0 of a mixed sba's
        // split sort elsewhere)
        const L0Args a{c->sba, lo, hi, ks.symbols, B, 1};
        const int w0 = width(0);
        const Dig d0 = dig_at(B, 0, w0);
        l0_dispatch(true, w0, false, a, d0, nt, nullptr, nullptr, 0, 0, NextDigits{});
        GK_TRY_HIP(c, hipGetLastError());
        rc = scan_offsets(w0, nc, misc, misc + 1, misc + 2, 1);
        if (rc != GK_OK) return rc;
        NextDigits ndg{dig_at(B, w0, width(1)), nd};
        if (p88) {  // the packed L0 (P88): nd / lo16_l0 set by the caller
            ndg.out16 = lo16_l0;
            ndg.pshi = p88_shi;
        }
        l0_dispatch(false, w0, true, a, d0, nt, c->keys[1], c->vals[1], nt, sink, ndg);
        GK_TRY_HIP(c, hipGetLastError());
        GK_TRY_HIP(c, hipMemcpyAsync(pieces, seg_base, 4u << w0, hipMemcpyDeviceToDevice, c->stream));
        GK_TRY_HIP(c, hipMemcpyAsync(pieces + (1u << w0), seg_cnt, 4u << w0, hipMemcpyDeviceToDevice, c->stream));
        return GK_OK;
    }

    // after a compact level: the (rare) sub-buckets that go to another global level get their keys
    // back in keys[out], so that level reads keys as usual (the digit bytes stay valid for it)
    int expand_big(int out) {
        if (!compact_now || nbig == 0) return GK_OK;
        hipLaunchKernelGGL(expand_compact_kernel, dim3(nbig, bucket_split(nbig)), dim3(256), 0, c->stream, big_start[cur_big],
                           big_len[cur_big], big_pref[cur_big], compact_hi, B, nd, c->keys[out], c->vals[out]);
        GK_TRY_HIP(c, hipGetLastError());
        return GK_OK;
    }

    // route nsub sub-buckets (seg_base / seg_cnt, or base / cnt) of a level; hi = key bits sorted
    // after it; sub-buckets under min_size elements are dropped (final as they stand)
    // ppref / pw / compact: see classify_kernel
    int classify(uint64_t nsub, int hi, int parity, int bigsel, const uint32_t *base = nullptr,
                 const uint32_t *cnt = nullptr, uint32_t min_size = 1, const uint64_t *ppref = nullptr, int pw = 0,
                 int compact = 0, bool read = true) {
        if (!base) base = seg_base;
        if (!cnt) cnt = seg_cnt;
        for (int k = 0; k < kLocal; ++k)
            GK_TRY_HIP(c, grow_keep(c, kLocName[k][0], nloc[k] + nsub, nloc[k], &loc[k][0]));
        for (int k = 0; k < kLocal; ++k)
            GK_TRY_HIP(c, grow_keep(c, kLocPrefName[k], nloc[k] + nsub, nloc[k], &loc_pref[k]));
        GK_TRY_HIP(c, grow_keep(c, "dn_start", ndone + nsub, ndone, &dn_start));
        GK_TRY_HIP(c, grow_keep(c, "dn_len", ndone + nsub, ndone, &dn_len));
        GK_TRY_HIP(c, grow_keep(c, "dn_par", ndone + nsub, ndone, &dn_par));
        GK_TRY_HIP(c, hipMemsetAsync(ctr + kCtrBig, 0, 4, c->stream));
        GK_TRY_HIP(c, hipMemsetAsync(sums, 0, 8 * kSumN, c->stream));
        timer_begin(c, "msd_classify", &slot);
        hipLaunchKernelGGL(classify_kernel, dim3((unsigned)((nsub + kClassT - 1) / kClassT)), dim3(kClassT), 0,
                           c->stream, base, cnt, nsub, hi, B, parity, lists(0, bigsel), ctr, sums, min_size, ppref, pw,
                           compact, (uint32_t)kPTile, ctiles);
        GK_TRY_HIP(c, hipGetLastError());
        timer_end(c, slot);
        return read ? classify_counts() : GK_OK;
    }

    // the lists classify wrote (and drop_uniform_dev re-routed), to the host
    int classify_counts() {
        int r = read_ctr();
        if (r != GK_OK) return r;
        for (int k = 0; k < kLocal; ++k) {
            nloc[k] = h[kCtrLoc + k];
            loc_elems[k] += hs[kCtrLoc + k];
        }
        ndone = h[kCtrDone];
        nbig = h[kCtrBig];
        big_elems = hs[kCtrBig];
        return GK_OK;
    }

    // drop_uniform with no read-back of its own, behind a classify that did not read its lists
    // either (the deep levels of a repeat-rich genome: one host round trip per level instead of
    // two): the next-level list's count stays on the device; `bound` >= that count sizes the grids
    // (the blocks past the count return at once).  Ends with classify_counts.
    int drop_uniform_dev(int out, uint32_t bound) {
        const uint32_t *nb_dev = ctr + kCtrBig;
        const unsigned split = bucket_split(bound);
        if (compact_now)
            hipLaunchKernelGGL(expand_compact_kernel, dim3(bound, split), dim3(256), 0, c->stream, big_start[cur_big],
                               big_len[cur_big], big_pref[cur_big], compact_hi, B, nd, c->keys[out], c->vals[out],
                               nb_dev);
        uint32_t *mixed;
        GK_TRY_HIP(c, scratch(c, "uni_mixed", bound, &mixed));
        GK_TRY_HIP(c, hipMemsetAsync(mixed, 0, 4ull * bound, c->stream));
        hipLaunchKernelGGL(uniform_flag_kernel, dim3(bound, split), dim3(256), 0, c->stream, big_start[cur_big],
                           big_len[cur_big], c->keys[out], mixed, nb_dev, ctr + kCtrNbCopy);
        // (the done list has room: classify grew it by every sub-bucket, and each goes to one list)
        GK_TRY_HIP(c, hipMemsetAsync(ctr + kCtrBig, 0, 4, c->stream));
        GK_TRY_HIP(c, hipMemsetAsync(sums + kCtrBig, 0, 8, c->stream));
        GK_TRY_HIP(c, hipMemsetAsync(sums + kSumTiles, 0, 16, c->stream));
        hipLaunchKernelGGL(route_uniform_kernel, dim3(grid_n(bound)), dim3(256), 0, c->stream, big_start[cur_big],
                           big_len[cur_big], big_pref[cur_big], bound, mixed, lists(0, cur_big ^ 1), out, ctr, sums,
                           (uint32_t)kPTile, ctiles, ctr + kCtrNbCopy);
        GK_TRY_HIP(c, hipGetLastError());
        cur_big ^= 1;
        return classify_counts();
    }

    // one global partition level (R-bit digits below the top hi bits) over tiles already in
    // t_start / t_count (T tiles, C chunks, nseg buckets), reading kin / vin, writing keys[out] /
    // vals[out] and the next level's digit bytes
    template <int R>
    void level_launch(int hi, int nw, const uint32_t *t_start, const uint32_t *t_count, uint64_t T,
                      const uint64_t *kin, const uint32_t *vin, int out, bool count) {
        if (count) {
            if (nd_ready)  // the previous pass wrote this level's digits
                hipLaunchKernelGGL(msd_count_nd_kernel<R>, dim3((unsigned)T), dim3(256), 0, c->stream, t_start,
                                   t_count, nd, tile_hist);
            else
                hipLaunchKernelGGL(msd_count_kernel<R>, dim3((unsigned)T), dim3(256), 0, c->stream, t_start, t_count,
                                   dig_at(B, hi, R), kin, tile_hist);
            return;
        }
        if (compact_now) {
            const int rem = B - hi - R;  // 9..40: key bits below this level's digit
            NextDigits ndg{dig_at(B, hi + R, 8), nd};
            ndg.lowmask = (uint32_t)((1ull << (rem - 8)) - 1);
            if (c79_in)  // the previous level wrote packed pairs
                hipLaunchKernelGGL((msd_pipe_kernel<kPT, kPI, R, 4, true, 0, true>), dim3(pgrid), dim3(kPT), 0,
                                   c->stream, t_start, t_count, dig_at(B, hi, R), tile_hist, kin, vin, c->keys[out],
                                   c->vals[out], (uint32_t)T, n, ndg, lo16, c79_shi);
            else
                hipLaunchKernelGGL((msd_pipe_kernel<kPT, kPI, R, 4, true>), dim3(pgrid), dim3(kPT), 0, c->stream,
                                   t_start, t_count, dig_at(B, hi, R), tile_hist, kin, vin, c->keys[out],
                                   c->vals[out], (uint32_t)T, n, ndg);
            return;
        }
        if (c79_out) {  // packed pairs for the compact level behind this one
            NextDigits ndg{dig_at(B, hi + R, nw), nd};
            ndg.out16 = lo16;
            ndg.pshi = c79_shi;
            if (p88_in) {  // reading the packed L0's output
                ndg.in8 = nd_l0;
                hipLaunchKernelGGL((msd_pipe_kernel<kPT, kPI, R, 5, true, 0, 2>), dim3(pgrid), dim3(kPT), 0, c->stream,
                                   t_start, t_count, dig_at(B, hi, R), tile_hist, kin, vin, c->keys[out], c->vals[out],
                                   (uint32_t)T, n, ndg, lo16_l0, p88_shi);
                return;
            }
            hipLaunchKernelGGL((msd_pipe_kernel<kPT, kPI, R, 5, true>), dim3(pgrid), dim3(kPT), 0, c->stream, t_start,
                               t_count, dig_at(B, hi, R), tile_hist, kin, vin, c->keys[out], c->vals[out],
                               (uint32_t)T, n, ndg);
            return;
        }
        const NextDigits ndg{dig_at(B, hi + R, nw), nd};
        if (nd_next)
            hipLaunchKernelGGL((msd_pipe_kernel<kPT, kPI, R, 0, true>), dim3(pgrid), dim3(kPT), 0, c->stream, t_start,
                               t_count, dig_at(B, hi, R), tile_hist, kin, vin, c->keys[out], c->vals[out],
                               (uint32_t)T, n, ndg);
        else
            hipLaunchKernelGGL((msd_pipe_kernel<kPT, kPI, R, 0, false>), dim3(pgrid), dim3(kPT), 0, c->stream,
                               t_start, t_count, dig_at(B, hi, R), tile_hist, kin, vin, c->keys[out], c->vals[out],
                               (uint32_t)T, n, ndg);
    }

    void level_dispatch(int level, int hi, const uint32_t *t_start, const uint32_t *t_count, uint64_t T,
                        const uint64_t *kin, const uint32_t *vin, int out, bool count) {
        const int w = width(level), nw = width(level + 1);
        if (w == 8) level_launch<8>(hi, nw, t_start, t_count, T, kin, vin, out, count);
        else if (w == 7) level_launch<7>(hi, nw, t_start, t_count, T, kin, vin, out, count);
        else level_launch<6>(hi, nw, t_start, t_count, T, kin, vin, out, count);
    }

    // the output format of a global level over nseg buckets holding elems elements (level_pass):
    //   nd_next  the next level's digit bytes are written (its sub-buckets are most likely big);
    //   compact  (low bits, start) + digit byte, 9 B out, when its sub-buckets will most likely all
    //            be finished locally and the key bits below the next 8-bit digit fit a u32;
    //   pairs    packed pairs (10 B + digit byte) when the next level is most likely compact (its
    //            sub-buckets local, its remaining bits <= 40) and this level's remaining key bits
    //            and the start fit 80 bits (GKM_TEST_PAIRS=1, tests: whenever the bits fit)
    struct LevelFormat {
        bool nd_next, compact, pairs;
    };
    LevelFormat level_format(int level, int hi, uint64_t elems, uint64_t nseg) const {
        LevelFormat f{};
        f.nd_next = nseg == 0 || (elems / nseg >> width(level)) >= (uint64_t)kBlockMax;
        const int rem = B - hi - width(level);
        f.compact = phase == 0 && !f.nd_next && rem >= 9 && rem <= 40 && width(level + 1) == 8 && !no_compact();
        const uint64_t next_mean = nseg ? (elems / nseg >> width(level)) >> width(level + 1) : 0;
        const int rem2 = rem - width(level + 1);
        const bool force = opt("GKM_TEST_PAIRS") != nullptr;  // (read per level: tests flip it)
        f.pairs = allow_c79 && !c79_in && phase == 0 && !f.compact && rem >= 33 && rem <= 48 && !no_compact() &&
                  (force || (f.nd_next && next_mean < (uint64_t)kBlockMax && rem2 >= 9 && rem2 <= 40 &&
                             width(level + 2) == 8 && width(level + 1) == 8));
        return f;
    }

    int level_pass(int level, int hi, const uint32_t *t_start, const uint32_t *t_count, uint64_t T, uint64_t C,
                   const uint32_t *s_cfirst, const uint32_t *s_nchunks, const uint32_t *s_start, uint64_t nseg,
                   const uint64_t *kin, const uint32_t *vin, int out) {
        timer_begin(c, nd_ready ? "msd_count_nd" : "msd_count", &slot);
        timer_units(c, slot, big_elems);
        level_dispatch(level, hi, t_start, t_count, T, kin, vin, out, true);
        GK_TRY_HIP(c, hipGetLastError());
        timer_end(c, slot);
        int rc = scan_offsets(width(level), C, s_cfirst, s_nchunks, s_start, nseg);
        if (rc != GK_OK) return rc;
        GK_TRY_HIP(c, scratch(c, "msd_nd", n + 64, &nd));
        // the next level's digit bytes, unless this level's sub-buckets will most likely all be
        // local (mean under kBlockMax); a next level then counts from the keys
        const LevelFormat lf = level_format(level, hi, big_elems, nseg);
        nd_next = lf.nd_next;
        compact_now = lf.compact;
        compact_hi = hi + width(level);
        c79_out = lf.pairs;
        const int rem = B - hi - width(level);
        if (c79_out) {
            c79_shi = 64 - rem;
            GK_TRY_HIP(c, scratch(c, "msd_lo16", n + 64, &lo16));
        }
        // the packed L0's output in, but no packed pairs out: back to (key, start) first
        if (p88_in && !c79_out) {
            if (pieces_level)  // (first_level_from_pieces expands its pieces itself beforehand)
                return fail(c, GK_E_HIP, "msd: packed L0 pieces reached a level that does not read them");
            if (int rc = p88_detach()) return rc;
            hipLaunchKernelGGL(expand_p88_kernel, dim3((unsigned)nseg, bucket_split(nseg)), dim3(256), 0, c->stream,
                               big_start[cur_big], big_len[cur_big], big_pref[cur_big], hi, B, p88_shi,
                               const_cast<uint64_t *>(kin), lo16_l0, nd_l0, const_cast<uint32_t *>(vin));
            GK_TRY_HIP(c, hipGetLastError());
            p88_in = false;
        }
        // packed pairs in, but not a compact level after all: back to (key, start) first
        if (c79_in && !compact_now) {
            hipLaunchKernelGGL(expand_pair_kernel, dim3((unsigned)nseg, bucket_split(nseg)), dim3(256), 0, c->stream,
                               big_start[cur_big], big_len[cur_big], big_pref[cur_big], hi, B, c79_shi,
                               const_cast<uint64_t *>(kin), lo16, const_cast<uint32_t *>(vin));
            GK_TRY_HIP(c, hipGetLastError());
            c79_in = false;
        }
        timer_begin(c, compact_now ? kPassNamesC[level & 7] : c79_out ? kPassNamesP[level & 7] : kPassNames[level & 7],
                    &slot);
        timer_units(c, slot, big_elems);
        level_dispatch(level, hi, t_start, t_count, T, kin, vin, out, false);
        GK_TRY_HIP(c, hipGetLastError());
        timer_end(c, slot);
        // a compact or packed-pair level wrote the next 8-bit digit too (the next count must not
        // read keys: pairs hold them shifted)
        nd_ready = nd_next || compact_now || c79_out;
        c79_in = c79_out;  // the next level's input format
        p88_in = false;
        return GK_OK;
    }

    // after a packed-pair level's classify: its local buckets (entries [before[k], nloc[k]) of the
    // generation-0 lists) back to (key, start) for the finishing kernels
    int expand_pair_locals(const uint64_t (&before)[kLocal], int out) {
        for (int k = 0; k < kLocal; ++k) {
            if (nloc[k] <= before[k]) continue;
            hipLaunchKernelGGL(expand_pair_list_kernel, dim3((unsigned)(nloc[k] - before[k])), dim3(256), 0,
                               c->stream, loc[k][0], loc_pref[k], (uint32_t)before[k], B, c79_shi, c->keys[out], lo16,
                               c->vals[out]);
            GK_TRY_HIP(c, hipGetLastError());
        }
        return GK_OK;
    }

    // first level from received buckets: pieces (off, len) of kin / vin, grouped by top-kGR-bit
    // bucket in ascending bucket order, pieces of a bucket in the order their elements must keep
    // level / hi: the level the pieces are partitioned at and the key bits already sorted (the
    // exchange's pieces: level 1 after kGR bits; the key-range select's chunks: level 0, no bits)
    int first_level_from_pieces(const uint64_t *kin, const uint32_t *vin, const uint64_t *poff, const uint64_t *plen,
                                const uint32_t *pbucket, uint32_t np, int level = 1, int hi = kGR) {
        std::vector<uint32_t> ts, tc, cf, cn, scf, snc, sst;
        std::vector<uint64_t> spf;  // the buckets' prefixes: their top-hi-bit values
        uint64_t out_base = 0;
        for (uint32_t i = 0; i < np;) {
            uint32_t j = i;
            uint64_t tot = 0;
            const uint64_t tile0 = ts.size();
            while (j < np && pbucket[j] == pbucket[i]) {
                for (uint64_t o = 0; o < plen[j]; o += kPTile) {
                    ts.push_back((uint32_t)(poff[j] + o));
                    tc.push_back((uint32_t)std::min<uint64_t>(kPTile, plen[j] - o));
                }
                tot += plen[j];
                ++j;
            }
            if (tot > 0) {
                const uint64_t nt = ts.size() - tile0;
                scf.push_back((uint32_t)cf.size());
                for (uint64_t t = 0; t < nt; t += ctiles) {
                    cf.push_back((uint32_t)(tile0 + t));
                    cn.push_back((uint32_t)std::min<uint64_t>(ctiles, nt - t));
                }
                snc.push_back((uint32_t)(cf.size() - scf.back()));
                sst.push_back((uint32_t)out_base);
                spf.push_back(pbucket[i]);
                out_base += tot;
            }
            i = j;
        }
        if (out_base != n) return fail(c, GK_E_ARG, "piece lengths do not add up to n");
        const uint64_t T = ts.size(), C = cf.size(), nseg = sst.size();
        if (nseg == 0) return GK_OK;
        int rc = tables(T, C, nseg);
        if (rc != GK_OK) return rc;
        uint32_t *t_start, *t_count, *s_cfirst, *s_nchunks, *s_st;
        GK_TRY_HIP(c, scratch(c, "t_start", T, &t_start));
        GK_TRY_HIP(c, scratch(c, "t_count", T, &t_count));
        GK_TRY_HIP(c, scratch(c, "s_cfirst", nseg, &s_cfirst));
        GK_TRY_HIP(c, scratch(c, "s_nchunks", nseg, &s_nchunks));
        GK_TRY_HIP(c, scratch(c, "s_pstart", nseg, &s_st));
        GK_TRY_HIP(c, hipMemcpyAsync(t_start, ts.data(), 4 * T, hipMemcpyHostToDevice, c->stream));
        GK_TRY_HIP(c, hipMemcpyAsync(t_count, tc.data(), 4 * T, hipMemcpyHostToDevice, c->stream));
        GK_TRY_HIP(c, hipMemcpyAsync(c_first, cf.data(), 4 * C, hipMemcpyHostToDevice, c->stream));
        GK_TRY_HIP(c, hipMemcpyAsync(c_ntiles, cn.data(), 4 * C, hipMemcpyHostToDevice, c->stream));
        GK_TRY_HIP(c, hipMemcpyAsync(s_cfirst, scf.data(), 4 * nseg, hipMemcpyHostToDevice, c->stream));
        GK_TRY_HIP(c, hipMemcpyAsync(s_nchunks, snc.data(), 4 * nseg, hipMemcpyHostToDevice, c->stream));
        GK_TRY_HIP(c, hipMemcpyAsync(s_st, sst.data(), 4 * nseg, hipMemcpyHostToDevice, c->stream));
        uint64_t *s_pref;
        GK_TRY_HIP(c, scratch(c, "s_ppref", nseg, &s_pref));
        GK_TRY_HIP(c, hipMemcpyAsync(s_pref, spf.data(), 8 * nseg, hipMemcpyHostToDevice, c->stream));
        GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
        big_elems = n;
        if (p88_in && !level_format(level, hi, n, nseg).pairs) {  // (prefetched packed L0: back to (key, start))
            if (int rd = p88_detach()) return rd;
            uint64_t *pdev;
            GK_TRY_HIP(c, scratch(c, "p88_pieces", 3 * np, &pdev));
            std::vector<uint64_t> hp(3 * (uint64_t)np);
            for (uint32_t j = 0; j < np; ++j) {
                hp[j] = poff[j];
                hp[np + j] = plen[j];
                hp[2 * (uint64_t)np + j] = pbucket[j];
            }
            GK_TRY_HIP(c, hipMemcpyAsync(pdev, hp.data(), 8 * hp.size(), hipMemcpyHostToDevice, c->stream));
            hipLaunchKernelGGL(expand_p88_pieces_kernel, dim3(np, bucket_split(np)), dim3(256), 0, c->stream, pdev,
                               np, hi, B, p88_shi, const_cast<uint64_t *>(kin), lo16_l0, nd_l0,
                               const_cast<uint32_t *>(vin));
            GK_TRY_HIP(c, hipGetLastError());
            GK_TRY_HIP(c, hipStreamSynchronize(c->stream));  // (hp is released at return)
            p88_in = false;
        }
        pieces_level = true;
        rc = level_pass(level, hi, t_start, t_count, T, C, s_cfirst, s_nchunks, s_st, nseg, kin, vin, 0);
        pieces_level = false;
        if (rc != GK_OK) return rc;
        cur_big = 0;
        uint64_t before[kLocal];
        for (int k = 0; k < kLocal; ++k) before[k] = nloc[k];
        rc = classify(nseg << width(level), hi + width(level), 0, cur_big, nullptr, nullptr, 1, s_pref, width(level),
                      compact_now ? 1 : 0);
        // (as levels(): a packed-pair level's local sub-buckets back to (key, start))
        if (rc == GK_OK && c79_out) rc = expand_pair_locals(before, 0);
        return rc == GK_OK ? expand_big(0) : rc;
    }

    // Multi-word keys, phase > 0: the head flags of the order so far (buffer 0) mark the groups of
    // equal earlier words; sort each group of >= 2 by the key word of symbols [sym0, sym0 + nsym).
    int next_phase(int sym0, int nsym) {
        uint32_t *g_start, *g_len;
        timer_begin(c, "msd_tie_groups", &slot);
        const unsigned ttiles = (unsigned)std::max<uint64_t>((n + kTieTile - 1) / kTieTile, 1);
        uint32_t *cf, *cl, *of, *ol;
        GK_TRY_HIP(c, scratch(c, "tie_cnt_f", ttiles + 1, &cf));
        GK_TRY_HIP(c, scratch(c, "tie_cnt_l", ttiles + 1, &cl));
        GK_TRY_HIP(c, scratch(c, "tie_off_f", ttiles + 1, &of));
        GK_TRY_HIP(c, scratch(c, "tie_off_l", ttiles + 1, &ol));
        hipLaunchKernelGGL(tie_bounds_kernel<false>, dim3(ttiles), dim3(256), 0, c->stream, heads, n, cf, cl, nullptr,
                           nullptr, nullptr, nullptr);
        GK_TRY_HIP(c, hipGetLastError());
        uint64_t ng = 0, ng2 = 0;
        GK_TRY_HIP(c, scan_u32_exclusive_pair(c, cf, of, cl, ol, ttiles, &ng, &ng2));
        GK_TRY_HIP(c, scratch(c, "tie_start", ng + 64, &g_start));
        GK_TRY_HIP(c, scratch(c, "tie_len", ng2 + 64, &g_len));
        hipLaunchKernelGGL(tie_bounds_kernel<true>, dim3(ttiles), dim3(256), 0, c->stream, heads, n, nullptr, nullptr,
                           of, ol, g_start, g_len);
        GK_TRY_HIP(c, hipGetLastError());
        if (ng != ng2) return fail(c, GK_E_HIP, "msd: tie group bounds do not pair up");
        if (ng > 0)
            hipLaunchKernelGGL(tie_run_lengths_kernel, dim3((unsigned)std::min<uint64_t>((ng + 255) / 256, 8192)),
                               dim3(256), 0, c->stream, g_start, g_len, ng);
        GK_TRY_HIP(c, hipGetLastError());
        timer_end(c, slot);
        if (ng == 0) return GK_OK;
        timer_begin(c, "msd_tie_encode", &slot);
        const unsigned grid = (unsigned)std::min<uint64_t>((ng + 3) / 4, (uint64_t)cus * 16);
        bool flat = ng > 4096;
        if (!flat) {  // few groups: flat too if they are large (one wave per group would be serial)
            std::vector<uint32_t> lens(ng);
            GK_TRY_HIP(c, hipMemcpyAsync(lens.data(), g_len, 4 * ng, hipMemcpyDeviceToHost, c->stream));
            GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
            uint64_t tot = 0;
            for (uint32_t v : lens) tot += v;
            flat = tot > (1u << 20);
        }
        if (flat) {  // many groups: the members listed from the head flags, then one thread per member
            uint32_t *mlist;
            // the list lives in the free key buffer (8 B per element; classify and the levels below
            // reuse it only after the encode has read the list)
            mlist = reinterpret_cast<uint32_t *>(c->keys[1]);
            hipLaunchKernelGGL(tie_members_kernel<false>, dim3(ttiles), dim3(256), 0, c->stream, heads, n, cf, nullptr,
                               nullptr);
            GK_TRY_HIP(c, hipGetLastError());
            uint64_t nm = 0;
            GK_TRY_HIP(c, scan_u32_exclusive_pub(c, cf, ttiles, of, &nm));
            hipLaunchKernelGGL(tie_members_kernel<true>, dim3(ttiles), dim3(256), 0, c->stream, heads, n, nullptr, of,
                               mlist);
            GK_TRY_HIP(c, hipGetLastError());
            const unsigned eg = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((nm + 255) / 256, (uint64_t)cus * 16));
            if (ks.bits == 2)
                hipLaunchKernelGGL(tie_encode_list_kernel<2>, dim3(eg), dim3(256), 0, c->stream, c->sba, mlist, (uint32_t)nm,
                                   c->vals[0], c->keys[0], sym0, nsym, ks.symbols, ks.canonical);
            else
                hipLaunchKernelGGL(tie_encode_list_kernel<4>, dim3(eg), dim3(256), 0, c->stream, c->sba, mlist, (uint32_t)nm,
                                   c->vals[0], c->keys[0], sym0, nsym, ks.symbols, ks.canonical);
        } else if (ks.bits == 2)
            hipLaunchKernelGGL(tie_encode_kernel<2>, dim3(grid), dim3(256), 0, c->stream, c->sba, g_start, g_len,
                               (uint32_t)ng, c->vals[0], c->keys[0], sym0, nsym, ks.symbols, ks.canonical);
        else
            hipLaunchKernelGGL(tie_encode_kernel<4>, dim3(grid), dim3(256), 0, c->stream, c->sba, g_start, g_len,
                               (uint32_t)ng, c->vals[0], c->keys[0], sym0, nsym, ks.symbols, ks.canonical);
        GK_TRY_HIP(c, hipGetLastError());
        timer_end(c, slot);
        B = ks.bits * nsym;
        ++phase;
        GK_TRY_HIP(c, hipMemsetAsync(ctr, 0, 4 * kCtrN, c->stream));
        ndone = 0;
        nbig = 0;
        for (int k = 0; k < kLocal; ++k) nloc[k] = loc_elems[k] = 0;
        nd_ready = false;
        c79_in = false;
        int rc = classify(ng, 0, 0, cur_big, g_start, g_len, 2);
        if (rc != GK_OK) return rc;
        rc = levels(1, 0, 0);
        if (rc != GK_OK) return rc;
        return finish();
    }

    // Prefix doubling (gkm_capi.hip sort_doubling): every run of >= 2 elements of keys[0] / vals[0]
    // that `flags` marks as one group (a 1 starts a group) sorted stably by the bkey-bit keys, in
    // place; the members' group heads in c->heads.  Elements outside those groups stay where they
    // are, so a round costs in proportion to the elements still tied, not to n.
    int sort_groups(const uint8_t *flags, int bkey) {
        uint32_t *g_start, *g_len;
        const unsigned ttiles = (unsigned)std::max<uint64_t>((n + kTieTile - 1) / kTieTile, 1);
        uint32_t *cf, *cl, *of, *ol;
        GK_TRY_HIP(c, scratch(c, "tie_cnt_f", ttiles + 1, &cf));
        GK_TRY_HIP(c, scratch(c, "tie_cnt_l", ttiles + 1, &cl));
        GK_TRY_HIP(c, scratch(c, "tie_off_f", ttiles + 1, &of));
        GK_TRY_HIP(c, scratch(c, "tie_off_l", ttiles + 1, &ol));
        hipLaunchKernelGGL(tie_bounds_kernel<false>, dim3(ttiles), dim3(256), 0, c->stream, flags, n, cf, cl, nullptr,
                           nullptr, nullptr, nullptr);
        GK_TRY_HIP(c, hipGetLastError());
        uint64_t ng = 0, ng2 = 0;
        GK_TRY_HIP(c, scan_u32_exclusive_pair(c, cf, of, cl, ol, ttiles, &ng, &ng2));
        if (ng != ng2) return fail(c, GK_E_HIP, "msd: tie group bounds do not pair up");
        if (ng == 0) return GK_OK;
        GK_TRY_HIP(c, scratch(c, "tie_start", ng + 64, &g_start));
        GK_TRY_HIP(c, scratch(c, "tie_len", ng + 64, &g_len));
        hipLaunchKernelGGL(tie_bounds_kernel<true>, dim3(ttiles), dim3(256), 0, c->stream, flags, n, nullptr, nullptr,
                           of, ol, g_start, g_len);
        GK_TRY_HIP(c, hipGetLastError());
        hipLaunchKernelGGL(tie_run_lengths_kernel, dim3((unsigned)std::min<uint64_t>((ng + 255) / 256, 8192)),
                           dim3(256), 0, c->stream, g_start, g_len, ng);
        GK_TRY_HIP(c, hipGetLastError());
        B = bkey;
        phase = 1;  // (no compact or packed-pair levels: later-phase rules)
        nd_ready = false;
        c79_in = false;
        int rc = classify(ng, 0, 0, cur_big, g_start, g_len, 2);
        if (rc != GK_OK) return rc;
        rc = levels(1, 0, 0);
        if (rc != GK_OK) return rc;
        return finish();
    }

    // before another global level: its buckets whose keys are all equal go to the done list
    // (checked once the big buckets hold few elements: after L1 of a random genome they hold
    // all of them and never are)
    int drop_uniform(int level, int out) {
        if (nbig == 0 || level < 1 || big_elems * 64 > std::max<uint64_t>(c->n, 1)) return GK_OK;
        uint32_t *mixed;
        GK_TRY_HIP(c, scratch(c, "uni_mixed", nbig, &mixed));
        GK_TRY_HIP(c, hipMemsetAsync(mixed, 0, 4ull * nbig, c->stream));
        hipLaunchKernelGGL(uniform_flag_kernel, dim3(nbig, bucket_split(nbig)), dim3(256), 0, c->stream,
                           big_start[cur_big], big_len[cur_big], c->keys[out], mixed);
        GK_TRY_HIP(c, grow_keep(c, "dn_start", ndone + nbig, ndone, &dn_start));
        GK_TRY_HIP(c, grow_keep(c, "dn_len", ndone + nbig, ndone, &dn_len));
        GK_TRY_HIP(c, grow_keep(c, "dn_par", ndone + nbig, ndone, &dn_par));
        GK_TRY_HIP(c, hipMemsetAsync(ctr + kCtrBig, 0, 4, c->stream));
        GK_TRY_HIP(c, hipMemsetAsync(sums + kCtrBig, 0, 8, c->stream));
        GK_TRY_HIP(c, hipMemsetAsync(sums + kSumTiles, 0, 16, c->stream));
        hipLaunchKernelGGL(route_uniform_kernel, dim3(grid_n(nbig)), dim3(256), 0, c->stream, big_start[cur_big],
                           big_len[cur_big], big_pref[cur_big], nbig, mixed, lists(0, cur_big ^ 1), out, ctr, sums,
                           (uint32_t)kPTile, ctiles);
        GK_TRY_HIP(c, hipGetLastError());
        cur_big ^= 1;
        int r = read_ctr();
        if (r != GK_OK) return r;
        ndone = h[kCtrDone];
        nbig = h[kCtrBig];
        big_elems = hs[kCtrBig];
        return GK_OK;
    }

    // global levels while the next-level list is non-empty; `in` holds the current buffer, hi
    // key bits are sorted
    // (c79_in carries over: a first level from pieces may have written packed pairs)
    int levels(int level, int hi, int in) {
        while (nbig > 0) {
            const int out = in ^ 1;
            uint32_t *ntl, *nch, *tfirst, *cfirst;
            GK_TRY_HIP(c, scratch(c, "s_ntiles", nbig, &ntl));
            GK_TRY_HIP(c, scratch(c, "s_nchunks", nbig, &nch));
            GK_TRY_HIP(c, scratch(c, "s_tfirst", nbig, &tfirst));
            GK_TRY_HIP(c, scratch(c, "s_cfirst", nbig, &cfirst));
            // the tile / chunk totals came with the list counters (classify, route_uniform)
            const uint64_t T = hs[kSumTiles], C = hs[kSumChunks];
            if (nbig <= kSegScanMax && !opt("GKM_TEST_SEG_SCAN_MULTI")) {
                hipLaunchKernelGGL(seg_tiles_scan_kernel, dim3(1), dim3(1024), 0, c->stream, big_len[cur_big], nbig,
                                   (uint32_t)kPTile, ctiles, tfirst, cfirst, nch);
                GK_TRY_HIP(c, hipGetLastError());
            } else {
                hipLaunchKernelGGL(seg_counts_kernel, dim3(grid_n(nbig)), dim3(256), 0, c->stream, big_len[cur_big],
                                   nbig, (uint32_t)kPTile, ctiles, ntl, nch);
                GK_TRY_HIP(c, hipGetLastError());
                GK_TRY_HIP(c, scan_u32_exclusive_pair_launch(c, ntl, tfirst, nch, cfirst, nbig));
            }
            if (opt("GKM_TEST_CHECK_TILES")) {  // (tests: the totals against the scans' own)
                uint32_t last[4];
                GK_TRY_HIP(c, hipMemcpyAsync(&last[0], tfirst + nbig - 1, 4, hipMemcpyDeviceToHost, c->stream));
                GK_TRY_HIP(c, hipMemcpyAsync(&last[1], cfirst + nbig - 1, 4, hipMemcpyDeviceToHost, c->stream));
                GK_TRY_HIP(c, hipMemcpyAsync(&last[2], nch + nbig - 1, 4, hipMemcpyDeviceToHost, c->stream));
                GK_TRY_HIP(c, hipMemcpyAsync(&last[3], big_len[cur_big] + nbig - 1, 4, hipMemcpyDeviceToHost, c->stream));
                GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
                if (last[0] + tiles_of(last[3], (uint32_t)kPTile) != T || last[1] + last[2] != C)
                    return fail(c, GK_E_HIP, "msd: level tile totals disagree with the bucket scan");
            }
            uint32_t *t_start, *t_count;
            GK_TRY_HIP(c, scratch(c, "t_start", T, &t_start));
            GK_TRY_HIP(c, scratch(c, "t_count", T, &t_count));
            int rc = tables(T, C, nbig);
            if (rc != GK_OK) return rc;
            hipLaunchKernelGGL(tile_table_kernel, dim3((unsigned)std::max<uint64_t>((std::max(T, C) + 255) / 256, 1)), dim3(256), 0,
                               c->stream, big_start[cur_big], big_len[cur_big], tfirst, cfirst, nbig,
                               (uint32_t)kPTile, (uint32_t)T, (uint32_t)C, ctiles, t_start, t_count, c_first, c_ntiles);
            const uint64_t in_big = big_elems;
            rc = level_pass(level, hi, t_start, t_count, T, C, cfirst, nch, big_start[cur_big], nbig, c->keys[in],
                            c->vals[in], out);
            if (rc != GK_OK) return rc;
            cur_big ^= 1;
            uint64_t before[kLocal];
            for (int k = 0; k < kLocal; ++k) before[k] = nloc[k];
            const uint64_t nsub = (uint64_t)nbig << width(level);
            // the level's input already small: its output's uniform buckets are dropped behind
            // the classify with one read-back for both (drop_uniform's rule, on the input's size)
            const bool fuse = !c79_out && level >= 1 && in_big * 64 <= std::max<uint64_t>(c->n, 1) &&
                              !opt("GKM_NO_FUSED_UNIFORM");
            rc = classify(nsub, hi + width(level), out, cur_big, nullptr, nullptr, 1, big_pref[cur_big ^ 1],
                          width(level), compact_now ? 1 : 0, !fuse);
            if (fuse) {
                const uint64_t bound = std::min<uint64_t>(nsub, in_big / ((uint64_t)kBlockMax + 1));
                if (rc == GK_OK) rc = bound ? drop_uniform_dev(out, (uint32_t)bound) : classify_counts();
            } else {
                if (rc == GK_OK && c79_out) rc = expand_pair_locals(before, out);
                if (rc == GK_OK) rc = expand_big(out);
                if (rc == GK_OK && !c79_out) rc = drop_uniform(level, out);  // (pairs: keys not comparable)
            }
            if (rc != GK_OK) return rc;
            ++level;
            hi += width(level - 1);
            in = out;
        }
        return GK_OK;
    }

    // one local class's kernel over a list of cnt buckets
    void local_launch(int k, uint32_t cnt, const uint2 *lst, uint64_t *k0, uint32_t *v0, const uint64_t *k1,
                      const uint32_t *v1, const Lists &nl, const Lists *d_nl, int round) {
        // common-prefix skip: re-listed buckets, later phases (repeats) and the block class; not
        // the first wave round of phase 0, where random keys differ right below the sorted bits
        const int skip = (round > 0 || phase > 0 || k == 3) ? 1 : 0;
        const uint32_t small = (round > 0 || phase > 0) ? kSmallLate : kSmall;
        // round 0 reads classify's entries, some of which may hold compact elements
        const CompactIn ci{round == 0 ? loc_pref[k] : nullptr, nd};
        // persistent grids of the workgroups that fit at once (occupancy API, per kernel)
        auto grid = [&](const void *fn, int threads) {
            int per_cu = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, threads, 0) != hipSuccess || per_cu < 1)
                per_cu = 1;
            uint64_t g = std::min<uint64_t>(cnt, (uint64_t)cus * per_cu);
            if (g >= 8) g = xcd_walk_off() ? g - ((g & 7) == 0) : (g & ~7ull);  // the wave kernels' XCD-aware walk
            return dim3((unsigned)g);
        };
        // wave classes: msd_wave_kernel<I, waves per SIMD, keys written>
        auto wave = [&](auto fn_wk, auto fn_nk) {
            const void *fn = wkeys ? (const void *)fn_wk : (const void *)fn_nk;
            if (wkeys)
                hipLaunchKernelGGL(fn_wk, grid(fn, 64), dim3(64), 0, c->stream, lst, cnt, B, k0, v0, k1, v1, heads,
                                   d_nl, ctr, skip, small, ci.pref, ci.nd);
            else
                hipLaunchKernelGGL(fn_nk, grid(fn, 64), dim3(64), 0, c->stream, lst, cnt, B, k0, v0, k1, v1, heads,
                                   d_nl, ctr, skip, small, ci.pref, ci.nd);
        };
        switch (k) {
        case 0:
            wave(msd_wave_kernel<4, kWaveOcc4, true, kWaveR4>, msd_wave_kernel<4, kWaveOcc4, false, kWaveR4>);
            break;
        case 1:
            if (exp_wave_copy() && exp_opt("GKM_EXP_WAVECOPY")[0] == '2') {  // timing only
                hipLaunchKernelGGL((msd_wave_copy2_kernel<8, kWaveOcc8>),
                                   grid((const void *)msd_wave_copy2_kernel<8, kWaveOcc8>, 64), dim3(64), 0,
                                   c->stream, lst, cnt, B, k0, v0, k1, v1, heads, ci.pref, ci.nd);
                break;
            }
            if (exp_wave_copy() && exp_opt("GKM_EXP_WAVECOPY")[0] == '3') {  // timing only
                hipLaunchKernelGGL((msd_wave_copy_kernel<8, kWaveOcc8, 1>),
                                   grid((const void *)msd_wave_copy_kernel<8, kWaveOcc8, 1>, 64), dim3(64), 0,
                                   c->stream, lst, cnt, B, k0, v0, k1, v1, heads, ci.pref, ci.nd);
                break;
            }
            if (exp_wave_copy() && exp_opt("GKM_EXP_WAVECOPY")[0] == '4') {  // timing only
                hipLaunchKernelGGL((msd_wave_copy_kernel<8, kWaveOcc8, 2>),
                                   grid((const void *)msd_wave_copy_kernel<8, kWaveOcc8, 2>, 64), dim3(64), 0,
                                   c->stream, lst, cnt, B, k0, v0, k1, v1, heads, ci.pref, ci.nd);
                break;
            }
            if (exp_wave_copy() && exp_opt("GKM_EXP_WAVECOPY")[0] == '5') {  // timing only
                hipLaunchKernelGGL(stream_copy_kernel, dim3(cus * 8), dim3(256), 0, c->stream, n, k1, nd, k0, v0, heads);
                break;
            }
            if (exp_wave_copy()) {  // timing experiments only: wrong output
                hipLaunchKernelGGL((msd_wave_copy_kernel<8, kWaveOcc8>),
                                   grid((const void *)msd_wave_copy_kernel<8, kWaveOcc8>, 64), dim3(64), 0,
                                   c->stream, lst, cnt, B, k0, v0, k1, v1, heads, ci.pref, ci.nd);
                break;
            }
            wave(msd_wave_kernel<8, kWaveOcc8, true, kWaveR8>, msd_wave_kernel<8, kWaveOcc8, false, kWaveR8>);
            break;
        case 2:
            wave(msd_wave_kernel<16, kWaveOcc16, true, kWaveR16>, msd_wave_kernel<16, kWaveOcc16, false, kWaveR16>);
            break;
        case 3:
            hipLaunchKernelGGL((msd_local_kernel<kBT, kBI, kBR>),
                               grid((const void *)msd_local_kernel<kBT, kBI, kBR>, kBT), dim3(kBT), 0, c->stream, lst,
                               cnt, B, k0, v0, k1, v1, heads, nl, ctr, skip,
                               (uint32_t)kSmall, wkeys, ci);  // the block class keeps kSmall: 96 measured slower (A/B)
            break;
        case 5: {
            // (A/B: GKM_BLOCK32_T512=1 -- 512 threads x 16 keys: half the per-wave counters to
            // zero and scan per bucket, half the waves)
            static const bool t512 = opt("GKM_BLOCK32_T512") != nullptr;
            if (t512)
                hipLaunchKernelGGL((msd_local_kernel<kBT, 2 * kBI, kBR2>),
                                   grid((const void *)msd_local_kernel<kBT, 2 * kBI, kBR2>, kBT), dim3(kBT), 0,
                                   c->stream, lst, cnt, B, k0, v0, k1, v1, heads, nl, ctr, skip, (uint32_t)kSmall,
                                   wkeys, ci);
            else
                hipLaunchKernelGGL((msd_local_kernel<kBT2, kBI, kBR2>),
                                   grid((const void *)msd_local_kernel<kBT2, kBI, kBR2>, kBT2), dim3(kBT2), 0,
                                   c->stream, lst, cnt, B, k0, v0, k1, v1, heads, nl, ctr, skip, (uint32_t)kSmall,
                                   wkeys, ci);
            break;
        }
        default:
            hipLaunchKernelGGL(msd_tiny_kernel, dim3((cnt + 255) / 256), dim3(256), 0, c->stream, lst, cnt, k0, v0, k1,
                               v1, heads, wkeys, ci, B);
        }
    }

    // local rounds (generation g lists -> re-listed sub-buckets in generation g ^ 1), done copies.
    int finish() {
        const uint64_t max_spill = n / (kSmall + 1) + 1024;
        uint64_t pending = 0;
        for (int k = 0; k < kLocal; ++k) {
            GK_TRY_HIP(c, grow_keep(c, kLocName[k][0], std::max<uint64_t>(nloc[k], max_spill), nloc[k], &loc[k][0]));
            GK_TRY_HIP(c, grow_keep(c, kLocName[k][1], max_spill, 0, &loc[k][1]));
            pending += nloc[k];
        }
        GK_TRY_HIP(c, grow_keep(c, "dn_start", ndone + max_spill, ndone, &dn_start));
        GK_TRY_HIP(c, grow_keep(c, "dn_len", ndone + max_spill, ndone, &dn_len));
        GK_TRY_HIP(c, grow_keep(c, "dn_par", ndone + max_spill, ndone, &dn_par));
        int g = 0, round = 0;
        while (pending > 0) {
            const int ng = g ^ 1;
            // the re-list counters of this round start from 0 (the done count carries on)
            GK_TRY_HIP(c, hipMemsetAsync(ctr + kCtrLoc, 0, 4 * kLocal, c->stream));
            const Lists nl = lists(ng, 0);
            Lists *d_nl = nullptr;
            GK_TRY_HIP(c, scratch(c, "lists_dev", 1, &d_nl));
            hipLaunchKernelGGL(lists_store_kernel, dim3(1), dim3(1), 0, c->stream, nl, d_nl);
            GK_TRY_HIP(c, hipGetLastError());
            for (int k = 0; k < kLocal; ++k) {
                if (!nloc[k]) continue;
                timer_begin(c, round == 0 ? kLocTimer[k][0] : kLocTimer[k][1], &slot);
                if (round == 0) timer_units(c, slot, loc_elems[k]);
                const uint32_t cnt = (uint32_t)nloc[k];
                uint64_t *k0 = c->keys[0], *k1 = c->keys[1];
                uint32_t *v0 = c->vals[0], *v1 = c->vals[1];
                const uint2 *lst = loc[k][g];
                static const bool trace = opt("GKM_MSD_TRACE") != nullptr;
                hipEvent_t t0 = nullptr, t1 = nullptr;
                if (trace) {
                    hipEventCreate(&t0);
                    hipEventCreate(&t1);
                    hipEventRecord(t0, c->stream);
                }
                local_launch(k, cnt, lst, k0, v0, k1, v1, nl, d_nl, round);
                GK_TRY_HIP(c, hipGetLastError());
                timer_end(c, slot);
                if (trace) {  // diagnostics: one line per local launch
                    hipEventRecord(t1, c->stream);
                    hipEventSynchronize(t1);
                    float ms = 0;
                    hipEventElapsedTime(&ms, t0, t1);
                    std::fprintf(stderr, "[msd] phase %d round %d class %d buckets %u: %.3f ms\n", phase, round, k,
                                 cnt, ms);
                    hipEventDestroy(t0);
                    hipEventDestroy(t1);
                }
            }
            int rc = read_ctr();
            if (rc != GK_OK) return rc;
            pending = 0;
            for (int k = 0; k < kLocal; ++k) {
                nloc[k] = h[kCtrLoc + k];
                pending += nloc[k];
            }
            ndone = h[kCtrDone];
            g = ng;
            if (++round > 64) return fail(c, GK_E_HIP, "msd local rounds did not converge");
        }
        if (ndone > 0) {
            hipLaunchKernelGGL(done_copy_kernel, dim3((unsigned)ndone, bucket_split(ndone)), dim3(256), 0, c->stream,
                               dn_start, dn_len,
                               dn_par, c->vals[1], c->vals[0], wkeys ? c->keys[1] : nullptr, c->keys[0], heads);
            GK_TRY_HIP(c, hipGetLastError());
        }
        c->heads = heads;
        c->heads_valid = true;
        c->cur = 0;
        return GK_OK;
    }
};

// The enumerated k-mers of the whole sequence (gk_sort's fixed-length path, k <= 64).  Keys of
// more than 64 bits are sorted in phases of one word (64 / bits symbols): phase 0 sorts every
// k-mer by its first word, each later phase sorts the groups of equal earlier words by the next.
int msd_sort(gk_ctx *c, const KeySpec &ks) {
    const int spw = 64 / ks.bits;
    const int nphase = (ks.symbols + spw - 1) / spw;
    MsdDriver d(c, ks);
    d.B = ks.bits * std::min(ks.symbols, spw);
    if (nphase == 1) d.enable_wide_l0();
    // canonical 2-bit keys with a full 64-bit first word (k >= 32; C5): an 8-bit L0 leaves 48 bits
    // behind the next level -- packed pairs there and a compact level after them, which the 7-bit
    // L0's 49 and 41 bits do not allow (C5 219-221 -> 216.7-216.9 ms, profiles/r4/l08_ab.txt; the
    // same change made C4, 62-bit keys, 5 ms slower)
    if (ks.bits == 2 && ks.canonical && d.B == 64 && !opt("GKM_LEVEL_BITS")) d.wsched[0] = 8;
    d.allow_c79 = opt("GKM_NO_PAIRS") == nullptr;
    d.wkeys = (nphase == 1 && (!ks.acgt_only || c->msd_force_keys)) ? 1 : 0;  // one-word keys end final in keys[0]
    c->msd_keys_final = d.wkeys != 0;
    timer_begin(c, "msd_total", &d.total_slot);
    int rc = d.init(c->n);
    if (rc != GK_OK) return rc;
    if (use_pack() && c->acgt && ks.bits == 2 && !ks.acgt_only) {  // both L0 passes read the packed sequence
        rc = pack_sequence(c, &d.pk_code, &d.pk_dol);
        if (rc != GK_OK) return rc;
        c->pk_fresh = false;
    } else if (c->res_pk && ks.bits == 2 && (c->acgt || ks.acgt_only)) {
        // the packed copy the transfer left beside the sba (gkm_xfer.hip): both L0 passes read 0.37 B
        // per position instead of packing the bytes in every tile.  Its stops are the non-ACGT bytes:
        // '$' on an ACGT sba, every byte that ends the ACGT-only k-mers of a mixed one (class A)
        d.pk_code = c->res_code;
        d.pk_dol = c->res_dol;
    }
    uint64_t found = 0;
    // the packed L0 output (P88) when the level behind it writes packed pairs
    d.p88 = d.p88_wanted();  // (multi-word keys: phase 0's first word; the tie phases read keys[0] / vals[0])
    d.p88_shi = 64 - (d.B - d.width(0) - 8);
    // The L0's output buffer: the one that makes the last global level write buffer 1, so that the
    // finishing kernels read buffer 1 and write buffer 0 instead of rewriting buffer 0 in place
    // (levels predicted from the mean bucket size; C3: L0, L1, L2 -> L0 writes buffer 1).  A/B on
    // one box (C3, 3 pairs): 67.3-68.3 against 67.7-68.8 ms.  GKM_L0_BUF=0/1 forces it.
    int l0b = 0;
    {
        uint64_t mean = c->n >> d.width(0);
        int lev = 0;
        for (int l = 1; mean > (uint64_t)kBlockMax && l < kMaxLevels; ++l, ++lev) mean >>= d.width(l);
        l0b = 1 ^ (lev & 1);
        if (const char *e = opt("GKM_L0_BUF")) l0b = std::atoi(e) & 1;
    }
    rc = d.run_l0(0, c->sba_len, c->keys[l0b], c->vals[l0b], c->elem_cap + 64, &found);
    if (rc != GK_OK) return rc;
    if (found != c->n) return fail(c, GK_E_HIP, "msd: k-mer count differs from the enumeration");
    rc = d.classify(1u << d.width(0), d.width(0), l0b, 0, nullptr, nullptr, 1, nullptr, d.width(0));
    if (rc != GK_OK) return rc;
    if (d.p88_in) rc = d.expand_p88_locals(l0b);  // (skewed genomes: L0 buckets finished locally)
    if (rc != GK_OK) return rc;
    rc = d.levels(1, d.width(0), l0b);
    if (rc != GK_OK) return rc;
    rc = d.finish();
    for (int ph = 1; ph < nphase && rc == GK_OK; ++ph)
        rc = d.next_phase(ph * spw, std::min(spw, ks.symbols - ph * spw));
    timer_end(c, d.total_slot);
    return rc;
}

// ---------------------------------------------------------------------------------------------
// Prefetched L0 (gk_sort_hint).  The end-to-end interval of a sort -- the sequence in host memory
// to the sorted product in HBM -- is the packed transfer (host-bound: ~20 ms for 3.1 Gb) followed
// by the sort, whose first pass (L0 count + partition, ~14 ms at C3) needs only the sequence.  With
// a hint, gk_set_sequence runs that pass while the sequence streams in: the k-mer starts [0, n) of
// an ACGT sba (any number of contigs: the '$' separators are stops of the L0 pass, round 6) are cut
// into regions of whole L0 tiles of positions; as soon as the transfer has
// unpacked a region's bytes (and its last tile's halo) on the context's stream, the region is
// counted, scanned and partitioned on the prefetch stream into keys[1] / vals[1] / the digit bytes
// at output indices from its first position (MsdDriver::l0_region), and its 2^w0 buckets become
// pieces.  gk_sort(k) then starts at the first level from those pieces (msd_sort_prefetched, the
// key-range shards' first_level_from_pieces) -- the same stable order: a bucket's pieces are taken
// in region order, i.e. start order.  Any other use of the buffers drops the prefetch (pre_drop).
// ---------------------------------------------------------------------------------------------
struct L0Prefetch {
    KeySpec ks{};
    uint64_t len = 0, n = 0;        // sba bytes, k-mer starts
    uint32_t nreg = 0, tpr = 0;     // regions, L0 tiles of the largest region
    uint32_t nc_max = 0, next = 0;  // chunk-table entries per region; next region to launch
    int w0 = 7, w1 = 8;
    bool p88 = false;               // the packed L0 output (MsdDriver::p88_wanted for n)
    int p88_shi = 0;
    uint32_t *tab = nullptr;        // per region: c_first[nc_max], c_ntiles[nc_max], misc[4]
    uint32_t *pieces = nullptr;     // per region: 2^w0 bases, then 2^w0 counts
    std::vector<uint64_t> first;    // first L0 tile of each region (+ the end)
    uint64_t lo(uint32_t r) const { return first[r] * kP0Tile; }
    uint64_t hi(uint32_t r) const { return std::min<uint64_t>(first[r + 1] * kP0Tile, n); }
    uint32_t tiles(uint32_t r) const { return (uint32_t)((hi(r) - lo(r) + kP0Tile - 1) / kP0Tile); }
    // bytes a region's tiles read: each tile loads its positions plus a 96-byte halo
    uint64_t need(uint32_t r) const { return std::min<uint64_t>(lo(r) + (uint64_t)tiles(r) * kP0Tile + 128, len); }
};

static KeySpec hint_spec(uint32_t k) {
    KeySpec ks{};
    ks.bits = 2;
    ks.symbols = (int)k;
    ks.min_len = (int)k;
    ks.words = 1;
    ks.total_bits = 2 * (int)k;
    return ks;
}

bool prefetch_matches(const gk_ctx *c, const KeySpec &ks) {
    return c->pre_valid && c->enumerated && ks.bits == 2 && ks.symbols == (int)c->pre_k &&
           ks.min_len == ks.symbols && ks.words == 1 && ks.lenbits == 0 && !ks.canonical &&
           c->n + ks.symbols - 1 <= c->sba_len;  // (acgt_only: the class A of a mixed sba, gkm_split.hip)
}

int prefetch_plan(gk_ctx *c, uint64_t len, L0Prefetch **out) {
    *out = nullptr;
    const uint32_t k = c->hint_k;
    if (k < 8 || k > 32 || len < (uint64_t)k + kP0Tile) return GK_OK;
    const KeySpec ks = hint_spec(k);
    MsdDriver d(c, ks);
    if (d.width(0) != 7 && d.width(0) != kGR) return GK_OK;  // (the wide L0 has its own tiles)
    auto *p = new L0Prefetch();
    p->ks = ks;
    p->len = len;
    p->n = len - k + 1;
    p->w0 = d.width(0);
    p->w1 = d.width(1);
    d.allow_c79 = opt("GKM_NO_PAIRS") == nullptr;
    d.n = p->n;
    p->p88 = d.p88_wanted();
    p->p88_shi = 64 - (d.B - p->w0 - 8);
    const uint64_t nt = (p->n + kP0Tile - 1) / kP0Tile;
    // regions: GKM_PREFETCH_REGIONS (default 16); the last region's pass is what the transfer
    // cannot hide
    const char *e = opt("GKM_PREFETCH_REGIONS");
    const uint64_t want = std::max<uint64_t>(1, e && *e ? std::strtoull(e, nullptr, 10) : 16);
    // equal regions, but the last one's share is cut into halving pieces (1/2, 1/4, 1/8, 1/8 of it):
    // the pass of the last region to land is what the transfer cannot hide
    const uint64_t tpr = std::max<uint64_t>(1, (nt + want - 1) / want);
    for (uint64_t f = 0; f < nt; f += tpr) {
        const uint64_t e = std::min(nt, f + tpr);
        if (e == nt && e - f >= 8) {
            const uint64_t m = e - f;
            for (uint64_t g : {f, f + m / 2, f + 3 * m / 4}) p->first.push_back(g);
            p->first.push_back(f + 7 * m / 8);
        } else {
            p->first.push_back(f);
        }
    }
    p->first.push_back(nt);
    p->nreg = (uint32_t)(p->first.size() - 1);
    p->tpr = (uint32_t)tpr;
    p->nc_max = (p->tpr + d.ctiles - 1) / d.ctiles;
    const uint32_t R = 1u << p->w0, stride = 2 * p->nc_max + 4;
    int rc = ensure_elems(c, len, 1);  // keys[1] / vals[1] by position (n <= len)
    if (rc != GK_OK) {
        delete p;
        return rc;
    }
    GK_TRY_HIP(c, msd_tables());
    uint8_t *ndp;
    uint32_t *dummy;
    if (!p->p88) GK_TRY_HIP(c, scratch(c, "msd_nd", len + 64, &ndp));  // (packed: in vals[1], MsdDriver::p88_place)
    GK_TRY_HIP(c, scratch(c, "pre_tables", (uint64_t)p->nreg * stride, &p->tab));
    GK_TRY_HIP(c, scratch(c, "pre_pieces", (uint64_t)p->nreg * 2 * R, &p->pieces));
    GK_TRY_HIP(c, scratch(c, "s_misc", 4, &dummy));
    rc = d.tables(p->tpr, p->nc_max, 1);
    if (rc != GK_OK) {
        delete p;
        return rc;
    }
    std::vector<uint32_t> h((uint64_t)p->nreg * stride, 0);
    for (uint32_t r = 0; r < p->nreg; ++r) {
        uint32_t *t = h.data() + (uint64_t)r * stride;
        const uint32_t ntr = p->tiles(r), ncr = (ntr + d.ctiles - 1) / d.ctiles;
        for (uint32_t j = 0; j < ncr; ++j) {
            t[j] = j * d.ctiles;
            t[p->nc_max + j] = std::min<uint32_t>(d.ctiles, ntr - j * d.ctiles);
        }
        t[2 * p->nc_max] = 0;                        // s_cfirst
        t[2 * p->nc_max + 1] = ncr;                  // s_nchunks
        t[2 * p->nc_max + 2] = (uint32_t)p->lo(r);   // s_start: outputs by position
    }
    GK_TRY_HIP(c, hipMemcpy(p->tab, h.data(), 4 * h.size(), hipMemcpyHostToDevice));
    if (!c->pre_stream) GK_TRY_HIP(c, hipStreamCreateWithFlags(&c->pre_stream, hipStreamNonBlocking));
    if (!c->pre_done) GK_TRY_HIP(c, hipEventCreateWithFlags(&c->pre_done, hipEventDisableTiming));
    while (c->pre_ev.size() < p->nreg) {
        hipEvent_t ev;
        GK_TRY_HIP(c, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        c->pre_ev.push_back(ev);
    }
    *out = p;
    return GK_OK;
}

int prefetch_launch(gk_ctx *c, L0Prefetch *p, uint64_t landed) {
    if (!p || p->next >= p->nreg || landed < p->need(p->next)) return GK_OK;
    // every unpack enqueued so far (on the transfer's unpack stream); the regions now covered wait
    // for them
    GK_TRY_HIP(c, hipEventRecord(c->pre_ev[p->next], c->unpack_stream ? c->unpack_stream : c->stream));
    GK_TRY_HIP(c, hipStreamWaitEvent(c->pre_stream, c->pre_ev[p->next], 0));
    // the regions run on the prefetch stream; every return below restores the context's stream
    struct StreamSwap {
        gk_ctx *c;
        hipStream_t keep;
        ~StreamSwap() { c->stream = keep; }
    } swap{c, c->stream};
    c->stream = c->pre_stream;
    MsdDriver d(c, p->ks);
    if (p->p88) {  // the regions' low start bits and digit bytes in vals[1] (p88_place)
        d.p88_place(1);
        d.nd = d.nd_l0;
        d.p88 = true;
        d.p88_shi = p->p88_shi;
    } else {
        GK_TRY_HIP(c, scratch(c, "msd_nd", p->len + 64, &d.nd));
    }
    const uint32_t R = 1u << p->w0, stride = 2 * p->nc_max + 4;
    int rc = GK_OK;
    int slot;
    timer_begin(c, "prefetch_l0", &slot);
    uint64_t units = 0;
    for (; rc == GK_OK && p->next < p->nreg && landed >= p->need(p->next); ++p->next) {
        const uint32_t r = p->next, ntr = p->tiles(r);
        rc = d.l0_region(p->lo(r), p->hi(r), ntr, (ntr + d.ctiles - 1) / d.ctiles, p->nc_max,
                         p->tab + (uint64_t)r * stride, p->len + 16, p->pieces + (uint64_t)r * 2 * R);
        units += p->hi(r) - p->lo(r);
    }
    timer_units(c, slot, units);
    timer_end(c, slot);
    return rc;
}

int prefetch_finish(gk_ctx *c, L0Prefetch *p, bool ok) {
    if (!p) return GK_OK;
    int rc = GK_OK;
    if (ok) rc = prefetch_launch(c, p, p->len);
    if (p->next > 0) {  // later work on the context's stream comes after the prefetch's
        GK_TRY_HIP(c, hipEventRecord(c->pre_done, c->pre_stream));
        GK_TRY_HIP(c, hipStreamWaitEvent(c->stream, c->pre_done, 0));
    }
    c->pre_valid = ok && rc == GK_OK && p->next == p->nreg;
    c->pre_k = (uint32_t)p->ks.symbols;
    c->pre_regions = p->nreg;
    c->pre_w0 = p->w0;
    c->pre_w1 = p->w1;
    c->pre_p88_shi = p->p88 ? p->p88_shi : 0;
    delete p;
    return rc;
}

// gk_sort(k) after a prefetched L0: the regions' buckets are the pieces of the first level
int msd_sort_prefetched(gk_ctx *c, const KeySpec &ks) {
    c->pre_valid = false;  // consumed
    MsdDriver d(c, ks);
    d.B = ks.total_bits;
    if (d.width(0) != c->pre_w0 || d.width(1) != c->pre_w1) return msd_sort(c, ks);  // (widths changed)
    d.allow_c79 = opt("GKM_NO_PAIRS") == nullptr;
    d.wkeys = (!ks.acgt_only || c->msd_force_keys) ? 1 : 0;  // one-word keys end final in keys[0] (as msd_sort)
    c->msd_keys_final = d.wkeys != 0;
    timer_begin(c, "msd_total", &d.total_slot);
    int rc = d.init(c->n);
    if (rc != GK_OK) return rc;
    const uint32_t R = 1u << c->pre_w0, nreg = c->pre_regions;
    uint32_t *pieces;
    GK_TRY_HIP(c, scratch(c, "pre_pieces", (uint64_t)nreg * 2 * R, &pieces));
    std::vector<uint32_t> h((uint64_t)nreg * 2 * R);
    GK_TRY_HIP(c, hipMemcpyAsync(h.data(), pieces, 4 * h.size(), hipMemcpyDeviceToHost, c->stream));
    GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
    std::vector<uint64_t> poff, plen;
    std::vector<uint32_t> pb;
    for (uint32_t b = 0; b < R; ++b)
        for (uint32_t r = 0; r < nreg; ++r) {  // a bucket's pieces in region order = start order
            const uint32_t cnt = h[(uint64_t)r * 2 * R + R + b];
            if (!cnt) continue;
            poff.push_back(h[(uint64_t)r * 2 * R + b]);
            plen.push_back(cnt);
            pb.push_back(b);
        }
    if (c->pre_p88_shi) {  // the regions wrote the packed L0 form (its side arrays in vals[1])
        d.p88_place(1);
        d.nd = d.nd_l0;
        d.p88_in = true;
        d.p88_shi = c->pre_p88_shi;
    } else {
        GK_TRY_HIP(c, scratch(c, "msd_nd", c->sba_len + 64, &d.nd));
    }
    d.nd_ready = true;  // the regions' L0 wrote the level-1 digit bytes
    rc = d.first_level_from_pieces(c->keys[1], c->vals[1], poff.data(), plen.data(), pb.data(),
                                   (uint32_t)poff.size(), 1, d.width(0));
    if (rc == GK_OK) rc = d.levels(2, d.width(0) + d.width(1), 0);
    if (rc == GK_OK) rc = d.finish();
    timer_end(c, d.total_slot);
    return rc;
}

// starts-only shards (GK_SHARD_STARTS_ONLY): key of the k-mer at every received start from the 2-bit
// packed copy (B <= 64 bits: the first word), and its next-level digit byte
__global__ __launch_bounds__(256) void keys_from_starts_kernel(const uint64_t *__restrict__ pk,
                                                                const uint32_t *__restrict__ vin, uint64_t n, int B,
                                                                Dig dn, uint64_t *__restrict__ kout,
                                                                uint8_t *__restrict__ nd) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const uint32_t s = vin[i], q = s >> 5, sh = (s & 31) * 2;
        const uint64_t A = pk[q];
        const uint64_t T = sh ? (A << sh) | (pk[q + 1] >> (64 - sh)) : A;
        const uint64_t key = T >> (64 - B);
        kout[i] = key;
        nd[i] = (uint8_t)dg_of(key, dn);
    }
}

static unsigned grid_of_n_msd(uint64_t n) { return (unsigned)std::min<uint64_t>((n + 255) / 256, 1u << 16); }

// multi-GPU send side: k-mers starting in [lo, hi) partitioned by their top kGR key bits
int msd_shard_partition(gk_ctx *c, const KeySpec &ks, uint64_t lo, uint64_t hi, uint64_t *kout, uint32_t *vout,
                        uint64_t cap, uint64_t *hist, uint64_t *count) {
    MsdDriver d(c, ks);
    d.B = ks.bits * std::min(ks.symbols, 64 / ks.bits);  // the first key word (see msd_sort)
    d.wsched[0] = kGR;  // the exchange splits by kGR-bit buckets (msd_radix_bits)
    GK_TRY_HIP(c, msd_tables());
    if (c->res_pk && c->acgt && ks.bits == 2) {  // both L0 passes read the transfer's packed copy
        d.pk_code = c->res_code;
        d.pk_dol = c->res_dol;
    }
    int rc = d.run_l0(lo, hi, kout, vout, cap, count);
    if (rc != GK_OK) return rc;
    std::vector<uint32_t> hc(kGRadix);
    GK_TRY_HIP(c, hipMemcpyAsync(hc.data(), d.seg_cnt, 4 * kGRadix, hipMemcpyDeviceToHost, c->stream));
    GK_TRY_HIP(c, hipStreamSynchronize(c->stream));  // the caller's exchange reads kout / vout next
    for (int i = 0; i < kGRadix; ++i) hist[i] = hc[i];
    return GK_OK;
}

// multi-GPU receive side: sort n received k-mers (buckets as pieces) into keys[0] / vals[0]
int msd_shard_sort(gk_ctx *c, const KeySpec &ks, const uint64_t *kin, const uint32_t *vin, const uint64_t *poff,
                   const uint64_t *plen, const uint32_t *pbucket, uint32_t np) {
    const int spw = 64 / ks.bits;
    const int nphase = (ks.symbols + spw - 1) / spw;
    MsdDriver d(c, ks);
    d.B = ks.bits * std::min(ks.symbols, spw);
    d.wkeys = (nphase == 1 && (!ks.acgt_only || c->msd_force_keys)) ? 1 : 0;  // one-word keys end final in keys[0]
    c->msd_keys_final = d.wkeys != 0;
    d.wsched[0] = kGR;  // pieces are kGR-bit buckets
    d.allow_c79 = opt("GKM_NO_PAIRS") == nullptr;
    timer_begin(c, "msd_total", &d.total_slot);
    int rc = d.init(c->n);
    if (rc != GK_OK) return rc;
    if (!kin) {
        // starts only (GK_SHARD_STARTS_ONLY): every received k-mer's key from the rank's own packed copy
        // of the sequence (a sender's piece holds ascending starts of one position range, so the
        // words read stay close), with the level-1 digit byte its count pass reads
        const uint64_t *pk = nullptr;
        const uint32_t *pd = nullptr;
        if (c->res_pk && c->acgt) {
            pk = c->res_code;
        } else {
            int rp = pack_sequence(c, &pk, &pd);
            if (rp != GK_OK) return rp;
        }
        GK_TRY_HIP(c, scratch(c, "msd_nd", c->n + 64, &d.nd));
        int slot;
        timer_begin(c, "shard_keys", &slot);
        timer_units(c, slot, c->n);
        hipLaunchKernelGGL(keys_from_starts_kernel, dim3(grid_of_n_msd(c->n)), dim3(256), 0, c->stream, pk, vin, c->n,
                           d.B, dig_at(d.B, kGR, d.width(1)), c->keys[1], d.nd);
        GK_TRY_HIP(c, hipGetLastError());
        timer_end(c, slot);
        kin = c->keys[1];
        d.nd_ready = true;
    }
    rc = d.first_level_from_pieces(kin, vin, poff, plen, pbucket, np);
    if (rc != GK_OK) return rc;
    rc = d.levels(2, kGR + d.width(1), 0);
    if (rc != GK_OK) return rc;
    rc = d.finish();
    for (int ph = 1; ph < nphase && rc == GK_OK; ++ph)
        rc = d.next_phase(ph * spw, std::min(spw, ks.symbols - ph * spw));
    timer_end(c, d.total_slot);
    return rc;
}

// One-word keys already in memory (keys[cur] / vals[cur], n = c->n; the low total_bits bits of
// each key significant), sorted stably by the MSD levels over the keys themselves -- 8-bit digits
// from the top, packed pairs and a compact level where the bits allow, the same finishing kernels --
// instead of one LSD pass per 8 bits: two global passes and the local rounds for 1e8 keys where
// the LSD sort made six.  Result in keys[0] / vals[0] (c->cur = 0), the keys final; radix_sort's
// contract otherwise (gkm_sort.hip).
int msd_sort_keys(gk_ctx *c, int total_bits) {
    KeySpec kk{};
    kk.bits = 8;  // (no sequence-derived L0: every level reads the keys, 8-bit digits)
    kk.symbols = (total_bits + 7) / 8;
    kk.min_len = 1;
    kk.words = 1;
    kk.total_bits = total_bits;
    MsdDriver d(c, kk);
    d.B = total_bits;
    d.wkeys = 1;
    d.allow_c79 = opt("GKM_NO_PAIRS") == nullptr;
    // digit widths: as few global levels as leave buckets of <= ~400 keys for the one-wave
    // finishing classes (1e8 keys: 6 + 6 + 6 bits, buckets of ~380), the bits spread evenly; two
    // 8-bit levels left 1.5 K-key buckets to the block-local class, which ran 3.6 ms for 1e8 keys
    if (!opt("GKM_LEVEL_BITS")) {
        int b = 0;
        while (b < total_bits && (c->n >> b) > 400) ++b;
        const int L = std::max(1, (b + 7) / 8);
        const int w = std::max(6, std::min(8, (b + L - 1) / L));
        for (int l = 0; l < kMaxLevels; ++l) d.wsched[l] = l < L ? w : kGR;
    }
    c->msd_keys_final = true;
    timer_begin(c, "msd_total", &d.total_slot);
    const int in = c->cur;
    int rc = d.init(c->n);
    if (rc != GK_OK) return rc;
    uint32_t *one;
    GK_TRY_HIP(c, scratch(c, "keys_bucket", 2, &one));
    const uint32_t hb[2] = {0, (uint32_t)c->n};
    GK_TRY_HIP(c, hipMemcpyAsync(one, hb, 8, hipMemcpyHostToDevice, c->stream));
    rc = d.classify(1, 0, in, 0, one, one + 1);  // all keys as one bucket, no bits sorted
    if (rc == GK_OK) rc = d.levels(0, 0, in);
    if (rc == GK_OK) rc = d.finish();
    c->cur = 0;
    timer_end(c, d.total_slot);
    return rc;
}

// sort_doubling's rounds: the tied groups of keys[0] / vals[0] (flags: 1 starts a group) sorted by
// their bkey-bit keys (MsdDriver::sort_groups)
int msd_sort_groups(gk_ctx *c, const uint8_t *flags, int bkey) {
    KeySpec kk{};
    kk.bits = 8;
    kk.symbols = (bkey + 7) / 8;
    kk.min_len = 1;
    kk.words = 1;
    kk.total_bits = bkey;
    MsdDriver d(c, kk);
    d.B = bkey;
    d.wkeys = 1;
    timer_begin(c, "msd_groups", &d.total_slot);
    int rc = d.init(c->n);
    if (rc == GK_OK) rc = d.sort_groups(flags, bkey);
    timer_end(c, d.total_slot);
    return rc;
}

int msd_radix_bits() { return kGR; }
hipError_t rank_mode_msd(int ballot) { return set_rank_ballot_here(ballot); }

// the key-range ranks fuse their select into the L0 when their digit share is >= 1 / this: the
// emulated C3 rank (tools/range_emulate.py, profiles/r5/emu_fused_ab.txt) ran 42.3 against 45.0 ms
// fused at N = 2, but 26.0 against 23.7 at N = 4 and 18.1 against 13.5 at N = 8 -- the L0 over the
// whole sequence costs ~7.7 ms even when it stores an eighth of it
constexpr uint64_t kFusedMaxRanks = 2;

// L0 digit width of the key-range shards: 7 bits for 2-bit keys (as msd_sort), 8 otherwise
static int range_width(const KeySpec &ks) { return ks.bits == 2 ? 7 : kGR; }

// Ownership digits of the key-range shards: the ranks' ranges are cut on the top 12 bits of 2-bit
// keys (k >= 6; 2k bits below), so a hot 7-bit L0 digit of a skewed genome is split between ranks;
// 4-bit keys keep 8 bits.  The first partition level after the select still uses range_width.
int range_own_bits(const KeySpec &ks) {
    const int B = ks.bits * std::min(ks.symbols, 64 / ks.bits);
    return ks.bits == 2 ? std::min(12, B) : std::min(kGR, B);
}

int msd_l0_histogram(gk_ctx *c, const KeySpec &ks, uint64_t lo, uint64_t hi, uint64_t *hist, int *bits) {
    MsdDriver d(c, ks);
    d.B = ks.bits * std::min(ks.symbols, 64 / ks.bits);  // the first key word (see msd_sort)
    GK_TRY_HIP(c, msd_tables());
    // the packed sequence is made here for the whole sba and kept for the gk_shard_sort_range
    // that follows (one packing per key-range step)
    if (use_pack() && c->acgt && ks.bits == 2) {
        int rp = pack_sequence(c, &d.pk_code, &d.pk_dol);
        if (rp != GK_OK) return rp;
    } else if (c->res_pk && ks.bits == 2 && (c->acgt || ks.acgt_only)) {  // the transfer's packed copy
        d.pk_code = c->res_code;
        d.pk_dol = c->res_dol;
    }
    const int ob = range_own_bits(ks);
    L0Args a{c->sba, lo, std::max(hi, lo), ks.symbols, d.B, ks.acgt_only};
    a.own_bits = ob;
    a.pk_code = d.pk_code;
    a.pk_dol = d.pk_dol;
    uint32_t *gh;
    GK_TRY_HIP(c, scratch(c, "own_hist", 4096, &gh));
    GK_TRY_HIP(c, hipMemsetAsync(gh, 0, 4 * 4096, c->stream));
    const uint32_t ntiles = (uint32_t)std::max<uint64_t>((a.hi - lo + kSTile - 1) / kSTile, 1);
    int slot;
    timer_begin(c, "histogram", &slot);
    timer_units(c, slot, a.hi - lo);
#define GK_HIST(B_, C_)                                                                                        \
    do {                                                                                                       \
        int per_cu = 0;                                                                                        \
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, own_hist_kernel<B_, C_>, kST, 0) !=          \
                hipSuccess || per_cu < 1)                                                                      \
            per_cu = 1;                                                                                        \
        const unsigned g = std::min<unsigned>(ntiles, d.cus * (unsigned)per_cu);                               \
        hipLaunchKernelGGL((own_hist_kernel<B_, C_>), dim3(g), dim3(kST), 0, c->stream, a, ntiles, gh);        \
    } while (0)
    if (ks.bits == 2 && !ks.canonical && a.pk_code && ks.symbols <= 32 && a.hi > lo && !opt("GKM_RSEL_OFF")) {
        int per_cu = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, own_hist_rsel_kernel, kRselW * 64, 0) != hipSuccess ||
            per_cu < 1)
            per_cu = 1;
        const uint64_t G = (a.hi + 31) / 32 - lo / 32;
        const uint64_t gpb = std::max<uint64_t>((G + (uint64_t)d.cus * per_cu - 1) / ((uint64_t)d.cus * per_cu), 1);
        hipLaunchKernelGGL(own_hist_rsel_kernel, dim3((unsigned)((G + gpb - 1) / gpb)), dim3(kRselW * 64), 0, c->stream,
                           a, gpb, gh);
    } else if (ks.bits == 2) { if (ks.canonical) GK_HIST(2, true); else GK_HIST(2, false); }
    else { if (ks.canonical) GK_HIST(4, true); else GK_HIST(4, false); }
#undef GK_HIST
    GK_TRY_HIP(c, hipGetLastError());
    timer_end(c, slot);
    std::vector<uint32_t> hc(1u << ob);
    GK_TRY_HIP(c, hipMemcpyAsync(hc.data(), gh, 4u << ob, hipMemcpyDeviceToHost, c->stream));
    GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
    for (int i = 0; i < (1 << ob); ++i) hist[i] = hc[i];
    *bits = ob;
    return GK_OK;
}

int msd_sort_range(gk_ctx *c, const KeySpec &ks, uint32_t digit_lo, uint32_t digit_hi, uint64_t *n_kept) {
    const int spw = 64 / ks.bits;
    const int nphase = (ks.symbols + spw - 1) / spw;
    MsdDriver d(c, ks);
    d.B = ks.bits * std::min(ks.symbols, spw);
    d.wkeys = (nphase == 1 && (!ks.acgt_only || c->msd_force_keys)) ? 1 : 0;  // one-word keys end final in keys[0]
    c->msd_keys_final = d.wkeys != 0;
    // packed-pair levels where the bits fit (the first level from the select's pieces has 55 bits
    // left at C3: its L1 writes the pairs)
    d.allow_c79 = opt("GKM_NO_PAIRS") == nullptr;
    d.wsched[0] = range_width(ks);
    timer_begin(c, "msd_total", &d.total_slot);
    GK_TRY_HIP(c, msd_tables());
    const uint64_t L = c->sba_len;
    const uint32_t ntiles = (uint32_t)std::max<uint64_t>((L + kSTile - 1) / kSTile, 1);
    const uint64_t nw = (uint64_t)ntiles * kSR * kSW;
    L0Args a{c->sba, 0, L, ks.symbols, d.B, ks.acgt_only};
    a.own_lo = digit_lo;
    a.own_span = digit_hi > digit_lo ? digit_hi - digit_lo : 0;
    a.own_bits = range_own_bits(ks);
    if (use_pack() && c->acgt && ks.bits == 2) {  // this step's gk_shard_histogram's packing, or pack now
        if (c->pk_fresh) {
            uint64_t *pc;
            uint32_t *pd;
            const uint64_t nwords = (L + kSbaPad) / 32;
            GK_TRY_HIP(c, scratch(c, "pk_code", nwords, &pc));
            GK_TRY_HIP(c, scratch(c, "pk_dol", nwords, &pd));
            a.pk_code = pc;
            a.pk_dol = pd;
        } else {
            int rp = pack_sequence(c, &a.pk_code, &a.pk_dol);
            if (rp != GK_OK) return rp;
        }
        c->pk_fresh = false;
        d.pk_code = a.pk_code;  // (the fused L0 reads it too)
        d.pk_dol = a.pk_dol;
    } else if (c->res_pk && ks.bits == 2 && (c->acgt || ks.acgt_only)) {  // the transfer's packed copy
        a.pk_code = c->res_code;
        a.pk_dol = c->res_dol;
        d.pk_code = c->res_code;
        d.pk_dol = c->res_dol;
    }
    // Fused select (round 5): when the rank keeps a large share of the k-mers, its L0 count and
    // partition run over the whole sequence and keep only the owned k-mers (msd0_pipe_kernel<...,
    // OWN>), as msd_sort's L0 does for all of them -- no select pass, no 13-byte write and re-read
    // per kept k-mer, and the packed L0 output.  With a small share the whole-sequence L0 (count,
    // packing and ranking of every position) costs more than the select it replaces.  The share is
    // estimated from the digit range; GKM_RANGE_FUSED=0/1 forces either path.
    {
        const int ob = range_own_bits(ks);
        const uint32_t span = digit_hi > digit_lo ? digit_hi - digit_lo : 0;
        bool fused = ks.bits == 2 && span > 0 && (uint64_t)span * kFusedMaxRanks >= (1ull << ob);
        if (const char *e = opt("GKM_RANGE_FUSED")) fused = ks.bits == 2 && span > 0 && e[0] == '1';
        if (fused) {
            c->n = 0;
            c->cur = 0;
            uint64_t found = 0;
            int rc = d.l0_count(0, L, digit_lo, span, &found, ob);
            if (rc != GK_OK) return rc;
            if (found > 0xFFFFFFFFull) return fail(c, GK_E_ARG, "more k-mers than uint32 start indices can address");
            *n_kept = found;
            if (found == 0) {
                timer_end(c, d.total_slot);
                return GK_OK;
            }
            rc = ensure_elems(c, found + 1, 1);
            if (rc != GK_OK) return rc;
            c->n = found;
            rc = d.init(found);
            if (rc != GK_OK) return rc;
            d.p88 = d.p88_wanted();
            d.p88_shi = 64 - (d.B - d.width(0) - 8);
            int l0b = 0;  // (as msd_sort: the last global level writes buffer 1)
            {
                uint64_t mean = found >> d.width(0);
                int lev = 0;
                for (int l = 1; mean > (uint64_t)kBlockMax && l < kMaxLevels; ++l, ++lev) mean >>= d.width(l);
                l0b = 1 ^ (lev & 1);
            }
            rc = d.l0_partition(c->keys[l0b], c->vals[l0b], c->elem_cap + 64, found);
            if (rc == GK_OK) rc = d.classify(1u << d.width(0), d.width(0), l0b, 0, nullptr, nullptr, 1, nullptr, d.width(0));
            if (rc == GK_OK && d.p88_in) rc = d.expand_p88_locals(l0b);
            if (rc == GK_OK) rc = d.levels(1, d.width(0), l0b);
            if (rc == GK_OK) rc = d.finish();
            for (int ph = 1; ph < nphase && rc == GK_OK; ++ph)
                rc = d.next_phase(ph * spw, std::min(spw, ks.symbols - ph * spw));
            timer_end(c, d.total_slot);
            return rc;
        }
    }
    const Dig d0 = dig_at(d.B, 0, d.width(0));
    const bool two_pass = select_two_pass();
    uint32_t *wave_cnt, *wave_off;
    GK_TRY_HIP(c, scratch(c, "sel_wave_cnt", nw + 1, &wave_cnt));
    GK_TRY_HIP(c, scratch(c, "sel_wave_off", nw + 1, &wave_off));
    c->n = 0;  // nothing in the buffers survives: ensure_elems copies none
    c->cur = 0;
    // single pass: chunks of tpw tiles per workgroup, one region of tpw * kSTile elements each in
    // keys[1] / vals[1] (room for every position: no count pass)
    uint32_t tpw = 1, nchunk = 0;
    auto launch = [&](int mode) {
        uint64_t *ko = mode ? c->keys[mode == 2 ? 1 : 0] : nullptr;
        uint32_t *vo = mode ? c->vals[mode == 2 ? 1 : 0] : nullptr;
        uint8_t *no = mode ? d.nd : nullptr;
        // persistent grid = the workgroups that fit at once (a second round of workgroups would
        // start only when the first ones have walked all their tiles)
#define GK_SEL(B_, C_, M_)                                                                                    \
    do {                                                                                                      \
        int per_cu = 0;                                                                                       \
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, msd0_select_kernel<B_, C_, M_>, kST, 0) !=  \
                hipSuccess ||                                                                                 \
            per_cu < 1)                                                                                       \
            per_cu = 1;                                                                                       \
        unsigned sgrid = std::min<unsigned>(ntiles, d.cus * (unsigned)per_cu);                                \
        if (M_ == 2) {                                                                                        \
            tpw = (ntiles + sgrid - 1) / sgrid;                                                               \
            sgrid = nchunk = (ntiles + tpw - 1) / tpw;                                                        \
        }                                                                                                     \
        hipLaunchKernelGGL((msd0_select_kernel<B_, C_, M_>), dim3(sgrid), dim3(kST), 0, c->stream, a, d0,     \
                           ntiles, tpw, wave_cnt, wave_off, ko, vo, no);                                      \
    } while (0)
#define GK_SEL_M(B_, C_)                                                                                      \
    do {                                                                                                      \
        if (mode == 0) GK_SEL(B_, C_, 0);                                                                     \
        else if (mode == 1) GK_SEL(B_, C_, 1);                                                                \
        else GK_SEL(B_, C_, 2);                                                                               \
    } while (0)
        if (ks.bits == 2 && ks.canonical) GK_SEL_M(2, true);
        else if (ks.bits == 2) GK_SEL_M(2, false);
        else if (ks.canonical) GK_SEL_M(4, true);
        else GK_SEL_M(4, false);
#undef GK_SEL_M
#undef GK_SEL
    };
    int slot;
    uint64_t found = 0;
    std::vector<uint64_t> poff, plen;
    if (two_pass) {
        timer_begin(c, "msd_select_count", &slot);
        timer_units(c, slot, L);
        launch(0);
        GK_TRY_HIP(c, hipGetLastError());
        GK_TRY_HIP(c, scan_u32_exclusive_pub(c, wave_cnt, nw, wave_off, &found));
        timer_end(c, slot);
        if (found > 0xFFFFFFFFull) return fail(c, GK_E_ARG, "more k-mers than uint32 start indices can address");
        int rc = ensure_elems(c, std::max<uint64_t>(found, 1), 1);
        if (rc != GK_OK) return rc;
        GK_TRY_HIP(c, scratch(c, "msd_nd", found + 64, &d.nd));
        timer_begin(c, "msd_select", &slot);
        timer_units(c, slot, found);
        launch(1);
        GK_TRY_HIP(c, hipGetLastError());
        timer_end(c, slot);
    } else if (ks.bits == 2 && !ks.canonical && a.pk_code && ks.symbols <= 32 && a.own_bits <= 32 &&
               !opt("GKM_RSEL_OFF")) {
        // the SWAR select over the packed copy: one region per wave (msd0_rsel_kernel)
        const uint64_t ngroups = (L + 31) / 32;
        int per_cu = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, msd0_rsel_kernel, kRselW * 64, 0) != hipSuccess ||
            per_cu < 1)
            per_cu = 1;
        uint64_t nwv = (uint64_t)d.cus * (unsigned)per_cu * kRselW;
        const uint64_t gpw = ((ngroups + nwv - 1) / nwv + 63) / 64 * 64;  // whole 64-group steps per wave
        nwv = (ngroups + gpw - 1) / gpw;
        const unsigned nblk = (unsigned)((nwv + kRselW - 1) / kRselW);
        const uint64_t cap = (uint64_t)nblk * kRselW * gpw * 32;  // every wave region is full-size
        if (cap > 0xFFFFFFFFull) return fail(c, GK_E_ARG, "sequence too long for uint32 start indices");
        int rc = ensure_elems(c, cap, 1);
        if (rc != GK_OK) return rc;
        GK_TRY_HIP(c, scratch(c, "msd_nd", cap + 64, &d.nd));
        GK_TRY_HIP(c, scratch(c, "sel_wave_cnt", (uint64_t)nblk * kRselW + 1, &wave_cnt));
        const int sh = 32 - a.own_bits;
        const uint32_t lo_w = (uint32_t)((uint64_t)a.own_lo << sh);
        const uint32_t spm1_w = (uint32_t)(((uint64_t)std::min<uint64_t>(a.own_span, 1ull << a.own_bits) << sh) - 1);
        timer_begin(c, "msd_select", &slot);
        timer_units(c, slot, L);
        if (a.own_span == 0) {
            GK_TRY_HIP(c, hipMemsetAsync(wave_cnt, 0, 4 * nwv, c->stream));
        } else {
            hipLaunchKernelGGL(msd0_rsel_kernel, dim3(nblk), dim3(kRselW * 64), 0, c->stream, a, d0, ngroups, gpw, lo_w,
                               spm1_w, wave_cnt, c->keys[1], c->vals[1], d.nd);
        }
        GK_TRY_HIP(c, hipGetLastError());
        timer_end(c, slot);
        std::vector<uint32_t> kc(nwv);
        GK_TRY_HIP(c, hipMemcpyAsync(kc.data(), wave_cnt, 4 * nwv, hipMemcpyDeviceToHost, c->stream));
        GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
        for (uint64_t w = 0; w < nwv; ++w) {
            if (!kc[w]) continue;
            poff.push_back(w * gpw * 32);
            plen.push_back(kc[w]);
            found += kc[w];
        }
        timer_units(c, slot, found);
        if (found > 0xFFFFFFFFull) return fail(c, GK_E_ARG, "more k-mers than uint32 start indices can address");
    } else {
        const uint64_t cap = (uint64_t)ntiles * kSTile;  // every chunk region is full-size
        if (cap > 0xFFFFFFFFull) return fail(c, GK_E_ARG, "sequence too long for uint32 start indices");
        int rc = ensure_elems(c, cap, 1);
        if (rc != GK_OK) return rc;
        GK_TRY_HIP(c, scratch(c, "msd_nd", cap + 64, &d.nd));
        timer_begin(c, "msd_select", &slot);
        timer_units(c, slot, L);
        launch(2);
        const uint64_t stride = (uint64_t)tpw * kSTile;  // each chunk's region (launch sets tpw)
        GK_TRY_HIP(c, hipGetLastError());
        timer_end(c, slot);
        std::vector<uint32_t> kc(nchunk);
        GK_TRY_HIP(c, hipMemcpyAsync(kc.data(), wave_cnt, 4 * (uint64_t)nchunk, hipMemcpyDeviceToHost, c->stream));
        GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
        for (uint32_t w = 0; w < nchunk; ++w) {
            if (!kc[w]) continue;
            poff.push_back((uint64_t)w * stride);
            plen.push_back(kc[w]);
            found += kc[w];
        }
        timer_units(c, slot, found);  // (stage rates: kept k-mers out, the whole sequence in)
        if (found > 0xFFFFFFFFull) return fail(c, GK_E_ARG, "more k-mers than uint32 start indices can address");
    }
    *n_kept = found;
    c->n = found;
    if (found == 0) {
        timer_end(c, d.total_slot);
        return GK_OK;
    }
    uint8_t *nd_keep = d.nd;
    int rc = d.init(found);
    if (rc != GK_OK) return rc;
    d.nd = nd_keep;
    d.nd_ready = true;  // the select wrote the L0 digit bytes
    if (two_pass) {
        // the kept k-mers as one bucket [0, found) with no key bits sorted
        uint32_t *one;
        GK_TRY_HIP(c, scratch(c, "sel_bucket", 2, &one));
        const uint32_t hb[2] = {0, (uint32_t)found};
        GK_TRY_HIP(c, hipMemcpyAsync(one, hb, 8, hipMemcpyHostToDevice, c->stream));
        rc = d.classify(1, 0, 0, 0, one, one + 1);
        if (rc == GK_OK) rc = d.levels(0, 0, 0);
    } else {
        // the chunks' regions of keys[1] / vals[1] are the pieces of one bucket, in position order;
        // the first level partitions them into [0, found) of keys[0] / vals[0]
        const std::vector<uint32_t> pb(poff.size(), 0u);
        rc = d.first_level_from_pieces(c->keys[1], c->vals[1], poff.data(), plen.data(), pb.data(),
                                       (uint32_t)poff.size(), 0, 0);
        if (rc == GK_OK) rc = d.levels(1, d.width(0), 0);
    }
    if (rc == GK_OK) rc = d.finish();
    for (int ph = 1; ph < nphase && rc == GK_OK; ++ph)
        rc = d.next_phase(ph * spw, std::min(spw, ks.symbols - ph * spw));
    timer_end(c, d.total_slot);
    return rc;
}

}  // namespace gkm

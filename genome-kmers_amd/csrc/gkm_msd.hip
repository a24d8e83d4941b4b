// gkm_msd.hip -- stable MSD radix sort of one-word k-mer keys (the C3 hot path), gfx950.
//
// Why MSD: an LSD sort of 62-bit keys moves every (key, start) pair 8 times.  Here each pass
// partitions only what is still unsorted, and the tail is finished one bucket per wave:
//   L0     encode + partition by the top 8 bits, straight from the sequence byte array
//   L1..   partition every bucket larger than kLocalMax by the next 8 bits (big buckets only)
//   local  every bucket <= kLocalMax: one wave loads it, counting-sorts it by the next digit in
//          LDS, finishes sub-buckets <= kSmall by rank-by-count, writes it once; larger
//          sub-buckets spill to another round (one more digit each round).
// For 3.1e9 random 31-mers: L0, L1, L2 and one local round -- 4 movements instead of 8.
//
// Every partition is STABLE (64-lane ballot-match ranking, tiles in input order) and every
// partition offset is known before the scatter starts (count pass + column scan of per-tile
// digit histograms): no decoupled look-back chain.  Stability + ascending-start input make equal
// k-mers come out ordered by start index, the reference's break_ties=True order
// (kmers.py:1710-1711); a bucket whose key bits are exhausted is already in final order.
#include <algorithm>
#include <cstdlib>

#include "gkm_internal.h"
#include "gkm_partition.h"

namespace gkm {

// partition tile shapes (T threads x I items, wave-striped; LDS staging of T*I keys) are template
// parameters of the host driver; msd_sort picks one (default 1024 x 12)
constexpr int kChunkTiles = 256;                       // tiles per scan chunk
constexpr int kLocalMax = 512;                         // buckets <= this are finished by one wave
constexpr int kLocalChunks = kLocalMax / 64;
constexpr int kSmall = 24;                             // sub-buckets <= this: rank-by-count

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
    int symbols, total_bits;
};

template <int BITS, int TILE>
struct L0Pack {
    static constexpr int kGroups = TILE / 32 + 2;             // 32-position groups packed
    static constexpr int kCodeWords = kGroups * BITS / 2 + 1;  // u64 words (+1 for the funnel)
};

// thread g < kGroups holds the 32 bytes of group g (two 16-B loads)
template <int BITS, int TILE>
__device__ __forceinline__ void l0_load(const uint8_t *__restrict__ src, uint4 &ra, uint4 &rb) {
    // threads past kGroups re-load the last group: no branch, so load counts stay static
    const uint32_t g = min((uint32_t)threadIdx.x, (uint32_t)L0Pack<BITS, TILE>::kGroups - 1);
    const uint4 *s4 = reinterpret_cast<const uint4 *>(src + 32 * g);
    ra = s4[0];
    rb = s4[1];
}

template <int BITS, int TILE>
__device__ __forceinline__ void l0_pack(const uint4 &ra, const uint4 &rb, uint64_t *s_code, uint32_t *s_dol,
                                        const uint8_t *lut4) {
    using P = L0Pack<BITS, TILE>;
    const int g = threadIdx.x;
    if (g < P::kGroups) {
        const uint32_t wv[8] = {ra.x, ra.y, ra.z, ra.w, rb.x, rb.y, rb.z, rb.w};
        uint64_t c0 = 0, c1 = 0;
        uint32_t dm = 0;
#pragma unroll
        for (int q = 0; q < 32; ++q) {
            const uint32_t ch = (wv[q >> 2] >> (8 * (q & 3))) & 0xFFu;
            dm = (dm << 1) | (ch == GK_DOLLAR ? 1u : 0u);
            if (BITS == 2) {
                c0 = (c0 << 2) | (((ch >> 1) ^ (ch >> 2)) & 3u);
            } else {
                const uint64_t v = lut4[ch];
                if (q < 16) c0 = (c0 << 4) | v; else c1 = (c1 << 4) | v;
            }
        }
        if (BITS == 2) {
            s_code[g] = c0;
        } else {
            s_code[2 * g] = c0;
            s_code[2 * g + 1] = c1;
        }
        s_dol[g] = dm;
    }
    if (g == 0) s_code[P::kCodeWords - 1] = 0;
}

template <int BITS>
__device__ __forceinline__ uint64_t l0_key(const uint64_t *s_code, uint32_t p, int B) {
    const uint32_t o = p * BITS, w = o >> 6, s = o & 63;
    uint64_t x = s_code[w] << s;
    if (s) x |= s_code[w + 1] >> (64 - s);
    return x >> (64 - B);
}

__device__ __forceinline__ bool l0_valid(const uint32_t *s_dol, uint32_t p, int S) {
    const uint32_t w = p >> 5, s = p & 31;
    const uint64_t x = (((uint64_t)s_dol[w] << 32) | s_dol[w + 1]) << s;
    return (x >> (64 - S)) == 0;
}

template <int BITS, int T, int I>
__global__ __launch_bounds__(T) void msd0_count_kernel(L0Args a, Dig d0, uint32_t *__restrict__ tile_hist) {
    constexpr int TILE = T * I;
    using P = L0Pack<BITS, TILE>;
    __shared__ uint64_t s_code[P::kCodeWords];
    __shared__ uint32_t s_dol[P::kGroups];
    __shared__ uint32_t s_hist[256];
    __shared__ uint8_t s_lut4[256];
    const int t = threadIdx.x;
    if (t < 256) {
        s_lut4[t] = c_code4_msd[t];
        s_hist[t] = 0;
    }
    lds_barrier();
    const uint64_t P0 = (uint64_t)blockIdx.x * TILE;
    uint4 ra, rb;
    l0_load<BITS, TILE>(a.sba + P0, ra, rb);
    l0_pack<BITS, TILE>(ra, rb, s_code, s_dol, s_lut4);
    lds_barrier();
#pragma unroll
    for (int i = 0; i < I; ++i) {
        const uint32_t p = i * T + t;
        if (l0_valid(s_dol, p, a.symbols)) atomicAdd(&s_hist[dg_of(l0_key<BITS>(s_code, p, a.total_bits), d0)], 1u);
    }
    lds_barrier();
    if (t < 256) tile_hist[(uint64_t)blockIdx.x * 256 + t] = s_hist[t];
}

// persistent (see msd_scatter_kernel): the next tile's bytes are loaded while runs are stored
template <int BITS, int T, int I>
__global__ __launch_bounds__(T) void msd0_scatter_kernel(L0Args a, Dig d0, const uint32_t *__restrict__ tile_off,
                                                         uint64_t *__restrict__ kout, uint32_t *__restrict__ vout,
                                                         uint32_t ntiles, uint64_t sink) {
    constexpr int TILE = T * I;
    using P = L0Pack<BITS, TILE>;
    using SM = PartSmem<T, I>;
    __shared__ __attribute__((aligned(16))) unsigned char s_raw[SM::kUnion];
    __shared__ uint64_t s_code[P::kCodeWords];
    __shared__ uint32_t s_dol[P::kGroups];
    __shared__ uint32_t s_toff[256];
    __shared__ uint32_t s_wsum[4];
    __shared__ uint32_t s_count;
    __shared__ uint8_t s_lut4[256];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t *s_wc = reinterpret_cast<uint32_t *>(s_raw);
    if (tid < 256) s_lut4[tid] = c_code4_msd[tid];
    const TileWalk walk(ntiles);
    uint4 ra, rb;
    uint32_t toff = 0;
    auto load = [&](uint32_t t) {
        l0_load<BITS, TILE>(a.sba + (uint64_t)t * TILE, ra, rb);
        toff = tile_off[(uint64_t)t * 256 + (tid & 255)];  // every lane loads: no branch
    };
    if (walk.first < walk.end) load(walk.first);
    __builtin_amdgcn_s_waitcnt(kVmcnt0);  // see msd_scatter_kernel
    for (uint32_t t = walk.first; t < walk.end; t += walk.step) {
        lds_barrier();  // the previous tile's runs have been read out of LDS
        for (int i = tid; i < SM::kWaves * 256; i += T) s_wc[i] = 0;
        if (tid < 256) s_toff[tid] = toff;
        l0_pack<BITS, TILE>(ra, rb, s_code, s_dol, s_lut4);
        lds_barrier();
        const uint64_t P0 = (uint64_t)t * TILE;
        uint64_t key[I];
        uint32_t val[I];
        bool valid[I];
        uint32_t p0 = wave * (I * 64) + lane;
        asm volatile("" : "+v"(p0));  // keep the per-item offsets inside the loop (no hoisting)
#pragma unroll
        for (int i = 0; i < I; ++i) {
            const uint32_t p = p0 + i * 64;
            valid[i] = l0_valid(s_dol, p, a.symbols);
            key[i] = l0_key<BITS>(s_code, p, a.total_bits);
            val[i] = (uint32_t)(P0 + p);
        }
        partition_stage<T, I>(key, val, valid, d0, s_raw, s_toff, s_wsum, &s_count);
        const uint32_t cnt = s_count;
        if (t + walk.step < walk.end) load(t + walk.step);
        partition_store<T, I, 0>(d0, s_raw, s_toff, cnt, sink, kout, vout);
    }
}

// ---------------------------------------------------------------------------------------------
// column-wise segmented exclusive scan of per-tile digit histograms -> per-tile digit offsets
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void chunk_sum_kernel(const uint32_t *__restrict__ tile_hist,
                                                        const uint32_t *__restrict__ c_first,
                                                        const uint32_t *__restrict__ c_ntiles,
                                                        uint32_t *__restrict__ chunk_hist) {
    const int d = threadIdx.x;
    const uint64_t f = c_first[blockIdx.x];
    const uint32_t nt = c_ntiles[blockIdx.x];
    uint32_t acc = 0;
    uint32_t i = 0;
    for (; i + 8 <= nt; i += 8) {
        uint32_t v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = tile_hist[(f + i + u) * 256 + d];
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; i < nt; ++i) acc += tile_hist[(f + i) * 256 + d];
    chunk_hist[(uint64_t)blockIdx.x * 256 + d] = acc;
}

// one block per bucket: chunk bases within the bucket, digit bases, digit counts
__global__ __launch_bounds__(256) void seg_scan_kernel(uint32_t *__restrict__ chunk_hist,
                                                       const uint32_t *__restrict__ s_cfirst,
                                                       const uint32_t *__restrict__ s_nchunks,
                                                       const uint32_t *__restrict__ s_start,
                                                       uint32_t *__restrict__ seg_base, uint32_t *__restrict__ seg_cnt) {
    __shared__ uint32_t s_wsum[4];
    const int d = threadIdx.x, lane = d & 63, wave = d >> 6;
    const uint64_t cf = s_cfirst[blockIdx.x];
    const uint32_t nc = s_nchunks[blockIdx.x];
    uint32_t run = 0;
    uint32_t i = 0;
    for (; i + 8 <= nc; i += 8) {
        uint32_t v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = chunk_hist[(cf + i + u) * 256 + d];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            chunk_hist[(cf + i + u) * 256 + d] = run;
            run += v[u];
        }
    }
    for (; i < nc; ++i) {
        const uint32_t v = chunk_hist[(cf + i) * 256 + d];
        chunk_hist[(cf + i) * 256 + d] = run;
        run += v;
    }
    uint32_t incl = run;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(incl, off);
        if (lane >= off) incl += y;
    }
    if (lane == 63) s_wsum[wave] = incl;
    __syncthreads();
    uint32_t pre = 0;
    for (int w = 0; w < wave; ++w) pre += s_wsum[w];
    const uint32_t base = s_start[blockIdx.x] + pre + incl - run;
    seg_base[(uint64_t)blockIdx.x * 256 + d] = base;
    seg_cnt[(uint64_t)blockIdx.x * 256 + d] = run;
    for (uint32_t c = 0; c < nc; ++c) chunk_hist[(cf + c) * 256 + d] += base;
}

__global__ __launch_bounds__(256) void tile_apply_kernel(uint32_t *__restrict__ tile_hist,
                                                         const uint32_t *__restrict__ c_first,
                                                         const uint32_t *__restrict__ c_ntiles,
                                                         const uint32_t *__restrict__ chunk_base) {
    const int d = threadIdx.x;
    const uint64_t f = c_first[blockIdx.x];
    const uint32_t nt = c_ntiles[blockIdx.x];
    uint32_t run = chunk_base[(uint64_t)blockIdx.x * 256 + d];
    uint32_t i = 0;
    for (; i + 8 <= nt; i += 8) {
        uint32_t v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = tile_hist[(f + i + u) * 256 + d];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            tile_hist[(f + i + u) * 256 + d] = run;
            run += v[u];
        }
    }
    for (; i < nt; ++i) {
        const uint32_t v = tile_hist[(f + i) * 256 + d];
        tile_hist[(f + i) * 256 + d] = run;
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

// sub-buckets of this level: > kLocalMax -> next level (or done when no digit is left),
// 1..kLocalMax -> local list (sorted from digit `level + 1` on by the local rounds)
__global__ __launch_bounds__(256) void classify_kernel(const uint32_t *__restrict__ seg_base,
                                                       const uint32_t *__restrict__ seg_cnt, int level, int has_next,
                                                       int parity, uint32_t *__restrict__ nb_start,
                                                       uint32_t *__restrict__ nb_len, uint32_t *__restrict__ ctr,
                                                       uint32_t *__restrict__ dn_start, uint32_t *__restrict__ dn_len,
                                                       uint8_t *__restrict__ dn_par, uint2 *__restrict__ local) {
    const int lane = threadIdx.x & 63;
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint32_t size = seg_cnt[i], st = seg_base[i];
    const bool big = size > (uint32_t)kLocalMax;
    const uint32_t a = wave_append(big && has_next, &ctr[0], lane);
    if (big && has_next) {
        nb_start[a] = st;
        nb_len[a] = size;
    }
    const uint32_t b = wave_append(big && !has_next, &ctr[1], lane);
    if (big && !has_next) {
        dn_start[b] = st;
        dn_len[b] = size;
        dn_par[b] = (uint8_t)parity;
    }
    const bool small = size >= 1 && !big;
    const uint32_t c = wave_append(small, &ctr[2], lane);
    if (small) local[c] = local_entry(st, size, level + 1, parity);
}

// tile + chunk tables of a bucket list (one thread per bucket)
__global__ __launch_bounds__(256) void tile_table_kernel(const uint32_t *__restrict__ s_start,
                                                         const uint32_t *__restrict__ s_len,
                                                         const uint32_t *__restrict__ s_tfirst,
                                                         const uint32_t *__restrict__ s_cfirst, uint32_t nseg, uint32_t tile,
                                                         uint32_t *__restrict__ t_start, uint32_t *__restrict__ t_count,
                                                         uint32_t *__restrict__ c_first, uint32_t *__restrict__ c_ntiles) {
    const uint32_t s = blockIdx.x * 256 + threadIdx.x;
    if (s >= nseg) return;
    const uint32_t st = s_start[s], len = s_len[s], tf = s_tfirst[s], cf = s_cfirst[s];
    const uint32_t nt = (len + tile - 1) / tile;
    for (uint32_t j = 0; j < nt; ++j) {
        t_start[tf + j] = st + j * tile;
        t_count[tf + j] = std::min<uint32_t>(tile, len - j * tile);
    }
    const uint32_t nc = (nt + kChunkTiles - 1) / kChunkTiles;
    for (uint32_t j = 0; j < nc; ++j) {
        c_first[cf + j] = tf + j * kChunkTiles;
        c_ntiles[cf + j] = std::min<uint32_t>(kChunkTiles, nt - j * kChunkTiles);
    }
}

__global__ __launch_bounds__(256) void seg_counts_kernel(const uint32_t *__restrict__ s_len, uint32_t nseg, uint32_t tile,
                                                         uint32_t *__restrict__ ntiles, uint32_t *__restrict__ nchunks) {
    const uint32_t s = blockIdx.x * 256 + threadIdx.x;
    if (s >= nseg) return;
    const uint32_t nt = (s_len[s] + tile - 1) / tile;
    ntiles[s] = nt;
    nchunks[s] = (nt + kChunkTiles - 1) / kChunkTiles;
}

// ---------------------------------------------------------------------------------------------
// local rounds: one wave per bucket of <= kLocalMax elements
// ---------------------------------------------------------------------------------------------
// Stable counting sort of the bucket by digit `level` (registers -> LDS), then per sub-bucket:
// singleton or key exhausted -> final; <= kSmall -> rank-by-count (full key, ties by position);
// larger -> written in stable order and re-listed for the next round with level + 1.
// Output always goes to buffer 0; the bucket is read fully before any write, so in place is safe.
__global__ __launch_bounds__(64) void msd_local_kernel(const uint2 *__restrict__ list, int B, uint64_t *k0, uint32_t *v0,
                                                       const uint64_t *__restrict__ k1, const uint32_t *__restrict__ v1,
                                                       uint2 *__restrict__ spill, uint32_t *__restrict__ spill_count) {
    __shared__ uint64_t s_k[kLocalMax];
    __shared__ uint32_t s_v[kLocalMax];
    __shared__ uint32_t s_cnt[256];
    __shared__ uint32_t s_strt[256];
    const int lane = threadIdx.x;
    const uint2 e = list[blockIdx.x];
    const uint64_t st = e.x;
    const uint32_t len = e.y >> 8;
    const int level = (e.y >> 1) & 127;
    const int par = e.y & 1;
    const uint64_t *sk = par ? k1 : k0;
    const uint32_t *sv = par ? v1 : v0;
    const int D = num_digits(B);

    if (len <= (uint32_t)kSmall || level >= D) {
        // tiny bucket (or key exhausted: stable order is final)
        if (level >= D) {
            if (par)
                for (uint32_t i = lane; i < len; i += 64) {
                    k0[st + i] = sk[st + i];
                    v0[st + i] = sv[st + i];
                }
            return;
        }
        uint64_t mk = 0;
        uint32_t mv = 0;
        if ((uint32_t)lane < len) {
            mk = sk[st + lane];
            mv = sv[st + lane];
        }
        uint32_t r = 0;
        for (uint32_t j = 0; j < len; ++j) {
            const uint64_t kj = __shfl(mk, (int)j);
            r += (kj < mk) || (kj == mk && j < (uint32_t)lane);
        }
        if ((uint32_t)lane < len) {
            k0[st + r] = mk;
            v0[st + r] = mv;
        }
        return;
    }

    // counting sort by digit `level`
    const Dig dd = digit_at(B, level);
    for (int i = lane; i < 256; i += 64) s_cnt[i] = 0;
    uint64_t key[kLocalChunks];
    uint32_t val[kLocalChunks], rk[kLocalChunks];
#pragma unroll
    for (int c = 0; c < kLocalChunks; ++c) {
        const uint32_t i = c * 64 + lane;
        const bool valid = i < len;
        key[c] = valid ? sk[st + i] : 0;
        val[c] = valid ? sv[st + i] : 0;
    }
#pragma unroll
    for (int c = 0; c < kLocalChunks; ++c) {
        rk[c] = 0;
        if ((uint32_t)c * 64 >= len) continue;  // wave-uniform
        const bool valid = c * 64 + lane < len;
        const uint32_t d = dg_of(key[c], dd);
        const uint64_t peers = match_peers(d, valid);
        const uint32_t rank_in = lanes_below(peers);
        const uint32_t old = s_cnt[d];
        if (valid && rank_in == 0) s_cnt[d] = old + (uint32_t)__popcll(peers);
        rk[c] = old + rank_in;
    }
    {
        uint32_t c4[4], s4 = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            c4[u] = s_cnt[lane * 4 + u];
            s4 += c4[u];
        }
        uint32_t incl = s4;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(incl, off);
            if (lane >= off) incl += y;
        }
        uint32_t run = incl - s4;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            s_strt[lane * 4 + u] = run;
            run += c4[u];
        }
    }
#pragma unroll
    for (int c = 0; c < kLocalChunks; ++c) {
        if (c * 64 + lane < len) {
            const uint32_t p = s_strt[dg_of(key[c], dd)] + rk[c];
            s_k[p] = key[c];
            s_v[p] = val[c];
        }
    }
    const bool last = level + 1 >= D;
    for (uint32_t c0 = 0; c0 < len; c0 += 64) {
        const uint32_t p = c0 + lane;
        bool respill = false;
        uint32_t sub_start = 0, sub_len = 0;
        if (p < len) {
            const uint64_t kk = s_k[p];
            const uint32_t vv = s_v[p];
            const uint32_t d = dg_of(kk, dd);
            const uint32_t size = s_cnt[d], sb = s_strt[d];
            uint32_t out = p;
            if (size > 1 && !last) {
                if (size <= (uint32_t)kSmall) {
                    const uint32_t me = p - sb;
                    uint32_t r = 0;
                    for (uint32_t j = 0; j < size; ++j) {
                        const uint64_t kj = s_k[sb + j];
                        r += (kj < kk) || (kj == kk && j < me);
                    }
                    out = sb + r;
                } else if (p == sb) {
                    respill = true;
                    sub_start = (uint32_t)st + sb;
                    sub_len = size;
                }
            }
            k0[st + out] = kk;
            v0[st + out] = vv;
        }
        const uint32_t slot = wave_append(respill, spill_count, lane);
        if (respill) spill[slot] = local_entry(sub_start, sub_len, level + 1, 0);
    }
}

__global__ __launch_bounds__(256) void done_copy_kernel(const uint32_t *__restrict__ dn_start,
                                                        const uint32_t *__restrict__ dn_len,
                                                        const uint8_t *__restrict__ dn_par, const uint64_t *__restrict__ k1,
                                                        const uint32_t *__restrict__ v1, uint64_t *__restrict__ k0,
                                                        uint32_t *__restrict__ v0) {
    const uint32_t s = blockIdx.x;
    if (!dn_par[s]) return;
    const uint64_t st = dn_start[s];
    const uint32_t len = dn_len[s];
    for (uint32_t i = threadIdx.x; i < len; i += 256) {
        k0[st + i] = k1[st + i];
        v0[st + i] = v1[st + i];
    }
}

// ---------------------------------------------------------------------------------------------
// host driver
// ---------------------------------------------------------------------------------------------
static int grid_n(uint64_t n, int cap = 8192) {
    uint64_t g = (n + 255) / 256;
    if (g < 1) g = 1;
    return (int)std::min<uint64_t>(g, (uint64_t)cap);
}

hipError_t scan_u32_exclusive_pub(gk_ctx *c, const uint32_t *in, uint64_t n, uint32_t *out, uint64_t *total);

// scan per-tile histograms of the bucket list (nseg buckets, C chunks) into per-tile offsets
static int scan_offsets(gk_ctx *c, uint32_t *tile_hist, uint32_t *chunk_hist, const uint32_t *c_first,
                        const uint32_t *c_ntiles, uint64_t C, const uint32_t *s_cfirst, const uint32_t *s_nchunks,
                        const uint32_t *s_start, uint64_t nseg, uint32_t *seg_base, uint32_t *seg_cnt) {
    hipLaunchKernelGGL(chunk_sum_kernel, dim3((unsigned)C), dim3(256), 0, c->stream, tile_hist, c_first, c_ntiles,
                       chunk_hist);
    hipLaunchKernelGGL(seg_scan_kernel, dim3((unsigned)nseg), dim3(256), 0, c->stream, chunk_hist, s_cfirst, s_nchunks,
                       s_start, seg_base, seg_cnt);
    hipLaunchKernelGGL(tile_apply_kernel, dim3((unsigned)C), dim3(256), 0, c->stream, tile_hist, c_first, c_ntiles,
                       chunk_hist);
    GK_TRY_HIP(c, hipGetLastError());
    return GK_OK;
}

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
    hipError_t r = hipMalloc(&np, bytes);
    if (r != hipSuccess) return r;
    if (e.first && keep) {
        r = hipMemcpyAsync(np, e.first, sizeof(T) * keep, hipMemcpyDeviceToDevice, c->stream);
        if (r != hipSuccess) return r;
        r = hipStreamSynchronize(c->stream);
        if (r != hipSuccess) return r;
    }
    if (e.first) hipFree(e.first);
    e.first = np;
    e.second = bytes;
    *p = static_cast<T *>(np);
    return hipSuccess;
}

// partition grid: 4 workgroups per CU (one resident at a time: LDS-bound), a multiple of 8 (equal
// shares per XCD); measured 4% faster than exactly one per CU (profiles/r1/README.md)
static unsigned persistent_grid(gk_ctx *c) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess || cus < 8) cus = 256;
    return (unsigned)(cus / 8 * 8 * 4);
}

static int read_ctr(gk_ctx *c, const uint32_t *d, uint32_t *h, int count) {
    GK_TRY_HIP(c, hipMemcpyAsync(h, d, 4 * count, hipMemcpyDeviceToHost, c->stream));
    GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
    return GK_OK;
}

template <int PT, int PI>
static int msd_sort_shape(gk_ctx *c, const KeySpec &ks) {
    constexpr uint32_t kPartTile = PT * PI;
    GK_TRY_HIP(c, msd_tables());
    int total_slot;
    timer_begin(c, "msd_total", &total_slot);
    const int B = ks.total_bits, D = num_digits(B);
    const uint64_t n = c->n, L = c->sba_len;
    uint32_t *ctr;  // [0] next-level buckets, [1] done buckets, [2] local entries, [3] spill entries
    GK_TRY_HIP(c, scratch(c, "msd_ctr", 4, &ctr));
    GK_TRY_HIP(c, hipMemsetAsync(ctr, 0, 16, c->stream));

    // ---- L0: one bucket (all k-mers), tiles over sba positions ----
    const uint64_t nt0 = (L + kPartTile - 1) / kPartTile;
    const uint64_t nc0 = (nt0 + kChunkTiles - 1) / kChunkTiles;
    uint32_t *tile_hist, *chunk_hist, *c_first, *c_ntiles, *s_misc, *seg_base, *seg_cnt;
    GK_TRY_HIP(c, scratch(c, "tile_hist", nt0 * 256, &tile_hist));
    GK_TRY_HIP(c, scratch(c, "chunk_hist", nc0 * 256, &chunk_hist));
    GK_TRY_HIP(c, scratch(c, "c_first", nc0, &c_first));
    GK_TRY_HIP(c, scratch(c, "c_ntiles", nc0, &c_ntiles));
    GK_TRY_HIP(c, scratch(c, "s_misc", 4, &s_misc));
    GK_TRY_HIP(c, scratch(c, "seg_base", 256, &seg_base));
    GK_TRY_HIP(c, scratch(c, "seg_cnt", 256, &seg_cnt));
    {
        std::vector<uint32_t> cf(nc0), cn(nc0);
        for (uint64_t j = 0; j < nc0; ++j) {
            cf[j] = (uint32_t)(j * kChunkTiles);
            cn[j] = (uint32_t)std::min<uint64_t>(kChunkTiles, nt0 - j * kChunkTiles);
        }
        const uint32_t misc[3] = {0, (uint32_t)nc0, 0};  // s_cfirst, s_nchunks, s_start
        GK_TRY_HIP(c, hipMemcpyAsync(c_first, cf.data(), 4 * nc0, hipMemcpyHostToDevice, c->stream));
        GK_TRY_HIP(c, hipMemcpyAsync(c_ntiles, cn.data(), 4 * nc0, hipMemcpyHostToDevice, c->stream));
        GK_TRY_HIP(c, hipMemcpyAsync(s_misc, misc, 12, hipMemcpyHostToDevice, c->stream));
        GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
    }
    L0Args a{c->sba, ks.symbols, B};
    const Dig d0 = digit_at(B, 0);
    const unsigned pgrid = persistent_grid(c);
    int slot;
    timer_begin(c, "msd_l0_count", &slot);
    if (ks.bits == 2)
        hipLaunchKernelGGL((msd0_count_kernel<2, PT, PI>), dim3((unsigned)nt0), dim3(PT), 0, c->stream, a, d0, tile_hist);
    else
        hipLaunchKernelGGL((msd0_count_kernel<4, PT, PI>), dim3((unsigned)nt0), dim3(PT), 0, c->stream, a, d0, tile_hist);
    GK_TRY_HIP(c, hipGetLastError());
    timer_end(c, slot);
    timer_begin(c, "msd_scan", &slot);
    int rc = scan_offsets(c, tile_hist, chunk_hist, c_first, c_ntiles, nc0, s_misc, s_misc + 1, s_misc + 2, 1,
                          seg_base, seg_cnt);
    if (rc != GK_OK) return rc;
    timer_end(c, slot);
    timer_begin(c, "msd_pass_l0", &slot);
    if (ks.bits == 2)
        hipLaunchKernelGGL((msd0_scatter_kernel<2, PT, PI>), dim3(pgrid), dim3(PT), 0, c->stream, a, d0, tile_hist,
                           c->keys[0], c->vals[0], (uint32_t)nt0, n);
    else
        hipLaunchKernelGGL((msd0_scatter_kernel<4, PT, PI>), dim3(pgrid), dim3(PT), 0, c->stream, a, d0, tile_hist,
                           c->keys[0], c->vals[0], (uint32_t)nt0, n);
    GK_TRY_HIP(c, hipGetLastError());
    timer_end(c, slot);

    // bucket lists (ping-pong), done list, local list
    const uint64_t max_big = n / kLocalMax + 2;
    uint32_t *lst_start[2], *lst_len[2], *dn_start, *dn_len;
    uint8_t *dn_par;
    uint2 *local;
    GK_TRY_HIP(c, scratch(c, "lstA_start", max_big, &lst_start[0]));
    GK_TRY_HIP(c, scratch(c, "lstA_len", max_big, &lst_len[0]));
    GK_TRY_HIP(c, scratch(c, "lstB_start", max_big, &lst_start[1]));
    GK_TRY_HIP(c, scratch(c, "lstB_len", max_big, &lst_len[1]));
    GK_TRY_HIP(c, scratch(c, "dn_start", max_big, &dn_start));
    GK_TRY_HIP(c, scratch(c, "dn_len", max_big, &dn_len));
    GK_TRY_HIP(c, scratch(c, "dn_par", max_big, &dn_par));
    GK_TRY_HIP(c, grow_keep(c, "local", 256, 0, &local));
    int li = 0;
    hipLaunchKernelGGL(classify_kernel, dim3(1), dim3(256), 0, c->stream, seg_base, seg_cnt, 0, D > 1 ? 1 : 0, 0,
                       lst_start[li], lst_len[li], ctr, dn_start, dn_len, dn_par, local);
    GK_TRY_HIP(c, hipGetLastError());
    uint32_t h[4];
    rc = read_ctr(c, ctr, h, 4);
    if (rc != GK_OK) return rc;
    uint32_t nbig = h[0], nlocal = h[2];

    // ---- L1..: partition big buckets by the next digit ----
    int level = 1, in = 0;
    while (nbig > 0 && level < D) {
        const int out = in ^ 1;
        uint32_t *ntl, *nch, *tfirst, *cfirst;
        GK_TRY_HIP(c, scratch(c, "s_ntiles", nbig, &ntl));
        GK_TRY_HIP(c, scratch(c, "s_nchunks", nbig, &nch));
        GK_TRY_HIP(c, scratch(c, "s_tfirst", nbig, &tfirst));
        GK_TRY_HIP(c, scratch(c, "s_cfirst", nbig, &cfirst));
        hipLaunchKernelGGL(seg_counts_kernel, dim3(grid_n(nbig, 1 << 30)), dim3(256), 0, c->stream, lst_len[li], nbig,
                           kPartTile, ntl, nch);
        GK_TRY_HIP(c, hipGetLastError());
        uint64_t T = 0, C = 0;
        GK_TRY_HIP(c, scan_u32_exclusive_pub(c, ntl, nbig, tfirst, &T));
        GK_TRY_HIP(c, scan_u32_exclusive_pub(c, nch, nbig, cfirst, &C));
        uint32_t *t_start, *t_count;
        GK_TRY_HIP(c, scratch(c, "t_start", T, &t_start));
        GK_TRY_HIP(c, scratch(c, "t_count", T, &t_count));
        GK_TRY_HIP(c, scratch(c, "tile_hist", T * 256, &tile_hist));
        GK_TRY_HIP(c, scratch(c, "chunk_hist", C * 256, &chunk_hist));
        GK_TRY_HIP(c, scratch(c, "c_first", C, &c_first));
        GK_TRY_HIP(c, scratch(c, "c_ntiles", C, &c_ntiles));
        GK_TRY_HIP(c, scratch(c, "seg_base", (uint64_t)nbig * 256, &seg_base));
        GK_TRY_HIP(c, scratch(c, "seg_cnt", (uint64_t)nbig * 256, &seg_cnt));
        GK_TRY_HIP(c, grow_keep(c, "local", (uint64_t)nlocal + 256ull * nbig, nlocal, &local));
        hipLaunchKernelGGL(tile_table_kernel, dim3(grid_n(nbig, 1 << 30)), dim3(256), 0, c->stream, lst_start[li],
                           lst_len[li], tfirst, cfirst, nbig, kPartTile, t_start, t_count, c_first, c_ntiles);
        const Dig dl = digit_at(B, level);
        timer_begin(c, "msd_count", &slot);
        hipLaunchKernelGGL(msd_count_kernel, dim3((unsigned)T), dim3(256), 0, c->stream, t_start, t_count, dl,
                           c->keys[in], tile_hist);
        GK_TRY_HIP(c, hipGetLastError());
        timer_end(c, slot);
        timer_begin(c, "msd_scan", &slot);
        rc = scan_offsets(c, tile_hist, chunk_hist, c_first, c_ntiles, C, cfirst, nch, lst_start[li], nbig, seg_base,
                          seg_cnt);
        if (rc != GK_OK) return rc;
        timer_end(c, slot);
        static const char *kPassNames[] = {"msd_pass_l0", "msd_pass_l1", "msd_pass_l2", "msd_pass_l3",
                                           "msd_pass_l4", "msd_pass_l5", "msd_pass_l6", "msd_pass_l7"};
        timer_begin(c, kPassNames[level & 7], &slot);
        hipLaunchKernelGGL((msd_scatter_kernel<PT, PI>), dim3(pgrid), dim3(PT), 0, c->stream, t_start, t_count, dl,
                           tile_hist, c->keys[in], c->vals[in], c->keys[out], c->vals[out], (uint32_t)T, n);
        GK_TRY_HIP(c, hipGetLastError());
        timer_end(c, slot);
        const bool has_next = level + 1 < D;
        const int lo = li ^ 1;
        GK_TRY_HIP(c, hipMemsetAsync(ctr, 0, 4, c->stream));
        timer_begin(c, "msd_classify", &slot);
        hipLaunchKernelGGL(classify_kernel, dim3(nbig), dim3(256), 0, c->stream, seg_base, seg_cnt, level,
                           has_next ? 1 : 0, out, lst_start[lo], lst_len[lo], ctr, dn_start, dn_len, dn_par, local);
        GK_TRY_HIP(c, hipGetLastError());
        timer_end(c, slot);
        rc = read_ctr(c, ctr, h, 4);
        if (rc != GK_OK) return rc;
        nbig = h[0];
        nlocal = h[2];
        li = lo;
        ++level;
        in = out;
    }

    // ---- local rounds: every bucket <= kLocalMax, written to buffer 0 ----
    uint2 *spill;
    GK_TRY_HIP(c, scratch(c, "spill", n / (kSmall + 1) + 256, &spill));
    GK_TRY_HIP(c, grow_keep(c, "local", std::max<uint64_t>(nlocal, n / (kSmall + 1) + 256), nlocal, &local));
    const uint2 *cur_list = local;
    uint32_t ncur = nlocal;
    int round = 0;
    while (ncur > 0) {
        GK_TRY_HIP(c, hipMemsetAsync(ctr + 3, 0, 4, c->stream));
        uint2 *out_list = (round % 2 == 0) ? spill : local;  // spills of round r live in the other list
        timer_begin(c, round == 0 ? "msd_local" : "msd_local_spill", &slot);
        hipLaunchKernelGGL(msd_local_kernel, dim3(ncur), dim3(64), 0, c->stream, cur_list, B, c->keys[0], c->vals[0],
                           c->keys[1], c->vals[1], out_list, ctr + 3);
        GK_TRY_HIP(c, hipGetLastError());
        timer_end(c, slot);
        rc = read_ctr(c, ctr + 3, &ncur, 1);
        if (rc != GK_OK) return rc;
        cur_list = out_list;
        ++round;
        if (round > 16) return fail(c, GK_E_HIP, "msd local rounds did not converge");
    }
    const uint32_t ndone = h[1];
    if (ndone > 0) {
        hipLaunchKernelGGL(done_copy_kernel, dim3(ndone), dim3(256), 0, c->stream, dn_start, dn_len, dn_par,
                           c->keys[1], c->vals[1], c->keys[0], c->vals[0]);
        GK_TRY_HIP(c, hipGetLastError());
    }
    timer_end(c, total_slot);
    c->cur = 0;
    return GK_OK;
}

int msd_sort(gk_ctx *c, const KeySpec &ks) {
    const char *e = getenv("GKM_MSD_SHAPE");  // tuning experiments only
    const int shape = e ? atoi(e) : 0;
    switch (shape) {
    case 1: return msd_sort_shape<512, 12>(c, ks);
    case 2: return msd_sort_shape<512, 16>(c, ks);
    case 3: return msd_sort_shape<256, 16>(c, ks);
    default: return msd_sort_shape<1024, 12>(c, ks);
    }
}

}  // namespace gkm

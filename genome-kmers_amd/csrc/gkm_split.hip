// gkm_split.hip -- fixed-length sort of a sequence with non-ACGT bytes (GRCh38: N runs), gfx950.
//
// A 4-bit key spends half its bits on an alphabet the data barely uses: with 16 symbols per word
// the first MSD word of a 31-mer covers 16 bases, most k-mers tie on it, and every 8-bit digit
// holds only ~25 live values of 256.  Here the k-mers are split by class:
//   A  every base in A/C/G/T   -> the 2-bit MSD sort (gkm_msd.hip, acgt_only L0): the C3 speed
//   B  some other IUPAC letter -> 4-bit keys, LSD radix sort of the (few) B starts
// and the two sorted runs are merged.  No A k-mer equals a B k-mer, so the merge is a pure
// interleave: each B group (run of equal B k-mers) lands before the first A k-mer greater than
// it (a binary search over the sorted A starts, comparing bytes in the reference's order,
// kmers.py:306-397), and every A k-mer moves up by the B k-mers placed before it.  Both runs are
// in (k-mer, start) order, so the merged order is the reference's break_ties=True order
// (kmers.py:1710-1711).  Canonical k-mers (gkm_canon.h) keep their class under reverse
// complement, so the split applies to them unchanged.
#include <algorithm>
#include <cstdio>
#include <cstring>

#include "gkm_canon.h"
#include "gkm_internal.h"
#include "gkm_swar.h"

namespace gkm {

hipError_t scan_u32_exclusive_pub(gk_ctx *c, const uint32_t *in, uint64_t n, uint32_t *out, uint64_t *total);
hipError_t scan_u32_exclusive_pair(gk_ctx *c, const uint32_t *in1, uint32_t *out1, const uint32_t *in2,
                                   uint32_t *out2, uint64_t n, uint64_t *total1, uint64_t *total2);

__constant__ uint8_t c_code4_split[256];
__constant__ uint8_t c_comp_split[256];  // the reference's complement (sequence_collection.py:402-433)
static bool g_split_tables = false;

static hipError_t split_tables() {
    if (g_split_tables) return hipSuccess;
    uint8_t code4[256] = {0};
    const char *order = "ABCDGHKMNRSTVWY";
    for (int i = 0; order[i]; ++i) code4[(uint8_t)order[i]] = (uint8_t)(i + 1);
    hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(c_code4_split), code4, 256);
    if (e != hipSuccess) return e;
    uint8_t comp[256];
    for (int i = 0; i < 256; ++i) comp[i] = (uint8_t)i;
    const char *pairs[] = {"AT", "CG", "RY", "KM", "BV", "DH"};
    for (const char *p : pairs) {
        comp[(uint8_t)p[0]] = (uint8_t)p[1];
        comp[(uint8_t)p[1]] = (uint8_t)p[0];
    }
    e = hipMemcpyToSymbol(HIP_SYMBOL(c_comp_split), comp, 256);
    if (e == hipSuccess) g_split_tables = true;
    return e;
}

// ---------------------------------------------------------------------------------------------
// class B starts: no '$' in [p, p + k) and some byte outside ACGT in it
// ---------------------------------------------------------------------------------------------
constexpr int kFlagTile = 8192;                  // positions per workgroup
constexpr int kFlagGroups = kFlagTile / 32 + 3;  // 32-position groups incl. a 64-position halo

// the S (<= 64) mask bits from p are all zero
__device__ __forceinline__ bool window_clear(const uint32_t *m, uint32_t p, int S) {
    const uint32_t w = p >> 5, s = p & 31;
    const uint64_t x = (((uint64_t)m[w] << 32) | m[w + 1]) << s;
    if (S <= 32) return (x >> (64 - S)) == 0;
    const uint64_t y = (((uint64_t)m[w + 1] << 32) | m[w + 2]) << s;
    return (x >> 32) == 0 && (y >> (96 - S)) == 0;
}

// Class-B k-mers: no '$' in [p, p + k) and some byte outside ACGT in it.  Homopolymers (one
// letter k times: GRCh38's ~150 M N bases give that many "N...N" k-mers, one group already in
// start order) skip the B sort (split_sort).
// Key-range shards (p4_lo, p4_hi != 0, 0x10000): only B k-mers whose (canonical) first four
// symbols, as a 16-bit 4-bit code, lie in [p4_lo, p4_hi) -- the rank's byte-order interval
// (split_sort's SplitRange).
__device__ __forceinline__ uint32_t b_prefix(const uint8_t *sba, uint64_t p, int k, bool hp, int canonical,
                                             const uint8_t *lut4, const uint8_t *comp, int ns) {
    uint32_t v = 0;
    if (hp) {  // one letter k times; canonical: the smaller of the letter and its complement
        uint32_t ch = sba[p];
        if (canonical) ch = min(ch, (uint32_t)comp[ch]);
        const uint32_t c4 = lut4[ch];
        for (int t = 0; t < ns; ++t) v = (v << 4) | c4;
        return v;
    }
    const uint8_t *b = sba + p;
    const bool rc = canonical && canon_is_rc<4>(b, k, lut4);
    for (int t = 0; t < ns; ++t) v = (v << 4) | canon_sym<4>(b, k, t, rc, lut4);
    return v;
}

// The class-B starts without flag arrays: per 8192-position tile, COUNT writes the numbers of
// non-homopolymer and homopolymer B k-mers (cnt[0][t], cnt[1][t]); after their scans, STORE
// writes each kind's start positions from the tile's offsets (thread order = position order:
// thread t owns positions 32 t .. 32 t + 31).  Key-range shards keep only the k-mers whose
// b_prefix4 lies in their interval.
template <bool STORE>
__global__ __launch_bounds__(256) void class_b_select_kernel(const uint8_t *__restrict__ sba, uint64_t base,
                                                             uint64_t L, int k,
                                                             int canonical, uint32_t p4_lo, uint32_t p4_hi, int pns,
                                                             uint32_t *__restrict__ cnt_r, uint32_t *__restrict__ cnt_h,
                                                             const uint32_t *__restrict__ off_r,
                                                             const uint32_t *__restrict__ off_h,
                                                             uint32_t *__restrict__ out_r, uint32_t *__restrict__ out_h) {
    __shared__ uint32_t s_dol[kFlagGroups], s_bad[kFlagGroups], s_diff[kFlagGroups];
    __shared__ uint8_t s_lut4[256], s_comp[256];
    __shared__ uint32_t s_w[2][4];
    // the store pass has nothing to do for a tile whose counts are zero: away from N runs and IUPAC
    // letters, that is almost every tile of a genome
    if (STORE && cnt_r[blockIdx.x] == 0 && cnt_h[blockIdx.x] == 0) return;
    s_lut4[threadIdx.x] = c_code4_split[threadIdx.x];
    s_comp[threadIdx.x] = c_comp_split[threadIdx.x];
    const bool ranged = p4_lo != 0 || p4_hi != (1u << (4 * pns));
    const uint64_t P0 = base + (uint64_t)blockIdx.x * kFlagTile;  // positions >= L are not taken
    // the tile's 256 groups and the 3 halo groups: every load issued before any flag work (a second
    // loop trip for the halo would double the load latency of the tile)
    static_assert(kFlagGroups - 256 <= 256, "one halo group per thread at most");
    const bool halo = threadIdx.x < kFlagGroups - 256;
    uint4 ld[2][2];
    uint32_t ldn[2];
    {
        const uint4 *src = reinterpret_cast<const uint4 *>(sba + P0 + 32ull * threadIdx.x);  // '$' pad after L
        ld[0][0] = src[0];
        ld[0][1] = src[1];
        ldn[0] = sba[P0 + 32ull * (threadIdx.x + 1)];
        if (halo) {
            ld[1][0] = src[512];  // group threadIdx.x + 256
            ld[1][1] = src[513];
            ldn[1] = sba[P0 + 32ull * (threadIdx.x + 257)];
        }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        if (h == 1 && !halo) break;
        const int g = threadIdx.x + 256 * h;
        const uint4 ra = ld[h][0], rb = ld[h][1];
        const uint32_t nxt = ldn[h];
        // SWAR, 8 positions per step: '$' flags, non-ACGT flags, and "differs from the next byte"
        // flags (each byte against its successor: the unit shifted down one byte, the next unit's
        // first byte on top)
        constexpr uint64_t kOnes = 0x0101010101010101ull;
        const uint64_t x[4] = {((uint64_t)ra.y << 32) | ra.x, ((uint64_t)ra.w << 32) | ra.z,
                               ((uint64_t)rb.y << 32) | rb.x, ((uint64_t)rb.w << 32) | rb.z};
        uint32_t dm = 0, bm = 0, fm = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint64_t nb = j < 3 ? (x[j + 1] & 0xFFu) : (uint64_t)nxt;
            const uint64_t y = (x[j] >> 8) | (nb << 56);
            dm = (dm << 8) | gather_flags8(zero_bytes(x[j] ^ (kOnes * GK_DOLLAR)));
            bm = (bm << 8) | gather_flags8(non_acgt_bytes(x[j]));
            fm = (fm << 8) | gather_flags8(~zero_bytes(x[j] ^ y) & (kOnes << 7));
        }
        s_dol[g] = dm;
        s_bad[g] = bm;
        s_diff[g] = fm;
    }
    __syncthreads();
    const uint32_t p0 = threadIdx.x * 32;
    uint32_t mr = 0, mh = 0;  // bit j: position p0 + j
    const uint32_t g = threadIdx.x;
    // inside a run of one non-ACGT letter (GRCh38's N runs) that covers every window of the
    // thread's 32 positions, all 32 start homopolymer B k-mers with the same (canonical) prefix
    const bool run = (s_bad[g] >> 31) != 0 && s_dol[g] == 0 && (k < 2 || window_clear(s_dol, p0 + 32, k - 1)) &&
                     s_diff[g] == 0 && (k < 3 || window_clear(s_diff, p0 + 32, k - 2)) && P0 + p0 + 31 < L;
    if (run) {
        bool keep = true;
        if (ranged) {
            const uint32_t p4 = b_prefix(sba, P0 + p0, k, true, canonical, s_lut4, s_comp, pns);
            keep = p4 >= p4_lo && p4 < p4_hi;
        }
        if (keep) mh = 0xFFFFFFFFu;
    } else if (s_bad[g] | s_bad[g + 1] | s_bad[g + 2]) {  // a non-ACGT byte nearby
        for (int j = 0; j < 32; ++j) {
            const uint32_t p = p0 + j;
            bool f = P0 + p < L && window_clear(s_dol, p, k) && !window_clear(s_bad, p, k);
            if (!f) continue;
            const bool hp = k == 1 || window_clear(s_diff, p, k - 1);
            if (ranged) {
                const uint32_t p4 = b_prefix(sba, P0 + p, k, hp, canonical, s_lut4, s_comp, pns);
                if (p4 < p4_lo || p4 >= p4_hi) continue;
            }
            if (hp) mh |= 1u << j;
            else mr |= 1u << j;
        }
    }
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t cr = (uint32_t)__popc(mr), ch = (uint32_t)__popc(mh), ir = cr, ih = ch;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t yr = __shfl_up(ir, o), yh = __shfl_up(ih, o);
        if (lane >= o) {
            ir += yr;
            ih += yh;
        }
    }
    if (lane == 63) {
        s_w[0][wave] = ir;
        s_w[1][wave] = ih;
    }
    __syncthreads();
    if (!STORE) {
        if (threadIdx.x == 0) {
            cnt_r[blockIdx.x] = s_w[0][0] + s_w[0][1] + s_w[0][2] + s_w[0][3];
            cnt_h[blockIdx.x] = s_w[1][0] + s_w[1][1] + s_w[1][2] + s_w[1][3];
        }
        return;
    }
    uint32_t orr = off_r[blockIdx.x] + ir - cr, oh = off_h[blockIdx.x] + ih - ch;
    for (uint32_t w = 0; w < wave; ++w) {
        orr += s_w[0][w];
        oh += s_w[1][w];
    }
    for (uint32_t m = mr; m; m &= m - 1) out_r[orr++] = (uint32_t)(P0 + p0 + __ffs(m) - 1);
    for (uint32_t m = mh; m; m &= m - 1) out_h[oh++] = (uint32_t)(P0 + p0 + __ffs(m) - 1);
}

// homopolymer k-mers by (canonical) letter: counts per letter; flags of one letter
__device__ __forceinline__ uint32_t homo_letter(const uint8_t *sba, uint32_t p, int canonical, const uint8_t *comp) {
    const uint32_t c = sba[p];
    return canonical ? min(c, (uint32_t)comp[c]) : c;
}

__global__ __launch_bounds__(256) void homo_count_kernel(const uint8_t *__restrict__ sba,
                                                         const uint32_t *__restrict__ hs, uint64_t n, int canonical,
                                                         uint32_t *__restrict__ counts) {
    __shared__ uint32_t s_c[256];
    __shared__ uint8_t s_comp[256];
    s_c[threadIdx.x] = 0;
    s_comp[threadIdx.x] = c_comp_split[threadIdx.x];
    __syncthreads();
    // the starts come in start order, so a wave mostly sees one letter (an N run): one LDS add per
    // wave then, not 64 to the same address
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const uint32_t l = homo_letter(sba, hs[i], canonical, s_comp);
        const uint32_t l0 = __builtin_amdgcn_readfirstlane(l);
        const uint64_t act = __ballot(1), same = __ballot(l == l0);
        if (same == act) {
            if ((threadIdx.x & 63) == (uint32_t)(__ffsll((long long)act) - 1)) atomicAdd(&s_c[l0], (uint32_t)__popcll(act));
        } else {
            atomicAdd(&s_c[l], 1u);
        }
    }
    __syncthreads();
    if (s_c[threadIdx.x]) atomicAdd(&counts[threadIdx.x], s_c[threadIdx.x]);
}

__global__ __launch_bounds__(256) void homo_flags_kernel(const uint8_t *__restrict__ sba,
                                                         const uint32_t *__restrict__ hs, uint64_t n, int canonical,
                                                         uint32_t letter, uint8_t *__restrict__ f) {
    __shared__ uint8_t s_comp[256];
    s_comp[threadIdx.x] = c_comp_split[threadIdx.x];
    __syncthreads();
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
        f[i] = homo_letter(sba, hs[i], canonical, s_comp) == letter ? 1 : 0;
}

__global__ __launch_bounds__(256) void gather_u32_kernel(const uint32_t *__restrict__ src,
                                                         const uint32_t *__restrict__ idx, uint64_t n,
                                                         uint32_t *__restrict__ dst) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) dst[i] = src[idx[i]];
}

// ---------------------------------------------------------------------------------------------
// key-range shards with position-sharded class-B selection (gk_shard_class_b)
// ---------------------------------------------------------------------------------------------
// Homopolymer starts (in start order) as runs: a run continues while the starts are consecutive
// and the (canonical) letter stays the same
__global__ __launch_bounds__(256) void homo_run_heads_kernel(const uint8_t *__restrict__ sba,
                                                             const uint32_t *__restrict__ hs, uint64_t n, int canonical,
                                                             uint8_t *__restrict__ f) {
    __shared__ uint8_t s_comp[256];
    s_comp[threadIdx.x] = c_comp_split[threadIdx.x];
    __syncthreads();
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const uint32_t p = hs[i];
        f[i] = (i == 0 || hs[i - 1] + 1 != p ||
                homo_letter(sba, hs[i - 1], canonical, s_comp) != homo_letter(sba, p, canonical, s_comp)) ? 1 : 0;
    }
}

// runs[3 g .. 3 g + 2] = (first start, number of starts, canonical letter)
__global__ __launch_bounds__(256) void homo_runs_kernel(const uint8_t *__restrict__ sba, const uint32_t *__restrict__ hs,
                                                        uint64_t n, const uint32_t *__restrict__ heads, uint64_t G,
                                                        int canonical, uint32_t *__restrict__ runs) {
    __shared__ uint8_t s_comp[256];
    s_comp[threadIdx.x] = c_comp_split[threadIdx.x];
    __syncthreads();
    for (uint64_t g = blockIdx.x * 256ull + threadIdx.x; g < G; g += (uint64_t)gridDim.x * 256) {
        const uint32_t p = hs[heads[g]];
        runs[3 * g] = p;
        runs[3 * g + 1] = (uint32_t)((g + 1 < G ? heads[g + 1] : n) - heads[g]);
        runs[3 * g + 2] = homo_letter(sba, p, canonical, s_comp);
    }
}

// ownership bin of each non-homopolymer B k-mer: the largest digit d with prefix(d) <= its prefix
// (prefix(d) = bins[d], ascending), counted into hist
__global__ __launch_bounds__(256) void b_bin_kernel(const uint8_t *__restrict__ sba, const uint32_t *__restrict__ st,
                                                    uint64_t n, int k, int canonical, int pns,
                                                    const uint32_t *__restrict__ bins, uint32_t nbins,
                                                    uint32_t *__restrict__ hist) {
    __shared__ uint8_t s_lut4[256], s_comp[256];
    s_lut4[threadIdx.x] = c_code4_split[threadIdx.x];
    s_comp[threadIdx.x] = c_comp_split[threadIdx.x];
    __syncthreads();
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const uint32_t x = b_prefix(sba, st[i], k, false, canonical, s_lut4, s_comp, pns);
        uint32_t lo = 0, hi = nbins;  // first bin with bins[d] > x
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (bins[mid] <= x) lo = mid + 1;
            else hi = mid;
        }
        atomicAdd(&hist[lo - 1], 1u);  // bins[0] == 0 <= x
    }
}

// keep flags of gathered non-homopolymer B starts: (canonical) prefix in [p4_lo, p4_hi)
__global__ __launch_bounds__(256) void b_keep_kernel(const uint8_t *__restrict__ sba, const uint32_t *__restrict__ st,
                                                     uint64_t n, int k, int canonical, int pns, uint32_t p4_lo,
                                                     uint32_t p4_hi, uint8_t *__restrict__ f) {
    __shared__ uint8_t s_lut4[256], s_comp[256];
    s_lut4[threadIdx.x] = c_code4_split[threadIdx.x];
    s_comp[threadIdx.x] = c_comp_split[threadIdx.x];
    __syncthreads();
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const uint32_t x = b_prefix(sba, st[i], k, false, canonical, s_lut4, s_comp, pns);
        f[i] = (x >= p4_lo && x < p4_hi) ? 1 : 0;
    }
}

// the owned homopolymer runs expanded into starts: run r = (first start, output offset)
__global__ __launch_bounds__(256) void expand_runs_kernel(const uint32_t *__restrict__ rs, const uint64_t *__restrict__ ro,
                                                          uint32_t nr, uint64_t n, uint32_t *__restrict__ out) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        uint32_t lo = 0, hi = nr;  // last run with ro[r] <= i
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (ro[mid] <= i) lo = mid;
            else hi = mid;
        }
        out[i] = rs[lo] + (uint32_t)(i - ro[lo]);
    }
}

// ---------------------------------------------------------------------------------------------
// group heads of the sorted B keys (W words, word-major)
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void key_heads_kernel(const uint64_t *__restrict__ keys, uint64_t n, int W,
                                                        uint8_t *__restrict__ heads) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        bool h = i == 0;
        for (int w = 0; w < W && !h; ++w) h = keys[(uint64_t)w * n + i] != keys[(uint64_t)w * n + i - 1];
        heads[i] = h ? 1 : 0;
    }
}

// ---------------------------------------------------------------------------------------------
// merge
// ---------------------------------------------------------------------------------------------
// sign of (k-mer at a) - (k-mer at b), canonical forms if canonical, in 4-bit codes (the
// reference's byte order; ACGT maps into them too)
__device__ __forceinline__ int kmer_cmp(const uint8_t *sba, uint32_t a, uint32_t b, int k, int canonical,
                                        const uint8_t *lut4) {
    const uint8_t *pa = sba + a, *pb = sba + b;
    const bool ra = canonical && canon_is_rc<4>(pa, k, lut4);
    const bool rb = canonical && canon_is_rc<4>(pb, k, lut4);
    for (int t = 0; t < k; ++t) {
        const uint32_t x = canon_sym<4>(pa, k, t, ra, lut4), y = canon_sym<4>(pb, k, t, rb, lut4);
        if (x != y) return x < y ? -1 : 1;
    }
    return 0;
}

// pos[g] = number of A k-mers smaller than B group g (lower bound over the sorted A starts)
__global__ __launch_bounds__(256) void b_group_pos_kernel(const uint8_t *__restrict__ sba, int k, int canonical,
                                                          const uint32_t *__restrict__ a_starts, uint64_t nA,
                                                          const uint32_t *__restrict__ b_starts,
                                                          const uint32_t *__restrict__ g_first, uint64_t G,
                                                          uint32_t *__restrict__ pos) {
    __shared__ uint8_t s_lut4[256];
    s_lut4[threadIdx.x] = c_code4_split[threadIdx.x];
    __syncthreads();
    for (uint64_t g = blockIdx.x * 256ull + threadIdx.x; g < G; g += (uint64_t)gridDim.x * 256) {
        const uint32_t sb = b_starts[g_first[g]];
        uint64_t lo = 0, hi = nA;
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            if (kmer_cmp(sba, a_starts[mid], sb, k, canonical, s_lut4) < 0) lo = mid + 1;
            else hi = mid;
        }
        pos[g] = (uint32_t)lo;
    }
}

// A element i goes to i + (B elements of the groups with pos <= i); it starts a group if its A
// predecessor does not share its k-mer or a B group lands right before it.  One workgroup per
// 4096 A elements: the group positions are sorted and there are few of them (thousands against
// billions of A elements), so almost every workgroup sees none inside its range and moves its
// elements by one constant shift -- a streaming copy; the rest search only the few positions
// inside their range.
constexpr int kMT = 256, kMI = 16, kMTile = kMT * kMI;

// number of entries of the ascending v[lo, hi) that are < x (lower) or <= x (upper), plus lo
__device__ __forceinline__ uint64_t bound_in(const uint32_t *v, uint64_t lo, uint64_t hi, uint64_t x, bool upper) {
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (upper ? (uint64_t)v[mid] <= x : (uint64_t)v[mid] < x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// With keys (W > 0): the A k-mers' final 2-bit keys (a_keys) are expanded to the W-word 4-bit keys
// of the merged order (out_keys, word-major with stride n).
template <int W>
__device__ __forceinline__ void put_key4(const uint64_t *a_keys, uint64_t i, int k, uint64_t *out_keys, uint64_t n,
                                         uint64_t o) {
    uint64_t w[W];
    expand4_key<W>(a_keys[i], k, w);
#pragma unroll
    for (int q = 0; q < W; ++q) out_keys[(uint64_t)q * n + o] = w[q];
}

// k > 32 (round 5, C5): the A k-mer at start s has no one-word MSD key to expand; its 2k-bit key is
// read from the 2-bit packed sequence (split_pack_kernel: 32 positions per word, position 0 on top)
// -- three consecutive words from two aligned 16-byte loads -- made canonical when asked and expanded to
// its W 4-bit words at the merged position.  The merge moves every A start anyway, so this replaces
// the separate key pass over the merged order (a 16-B row per position of the sequence, written in
// full, then one random row per k-mer: 11.5 + 85 ms at C5) with the random read alone.
// The three words come from two aligned 16-byte loads (words 2 j .. 2 j + 3, j = g / 2), issued by
// the caller for several k-mers before any is used (loads in flight, as the row gather of round 3).
#ifndef GKM_MERGE_PK16
#define GKM_MERGE_PK16 0
#endif
__device__ __forceinline__ void packed_pair_load(const uint64_t *__restrict__ pk, uint32_t s, uint4 &a, uint4 &b) {
    if (GKM_MERGE_PK16) {  // (A/B: two aligned 16-byte loads -- 97.5 against 86-87 ms of C5 merge)
        const uint4 *p4 = reinterpret_cast<const uint4 *>(pk) + ((s >> 5) >> 1);
        a = p4[0];
        b = p4[1];
        return;
    }
    // the three words g .. g + 2, placed where put_key4_packed looks for them
    const uint64_t g = s >> 5;
    const uint64_t x0 = pk[g], x1 = pk[g + 1], x2 = pk[g + 2];
    const bool odd = (g & 1) != 0;
    const uint64_t w0 = odd ? 0 : x0, w1 = odd ? x0 : x1, w2 = odd ? x1 : x2, w3 = odd ? x2 : 0;
    a = make_uint4((uint32_t)w0, (uint32_t)(w0 >> 32), (uint32_t)w1, (uint32_t)(w1 >> 32));
    b = make_uint4((uint32_t)w2, (uint32_t)(w2 >> 32), (uint32_t)w3, (uint32_t)(w3 >> 32));
}

template <int W>
__device__ __forceinline__ void put_key4_packed(const uint4 &qa, const uint4 &qb, uint32_t s, int k, bool canonical,
                                                uint64_t *out_keys, uint64_t n, uint64_t o) {
    const uint64_t w0 = ((uint64_t)qa.y << 32) | qa.x, w1 = ((uint64_t)qa.w << 32) | qa.z;
    const uint64_t w2 = ((uint64_t)qb.y << 32) | qb.x, w3 = ((uint64_t)qb.w << 32) | qb.z;
    const bool odd = ((s >> 5) & 1u) != 0;
    const uint64_t c0 = odd ? w1 : w0, c1 = odd ? w2 : w1, c2 = odd ? w3 : w2;
    const int sh = 2 * (int)(s & 31u);
    uint64_t hi = sh ? (c0 << sh) | (c1 >> (64 - sh)) : c0;  // symbols s .. s + 63, left-aligned
    uint64_t lo = sh ? (c1 << sh) | (c2 >> (64 - sh)) : c1;
    const int r = 128 - 2 * k;  // right-align the k symbols (33 <= k <= 63: 2 <= r <= 62)
    lo = (lo >> r) | (hi << (64 - r));
    hi >>= r;
    if (canonical) canon2(k, hi, lo);
    uint64_t w[W];
    key_from_2bit<W, 4>(hi, lo, k, w);
#pragma unroll
    for (int q = 0; q < W; ++q) out_keys[(uint64_t)q * n + o] = w[q];
}

// 2-bit codes of the sequence, 32 positions per word (bytes other than A/C/G/T get some code: only
// ACGT-only windows are read back)
__global__ __launch_bounds__(256) void split_pack_kernel(const uint8_t *__restrict__ sba, uint64_t nwords,
                                                         uint64_t *__restrict__ code) {
    for (uint64_t g = blockIdx.x * 256ull + threadIdx.x; g < nwords; g += (uint64_t)gridDim.x * 256) {
        const uint64_t *p = reinterpret_cast<const uint64_t *>(sba + 32 * g);
        const uint64_t a = p[0], b = p[1], c = p[2], d = p[3];
        code[g] = ((uint64_t)pack2_8e(a) << 48) | ((uint64_t)pack2_8e(b) << 32) | ((uint64_t)pack2_8e(c) << 16) |
                  pack2_8e(d);
    }
}

// PK: the A keys come from the packed sequence (put_key4_packed), not from a_keys
template <int W, bool PK = false>
__global__ __launch_bounds__(kMT) void merge_a_kernel(const uint32_t *__restrict__ a_starts,
                                                      const uint8_t *__restrict__ a_heads, uint64_t nA,
                                                      const uint32_t *__restrict__ pos,
                                                      const uint32_t *__restrict__ g_first, uint64_t G, uint64_t nB,
                                                      uint32_t *__restrict__ out, uint8_t *__restrict__ out_heads,
                                                      const uint64_t *__restrict__ a_keys, int k,
                                                      uint64_t *__restrict__ out_keys,
                                                      const uint64_t *__restrict__ pk = nullptr, int canonical = 0) {
    __shared__ uint64_t s_g[3];  // ub(i0), lb(i0), groups with pos < i1
    const uint64_t i0 = (uint64_t)blockIdx.x * kMTile;
    const uint64_t i1 = min(i0 + kMTile, nA);
    if (threadIdx.x == 0) {
        s_g[0] = bound_in(pos, 0, G, i0, true);
        s_g[1] = bound_in(pos, 0, s_g[0], i0, false);
        s_g[2] = bound_in(pos, s_g[0], G, i1, false);
    }
    __syncthreads();
    const uint64_t g0 = s_g[0], lb0 = s_g[1], g1 = s_g[2];
    if (g1 == g0) {  // no B group lands inside (i0, i1): one shift for the whole range
        const uint64_t shift = g0 < G ? g_first[g0] : nB;
        if (PK) {  // kU k-mers per thread at a time: their starts, then all their sequence reads
#ifndef GKM_MERGE_U
#define GKM_MERGE_U 2  // (A/B at C5, profiles/r5/ab_merge_keys.txt: 1 / 2 / 4 -> 85.9-86.4 / 85.5 / 86.9-87.4 ms)
#endif
            constexpr int kU = GKM_MERGE_U;
            for (uint64_t i = i0 + threadIdx.x; i < i1; i += kMT * kU) {
                uint32_t st[kU];
                uint4 qa[kU], qb[kU];
#pragma unroll
                for (int u = 0; u < kU; ++u) st[u] = i + u * kMT < i1 ? a_starts[i + u * kMT] : a_starts[i];
#pragma unroll
                for (int u = 0; u < kU; ++u) packed_pair_load(pk, st[u], qa[u], qb[u]);
#pragma unroll
                for (int u = 0; u < kU; ++u) {
                    const uint64_t j = i + u * kMT;
                    if (j >= i1) continue;
                    out[j + shift] = st[u];
                    out_heads[j + shift] = (a_heads[j] || (j == i0 && g0 > lb0)) ? 1 : 0;
                    put_key4_packed<(W ? W : 1)>(qa[u], qb[u], st[u], k, canonical != 0, out_keys, nA + nB, j + shift);
                }
            }
            return;
        }
        for (uint64_t i = i0 + threadIdx.x; i < i1; i += kMT) {
            out[i + shift] = a_starts[i];
            out_heads[i + shift] = (a_heads[i] || (i == i0 && g0 > lb0)) ? 1 : 0;
            if (W) put_key4<(W ? W : 1)>(a_keys, i, k, out_keys, nA + nB, i + shift);
        }
        return;
    }
    for (uint64_t i = i0 + threadIdx.x; i < i1; i += kMT) {
        const uint64_t ub = bound_in(pos, g0, g1, i, true);
        const uint64_t lb = i == i0 ? lb0 : bound_in(pos, g0, ub, i, false);
        const uint64_t shift = ub < G ? g_first[ub] : nB;
        const uint32_t st = a_starts[i];
        out[i + shift] = st;
        out_heads[i + shift] = (a_heads[i] || ub > lb) ? 1 : 0;
        if (PK) {
            uint4 qa, qb;
            packed_pair_load(pk, st, qa, qb);
            put_key4_packed<(W ? W : 1)>(qa, qb, st, k, canonical != 0, out_keys, nA + nB, i + shift);
        } else if (W) {
            put_key4<(W ? W : 1)>(a_keys, i, k, out_keys, nA + nB, i + shift);
        }
    }
}

// B element j of group g goes to j + pos[g]; per 4096 B elements, the groups they span
// With keys (W > 0): the B k-mers' 4-bit keys (b_keys, word-major with stride nB) go along.
template <int W>
__global__ __launch_bounds__(kMT) void merge_b_kernel(const uint32_t *__restrict__ b_starts,
                                                      const uint8_t *__restrict__ b_heads, uint64_t nB,
                                                      const uint32_t *__restrict__ pos,
                                                      const uint32_t *__restrict__ g_first, uint64_t G,
                                                      uint32_t *__restrict__ out, uint8_t *__restrict__ out_heads,
                                                      const uint64_t *__restrict__ b_keys, uint64_t n,
                                                      uint64_t *__restrict__ out_keys) {
    __shared__ uint64_t s_g[2];  // group of j0, groups starting at or before j1 - 1
    const uint64_t j0 = (uint64_t)blockIdx.x * kMTile;
    const uint64_t j1 = min(j0 + kMTile, nB);
    if (threadIdx.x == 0) {
        s_g[0] = bound_in(g_first, 0, G, j0, true) - 1;
        s_g[1] = bound_in(g_first, s_g[0], G, j1 - 1, true);
    }
    __syncthreads();
    const uint64_t ga = s_g[0], gb = s_g[1];
    for (uint64_t j = j0 + threadIdx.x; j < j1; j += kMT) {
        const uint64_t g = gb == ga + 1 ? ga : bound_in(g_first, ga, gb, j, true) - 1;
        out[j + pos[g]] = b_starts[j];
        out_heads[j + pos[g]] = b_heads[j];
#pragma unroll
        for (int q = 0; q < W; ++q) out_keys[(uint64_t)q * n + j + pos[g]] = b_keys[(uint64_t)q * nB + j];
    }
}

// keys of the A k-mers when no B k-mer exists: the 2-bit keys expanded in place of the merge
template <int W>
__global__ __launch_bounds__(256) void expand_keys_kernel(const uint64_t *__restrict__ a_keys, uint64_t n, int k,
                                                          uint64_t *__restrict__ out_keys) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
        put_key4<W>(a_keys, i, k, out_keys, n, i);
}

__global__ __launch_bounds__(256) void fill_u64_kernel(uint64_t *__restrict__ p, uint64_t n, uint64_t v) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) p[i] = v;
}

static unsigned grid_of_n(uint64_t n) { return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((n + 255) / 256, 16384)); }

static const char kAlpha4[] = "$ABCDGHKMNRSTVWY";  // 4-bit code = index

static uint32_t letter_code4(uint32_t ch) {
    const char *at = ch ? std::strchr(kAlpha4, (int)ch) : nullptr;
    return at ? (uint32_t)(at - kAlpha4) : 0;
}

// the pns-symbol 4-bit prefix of a homopolymer k-mer of (canonical) letter ch
static uint32_t homo_prefix(uint32_t ch, int pns) {
    uint32_t v = 0;
    for (int t = 0; t < pns; ++t) v = (v << 4) | letter_code4(ch);
    return v;
}

// Class-B k-mers starting in [lo, hi) for key-range shards (gk_shard_class_b): the non-homopolymer
// starts and the homopolymer runs (first start, count, canonical letter) to the host, in start
// order, and their ownership bins added to hist (bins[d] = the pns-symbol prefix of digit d's
// smallest k-mer, ascending; a homopolymer k-mer weighs homo_w16 / 16 of a k-mer)
int split_shard_class_b(gk_ctx *c, const KeySpec &ks, uint64_t lo, uint64_t hi, const std::vector<uint32_t> &bins,
                        int pns, uint32_t homo_w16, uint64_t *hist, std::vector<uint32_t> *rest,
                        std::vector<uint32_t> *runs) {
    rest->clear();
    runs->clear();
    hi = std::min<uint64_t>(hi, c->sba_len);
    if (hi <= lo) return GK_OK;
    if (lo % 32) return fail(c, GK_E_ARG, "shard lo must be a multiple of 32");
    GK_TRY_HIP(c, split_tables());
    const int k = ks.symbols;
    const unsigned ftiles = (unsigned)((hi - lo + kFlagTile - 1) / kFlagTile);
    uint32_t *cr, *chh, *orr, *ohh, *rs, *hs;
    GK_TRY_HIP(c, scratch(c, "split_cnt_r", ftiles + 1, &cr));
    GK_TRY_HIP(c, scratch(c, "split_cnt_h", ftiles + 1, &chh));
    GK_TRY_HIP(c, scratch(c, "split_off_r", ftiles + 1, &orr));
    GK_TRY_HIP(c, scratch(c, "split_off_h", ftiles + 1, &ohh));
    int slot;
    timer_begin(c, "split_b_select", &slot);
    const uint32_t all = 1u << (4 * 4);
    hipLaunchKernelGGL(class_b_select_kernel<false>, dim3(ftiles), dim3(256), 0, c->stream, c->sba, lo, hi, k,
                       ks.canonical, 0u, all, 4, cr, chh, nullptr, nullptr, nullptr, nullptr);
    GK_TRY_HIP(c, hipGetLastError());
    uint64_t nR = 0, nH = 0;
    GK_TRY_HIP(c, scan_u32_exclusive_pair(c, cr, orr, chh, ohh, ftiles, &nR, &nH));
    GK_TRY_HIP(c, scratch(c, "split_b_st0", nR + 64, &rs));
    GK_TRY_HIP(c, scratch(c, "split_h_st", nH + 64, &hs));
    hipLaunchKernelGGL(class_b_select_kernel<true>, dim3(ftiles), dim3(256), 0, c->stream, c->sba, lo, hi, k,
                       ks.canonical, 0u, all, 4, cr, chh, orr, ohh, rs, hs);
    GK_TRY_HIP(c, hipGetLastError());
    timer_end(c, slot);
    const uint32_t nbins = (uint32_t)bins.size();
    if (nR > 0) {
        rest->resize(nR);
        GK_TRY_HIP(c, hipMemcpyAsync(rest->data(), rs, 4 * nR, hipMemcpyDeviceToHost, c->stream));
        uint32_t *d_bins, *d_hist;
        GK_TRY_HIP(c, scratch(c, "split_bins", nbins, &d_bins));
        GK_TRY_HIP(c, scratch(c, "split_bhist", nbins, &d_hist));
        GK_TRY_HIP(c, hipMemcpyAsync(d_bins, bins.data(), 4 * nbins, hipMemcpyHostToDevice, c->stream));
        GK_TRY_HIP(c, hipMemsetAsync(d_hist, 0, 4 * nbins, c->stream));
        hipLaunchKernelGGL(b_bin_kernel, dim3(grid_of_n(nR)), dim3(256), 0, c->stream, c->sba, rs, nR, k, ks.canonical,
                           pns, d_bins, nbins, d_hist);
        GK_TRY_HIP(c, hipGetLastError());
        std::vector<uint32_t> bh(nbins);
        GK_TRY_HIP(c, hipMemcpyAsync(bh.data(), d_hist, 4 * nbins, hipMemcpyDeviceToHost, c->stream));
        GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
        for (uint32_t d = 0; d < nbins; ++d) hist[d] += bh[d];
    }
    if (nH > 0) {
        uint8_t *f;
        uint32_t *heads, *d_runs;
        GK_TRY_HIP(c, scratch(c, "split_h_lf", nH + 64, &f));
        GK_TRY_HIP(c, scratch(c, "split_h_idx", nH + 64, &heads));
        hipLaunchKernelGGL(homo_run_heads_kernel, dim3(grid_of_n(nH)), dim3(256), 0, c->stream, c->sba, hs, nH,
                           ks.canonical, f);
        GK_TRY_HIP(c, hipGetLastError());
        uint64_t G = 0;
        GK_TRY_HIP(c, select_flags(c, f, nH, heads, &G));
        GK_TRY_HIP(c, scratch(c, "split_runs", 3 * G + 64, &d_runs));
        hipLaunchKernelGGL(homo_runs_kernel, dim3(grid_of_n(G)), dim3(256), 0, c->stream, c->sba, hs, nH, heads, G,
                           ks.canonical, d_runs);
        GK_TRY_HIP(c, hipGetLastError());
        runs->resize(3 * G);
        GK_TRY_HIP(c, hipMemcpyAsync(runs->data(), d_runs, 12 * G, hipMemcpyDeviceToHost, c->stream));
        GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
        for (uint64_t g = 0; g < G; ++g) {
            const uint32_t x = homo_prefix((*runs)[3 * g + 2], pns);
            const uint64_t d = (uint64_t)(std::upper_bound(bins.begin(), bins.end(), x) - bins.begin()) - 1;
            hist[d] += ((uint64_t)(*runs)[3 * g + 1] * homo_w16 + 15) / 16;
        }
    }
    GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
    return GK_OK;
}

// ---------------------------------------------------------------------------------------------
// driver
// ---------------------------------------------------------------------------------------------
int split_sort(gk_ctx *c, const KeySpec &ks, bool *used, const SplitRange *rg) {
    *used = false;
    const uint64_t L = c->sba_len;
    const uint64_t n = rg ? L : c->n;  // key-range shards: the k-mer count is not known yet (<= L)
    const int k = ks.symbols;
    if (k > 64 || ks.bits != 4 || ks.lenbits || ks.symbols != ks.min_len) return GK_OK;
    if (rg && k < rg->pns) return fail(c, GK_E_ARG, "split: key-range shards need k >= the prefix length");
    GK_TRY_HIP(c, split_tables());
    c->split_keys_final = false;
    // final keys: the sorted order leaves with its W-word 4-bit keys -- B's from their own sort, A's
    // written by the merge: expanded from the one-word 2-bit MSD keys (k <= 32), or read from a
    // 2-bit packed copy of the sequence (k <= 63, round 5; GKM_NO_MERGE_KEYS=1: the re-encode after
    // the sort instead) -- and needs no re-encode
    const bool a_packed = k > 32 && k <= 63 && !opt("GKM_NO_MERGE_KEYS");
    const int WK = k <= 32 || a_packed ? ks.words : 0;
    int slot;
    // 1. class B starts: homopolymers (one letter k times) apart from the rest
    uint32_t *b_st[2], *h_st;
    const unsigned ftiles = (unsigned)((L + kFlagTile - 1) / kFlagTile);
    uint32_t *cr, *chh, *orr, *ohh;
    GK_TRY_HIP(c, scratch(c, "split_cnt_r", ftiles + 1, &cr));
    GK_TRY_HIP(c, scratch(c, "split_cnt_h", ftiles + 1, &chh));
    GK_TRY_HIP(c, scratch(c, "split_off_r", ftiles + 1, &orr));
    GK_TRY_HIP(c, scratch(c, "split_off_h", ftiles + 1, &ohh));
    const int pns = rg ? rg->pns : 4;
    const uint32_t p4_lo = rg ? rg->p4_lo : 0u, p4_hi = rg ? rg->p4_hi : (1u << (4 * pns));
    uint64_t nR = 0, nH = 0;
    if (rg && rg->given) {
        // 1'. the B k-mers of every rank's position share, gathered (gk_shard_class_b): keep the
        // non-homopolymer ones whose prefix is in the rank's interval, expand the owned runs
        timer_begin(c, "split_b_given", &slot);
        uint32_t *g_rest = nullptr;
        uint8_t *f;
        if (rg->n_rest > 0) {
            GK_TRY_HIP(c, scratch(c, "split_g_rest", rg->n_rest + 64, &g_rest));
            GK_TRY_HIP(c, scratch(c, "split_h_lf", rg->n_rest + 64, &f));
            GK_TRY_HIP(c, scratch(c, "split_h_idx", rg->n_rest + 64, &b_st[1]));
            GK_TRY_HIP(c, hipMemcpyAsync(g_rest, rg->rest, 4 * rg->n_rest, hipMemcpyHostToDevice, c->stream));
            hipLaunchKernelGGL(b_keep_kernel, dim3(grid_of_n(rg->n_rest)), dim3(256), 0, c->stream, c->sba, g_rest,
                               rg->n_rest, k, ks.canonical, pns, p4_lo, p4_hi, f);
            GK_TRY_HIP(c, hipGetLastError());
            GK_TRY_HIP(c, select_flags(c, f, rg->n_rest, b_st[1], &nR));
        }
        std::vector<uint32_t> own_s;
        std::vector<uint64_t> own_o;
        for (uint64_t g = 0; g < rg->n_runs; ++g) {
            const uint32_t x = homo_prefix(rg->runs[3 * g + 2], pns);
            if (x < p4_lo || x >= p4_hi) continue;
            own_s.push_back(rg->runs[3 * g]);
            own_o.push_back(nH);
            nH += rg->runs[3 * g + 1];
        }
        GK_TRY_HIP(c, scratch(c, "split_b_st0", nR + 64, &b_st[0]));
        GK_TRY_HIP(c, scratch(c, "split_h_st", nH + 64, &h_st));
        if (nR > 0) {
            hipLaunchKernelGGL(gather_u32_kernel, dim3(grid_of_n(nR)), dim3(256), 0, c->stream, g_rest, b_st[1], nR,
                               b_st[0]);
            GK_TRY_HIP(c, hipGetLastError());
        }
        if (nH > 0) {
            uint32_t *d_rs;
            uint64_t *d_ro;
            GK_TRY_HIP(c, scratch(c, "split_own_rs", own_s.size() + 1, &d_rs));
            GK_TRY_HIP(c, scratch(c, "split_own_ro", own_o.size() + 1, &d_ro));
            GK_TRY_HIP(c, hipMemcpyAsync(d_rs, own_s.data(), 4 * own_s.size(), hipMemcpyHostToDevice, c->stream));
            GK_TRY_HIP(c, hipMemcpyAsync(d_ro, own_o.data(), 8 * own_o.size(), hipMemcpyHostToDevice, c->stream));
            hipLaunchKernelGGL(expand_runs_kernel, dim3(grid_of_n(nH)), dim3(256), 0, c->stream, d_rs, d_ro,
                               (uint32_t)own_s.size(), nH, h_st);
            GK_TRY_HIP(c, hipGetLastError());
            GK_TRY_HIP(c, hipStreamSynchronize(c->stream));  // own_s / own_o leave scope
        }
        timer_end(c, slot);
    } else {
    timer_begin(c, "split_b_select", &slot);
    hipLaunchKernelGGL(class_b_select_kernel<false>, dim3(ftiles), dim3(256), 0, c->stream, c->sba, 0ull, L, k,
                       ks.canonical, p4_lo, p4_hi, pns, cr, chh, nullptr, nullptr, nullptr, nullptr);
    GK_TRY_HIP(c, hipGetLastError());
    GK_TRY_HIP(c, scan_u32_exclusive_pair(c, cr, orr, chh, ohh, ftiles, &nR, &nH));
    GK_TRY_HIP(c, scratch(c, "split_b_st0", nR + 64, &b_st[0]));
    GK_TRY_HIP(c, scratch(c, "split_h_st", nH + 64, &h_st));
    hipLaunchKernelGGL(class_b_select_kernel<true>, dim3(ftiles), dim3(256), 0, c->stream, c->sba, 0ull, L, k,
                       ks.canonical, p4_lo, p4_hi, pns, cr, chh, orr, ohh, b_st[0], h_st);
    GK_TRY_HIP(c, hipGetLastError());
    timer_end(c, slot);
    }
    const uint64_t nB = nR + nH;
    if (nB > n) return fail(c, GK_E_HIP, "split: more class-B k-mers than k-mers");
    if (!rg && nB * 4 > n) return GK_OK;  // mostly non-ACGT k-mers: the plain 4-bit MSD is the better sort
    *used = true;
    uint64_t nA = rg ? 0 : n - nB;

    // 2. sort the non-homopolymer B k-mers: 4-bit keys, LSD (on a swapped-in context of nR elements)
    uint64_t *b_k[2];
    uint8_t *b_heads;
    int bres = 0;
    GK_TRY_HIP(c, scratch(c, "split_b_st1", nB + 64, &b_st[1]));
    if (nH > 0 && nR + 64 < nB + 64) {  // b_st[0] also receives the assembled B order (bres flips)
        uint32_t *grown;
        GK_TRY_HIP(c, scratch(c, "split_b_st0g", nB + 64, &grown));
        GK_TRY_HIP(c, hipMemcpyAsync(grown, b_st[0], 4 * nR, hipMemcpyDeviceToDevice, c->stream));
        b_st[0] = grown;
    }
    GK_TRY_HIP(c, scratch(c, "split_b_heads", nB + 64, &b_heads));
    if (nR > 0) {
        const int W = ks.words;
        if (rg) {  // key-range shards: nothing sized the radix state for this context yet
            const uint64_t sv_n = c->n;
            c->n = 0;  // (no start array to keep)
            const int re = ensure_elems(c, std::max<uint64_t>(c->elem_cap, nR + 1), 1);
            c->n = sv_n;
            if (re != GK_OK) return re;
        }
        GK_TRY_HIP(c, scratch(c, "split_b_k0", W * (nR + 64), &b_k[0]));
        GK_TRY_HIP(c, scratch(c, "split_b_k1", W * (nR + 64), &b_k[1]));
        const uint64_t sv_n = c->n;
        uint64_t *sv_k[2] = {c->keys[0], c->keys[1]};
        uint32_t *sv_v[2] = {c->vals[0], c->vals[1]};
        const int sv_cur = c->cur;
        c->n = nR;
        c->keys[0] = b_k[0];
        c->keys[1] = b_k[1];
        c->vals[0] = b_st[0];
        c->vals[1] = b_st[1];
        c->cur = 0;
        timer_begin(c, "split_b_encode", &slot);
        hipError_t e = launch_encode_gather(c, ks, b_st[0], nR, b_k[0]);
        timer_end(c, slot);
        int rc = e == hipSuccess ? radix_sort(c, W, ks.total_bits, false) : GK_E_HIP;
        bres = c->cur;
        c->n = sv_n;
        c->keys[0] = sv_k[0];
        c->keys[1] = sv_k[1];
        c->vals[0] = sv_v[0];
        c->vals[1] = sv_v[1];
        c->cur = sv_cur;
        if (e != hipSuccess) return hip_fail(c, e, "split: encode B");
        if (rc != GK_OK) return rc;
        hipLaunchKernelGGL(key_heads_kernel, dim3(grid_of_n(nR)), dim3(256), 0, c->stream, b_k[bres], nR, W, b_heads);
        GK_TRY_HIP(c, hipGetLastError());
    }
    // B's final keys (word-major, stride nB): the rest's sorted keys, with the homopolymer groups'
    // constant keys spliced in below
    const uint64_t *b_keys = nR > 0 ? b_k[bres] : nullptr;
    uint64_t *bkf = nullptr;
    if (WK && nH > 0) GK_TRY_HIP(c, scratch(c, "split_b_kf", (uint64_t)WK * (nB + 64), &bkf));
    if (nH > 0) {
        // 2b. the homopolymer groups (one per (canonical) letter, members in start order) go into
        // the sorted B run at their insertion points: at most 15 segment copies
        timer_begin(c, "split_b_homo", &slot);
        uint32_t *cnt;
        GK_TRY_HIP(c, scratch(c, "split_h_cnt", 256, &cnt));
        GK_TRY_HIP(c, hipMemsetAsync(cnt, 0, 4 * 256, c->stream));
        hipLaunchKernelGGL(homo_count_kernel, dim3(grid_of_n(nH)), dim3(256), 0, c->stream, c->sba, h_st, nH,
                           ks.canonical, cnt);
        GK_TRY_HIP(c, hipGetLastError());
        std::vector<uint32_t> hc(256);
        GK_TRY_HIP(c, hipMemcpyAsync(hc.data(), cnt, 4 * 256, hipMemcpyDeviceToHost, c->stream));
        GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
        std::vector<uint32_t> letters;  // ascending byte = ascending key of letter^k
        for (int ch = 0; ch < 256; ++ch)
            if (hc[ch]) letters.push_back((uint32_t)ch);
        // groups by letter, in letter order, into grp (stable: h_st is in start order)
        uint32_t *grp = h_st, *tmp_idx, *grp2;
        if (letters.size() > 1) {
            uint8_t *lf;
            GK_TRY_HIP(c, scratch(c, "split_h_lf", nH + 64, &lf));
            GK_TRY_HIP(c, scratch(c, "split_h_idx", nH + 64, &tmp_idx));
            GK_TRY_HIP(c, scratch(c, "split_h_grp", nH + 64, &grp2));
            uint64_t at = 0;
            for (uint32_t ch : letters) {
                hipLaunchKernelGGL(homo_flags_kernel, dim3(grid_of_n(nH)), dim3(256), 0, c->stream, c->sba, h_st, nH,
                                   ks.canonical, ch, lf);
                uint64_t m = 0;
                GK_TRY_HIP(c, select_flags(c, lf, nH, tmp_idx, &m));
                hipLaunchKernelGGL(gather_u32_kernel, dim3(grid_of_n(m)), dim3(256), 0, c->stream, h_st, tmp_idx, m,
                                   grp2 + at);
                GK_TRY_HIP(c, hipGetLastError());
                at += m;
            }
            grp = grp2;
        }
        // insertion points: the number of sorted non-homopolymer B k-mers below each group's k-mer
        std::vector<uint32_t> ins(letters.size(), 0), first(letters.size());
        {
            uint64_t at = 0;
            for (size_t g = 0; g < letters.size(); ++g) {
                first[g] = (uint32_t)at;
                at += hc[letters[g]];
            }
        }
        if (nR > 0) {
            uint32_t *d_first, *d_pos;
            GK_TRY_HIP(c, scratch(c, "split_h_first", letters.size() + 1, &d_first));
            GK_TRY_HIP(c, scratch(c, "split_h_pos", letters.size() + 1, &d_pos));
            GK_TRY_HIP(c, hipMemcpyAsync(d_first, first.data(), 4 * letters.size(), hipMemcpyHostToDevice, c->stream));
            hipLaunchKernelGGL(b_group_pos_kernel, dim3(1), dim3(256), 0, c->stream, c->sba, k, ks.canonical,
                               b_st[bres], nR, grp, d_first, (uint64_t)letters.size(), d_pos);
            GK_TRY_HIP(c, hipGetLastError());
            GK_TRY_HIP(c, hipMemcpyAsync(ins.data(), d_pos, 4 * letters.size(), hipMemcpyDeviceToHost, c->stream));
            GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
        }
        // assemble the B order into the other start buffer (+ heads into a fresh array)
        uint32_t *fst = b_st[bres ^ 1];
        uint8_t *fhd;
        GK_TRY_HIP(c, scratch(c, "split_b_heads2", nB + 64, &fhd));
        uint64_t rcur = 0, out = 0;
        auto copy_rest = [&](uint64_t upto) -> hipError_t {
            const uint64_t m = upto - rcur;
            if (!m) return hipSuccess;
            hipError_t e = hipMemcpyAsync(fst + out, b_st[bres] + rcur, 4 * m, hipMemcpyDeviceToDevice, c->stream);
            if (e == hipSuccess)
                e = hipMemcpyAsync(fhd + out, b_heads + rcur, m, hipMemcpyDeviceToDevice, c->stream);
            for (int q = 0; q < WK && e == hipSuccess; ++q)
                e = hipMemcpyAsync(bkf + (uint64_t)q * nB + out, b_keys + (uint64_t)q * nR + rcur, 8 * m,
                                   hipMemcpyDeviceToDevice, c->stream);
            rcur = upto;
            out += m;
            return e;
        };
        for (size_t g = 0; g < letters.size(); ++g) {
            GK_TRY_HIP(c, copy_rest(ins[g]));
            const uint64_t m = hc[letters[g]];
            GK_TRY_HIP(c, hipMemcpyAsync(fst + out, grp + first[g], 4 * m, hipMemcpyDeviceToDevice, c->stream));
            GK_TRY_HIP(c, hipMemsetAsync(fhd + out, 0, m, c->stream));
            GK_TRY_HIP(c, hipMemsetAsync(fhd + out, 1, 1, c->stream));  // one group: one head
            if (WK) {  // the group's k-mer: its (canonical) letter k times
                const uint64_t c4 = letter_code4(letters[g]);
                for (int q = 0; q < WK; ++q) {  // q: word from the most significant end
                    uint64_t v = 0;
                    const int lo_sym = 16 * (WK - 1 - q);  // nibble index of the word's bit 0
                    for (int j = lo_sym; j < std::min(lo_sym + 16, k); ++j) v |= c4 << (4 * (j - lo_sym));
                    hipLaunchKernelGGL(fill_u64_kernel, dim3(grid_of_n(m)), dim3(256), 0, c->stream,
                                       bkf + (uint64_t)q * nB + out, m, v);
                }
                GK_TRY_HIP(c, hipGetLastError());
            }
            out += m;
        }
        GK_TRY_HIP(c, copy_rest(nR));
        b_heads = fhd;
        bres ^= 1;
        b_keys = bkf;
        timer_end(c, slot);
    }

    // 3. sort A: the 2-bit MSD over the ACGT-only k-mers (its count is checked against nA)
    KeySpec ka = ks;
    ka.bits = 2;
    ka.total_bits = 2 * k;
    ka.words = (ka.total_bits + 63) / 64;
    ka.acgt_only = 1;
    int rc;
    const uint64_t *a_keys = nullptr;  // A's final 2-bit keys (WK, k <= 32)
    c->msd_force_keys = WK > 0 && !a_packed;
    if (rg) {  // the rank's ACGT-only k-mers: select + MSD (gkm_msd.hip); room for the merge after
        rc = msd_sort_range(c, ka, rg->d_lo, rg->d_hi, &nA);
        c->msd_force_keys = false;
        if (rc != GK_OK) return rc;
        c->have_starts = true;
        a_keys = a_packed ? nullptr : c->keys[0];
        if (WK && !a_packed && nA + nB + 1 > c->elem_cap) {  // growing the buffers below does not keep the keys
            uint64_t *ak;
            GK_TRY_HIP(c, scratch(c, "split_a_keys", nA + 64, &ak));
            GK_TRY_HIP(c, hipMemcpyAsync(ak, c->keys[0], 8 * nA, hipMemcpyDeviceToDevice, c->stream));
            a_keys = ak;
        }
        rc = ensure_elems(c, nA + nB + 1, 1);  // keeps vals[0] (nA)
        if (rc != GK_OK) return rc;
        // the merge's output buffer at its final width now, not mid-merge (keys[0] may hold A's
        // keys: it is only regrown on the nA == 0 path below, where they are not used)
        if (WK && a_keys != c->keys[1])
            if (int r = grow_key_buffer(c, 1, WK)) return r;
        c->n = nA + nB;
    } else {
        // both key buffers at the final key width before the A sort (which uses word 0 of each):
        // nothing is freed or re-allocated between the A sort and the merge -- except with a
        // prefetched class-A L0 (gk_sort_hint) in keys[1] / vals[1]: keys[1] grows after the A sort,
        // whose result is in buffer 0 (keys[1] is its scratch by then)
        c->n = nA;
        const bool pre = nA > 0 && prefetch_matches(c, ka);
        c->n = n;
        if (WK) {
            if (!a_packed)
                if (int r = grow_key_buffer(c, 0, WK)) return r;
            if (!pre)
                if (int r = grow_key_buffer(c, 1, WK)) return r;
        }
        c->n = nA;
        rc = nA > 0 ? (pre ? msd_sort_prefetched(c, ka) : msd_sort(c, ka)) : GK_OK;
        c->msd_force_keys = false;
        c->n = n;
        if (rc != GK_OK) return rc;
        if (pre && WK) {
            if (c->cur != 0) return fail(c, GK_E_STATE, "split sort: the prefetched A sort did not end in buffer 0");
            if (int r = grow_key_buffer(c, 1, WK)) return r;
        }
        a_keys = a_packed ? nullptr : c->keys[0];
    }
    if (nA == 0) {  // all B: the B order is the order
        GK_TRY_HIP(c, hipMemcpyAsync(c->vals[0], b_st[bres], 4 * nB, hipMemcpyDeviceToDevice, c->stream));
        uint8_t *hd;
        GK_TRY_HIP(c, scratch(c, "split_heads", n + 64, &hd));
        GK_TRY_HIP(c, hipMemcpyAsync(hd, b_heads, nB, hipMemcpyDeviceToDevice, c->stream));
        if (WK) {  // (the B keys alone: A's packed-sequence path is not involved)
            if (b_keys == c->keys[0]) return fail(c, GK_E_STATE, "split sort: B keys alias the key buffer");
            if (int r = grow_key_buffer(c, 0, WK)) return r;
            GK_TRY_HIP(c, hipMemcpyAsync(c->keys[0], b_keys, 8 * (uint64_t)WK * nB, hipMemcpyDeviceToDevice,
                                         c->stream));  // stride nB == n
            c->split_keys_final = true;
        }
        c->cur = 0;
        c->heads = hd;
        c->heads_valid = true;
        return GK_OK;
    }
    if (nB == 0) {  // msd_sort left vals[0] / heads in place; A's keys expanded next to them
        if (WK && !a_packed) {  // (k > 32: the keys are re-encoded after the sort)
            if (a_keys == c->keys[1]) return fail(c, GK_E_STATE, "split sort: A keys alias the output buffer");
            if (int r = grow_key_buffer(c, 1, WK)) return r;
            const uint64_t nn = nA;
            if (WK == 1)
                hipLaunchKernelGGL(expand_keys_kernel<1>, dim3(grid_of_n(nn)), dim3(256), 0, c->stream, a_keys, nn, k,
                                   c->keys[1]);
            else
                hipLaunchKernelGGL(expand_keys_kernel<2>, dim3(grid_of_n(nn)), dim3(256), 0, c->stream, a_keys, nn, k,
                                   c->keys[1]);
            GK_TRY_HIP(c, hipGetLastError());
            GK_TRY_HIP(c, hipMemcpyAsync(c->vals[1], c->vals[0], 4 * nn, hipMemcpyDeviceToDevice, c->stream));
            c->cur = 1;
            c->split_keys_final = true;
        }
        return GK_OK;
    }

    // 4. merge: B groups, their insertion points in A, the interleave into vals[1] + heads
    timer_begin(c, "split_merge", &slot);
    uint32_t *g_first, *pos;
    uint64_t G = 0;
    GK_TRY_HIP(c, scratch(c, "split_g_first", nB + 64, &g_first));
    GK_TRY_HIP(c, select_flags(c, b_heads, nB, g_first, &G));
    GK_TRY_HIP(c, scratch(c, "split_pos", G + 64, &pos));
    hipLaunchKernelGGL(b_group_pos_kernel, dim3(grid_of_n(G)), dim3(256), 0, c->stream, c->sba, k, ks.canonical,
                       c->vals[0], nA, b_st[bres], g_first, G, pos);
    GK_TRY_HIP(c, hipGetLastError());
    uint8_t *hd;
    GK_TRY_HIP(c, scratch(c, "split_heads", n + 64, &hd));
    if (WK) {  // (a no-op after the pre-sizing above; a_keys / b_keys never live in keys[1])
        if (a_keys == c->keys[1] || b_keys == c->keys[1])
            return fail(c, GK_E_STATE, "split sort: input keys alias the merge output buffer");
        int r = grow_key_buffer(c, 1, WK);
        if (r != GK_OK) return r;
    }
    const dim3 ga((unsigned)((nA + kMTile - 1) / kMTile)), gb((unsigned)((nB + kMTile - 1) / kMTile));
    uint64_t *ok = c->keys[1];
    if (a_packed) {
        // the 2-bit packed sequence: three words past every start (the sba's '$' pad covers them)
        // (the transfer's resident packed copy when there is one: the same codes at every position)
        const uint64_t nwords = (L + kSbaPad) / 32;
        const uint64_t *pk = c->res_pk ? c->res_code : nullptr;
        if (!pk) {
            uint64_t *own;
            GK_TRY_HIP(c, scratch(c, "split_pk", nwords, &own));
            hipLaunchKernelGGL(split_pack_kernel, dim3((unsigned)std::min<uint64_t>((nwords + 255) / 256, 65536)),
                               dim3(256), 0, c->stream, c->sba, nwords, own);
            GK_TRY_HIP(c, hipGetLastError());
            pk = own;
        }
#define GK_MERGE_PK(W_)                                                                                         \
    do {                                                                                                        \
        hipLaunchKernelGGL((merge_a_kernel<W_, true>), ga, dim3(kMT), 0, c->stream, c->vals[0], c->heads, nA,     \
                           pos, g_first, G, nB, c->vals[1], hd, nullptr, k, ok, pk, ks.canonical);               \
        hipLaunchKernelGGL(merge_b_kernel<W_>, gb, dim3(kMT), 0, c->stream, b_st[bres], b_heads, nB, pos,         \
                           g_first, G, c->vals[1], hd, b_keys, nA + nB, ok);                                     \
    } while (0)
        if (WK == 3) GK_MERGE_PK(3);
        else if (WK == 4) GK_MERGE_PK(4);
        else return fail(c, GK_E_STATE, "split sort: packed-sequence keys need 3 or 4 key words");
#undef GK_MERGE_PK
        GK_TRY_HIP(c, hipGetLastError());
        c->split_keys_final = true;
        timer_end(c, slot);
        c->cur = 1;
        c->heads = hd;
        c->heads_valid = true;
        return GK_OK;
    }
    switch (WK) {
    case 0:
        hipLaunchKernelGGL(merge_a_kernel<0>, ga, dim3(kMT), 0, c->stream, c->vals[0], c->heads, nA, pos, g_first, G,
                           nB, c->vals[1], hd, nullptr, k, nullptr);
        hipLaunchKernelGGL(merge_b_kernel<0>, gb, dim3(kMT), 0, c->stream, b_st[bres], b_heads, nB, pos, g_first, G,
                           c->vals[1], hd, nullptr, n, nullptr);
        break;
    case 1:
        hipLaunchKernelGGL(merge_a_kernel<1>, ga, dim3(kMT), 0, c->stream, c->vals[0], c->heads, nA, pos, g_first, G,
                           nB, c->vals[1], hd, a_keys, k, ok);
        hipLaunchKernelGGL(merge_b_kernel<1>, gb, dim3(kMT), 0, c->stream, b_st[bres], b_heads, nB, pos, g_first, G,
                           c->vals[1], hd, b_keys, nA + nB, ok);
        break;
    default:
        hipLaunchKernelGGL(merge_a_kernel<2>, ga, dim3(kMT), 0, c->stream, c->vals[0], c->heads, nA, pos, g_first, G,
                           nB, c->vals[1], hd, a_keys, k, ok);
        hipLaunchKernelGGL(merge_b_kernel<2>, gb, dim3(kMT), 0, c->stream, b_st[bres], b_heads, nB, pos, g_first, G,
                           c->vals[1], hd, b_keys, nA + nB, ok);
    }
    GK_TRY_HIP(c, hipGetLastError());
    c->split_keys_final = WK > 0;
    timer_end(c, slot);
    c->cur = 1;
    c->heads = hd;
    c->heads_valid = true;
    return GK_OK;
}

}  // namespace gkm

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

#include "gkm_canon.h"
#include "gkm_internal.h"

namespace gkm {

__constant__ uint8_t c_code4_split[256];
static bool g_split_tables = false;

static hipError_t split_tables() {
    if (g_split_tables) return hipSuccess;
    uint8_t code4[256] = {0};
    const char *order = "ABCDGHKMNRSTVWY";
    for (int i = 0; order[i]; ++i) code4[(uint8_t)order[i]] = (uint8_t)(i + 1);
    hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(c_code4_split), code4, 256);
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

__global__ __launch_bounds__(256) void class_b_flags_kernel(const uint8_t *__restrict__ sba, uint64_t L, int k,
                                                            uint8_t *__restrict__ flags) {
    __shared__ uint32_t s_dol[kFlagGroups], s_bad[kFlagGroups];
    const uint64_t P0 = (uint64_t)blockIdx.x * kFlagTile;
    for (int g = threadIdx.x; g < kFlagGroups; g += 256) {
        const uint4 *src = reinterpret_cast<const uint4 *>(sba + P0 + 32ull * g);  // '$' pad after L
        const uint4 ra = src[0], rb = src[1];
        const uint32_t wv[8] = {ra.x, ra.y, ra.z, ra.w, rb.x, rb.y, rb.z, rb.w};
        uint32_t dm = 0, bm = 0;
#pragma unroll
        for (int q = 0; q < 32; ++q) {
            const uint32_t ch = (wv[q >> 2] >> (8 * (q & 3))) & 0xFFu;
            dm = (dm << 1) | (ch == GK_DOLLAR ? 1u : 0u);
            bm = (bm << 1) | ((ch == 'A' || ch == 'C' || ch == 'G' || ch == 'T') ? 0u : 1u);
        }
        s_dol[g] = dm;
        s_bad[g] = bm;
    }
    __syncthreads();
    // thread t: positions 32 t .. 32 t + 31 -> 32 flag bytes (two 16-B stores)
    const uint32_t p0 = threadIdx.x * 32;
    uint32_t out[8];
#pragma unroll
    for (int w = 0; w < 8; ++w) {
        uint32_t v = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const uint32_t p = p0 + 4 * w + b;
            const bool f = P0 + p < L && window_clear(s_dol, p, k) && !window_clear(s_bad, p, k);
            v |= (f ? 1u : 0u) << (8 * b);
        }
        out[w] = v;
    }
    if (P0 + p0 < L) {
        uint4 *dst = reinterpret_cast<uint4 *>(flags + P0 + p0);
        dst[0] = make_uint4(out[0], out[1], out[2], out[3]);
        dst[1] = make_uint4(out[4], out[5], out[6], out[7]);
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

__global__ __launch_bounds__(kMT) void merge_a_kernel(const uint32_t *__restrict__ a_starts,
                                                      const uint8_t *__restrict__ a_heads, uint64_t nA,
                                                      const uint32_t *__restrict__ pos,
                                                      const uint32_t *__restrict__ g_first, uint64_t G, uint64_t nB,
                                                      uint32_t *__restrict__ out, uint8_t *__restrict__ out_heads) {
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
        for (uint64_t i = i0 + threadIdx.x; i < i1; i += kMT) {
            out[i + shift] = a_starts[i];
            out_heads[i + shift] = (a_heads[i] || (i == i0 && g0 > lb0)) ? 1 : 0;
        }
        return;
    }
    for (uint64_t i = i0 + threadIdx.x; i < i1; i += kMT) {
        const uint64_t ub = bound_in(pos, g0, g1, i, true);
        const uint64_t lb = i == i0 ? lb0 : bound_in(pos, g0, ub, i, false);
        const uint64_t shift = ub < G ? g_first[ub] : nB;
        out[i + shift] = a_starts[i];
        out_heads[i + shift] = (a_heads[i] || ub > lb) ? 1 : 0;
    }
}

// B element j of group g goes to j + pos[g]; per 4096 B elements, the groups they span
__global__ __launch_bounds__(kMT) void merge_b_kernel(const uint32_t *__restrict__ b_starts,
                                                      const uint8_t *__restrict__ b_heads, uint64_t nB,
                                                      const uint32_t *__restrict__ pos,
                                                      const uint32_t *__restrict__ g_first, uint64_t G,
                                                      uint32_t *__restrict__ out, uint8_t *__restrict__ out_heads) {
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
    }
}

static unsigned grid_of_n(uint64_t n) { return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((n + 255) / 256, 16384)); }

// ---------------------------------------------------------------------------------------------
// driver
// ---------------------------------------------------------------------------------------------
int split_sort(gk_ctx *c, const KeySpec &ks, bool *used) {
    *used = false;
    const uint64_t n = c->n, L = c->sba_len;
    const int k = ks.symbols;
    if (k > 64 || ks.bits != 4 || ks.lenbits || ks.symbols != ks.min_len) return GK_OK;
    GK_TRY_HIP(c, split_tables());
    int slot;
    // 1. class B starts
    uint8_t *fB;
    uint32_t *b_st[2];
    GK_TRY_HIP(c, scratch(c, "split_flags", L + kFlagTile + 64, &fB));
    timer_begin(c, "split_b_select", &slot);
    hipLaunchKernelGGL(class_b_flags_kernel, dim3((unsigned)((L + kFlagTile - 1) / kFlagTile)), dim3(256), 0,
                       c->stream, c->sba, L, k, fB);
    GK_TRY_HIP(c, hipGetLastError());
    uint64_t nB = 0;
    // count first: the select output needs nB entries, which may be up to n
    GK_TRY_HIP(c, scratch(c, "split_b_st0", n + 64, &b_st[0]));
    GK_TRY_HIP(c, select_flags(c, fB, L, b_st[0], &nB));
    timer_end(c, slot);
    if (nB > n) return fail(c, GK_E_HIP, "split: more class-B k-mers than k-mers");
    if (nB * 4 > n) return GK_OK;  // mostly non-ACGT k-mers: the plain 4-bit MSD is the better sort
    *used = true;
    const uint64_t nA = n - nB;

    // 2. sort B: 4-bit keys, LSD (on a swapped-in context of nB elements)
    uint64_t *b_k[2];
    uint8_t *b_heads;
    int bres = 0;
    if (nB > 0) {
        const int W = ks.words;
        GK_TRY_HIP(c, scratch(c, "split_b_st1", nB + 64, &b_st[1]));
        GK_TRY_HIP(c, scratch(c, "split_b_k0", W * (nB + 64), &b_k[0]));
        GK_TRY_HIP(c, scratch(c, "split_b_k1", W * (nB + 64), &b_k[1]));
        GK_TRY_HIP(c, scratch(c, "split_b_heads", nB + 64, &b_heads));
        const uint64_t sv_n = c->n;
        uint64_t *sv_k[2] = {c->keys[0], c->keys[1]};
        uint32_t *sv_v[2] = {c->vals[0], c->vals[1]};
        const int sv_cur = c->cur;
        c->n = nB;
        c->keys[0] = b_k[0];
        c->keys[1] = b_k[1];
        c->vals[0] = b_st[0];
        c->vals[1] = b_st[1];
        c->cur = 0;
        timer_begin(c, "split_b_encode", &slot);
        hipError_t e = launch_encode_gather(c, ks, b_st[0], nB, b_k[0]);
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
        hipLaunchKernelGGL(key_heads_kernel, dim3(grid_of_n(nB)), dim3(256), 0, c->stream, b_k[bres], nB, W, b_heads);
        GK_TRY_HIP(c, hipGetLastError());
    }

    // 3. sort A: the 2-bit MSD over the ACGT-only k-mers (its count is checked against nA)
    KeySpec ka = ks;
    ka.bits = 2;
    ka.total_bits = 2 * k;
    ka.words = (ka.total_bits + 63) / 64;
    ka.acgt_only = 1;
    c->n = nA;
    int rc = nA > 0 ? msd_sort(c, ka) : GK_OK;
    c->n = n;
    if (rc != GK_OK) return rc;
    if (nA == 0) {  // all B: the B order is the order
        GK_TRY_HIP(c, hipMemcpyAsync(c->vals[0], b_st[bres], 4 * nB, hipMemcpyDeviceToDevice, c->stream));
        uint8_t *hd;
        GK_TRY_HIP(c, scratch(c, "split_heads", n + 64, &hd));
        GK_TRY_HIP(c, hipMemcpyAsync(hd, b_heads, nB, hipMemcpyDeviceToDevice, c->stream));
        c->cur = 0;
        c->heads = hd;
        c->heads_valid = true;
        return GK_OK;
    }
    if (nB == 0) return GK_OK;  // msd_sort left vals[0] / heads in place

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
    hipLaunchKernelGGL(merge_a_kernel, dim3((unsigned)((nA + kMTile - 1) / kMTile)), dim3(kMT), 0, c->stream,
                       c->vals[0], c->heads, nA, pos, g_first, G, nB, c->vals[1], hd);
    hipLaunchKernelGGL(merge_b_kernel, dim3((unsigned)((nB + kMTile - 1) / kMTile)), dim3(kMT), 0, c->stream,
                       b_st[bres], b_heads, nB, pos, g_first, G, c->vals[1], hd);
    GK_TRY_HIP(c, hipGetLastError());
    timer_end(c, slot);
    c->cur = 1;
    c->heads = hd;
    c->heads_valid = true;
    return GK_OK;
}

}  // namespace gkm

// gkm_encode.hip -- enumerate + encode kernels (gfx950).
//
// Reference behaviour restated here (paths relative to the reference's src/genome_kmers/):
//   enumerate   kmers.py:789-861      starts = concat_s arange(seg_start_s, seg_end_s - min_k + 2)
//   order       kmers.py:306-397      byte-wise lexicographic, '$'/end-of-array terminates (less)
//   alphabet    sequence_collection.py:441-458, 694-697  {A,C,G,T,R,Y,S,W,K,M,B,D,H,V,N,$}
// The encoders turn the k-mer at a start into an integer whose unsigned order equals that byte
// order: 2-bit codes when the sba is pure ACGT, 4-bit codes ('$' = 0) otherwise.
#include <cstdlib>
#include <vector>

#include "gkm_canon.h"
#include "gkm_internal.h"
#include "gkm_swar.h"

namespace gkm {

// '$' -> 0 ; A B C D G H K M N R S T V W Y -> 1..15 (ASCII order preserved)
__constant__ uint8_t c_code4[256];
// 0: A,C,G,T or '$'   1: other IUPAC letter   2: byte not allowed
__constant__ uint8_t c_class[256];

static bool g_tables_ready = false;

static hipError_t init_tables() {
    if (g_tables_ready) return hipSuccess;
    uint8_t code4[256] = {0}, cls[256];
    const char *order = "ABCDGHKMNRSTVWY";
    for (int i = 0; i < 256; ++i) cls[i] = 2;
    for (int i = 0; order[i]; ++i) {
        code4[(uint8_t)order[i]] = (uint8_t)(i + 1);
        cls[(uint8_t)order[i]] = 1;
    }
    cls['A'] = cls['C'] = cls['G'] = cls['T'] = 0;
    cls[GK_DOLLAR] = 0;
    hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(c_code4), code4, 256);
    if (e != hipSuccess) return e;
    e = hipMemcpyToSymbol(HIP_SYMBOL(c_class), cls, 256);
    if (e != hipSuccess) return e;
    g_tables_ready = true;
    return hipSuccess;
}

struct KS {  // POD copy of KeySpec for kernels
    int bits, symbols, lenbits, min_len, words, total_bits, digits, canonical;
};

static KS pod(const KeySpec &k) {
    return KS{k.bits, k.symbols, k.lenbits, k.min_len, k.words, k.total_bits, k.digits(), k.canonical};
}

__device__ __forceinline__ uint32_t code2(uint32_t c) { return ((c >> 1) ^ (c >> 2)) & 3u; }

template <int BITS>
__device__ __forceinline__ uint32_t sym_code(uint32_t c, const uint8_t *lut4) {
    if (BITS == 2) return code2(c);
    if (BITS == 3) return c == GK_DOLLAR ? 0u : code2(c) + 1u;
    return lut4[c];
}

// segment index of sba position p: last s with seg[s] <= p
__device__ __forceinline__ uint32_t seg_of(const uint32_t *__restrict__ seg, uint32_t nseg, uint64_t p) {
    uint32_t lo = 0, hi = nseg;
    while (hi - lo > 1) {
        uint32_t mid = (lo + hi) >> 1;
        if ((uint64_t)seg[mid] <= p) lo = mid; else hi = mid;
    }
    return lo;
}

// ---------------------------------------------------------------------------------------------
// alphabet / '$' census of the sba (sequence_collection.py:694-697)
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void alphabet_kernel(const uint8_t *__restrict__ sba, uint64_t L,
                                                       uint32_t *__restrict__ out) {
    uint32_t cls_or = 0, dollars = 0;
    uint64_t nchunk = L / 16;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nchunk;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint4 v = reinterpret_cast<const uint4 *>(sba)[i];
        uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                uint32_t c = (w[k] >> (8 * b)) & 0xFF;
                cls_or |= 1u << c_class[c];
                dollars += (c == GK_DOLLAR);
            }
        }
    }
    if (blockIdx.x == 0) {
        for (uint64_t i = nchunk * 16 + threadIdx.x; i < L; i += blockDim.x) {
            uint32_t c = sba[i];
            cls_or |= 1u << c_class[c];
            dollars += (c == GK_DOLLAR);
        }
    }
    // wave reduce
    for (int off = 32; off > 0; off >>= 1) {
        cls_or |= __shfl_xor(cls_or, off);
        dollars += __shfl_xor(dollars, off);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicOr(&out[0], cls_or);
        atomicAdd(&out[1], dollars);
    }
}

hipError_t launch_alphabet_range(gk_ctx *c, const uint8_t *p, uint64_t len, uint32_t *d_flags) {
    hipError_t e = init_tables();
    if (e != hipSuccess) return e;
    const uint64_t chunks = len / 16 + 1;
    const int grid = (int)std::min<uint64_t>((chunks + 255) / 256, 2048);
    hipLaunchKernelGGL(alphabet_kernel, dim3(grid), dim3(256), 0, c->stream, p, len, d_flags);
    return hipGetLastError();
}

hipError_t launch_alphabet(gk_ctx *c, uint32_t *d_flags) {
    hipError_t e = init_tables();
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(d_flags, 0, 8, c->stream);
    if (e != hipSuccess) return e;
    uint64_t chunks = c->sba_len / 16 + 1;
    int grid = (int)std::min<uint64_t>((chunks + 255) / 256, 2048);
    hipLaunchKernelGGL(alphabet_kernel, dim3(grid), dim3(256), 0, c->stream, c->sba, c->sba_len, d_flags);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// enumerate (kmers.py:789-835): out[j] = seg[s] + (j - cumk[s])
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void enumerate_kernel(const uint32_t *__restrict__ seg,
                                                        const uint64_t *__restrict__ cumk, uint32_t nseg,
                                                        uint64_t n, uint32_t *__restrict__ out) {
    for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < n; j += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t lo = 0, hi = nseg;
        while (hi - lo > 1) {
            uint32_t mid = (lo + hi) >> 1;
            if (cumk[mid] <= j) lo = mid; else hi = mid;
        }
        out[j] = (uint32_t)(seg[lo] + (j - cumk[lo]));
    }
}

hipError_t launch_enumerate(gk_ctx *c, uint32_t min_k, uint32_t *out) {
    // cumulative k-mer counts per segment, built on the host from the segment table
    const std::vector<uint32_t> &hseg = c->hseg;
    hipError_t e;
    std::vector<uint64_t> cum(c->nseg + 1, 0);
    for (uint64_t s = 0; s < c->nseg; ++s) {
        uint64_t end = (s + 1 == c->nseg) ? c->sba_len - 1 : (uint64_t)hseg[s + 1] - 2;
        cum[s + 1] = cum[s] + (end - hseg[s] + 1 - min_k + 1);
    }
    e = ensure(reinterpret_cast<void **>(&c->cumk), &c->cumk_cap, 8 * (c->nseg + 1));
    if (e != hipSuccess) return e;
    uint64_t *dcum = c->cumk;
    e = hipMemcpyAsync(dcum, cum.data(), 8 * (c->nseg + 1), hipMemcpyHostToDevice, c->stream);
    if (e != hipSuccess) return e;
    int grid = (int)std::min<uint64_t>((c->n + 255) / 256, 8192);
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL(enumerate_kernel, dim3(grid), dim3(256), 0, c->stream, c->seg, dcum, (uint32_t)c->nseg, c->n,
                       out);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    return hipStreamSynchronize(c->stream);  // cum is a stack buffer
}

// ---------------------------------------------------------------------------------------------
// validate user-provided starts: every start needs min_k bases before '$' (kmers.py:1715-1727)
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void validate_starts_kernel(const uint8_t *__restrict__ sba, uint64_t L,
                                                              const uint32_t *__restrict__ starts, uint64_t n,
                                                              uint32_t min_k, uint32_t *__restrict__ bad) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t p = starts[i];
        bool ok = p < L;
        for (uint32_t t = 0; ok && t < min_k; ++t) ok = (p + t < L) && sba[p + t] != GK_DOLLAR;
        if (!ok) atomicAdd(bad, 1u);
    }
}

hipError_t launch_validate_starts(gk_ctx *c, const uint32_t *starts, uint64_t n, uint32_t min_k, uint32_t *d_bad) {
    hipError_t e = hipMemsetAsync(d_bad, 0, 4, c->stream);
    if (e != hipSuccess) return e;
    int grid = (int)std::min<uint64_t>((n + 255) / 256, 8192);
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL(validate_starts_kernel, dim3(grid), dim3(256), 0, c->stream, c->sba, c->sba_len, starts, n,
                       min_k, d_bad);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// key assembly helpers
// ---------------------------------------------------------------------------------------------
template <int W>
__device__ __forceinline__ void bi_shl_or(uint64_t (&w)[W], int s, uint64_t v) {
#pragma unroll
    for (int k = 0; k < W - 1; ++k) w[k] = (w[k] << s) | (w[k + 1] >> (64 - s));
    w[W - 1] = (w[W - 1] << s) | v;
}

// key of the window bytes[0 .. symbols-1] (bytes past the pad are '$')
template <int W, int BITS, bool BOUNDED, typename ByteFn>
__device__ __forceinline__ void window_key(const KS &ks, ByteFn byte_at, const uint8_t *lut4, uint64_t (&w)[W]) {
#pragma unroll
    for (int k = 0; k < W; ++k) w[k] = 0;
    int len = ks.symbols;
    bool term = false;
    for (int t = 0; t < ks.symbols; ++t) {
        uint32_t ch = byte_at(t);
        if (BOUNDED && !term && ch == GK_DOLLAR) {
            term = true;
            len = t;
        }
        uint32_t sym = (BOUNDED && term) ? 0u : sym_code<BITS>(ch, lut4);
        bi_shl_or<W>(w, BITS, sym);
    }
    if (BOUNDED && ks.lenbits > 0) bi_shl_or<W>(w, ks.lenbits, (uint64_t)len);
}

// ---------------------------------------------------------------------------------------------
// encode over positions (enumerated starts): fixed length, one word, rolling 2-/4-bit encode
//   - the tile's sba bytes (+ halo) are staged in LDS with 16-B loads
//   - thread t rolls over 16 consecutive positions: key = (key << b | code) & mask
//   - keys are transposed through LDS so the HBM writes are coalesced
//   - all digit histograms of the radix sort are accumulated in the same pass
// ---------------------------------------------------------------------------------------------
constexpr int kRollR = 16;
constexpr int kRollPitch = 257;  // 256 threads + 1: conflict-free transposed reads

template <int BITS>
__global__ __launch_bounds__(256) void encode_roll_w1_kernel(const uint8_t *__restrict__ sba, uint64_t L,
                                                             const uint32_t *__restrict__ seg, uint32_t nseg, KS ks,
                                                             uint64_t *__restrict__ keys, uint32_t *__restrict__ vals,
                                                             uint32_t *__restrict__ ghist) {
    __shared__ __attribute__((aligned(16))) uint8_t s_bytes[kEncodeTile + 256];
    __shared__ uint64_t s_keys[kRollR * kRollPitch];
    __shared__ uint32_t s_vmask[256];
    __shared__ uint32_t s_hist[8 * 256];
    __shared__ uint8_t s_lut4[256];
    __shared__ uint32_t s_tile_seg, s_tile_has_dollar;

    const int t = threadIdx.x;
    const int S = ks.symbols;
    const int D = ks.digits;
    const uint64_t mask = ks.total_bits >= 64 ? ~0ull : ((1ull << ks.total_bits) - 1);
    s_lut4[t] = c_code4[t];
    for (int i = t; i < 8 * 256; i += 256) s_hist[i] = 0;

    const uint64_t ntiles = (L + kEncodeTile - 1) / kEncodeTile;
    for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const uint64_t P0 = tile * kEncodeTile;
        __syncthreads();
        // stage bytes [P0, P0 + 4096 + 256): 16 B per thread + 16 extra chunks
        {
            const uint4 *src = reinterpret_cast<const uint4 *>(sba + P0);
            uint4 *dst = reinterpret_cast<uint4 *>(s_bytes);
            dst[t] = src[t];
            if (t < 16) dst[256 + t] = src[256 + t];
        }
        if (t == 0) {
            s_tile_seg = seg_of(seg, nseg, P0);
            s_tile_has_dollar = 0;
        }
        __syncthreads();
        // any '$' in the staged window? (decides the cheap segment lookup)
        {
            const uint32_t *w32 = reinterpret_cast<const uint32_t *>(s_bytes);
            bool d = false;
            for (int i = t; i < (kEncodeTile + 256) / 4; i += 256) {
                uint32_t v = w32[i] ^ 0x24242424u;  // zero byte where '$'
                d |= ((v - 0x01010101u) & ~v & 0x80808080u) != 0;
            }
            if (__any(d) && (t & 63) == 0) s_tile_has_dollar = 1;
        }
        // rolling encode of positions 16t .. 16t+15
        {
            const int q0 = t * kRollR;
            uint64_t key = 0;
            int last_dollar = -1000;
            uint32_t vm = 0;
            const int steps = S - 1 + kRollR;
            for (int i = 0; i < steps; ++i) {
                uint32_t ch = s_bytes[q0 + i];
                if (ch == GK_DOLLAR) last_dollar = i;
                key = ((key << BITS) | sym_code<BITS>(ch, s_lut4)) & mask;
                int j = i - (S - 1);
                if (j >= 0) {
                    s_keys[j * kRollPitch + t] = key;
                    if (last_dollar < j) vm |= 1u << j;
                }
            }
            s_vmask[t] = vm;
        }
        __syncthreads();
        const bool has_dollar = s_tile_has_dollar != 0;
        const uint32_t tseg = s_tile_seg;
#pragma unroll 4
        for (int i = 0; i < kRollR; ++i) {
            const int q = t + 256 * i;
            const int owner = q >> 4, j = q & 15;
            const uint64_t p = P0 + q;
            if (((s_vmask[owner] >> j) & 1u) && p < L) {
                uint64_t key = s_keys[j * kRollPitch + owner];
                uint32_t s = has_dollar ? seg_of(seg, nseg, p) : tseg;
                uint64_t o = p - (uint64_t)ks.min_len * s;
                keys[o] = key;
                vals[o] = (uint32_t)p;
                for (int d = 0; d < D; ++d) atomicAdd(&s_hist[d * 256 + ((key >> (8 * d)) & 0xFF)], 1u);
            }
        }
    }
    __syncthreads();
    for (int i = t; i < D * 256; i += 256) {
        uint32_t v = s_hist[i];
        if (v) atomicAdd(&ghist[i], v);
    }
}

// ---------------------------------------------------------------------------------------------
// bounded variable-length keys of one word (2-bit ACGT with a length field, the 3-bit doubling
// seeds), rolling: thread t rolls the raw window over positions 16t .. 16t+15 as encode_roll_w1
// does, and a '$' bitmask of its bytes gives each position's first '$' -- the symbols from it on
// are zeroed and the length field is min(len, symbols), window_key's encoding (sort_keys' MSD path:
// no digit histograms).  The per-position byte loop of encode_generic_kernel ran 1.05 ms for 1e8
// positions of the reference's profiling workload.
// ---------------------------------------------------------------------------------------------
// HIST: the LSD sort's digit histograms of the stored keys as well (ks.digits of them; LDS counts
// flushed once per workgroup), in place of encode_generic_kernel's for the LSD route
template <int BITS, bool HIST>
__global__ __launch_bounds__(256) void encode_roll_bounded_kernel(const uint8_t *__restrict__ sba, uint64_t L,
                                                                  const uint32_t *__restrict__ seg, uint32_t nseg,
                                                                  KS ks, uint64_t *__restrict__ keys,
                                                                  uint32_t *__restrict__ vals,
                                                                  uint32_t *__restrict__ ghist) {
    __shared__ __attribute__((aligned(16))) uint8_t s_bytes[kEncodeTile + 256];
    __shared__ uint64_t s_keys[kRollR * kRollPitch];
    __shared__ uint32_t s_vmask[256];
    __shared__ uint32_t s_tile_seg, s_tile_has_dollar;
    __shared__ uint32_t s_hist[HIST ? 8 * 256 : 1];
    const int t = threadIdx.x;
    const int D = HIST ? ks.digits : 0;  // <= 8 (one word)
    if (HIST)
        for (int i = t; i < D * 256; i += 256) s_hist[i] = 0;
    const int S = ks.symbols;  // <= 32 (the caller checks)
    const uint64_t symmask = BITS * S >= 64 ? ~0ull : ((1ull << (BITS * S)) - 1);
    const uint64_t ntiles = (L + kEncodeTile - 1) / kEncodeTile;
    for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const uint64_t P0 = tile * kEncodeTile;
        __syncthreads();
        {
            const uint4 *src = reinterpret_cast<const uint4 *>(sba + P0);
            uint4 *dst = reinterpret_cast<uint4 *>(s_bytes);
            dst[t] = src[t];
            if (t < 16) dst[256 + t] = src[256 + t];
        }
        if (t == 0) {
            s_tile_seg = seg_of(seg, nseg, P0);
            s_tile_has_dollar = 0;
        }
        __syncthreads();
        {
            const uint32_t *w32 = reinterpret_cast<const uint32_t *>(s_bytes);
            bool d = false;
            for (int i = t; i < (kEncodeTile + 256) / 4; i += 256) {
                uint32_t v = w32[i] ^ 0x24242424u;  // zero byte where '$'
                d |= ((v - 0x01010101u) & ~v & 0x80808080u) != 0;
            }
            if (__any(d) && (t & 63) == 0) s_tile_has_dollar = 1;
        }
        {
            const int q0 = t * kRollR;
            const int span = S - 1 + kRollR;  // <= 47 bytes
            uint64_t dm = 0;                  // bit i: byte q0 + i is '$'
            uint64_t raw = 0;
            uint32_t vm = 0;
            for (int i = 0; i < span; ++i) {
                const uint32_t ch = s_bytes[q0 + i];
                if (ch == GK_DOLLAR) dm |= 1ull << i;
                raw = ((raw << BITS) | sym_code<BITS>(ch, nullptr)) & symmask;
                const int j = i - (S - 1);
                if (j >= 0) {
                    const uint64_t dj = dm >> j;  // '$' at window offsets
                    const int first = dj ? min(S, (int)__builtin_ctzll(dj)) : S;
                    uint64_t k = first < S ? raw & ~((1ull << (BITS * (S - first))) - 1) : raw;
                    if (ks.lenbits > 0) k = (k << ks.lenbits) | (uint64_t)first;
                    s_keys[j * kRollPitch + t] = k;
                    if (first >= ks.min_len) vm |= 1u << j;
                }
            }
            s_vmask[t] = vm;
        }
        __syncthreads();
        const bool has_dollar = s_tile_has_dollar != 0;
        const uint32_t tseg = s_tile_seg;
#pragma unroll 4
        for (int i = 0; i < kRollR; ++i) {
            const int q = t + 256 * i;
            const int owner = q >> 4, j = q & 15;
            const uint64_t p = P0 + q;
            if (((s_vmask[owner] >> j) & 1u) && p < L) {
                const uint32_t sg = has_dollar ? seg_of(seg, nseg, p) : tseg;
                const uint64_t o = p - (uint64_t)ks.min_len * sg;
                const uint64_t key = s_keys[j * kRollPitch + owner];
                keys[o] = key;
                vals[o] = (uint32_t)p;
                if (HIST)
                    for (int d = 0; d < D; ++d) atomicAdd(&s_hist[d * 256 + ((key >> (8 * d)) & 0xFF)], 1u);
            }
        }
    }
    if (HIST) {
        __syncthreads();
        for (int i = t; i < D * 256; i += 256) {
            const uint32_t v = s_hist[i];
            if (v) atomicAdd(&ghist[i], v);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// generic encode over positions: any width W, bounded (padded) keys; one key per thread from LDS
// ---------------------------------------------------------------------------------------------
template <int W, int BITS, bool BOUNDED>
__global__ __launch_bounds__(256) void encode_generic_kernel(const uint8_t *__restrict__ sba, uint64_t L,
                                                             const uint32_t *__restrict__ seg, uint32_t nseg, KS ks,
                                                             uint64_t n, uint64_t *__restrict__ keys,
                                                             uint32_t *__restrict__ vals, uint32_t *__restrict__ ghist) {
    __shared__ __attribute__((aligned(16))) uint8_t s_bytes[kEncodeTile + 512];
    __shared__ uint32_t s_hist[kMaxWords * 8 * 256];
    __shared__ uint8_t s_lut4[256];
    const int t = threadIdx.x;
    const int D = ks.digits;
    s_lut4[t] = c_code4[t];
    for (int i = t; i < D * 256; i += 256) s_hist[i] = 0;
    const uint64_t ntiles = (L + kEncodeTile - 1) / kEncodeTile;
    for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const uint64_t P0 = tile * kEncodeTile;
        __syncthreads();
        {
            const uint4 *src = reinterpret_cast<const uint4 *>(sba + P0);
            uint4 *dst = reinterpret_cast<uint4 *>(s_bytes);
            dst[t] = src[t];
            if (t < 32) dst[256 + t] = src[256 + t];
        }
        __syncthreads();
        for (int i = 0; i < kEncodeTile / 256; ++i) {
            const int q = t + 256 * i;
            const uint64_t p = P0 + q;
            if (p >= L) break;
            bool valid = true;
            for (int k = 0; k < ks.min_len; ++k) valid &= s_bytes[q + k] != GK_DOLLAR;
            if (!valid) continue;
            uint64_t w[W];
            window_key<W, BITS, BOUNDED>(ks, [&](int k) { return (uint32_t)s_bytes[q + k]; }, s_lut4, w);
            uint32_t s = seg_of(seg, nseg, p);
            uint64_t o = p - (uint64_t)ks.min_len * s;
#pragma unroll
            for (int k = 0; k < W; ++k) keys[(uint64_t)k * n + o] = w[k];
            vals[o] = (uint32_t)p;
            for (int d = 0; d < D; ++d) {
                int word = W - 1 - (d >> 3);
                atomicAdd(&s_hist[d * 256 + ((w[word] >> (8 * (d & 7))) & 0xFF)], 1u);
            }
        }
    }
    __syncthreads();
    for (int i = t; i < D * 256; i += 256) {
        uint32_t v = s_hist[i];
        if (v) atomicAdd(&ghist[i], v);
    }
}

// ---------------------------------------------------------------------------------------------
// gather encode: keys of arbitrary starts (user-provided or re-sorted arrays)
// ---------------------------------------------------------------------------------------------
// Fixed-length keys (k <= 64) of windows holding only A, C, G, T -- ~95 % of a GRCh38-like genome,
// all of a random one -- without a per-byte loop: the window is read as 8-byte words (a funnel
// shift per word aligns it to the start), 8 bytes become 16 bits of 2-bit codes by SWAR
// (pack2_8), the canonical choice is one 128-bit compare against the bit-reversed complement, and
// 4-bit keys expand the 2-bit codes nibble by nibble (A 1, C 3, G 5, T 12: 2 s + 1, + 5 for T).
// Windows with another byte take the per-byte path below.

// the k (<= 64) symbols from sba[s] as a right-aligned 2k-bit value (hi:lo); false if a window
// byte is not A, C, G or T (reads up to 72 bytes from s & ~7: the sba carries a '$' pad)
__device__ __forceinline__ bool window2_acgt(const uint8_t *sba, uint64_t s, int k, uint64_t &hi, uint64_t &lo) {
    const uint64_t a = s & ~7ull;
    const int sh = (int)(s - a) * 8;
    const uint64_t *p = reinterpret_cast<const uint64_t *>(sba + a);
    uint64_t prev = p[0];
    uint64_t bad = 0;
    hi = lo = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        if (8 * j >= k) break;
        const uint64_t nxt = p[j + 1];
        const uint64_t w = sh ? (prev >> sh) | (nxt << (64 - sh)) : prev;
        prev = nxt;
        const int nb = min(8, k - 8 * j);
        const uint64_t m = nb == 8 ? ~0ull : ((1ull << (8 * nb)) - 1);
        bad |= non_acgt_bytes(w) & m;
        const uint32_t v = pack2_8e(w) >> (16 - 2 * nb);
        hi = (hi << (2 * nb)) | (lo >> (64 - 2 * nb));
        lo = (lo << (2 * nb)) | v;
    }
    return bad == 0;
}

// the W key words of the fixed-length k-mer at st: SWAR for windows of A/C/G/T, per symbol otherwise
template <int W, int BITS>
__device__ __forceinline__ void fast_window_key(const uint8_t *__restrict__ sba, const KS &ks, uint32_t st,
                                                const uint8_t *s_lut4, uint64_t (&w)[W]) {
    const int k = ks.symbols;
    uint64_t hi, lo;
    if (window2_acgt(sba, st, k, hi, lo)) {
        if (ks.canonical) canon2(k, hi, lo);
        key_from_2bit<W, BITS>(hi, lo, k, w);
    } else {
        const uint8_t *b = sba + st;
        if (ks.canonical) {
            const bool rc = canon_is_rc<BITS>(b, k, s_lut4);
#pragma unroll
            for (int q = 0; q < W; ++q) w[q] = 0;
            for (int t = 0; t < k; ++t) bi_shl_or<W>(w, BITS, canon_sym<BITS>(b, k, t, rc, s_lut4));
        } else {
            window_key<W, BITS, false>(ks, [&](int q) { return (uint32_t)b[q]; }, s_lut4, w);
        }
    }
}

template <int W, int BITS>
__global__ __launch_bounds__(256) void encode_gather_fast_kernel(const uint8_t *__restrict__ sba, KS ks,
                                                                 const uint32_t *__restrict__ starts, uint64_t n,
                                                                 uint64_t *__restrict__ keys) {
    __shared__ uint8_t s_lut4[256];
    s_lut4[threadIdx.x] = c_code4[threadIdx.x];
    __syncthreads();
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t w[W];
        fast_window_key<W, BITS>(sba, ks, starts[i], s_lut4, w);
#pragma unroll
        for (int q = 0; q < W; ++q) keys[(uint64_t)q * n + i] = w[q];
    }
}

// Keys through an enumeration-order table (multi-word keys of a sorted enumeration, C5: 4 words).
// The gather above reads each sorted start's window from the sequence -- 64-72 unaligned bytes at
// a random position, about two random 64-B sectors per k-mer (236 ms at C5).  Here every key is
// computed once in enumeration order (sequential reads, contiguous AoS writes) and each sorted
// start then reads its W aligned words: one random row per k-mer.  Enumeration index of a start
// p in contig s: kb[s] + (p - seg[s]), kb = exclusive prefix of the contigs' k-mer counts.
constexpr int kSegLds = 2048;  // contig tables staged in LDS up to this many contigs

// the last s with tab[s] <= x (tab ascending, tab[0] <= x)
__device__ __forceinline__ uint32_t last_le(const uint32_t *tab, uint32_t n, uint32_t x) {
    uint32_t lo = 0, hi = n;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (tab[mid] <= x) lo = mid;
        else hi = mid;
    }
    return lo;
}

template <int W, int BITS>
__global__ __launch_bounds__(256) void key_table_kernel(const uint8_t *__restrict__ sba, KS ks,
                                                        const uint32_t *__restrict__ seg, const uint32_t *__restrict__ kb,
                                                        uint32_t nseg, uint64_t n, uint64_t *__restrict__ table) {
    __shared__ uint8_t s_lut4[256];
    __shared__ uint32_t s_seg[kSegLds], s_kb[kSegLds];
    s_lut4[threadIdx.x] = c_code4[threadIdx.x];
    const bool lds = nseg <= (uint32_t)kSegLds;
    if (lds)
        for (uint32_t i = threadIdx.x; i < nseg; i += 256) {
            s_seg[i] = seg[i];
            s_kb[i] = kb[i];
        }
    __syncthreads();
    const uint32_t *tseg = lds ? s_seg : seg, *tkb = lds ? s_kb : kb;
    for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < n; j += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t s = last_le(tkb, nseg, (uint32_t)j);  // contigs without k-mers share kb: the last wins
        uint64_t w[W];
        fast_window_key<W, BITS>(sba, ks, tseg[s] + ((uint32_t)j - tkb[s]), s_lut4, w);
#pragma unroll
        for (int q = 0; q < W; ++q) table[j * W + q] = w[q];
    }
}

template <int W>
__global__ __launch_bounds__(256) void table_gather_kernel(const uint32_t *__restrict__ starts,
                                                           const uint32_t *__restrict__ seg,
                                                           const uint32_t *__restrict__ kb, uint32_t nseg, uint64_t n,
                                                           const uint64_t *__restrict__ table,
                                                           uint64_t *__restrict__ keys) {
    __shared__ uint32_t s_seg[kSegLds], s_kb[kSegLds];
    const bool lds = nseg <= (uint32_t)kSegLds;
    if (lds)
        for (uint32_t i = threadIdx.x; i < nseg; i += 256) {
            s_seg[i] = seg[i];
            s_kb[i] = kb[i];
        }
    __syncthreads();
    const uint32_t *tseg = lds ? s_seg : seg, *tkb = lds ? s_kb : kb;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t p = starts[i];
        const uint32_t s = last_le(tseg, nseg, p);
        const uint64_t j = (uint64_t)tkb[s] + (p - tseg[s]);
        uint64_t w[W];
        if constexpr (W == 4) {
            const uint4 *r = reinterpret_cast<const uint4 *>(table + j * 4);
            const uint4 a = r[0], b = r[1];
            w[0] = ((uint64_t)a.y << 32) | a.x;
            w[1] = ((uint64_t)a.w << 32) | a.z;
            w[2] = ((uint64_t)b.y << 32) | b.x;
            w[3] = ((uint64_t)b.w << 32) | b.z;
        } else if constexpr (W == 2) {
            const uint4 a = *reinterpret_cast<const uint4 *>(table + j * 2);
            w[0] = ((uint64_t)a.y << 32) | a.x;
            w[1] = ((uint64_t)a.w << 32) | a.z;
        } else {
#pragma unroll
            for (int q = 0; q < W; ++q) w[q] = table[j * W + q];
        }
#pragma unroll
        for (int q = 0; q < W; ++q) keys[(uint64_t)q * n + i] = w[q];
    }
}

template <int W, int BITS>
static hipError_t table_gather_w(gk_ctx *c, const KS &k, const uint32_t *starts, uint64_t n, uint64_t *keys,
                                 uint64_t *table, const uint32_t *kb) {
    const int grid = (int)std::min<uint64_t>((n + 255) / 256, 8192);
    hipLaunchKernelGGL((key_table_kernel<W, BITS>), dim3(grid), dim3(256), 0, c->stream, c->sba, k, c->seg, kb,
                       (uint32_t)c->nseg, n, table);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((table_gather_kernel<W>), dim3(grid), dim3(256), 0, c->stream, starts, c->seg, kb,
                       (uint32_t)c->nseg, n, table, keys);
    return hipGetLastError();
}

// Keys through a position-indexed table of 2-bit rows (k <= 63; C5's canonical 63-mers under a
// 4-bit key spec).  The enumeration-order table above computes every key from its own window (a
// contig search, 9 unaligned words, a SWAR pack and a 4-bit expansion per k-mer: 64 ms at C5) and
// stores W words per row (99 GB at C5).  Here a lane computes the keys of kRowPos consecutive
// positions: the first window by SWAR from aligned words, the next ones by rolling the forward and
// reverse-complement values one symbol at a time, and it stores 16 B per position (hi, lo of the
// 2-bit key; 49 GB at C5).  A window holding a byte other than A/C/G/T (IUPAC, N, the '$'
// separators and pad) gets a marker row -- bit 63 of hi, which a 2-bit key of <= 63 symbols never
// sets -- and the gather computes those keys from the window itself.  The gather reads the row of
// each sorted start at its sba position (no contig search) and expands it to the key spec.
constexpr int kRowPos = 16;  // positions per lane
constexpr uint64_t kRowMarker = 1ull << 63;

// Rows leave through LDS: a lane's kRowPos rows are consecutive positions, so stored straight from
// the lane every store instruction would write 64 separate 16-B pieces (3.1e9 partial-line write
// requests at C5: 22 ms); staged per wave in halves of 8 rows, each store writes whole lines.
__global__ __launch_bounds__(256) void key_rows2_kernel(const uint8_t *__restrict__ sba, uint64_t sba_len, int k,
                                                        int canonical, uint64_t *__restrict__ rows) {
    constexpr int kHalf = kRowPos / 2;
    __shared__ uint4 s_rows[4][64 * kHalf + 64];  // per wave; row q at q + q / 8 (conflict-free writes)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint4 *sr = s_rows[wave];
    const uint64_t ng = (sba_len + kRowPos - 1) / kRowPos;
    const int s = 128 - 2 * k;  // right-alignment shift of the first 64 symbols (2 <= s < 128)
    const uint64_t mhi = k > 32 ? (~0ull >> (128 - 2 * k)) : 0ull;
    const uint64_t mlo = k >= 32 ? ~0ull : ((1ull << (2 * k)) - 1);
    const int top = 2 * k - 2;  // bit of the newest symbol's complement in the reverse strand
    // wave-uniform trips: every lane reaches the staging below
    for (uint64_t gw = blockIdx.x * 256ull + wave * 64; gw < ng; gw += (uint64_t)gridDim.x * 256) {
        const uint64_t g = gw + lane;
        const uint64_t p0 = (g < ng ? g : 0) * kRowPos;  // (a lane past the end computes rows it does not store)
        const uint64_t *src = reinterpret_cast<const uint64_t *>(sba + p0);  // 16-B aligned
        // the first window (bytes 0..k-1 after p0): 8 words = 64 symbols left-aligned in fh:fl
        uint64_t fh = 0, fl = 0;
        int lb = -1;  // the last non-ACGT byte so far (relative to p0)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint64_t x = src[j];
            const uint64_t v = pack2_8e(x);  // byte 0 in the most significant pair
            if (j < 4) fh |= v << (48 - 16 * j);
            else fl |= v << (48 - 16 * (j - 4));
            const int nb = min(8, max(0, k - 8 * j));
            const uint64_t m = non_acgt_bytes(x) & (nb == 8 ? ~0ull : ((1ull << (8 * nb)) - 1));
            if (m) lb = 8 * j + ((63 - __builtin_clzll(m)) >> 3);
        }
        if (s >= 64) {
            fl = fh >> (s - 64);
            fh = 0;
        } else {
            fl = (fl >> s) | (fh << (64 - s));
            fh >>= s;
        }
        // its reverse complement, right-aligned (canon2's construction)
        uint64_t rh = rev_pairs(~fl), rl = rev_pairs(~fh);
        if (s >= 64) {
            rl = rh >> (s - 64);
            rh = 0;
        } else {
            rl = (rl >> s) | (rh << (64 - s));
            rh >>= s;
        }
        // bytes k .. k + 14 after p0: the symbols rolled in for positions 1 .. 15
        const uint64_t a = p0 + (uint64_t)k;
        const uint64_t *q = reinterpret_cast<const uint64_t *>(sba + (a & ~7ull));
        const int sh = (int)(a & 7) * 8;
        const uint64_t u0 = q[0], u1 = q[1], u2 = q[2];
        const uint64_t n0 = sh ? (u0 >> sh) | (u1 << (64 - sh)) : u0;
        const uint64_t n1 = sh ? (u1 >> sh) | (u2 << (64 - sh)) : u1;
        const uint64_t c0 = ((n0 >> 1) ^ (n0 >> 2)) & 0x0303030303030303ull;
        const uint64_t c1 = ((n1 >> 1) ^ (n1 >> 2)) & 0x0303030303030303ull;
        const uint64_t b0 = non_acgt_bytes(n0), b1 = non_acgt_bytes(n1);
#pragma unroll
        for (int half = 0; half < 2; ++half) {
#pragma unroll
            for (int rr = 0; rr < kHalf; ++rr) {
                const int r = half * kHalf + rr;
                if (r > 0) {  // roll in byte k - 1 + r
                    const int i = r - 1;
                    const uint64_t c = ((i < 8 ? c0 : c1) >> (8 * (i & 7))) & 3;
                    if (((i < 8 ? b0 : b1) >> (8 * (i & 7) + 7)) & 1) lb = k - 1 + r;
                    fh = ((fh << 2) | (fl >> 62)) & mhi;
                    fl = ((fl << 2) | c) & mlo;
                    rl = (rl >> 2) | (rh << 62);
                    rh >>= 2;
                    if (top >= 64) rh |= (3 - c) << (top - 64);
                    else rl |= (3 - c) << top;
                }
                uint64_t h = fh, l = fl;
                if (canonical && (rh < fh || (rh == fh && rl < fl))) {
                    h = rh;
                    l = rl;
                }
                if (lb >= r) {
                    h = kRowMarker;
                    l = 0;
                }
                const int qi = lane * kHalf + rr;
                sr[qi + (qi >> 3)] = make_uint4((uint32_t)h, (uint32_t)(h >> 32), (uint32_t)l, (uint32_t)(l >> 32));
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
            // staged row qi = lane' * 8 + rr' is position gw * 16 + 16 lane' + 8 half + rr': runs of 8
            // rows (128 B, line-aligned) per lane'
#pragma unroll
            for (int j = 0; j < kHalf; ++j) {
                const int qi = j * 64 + lane;
                const uint64_t pos = (gw + (uint64_t)(qi >> 3)) * kRowPos + half * kHalf + (qi & 7);
                const uint4 v = sr[qi + (qi >> 3)];
                if (pos < sba_len) *reinterpret_cast<uint4 *>(rows + 2 * pos) = v;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
            __builtin_amdgcn_wave_barrier();  // the staging is read before the next half overwrites it
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
        }
    }
}

// The gather proper is a small kernel (many waves, U rows in flight per lane). Each random 16-B row
// costs a whole 128-B line of HBM reads (391 GB per C5 launch, profiles/r3/prof_c5_end2: 5.6 TB/s
// with the key writes); non-temporal row loads measured the same.  The keys of marker rows --
// about 5 % of C5's k-mers, the N runs, sorted together -- are left to row2_fix_kernel through a
// list appended per wave (one atomic per wave).  With the per-byte path inlined in the gather, its registers cut the waves in flight
// and the gather took 125 ms at C5 against 93 ms for the W-word rows.
template <int W, int BITS>
__global__ __launch_bounds__(256) void row2_gather_kernel(KS ks, const uint32_t *__restrict__ starts, uint64_t n,
                                                          const uint64_t *__restrict__ rows,
                                                          uint64_t *__restrict__ keys, uint32_t *__restrict__ fix_cnt,
                                                          uint32_t *__restrict__ fix_idx) {
#ifndef GKM_ROW_U
#define GKM_ROW_U 4
#endif
    constexpr int U = GKM_ROW_U;  // rows in flight per lane (A/B knob)
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const int lane = threadIdx.x & 63;
    for (uint64_t i0 = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i0 < n + (U - 1) * stride; i0 += U * stride) {
        uint32_t p[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = i0 + u * stride;
            p[u] = i < n ? starts[i] : 0u;
        }
        uint4 r[U];
#pragma unroll
        for (int u = 0; u < U; ++u) r[u] = *reinterpret_cast<const uint4 *>(rows + 2 * (uint64_t)p[u]);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = i0 + u * stride;
            const uint64_t hi = ((uint64_t)r[u].y << 32) | r[u].x, lo = ((uint64_t)r[u].w << 32) | r[u].z;
            const bool mk = i < n && (hi & kRowMarker);
            const uint64_t m = __ballot(mk);
            if (m) {  // wave-uniform
                const int leader = __builtin_ctzll(m);
                uint32_t base = 0;
                if (lane == leader) base = atomicAdd(fix_cnt, (uint32_t)__popcll(m));
                base = __shfl(base, leader);
                if (mk)
                    fix_idx[base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] = (uint32_t)i;
            }
            if (i < n && !mk) {
                uint64_t w[W];
                key_from_2bit<W, BITS>(hi, lo, ks.symbols, w);
#pragma unroll
                for (int q = 0; q < W; ++q) keys[(uint64_t)q * n + i] = w[q];
            }
        }
    }
}

// true iff the k (<= 64) bytes from sba[s] all equal ch (8-byte loads from s & ~7, as window2_acgt)
__device__ __forceinline__ bool window_homo(const uint8_t *sba, uint64_t s, int k, uint32_t ch) {
    const uint64_t pat = 0x0101010101010101ull * ch;
    const uint64_t a = s & ~7ull;
    const int sh = (int)(s - a) * 8;
    const uint64_t *p = reinterpret_cast<const uint64_t *>(sba + a);
    uint64_t prev = p[0], diff = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        if (8 * j >= k) break;
        const uint64_t nxt = p[j + 1];
        const uint64_t w = sh ? (prev >> sh) | (nxt << (64 - sh)) : prev;
        prev = nxt;
        const int nb = min(8, k - 8 * j);
        diff |= (w ^ pat) & (nb == 8 ? ~0ull : ((1ull << (8 * nb)) - 1));
    }
    return diff == 0;
}

// keys of the sorted entries whose rows are markers (a window with a non-ACGT byte), from the window.
// Homopolymers (one letter k times: GRCh38's N runs, ~150 M of C5's markers, sorted together) take
// a short path: the letter's code -- canonical: the smaller of it and its complement's -- k times.
template <int W, int BITS>
__global__ __launch_bounds__(256) void row2_fix_kernel(const uint8_t *__restrict__ sba, KS ks,
                                                       const uint32_t *__restrict__ starts, uint64_t n,
                                                       const uint32_t *__restrict__ fix_cnt,
                                                       const uint32_t *__restrict__ fix_idx,
                                                       uint64_t *__restrict__ keys) {
    __shared__ uint8_t s_lut4[256];
    s_lut4[threadIdx.x] = c_code4[threadIdx.x];
    __syncthreads();
    const uint32_t cnt = *fix_cnt;
    for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < cnt; j += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t i = fix_idx[j];
        const uint32_t p = starts[i];
        uint64_t w[W];
        const uint32_t ch = sba[p];
        if (BITS == 4 && window_homo(sba, p, ks.symbols, ch)) {
            uint32_t code = s_lut4[ch];
            if (ks.canonical) code = min(code, comp_sym<4>(code));
            const uint64_t rep = (uint64_t)code * 0x1111111111111111ull;
#pragma unroll
            for (int q = 0; q < W; ++q) {  // q: word from the least significant end (key_from_2bit)
                const int left = ks.symbols - 16 * q;
                w[W - 1 - q] = left >= 16 ? rep : left <= 0 ? 0ull : rep & (~0ull >> (64 - 4 * left));
            }
        } else {
            fast_window_key<W, BITS>(sba, ks, p, s_lut4, w);
        }
#pragma unroll
        for (int q = 0; q < W; ++q) keys[(uint64_t)q * n + i] = w[q];
    }
}

template <int W, int BITS>
static hipError_t row2_gather_w(gk_ctx *c, const KS &k, const uint32_t *starts, uint64_t n, uint64_t *keys,
                                uint64_t *rows, uint32_t *fix_cnt, uint32_t *fix_idx) {
    const uint64_t ng = (c->sba_len + kRowPos - 1) / kRowPos;
    const int g1 = (int)std::max<uint64_t>(1, std::min<uint64_t>((ng + 255) / 256, 8192));
    hipLaunchKernelGGL(key_rows2_kernel, dim3(g1), dim3(256), 0, c->stream, c->sba, (uint64_t)c->sba_len, k.symbols,
                       k.canonical, rows);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(fix_cnt, 0, 4, c->stream);
    if (e != hipSuccess) return e;
    const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>((n + 255) / 256, 8192));
    hipLaunchKernelGGL((row2_gather_kernel<W, BITS>), dim3(grid), dim3(256), 0, c->stream, k, starts, n, rows, keys,
                       fix_cnt, fix_idx);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((row2_fix_kernel<W, BITS>), dim3(2048), dim3(256), 0, c->stream, c->sba, k, starts, n, fix_cnt,
                       fix_idx, keys);
    return hipGetLastError();
}

template <int W, int BITS, bool BOUNDED>
__global__ __launch_bounds__(256) void encode_gather_kernel(const uint8_t *__restrict__ sba, KS ks,
                                                            const uint32_t *__restrict__ starts, uint64_t n,
                                                            uint64_t *__restrict__ keys) {
    __shared__ uint8_t s_lut4[256];
    s_lut4[threadIdx.x] = c_code4[threadIdx.x];
    __syncthreads();
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint8_t *b = sba + starts[i];
        uint64_t w[W];
        if (!BOUNDED && (BITS == 2 || BITS == 4) && ks.canonical) {  // fixed length: canonical strand
            const bool rc = canon_is_rc<(BITS == 2 ? 2 : 4)>(b, ks.symbols, s_lut4);
#pragma unroll
            for (int k = 0; k < W; ++k) w[k] = 0;
            for (int t = 0; t < ks.symbols; ++t)
                bi_shl_or<W>(w, BITS, canon_sym<(BITS == 2 ? 2 : 4)>(b, ks.symbols, t, rc, s_lut4));
        } else {
            window_key<W, BITS, BOUNDED>(ks, [&](int k) { return (uint32_t)b[k]; }, s_lut4, w);
        }
#pragma unroll
        for (int k = 0; k < W; ++k) keys[(uint64_t)k * n + i] = w[k];
    }
}

template <int BITS>
__global__ __launch_bounds__(256) void canon_strand_kernel(const uint8_t *__restrict__ sba, int k,
                                                           const uint32_t *__restrict__ starts, uint64_t n,
                                                           uint8_t *__restrict__ out) {
    __shared__ uint8_t s_lut4[256];
    s_lut4[threadIdx.x] = c_code4[threadIdx.x];
    __syncthreads();
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        out[i] = canon_is_rc<BITS>(sba + starts[i], k, s_lut4) ? 1 : 0;
}

hipError_t launch_canon_strands(gk_ctx *c, const KeySpec &ks, const uint32_t *starts, uint64_t n, uint8_t *out) {
    hipError_t e = init_tables();
    if (e != hipSuccess) return e;
    const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>((n + 255) / 256, 8192));
    if (ks.bits == 2)
        hipLaunchKernelGGL(canon_strand_kernel<2>, dim3(grid), dim3(256), 0, c->stream, c->sba, ks.symbols, starts, n,
                           out);
    else
        hipLaunchKernelGGL(canon_strand_kernel<4>, dim3(grid), dim3(256), 0, c->stream, c->sba, ks.symbols, starts, n,
                           out);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// dispatch
// ---------------------------------------------------------------------------------------------
template <int W, int BITS, bool BOUNDED>
static hipError_t dispatch_generic(gk_ctx *c, const KS &k, uint64_t *keys, uint32_t *vals, uint32_t *hist, int grid) {
    hipLaunchKernelGGL((encode_generic_kernel<W, BITS, BOUNDED>), dim3(grid), dim3(256), 0, c->stream, c->sba,
                       c->sba_len, c->seg, (uint32_t)c->nseg, k, c->n, keys, vals, hist);
    return hipGetLastError();
}

template <int BITS, bool BOUNDED>
static hipError_t dispatch_generic_w(gk_ctx *c, const KS &k, uint64_t *keys, uint32_t *vals, uint32_t *hist, int grid) {
    switch (k.words) {
    case 1: return dispatch_generic<1, BITS, BOUNDED>(c, k, keys, vals, hist, grid);
    case 2: return dispatch_generic<2, BITS, BOUNDED>(c, k, keys, vals, hist, grid);
    case 3: return dispatch_generic<3, BITS, BOUNDED>(c, k, keys, vals, hist, grid);
    case 4: return dispatch_generic<4, BITS, BOUNDED>(c, k, keys, vals, hist, grid);
    }
    return hipErrorInvalidValue;
}

hipError_t launch_encode_positions(gk_ctx *c, const KeySpec &ks, uint64_t *keys, uint32_t *vals, uint32_t *hist) {
    hipError_t e = init_tables();
    if (e != hipSuccess) return e;
    KS k = pod(ks);
    if (hist == nullptr) k.digits = 0;  // no digit histograms (the MSD sort counts its own)
    if (k.digits) {
        e = hipMemsetAsync(hist, 0, sizeof(uint32_t) * 256 * k.digits, c->stream);
        if (e != hipSuccess) return e;
    }
    const uint64_t ntiles = (c->sba_len + kEncodeTile - 1) / kEncodeTile;
    int grid = (int)std::min<uint64_t>(ntiles, 256 * 6);
    if (grid < 1) grid = 1;
    const bool bounded = ks.symbols != ks.min_len;
    if (!bounded && ks.words == 1 && (ks.bits == 2 || ks.bits == 4) && ks.symbols <= 64) {
        if (ks.bits == 2)
            hipLaunchKernelGGL(encode_roll_w1_kernel<2>, dim3(grid), dim3(256), 0, c->stream, c->sba, c->sba_len,
                               c->seg, (uint32_t)c->nseg, k, keys, vals, hist);
        else
            hipLaunchKernelGGL(encode_roll_w1_kernel<4>, dim3(grid), dim3(256), 0, c->stream, c->sba, c->sba_len,
                               c->seg, (uint32_t)c->nseg, k, keys, vals, hist);
        return hipGetLastError();
    }
    static const bool no_roll = opt("GKM_NO_ROLL_BOUNDED") != nullptr;  // (A/B)
    static const bool no_roll_hist = opt("GKM_NO_ROLL_HIST") != nullptr;  // (A/B)
    if (bounded && (hist == nullptr || (!no_roll_hist && k.digits <= 8)) && ks.words == 1 &&
        (ks.bits == 2 || ks.bits == 3) && ks.symbols <= 32 && ks.min_len >= 1 && !no_roll) {
        auto go = [&](auto fn) {
            hipLaunchKernelGGL(fn, dim3(grid), dim3(256), 0, c->stream, c->sba, c->sba_len, c->seg, (uint32_t)c->nseg,
                               k, keys, vals, hist);
        };
        if (ks.bits == 2)
            hist ? go(encode_roll_bounded_kernel<2, true>) : go(encode_roll_bounded_kernel<2, false>);
        else
            hist ? go(encode_roll_bounded_kernel<3, true>) : go(encode_roll_bounded_kernel<3, false>);
        return hipGetLastError();
    }
    if (ks.bits == 2) return bounded ? dispatch_generic_w<2, true>(c, k, keys, vals, hist, grid)
                                     : dispatch_generic_w<2, false>(c, k, keys, vals, hist, grid);
    if (ks.bits == 3) return dispatch_generic_w<3, true>(c, k, keys, vals, hist, grid);
    return bounded ? dispatch_generic_w<4, true>(c, k, keys, vals, hist, grid)
                   : dispatch_generic_w<4, false>(c, k, keys, vals, hist, grid);
}

// sort_doubling's first round: the rank of p + o after the seed sort orders like the seed key of
// p + o, so the tied elements take that key from their window instead of every position being
// ranked first (a random 4-byte scatter per position)
template <int BITS>
__global__ __launch_bounds__(256) void member_seed_key_kernel(const uint8_t *__restrict__ sba, KS ks,
                                                              const uint8_t *__restrict__ flags,
                                                              const uint32_t *__restrict__ vals,
                                                              const uint32_t *__restrict__ seg, uint32_t nseg,
                                                              uint64_t L, uint64_t o, uint64_t n,
                                                              uint64_t *__restrict__ keys) {
    __shared__ uint8_t s_lut4[256];
    s_lut4[threadIdx.x] = c_code4[threadIdx.x];
    __syncthreads();
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        if (flags[i] != 0 && (i + 1 >= n || flags[i + 1] != 0)) continue;  // a group of one
        const uint64_t p = vals[i];
        const uint64_t q = p + o;
        if (q > seg_end_of(seg, nseg, L, p)) {
            keys[i] = 0;
            continue;
        }
        uint64_t w[1];
        window_key<1, BITS, true>(ks, [&](int k) { return (uint32_t)sba[q + k]; }, s_lut4, w);
        keys[i] = w[0];
    }
}

hipError_t launch_member_seed_keys(gk_ctx *c, const KeySpec &seed, const uint8_t *flags, const uint32_t *vals,
                                   uint64_t o, uint64_t n, uint64_t *keys) {
    hipError_t e = init_tables();
    if (e != hipSuccess) return e;
    const KS k = pod(seed);
    const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>((n + 255) / 256, 8192));
    if (seed.bits == 2)
        hipLaunchKernelGGL(member_seed_key_kernel<2>, dim3(grid), dim3(256), 0, c->stream, c->sba, k, flags, vals, c->seg,
                           (uint32_t)c->nseg, (uint64_t)c->sba_len, o, n, keys);
    else if (seed.bits == 3)
        hipLaunchKernelGGL(member_seed_key_kernel<3>, dim3(grid), dim3(256), 0, c->stream, c->sba, k, flags, vals, c->seg,
                           (uint32_t)c->nseg, (uint64_t)c->sba_len, o, n, keys);
    else
        hipLaunchKernelGGL(member_seed_key_kernel<4>, dim3(grid), dim3(256), 0, c->stream, c->sba, k, flags, vals, c->seg,
                           (uint32_t)c->nseg, (uint64_t)c->sba_len, o, n, keys);
    return hipGetLastError();
}

template <int W, int BITS, bool BOUNDED>
static hipError_t gather_w(gk_ctx *c, const KS &k, const uint32_t *starts, uint64_t n, uint64_t *keys) {
    int grid = (int)std::min<uint64_t>((n + 255) / 256, 8192);
    if (grid < 1) grid = 1;
    static const bool slow = opt("GKM_GATHER_SLOW") != nullptr;  // A/B of the per-byte path
    if constexpr (!BOUNDED && (BITS == 2 || BITS == 4))
        if (k.symbols <= 64 && !slow) {
            hipLaunchKernelGGL((encode_gather_fast_kernel<W, BITS>), dim3(grid), dim3(256), 0, c->stream, c->sba, k,
                               starts, n, keys);
            return hipGetLastError();
        }
    hipLaunchKernelGGL((encode_gather_kernel<W, BITS, BOUNDED>), dim3(grid), dim3(256), 0, c->stream, c->sba, k,
                       starts, n, keys);
    return hipGetLastError();
}

template <int BITS, bool BOUNDED>
static hipError_t gather_dispatch(gk_ctx *c, const KS &k, const uint32_t *starts, uint64_t n, uint64_t *keys) {
    switch (k.words) {
    case 1: return gather_w<1, BITS, BOUNDED>(c, k, starts, n, keys);
    case 2: return gather_w<2, BITS, BOUNDED>(c, k, starts, n, keys);
    case 3: return gather_w<3, BITS, BOUNDED>(c, k, starts, n, keys);
    case 4: return gather_w<4, BITS, BOUNDED>(c, k, starts, n, keys);
    }
    return hipErrorInvalidValue;
}

hipError_t launch_encode_table_gather(gk_ctx *c, const KeySpec &ks, const uint32_t *starts, uint64_t n,
                                      uint64_t *keys, uint64_t *table, uint64_t table_bytes) {
    hipError_t e = init_tables();
    if (e != hipSuccess) return e;
    KS k = pod(ks);
    // the position-indexed 2-bit rows when they fit the table buffer (k <= 63)
    static const bool enum_rows = opt("GKM_KEY_TABLE_ENUM") != nullptr;  // (A/B: the W-word rows)
    // (the rows, then the fix-up list of marker entries -- at most n -- in the same buffer)
    const uint64_t rows_bytes = 16 * (((uint64_t)c->sba_len + kRowPos - 1) / kRowPos * kRowPos);
    if (!enum_rows && ks.symbols <= 63 && rows_bytes + 4 * (n + 64) <= table_bytes) {
        uint32_t *fix_idx = reinterpret_cast<uint32_t *>(reinterpret_cast<uint8_t *>(table) + rows_bytes);
        uint32_t *fix_cnt = nullptr;
        if (scratch(c, "rows_fix_cnt", 64, &fix_cnt) != hipSuccess) return hipErrorOutOfMemory;
        if (ks.bits == 2 && ks.words == 2) e = row2_gather_w<2, 2>(c, k, starts, n, keys, table, fix_cnt, fix_idx);
        else if (ks.bits == 4 && ks.words == 2) e = row2_gather_w<2, 4>(c, k, starts, n, keys, table, fix_cnt, fix_idx);
        else if (ks.bits == 4 && ks.words == 3) e = row2_gather_w<3, 4>(c, k, starts, n, keys, table, fix_cnt, fix_idx);
        else if (ks.bits == 4 && ks.words == 4) e = row2_gather_w<4, 4>(c, k, starts, n, keys, table, fix_cnt, fix_idx);
        else return hipErrorNotSupported;
        return e;
    }
    // kb: exclusive prefix of the contigs' k-mer counts (kmers.py:837-861 counts)
    std::vector<uint32_t> kb(c->nseg);
    uint64_t acc = 0;
    for (uint64_t s = 0; s < c->nseg; ++s) {
        kb[s] = (uint32_t)acc;
        const uint64_t end = (s + 1 == c->nseg) ? c->sba_len - 1 : (uint64_t)c->hseg[s + 1] - 2;
        const uint64_t len = end - c->hseg[s] + 1;
        if (len >= (uint64_t)ks.symbols) acc += len - ks.symbols + 1;
    }
    if (acc != n) return hipErrorNotSupported;  // not the whole enumeration: the caller gathers windows
    uint32_t *d_kb = nullptr;
    if (scratch(c, "enc_kb", std::max<uint64_t>(c->nseg, 1), &d_kb) != hipSuccess) return hipErrorOutOfMemory;
    e = hipMemcpyAsync(d_kb, kb.data(), 4 * c->nseg, hipMemcpyHostToDevice, c->stream);
    if (e != hipSuccess) return e;
    if (ks.bits == 2) {
        switch (ks.words) {
        case 2: e = table_gather_w<2, 2>(c, k, starts, n, keys, table, d_kb); break;
        default: return hipErrorNotSupported;
        }
    } else {
        switch (ks.words) {
        case 2: e = table_gather_w<2, 4>(c, k, starts, n, keys, table, d_kb); break;
        case 3: e = table_gather_w<3, 4>(c, k, starts, n, keys, table, d_kb); break;
        case 4: e = table_gather_w<4, 4>(c, k, starts, n, keys, table, d_kb); break;
        default: return hipErrorNotSupported;
        }
    }
    if (e != hipSuccess) return e;
    return hipStreamSynchronize(c->stream);  // kb (host vector) was read by an async copy
}

hipError_t launch_encode_gather(gk_ctx *c, const KeySpec &ks, const uint32_t *starts, uint64_t n, uint64_t *keys) {
    hipError_t e = init_tables();
    if (e != hipSuccess) return e;
    KS k = pod(ks);
    const bool bounded = ks.symbols != ks.min_len;
    if (ks.bits == 2) return bounded ? gather_dispatch<2, true>(c, k, starts, n, keys)
                                     : gather_dispatch<2, false>(c, k, starts, n, keys);
    if (ks.bits == 3) return gather_dispatch<3, true>(c, k, starts, n, keys);
    return bounded ? gather_dispatch<4, true>(c, k, starts, n, keys) : gather_dispatch<4, false>(c, k, starts, n, keys);
}

}  // namespace gkm

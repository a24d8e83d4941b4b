// gkm_canon.h -- canonical k-mers: the smaller of a k-mer and its reverse complement (gfx950).
//
// The complement is the reference's IUPAC mapping (SequenceCollection._get_complement_mapping_array,
// sequence_collection.py:402-433; reverse_complement_sba :42-73): A<->T C<->G R<->Y K<->M B<->V
// D<->H, S W N self-complementary.  The reference defines no canonical k-mer (kmers.py:689-696 only
// raises for other strands), so "canonical" here is this build's extension: min(x, revcomp(x))
// under the reference's byte order (kmers.py:306-397) for fixed-length k-mers.  The symbol codes
// are order-isomorphic to that byte order, so the comparison runs on codes:
//   2-bit (ACGT data)   A0 C1 G2 T3            complement = 3 - c
//   4-bit (IUPAC data)  $0 A1 B2 C3 D4 G5 H6 K7 M8 N9 R10 S11 T12 V13 W14 Y15
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gkm {

// nibble c of kComp4 = code of the complement of code c (4-bit codes)
//   c:    0  1  2  3  4  5  6  7  8  9 10 11 12 13 14 15
//   comp: 0 12 13  5  6  3  4  8  7  9 15 11  1  2 14 10
constexpr uint64_t kComp4 = 0xAE21BF9784365DC0ull;

template <int BITS>
__device__ __forceinline__ uint32_t comp_sym(uint32_t s) {
    if (BITS == 2) return 3u - s;
    return (uint32_t)(kComp4 >> (4 * s)) & 15u;
}

// symbol code of an sba byte (2-bit: ACGT only; 4-bit: lut4 maps '$' and IUPAC letters)
template <int BITS>
__device__ __forceinline__ uint32_t canon_code(uint32_t ch, const uint8_t *lut4) {
    if (BITS == 2) return ((ch >> 1) ^ (ch >> 2)) & 3u;
    return lut4[ch];
}

// reverse complement of the n right-aligned symbols of x (n * BITS <= 64)
template <int BITS>
__device__ __forceinline__ uint64_t revcomp_word(uint64_t x, int n) {
    uint64_t y;
    if (BITS == 2) {
        y = __builtin_bitreverse64(~x);  // complement, groups (and their bit pairs) reversed
        y = ((y >> 1) & 0x5555555555555555ull) | ((y & 0x5555555555555555ull) << 1);
        return y >> (64 - 2 * n);
    }
    y = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) y |= (uint64_t)comp_sym<4>((uint32_t)(x >> (4 * j)) & 15u) << (4 * j);
    y = __builtin_bswap64(y);
    y = ((y >> 4) & 0x0F0F0F0F0F0F0F0Full) | ((y & 0x0F0F0F0F0F0F0F0Full) << 4);
    return y >> (64 - 4 * n);
}

// true iff the reverse complement of the k-mer b[0..k) is strictly smaller than the k-mer
template <int BITS>
__device__ __forceinline__ bool canon_is_rc(const uint8_t *b, int k, const uint8_t *lut4) {
    for (int j = 0; j < k; ++j) {
        const uint32_t f = canon_code<BITS>(b[j], lut4);
        const uint32_t r = comp_sym<BITS>(canon_code<BITS>(b[k - 1 - j], lut4));
        if (f != r) return r < f;
    }
    return false;  // palindrome: both strands equal
}

// symbol t of the canonical k-mer
template <int BITS>
__device__ __forceinline__ uint32_t canon_sym(const uint8_t *b, int k, int t, bool rc, const uint8_t *lut4) {
    return rc ? comp_sym<BITS>(canon_code<BITS>(b[k - 1 - t], lut4)) : canon_code<BITS>(b[t], lut4);
}

}  // namespace gkm

// SWAR helpers over 8 sequence bytes (gkm_msd.hip's L0 packing, gkm_split.hip's class-B flags)
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

namespace gkm {

// SWAR over 8 bytes (byte 0 = the first position): bit 7 of each byte set iff the byte is zero
__device__ __forceinline__ uint64_t zero_bytes(uint64_t y) {
    constexpr uint64_t k7F = 0x7F7F7F7F7F7F7F7Full;
    return ~(((y & k7F) + k7F) | y | k7F);
}

// the 8 flag bits (bit 7 of each byte) as one byte, position 0 in the most significant bit
__device__ __forceinline__ uint32_t gather_flags8(uint64_t z) {
    uint64_t t = __builtin_bswap64(z) >> 7;
    t = (t | (t >> 7)) & 0x0003000300030003ull;
    t = (t | (t >> 14)) & 0x0000000F0000000Full;
    return (uint32_t)((t | (t >> 28)) & 0xFFu);
}

// bit 7 of each byte set iff the byte is not one of A, C, G, T
__device__ __forceinline__ uint64_t non_acgt_bytes(uint64_t x) {
    constexpr uint64_t kOnes = 0x0101010101010101ull;
    return ~(zero_bytes(x ^ (kOnes * 'A')) | zero_bytes(x ^ (kOnes * 'C')) | zero_bytes(x ^ (kOnes * 'G')) |
             zero_bytes(x ^ (kOnes * 'T'))) &
           (kOnes << 7);
}

// 16 2-bit symbols (x, right-aligned, A0 C1 G2 T3) as 16 4-bit codes of the 4-bit alphabet
// '$' A B C D G H K M N R S T V W Y (A 1, C 3, G 5, T 12: 2 s + 1, plus 5 for T), one per nibble
__device__ __forceinline__ uint64_t expand4_16(uint32_t x) {
    uint64_t v = x;
    v = (v | (v << 16)) & 0x0000FFFF0000FFFFull;
    v = (v | (v << 8)) & 0x00FF00FF00FF00FFull;
    v = (v | (v << 4)) & 0x0F0F0F0F0F0F0F0Full;
    v = (v | (v << 2)) & 0x3333333333333333ull;  // one symbol per nibble
    const uint64_t t = v & (v >> 1) & 0x1111111111111111ull;  // T
    return (v << 1) + 0x1111111111111111ull + t * 5;
}

// the W-word 4-bit key (most significant word first) of k <= 32 symbols given as a right-aligned
// 2-bit key (the ACGT-only k-mers' MSD keys)
template <int W>
__device__ __forceinline__ void expand4_key(uint64_t key2, int k, uint64_t (&w)[W]) {
#pragma unroll
    for (int q = 0; q < W; ++q) {  // q: word from the least significant end
        uint64_t e = q < 2 ? expand4_16((uint32_t)(key2 >> (32 * q))) : 0ull;
        const int left = k - 16 * q;  // symbols in this word
        if (left < 16) e &= left <= 0 ? 0ull : (~0ull >> (64 - 4 * left));
        w[W - 1 - q] = e;
    }
}

// (below: gkm_encode.hip's key encoders and gkm_split.hip's merge, which gathers the class-A keys
// of k > 32 from a 2-bit packed copy of the sequence)

// 2-bit codes (A0 C1 G2 T3) of 8 bytes as 16 bits, byte 0 in the most significant pair
__device__ __forceinline__ uint32_t pack2_8e(uint64_t x) {
    uint64_t t = __builtin_bswap64(((x >> 1) ^ (x >> 2)) & 0x0303030303030303ull);
    t = (t | (t >> 6)) & 0x000F000F000F000Full;
    t = (t | (t >> 12)) & 0x000000FF000000FFull;
    return (uint32_t)((t | (t >> 24)) & 0xFFFFu);
}

// the 32 2-bit groups of x in reverse order
__device__ __forceinline__ uint64_t rev_pairs(uint64_t x) {
    x = __builtin_bswap64(x);
    x = ((x >> 4) & 0x0F0F0F0F0F0F0F0Full) | ((x & 0x0F0F0F0F0F0F0F0Full) << 4);
    return ((x >> 2) & 0x3333333333333333ull) | ((x & 0x3333333333333333ull) << 2);
}

// canonical = min(k-mer, reverse complement) of a right-aligned 2k-bit value, in place
__device__ __forceinline__ void canon2(int k, uint64_t &hi, uint64_t &lo) {
    uint64_t rh = rev_pairs(~lo), rl = rev_pairs(~hi);  // complement, 64 groups reversed (left-aligned)
    const int s = 128 - 2 * k;
    if (s >= 64) {
        rl = rh >> (s - 64);
        rh = 0;
    } else if (s > 0) {
        rl = (rl >> s) | (rh << (64 - s));
        rh >>= s;
    }
    if (rh < hi || (rh == hi && rl < lo)) {
        hi = rh;
        lo = rl;
    }
}

// the W key words (BITS-bit symbols) of a k-symbol ACGT k-mer given as a right-aligned 2k-bit value
template <int W, int BITS>
__device__ __forceinline__ void key_from_2bit(uint64_t hi, uint64_t lo, int k, uint64_t (&w)[W]) {
    if (BITS == 2) {
        w[W - 1] = lo;
        if (W > 1) w[0] = hi;
    } else {
        const uint64_t part[4] = {lo & 0xFFFFFFFFull, lo >> 32, hi & 0xFFFFFFFFull, hi >> 32};
#pragma unroll
        for (int q = 0; q < W; ++q) {  // q: word from the least significant end
            uint64_t e = expand4_16((uint32_t)part[q]);
            const int left = k - 16 * q;  // symbols in this word
            if (left < 16) e &= left <= 0 ? 0ull : (~0ull >> (64 - 4 * left));
            w[W - 1 - q] = e;
        }
    }
}

// One word of the 2-bit packed sequence layout (gkm_msd.hip pack2_kernel, the L0 kernels' LDS
// tiles): 32 bytes from p (16-byte aligned) -> their 2-bit codes (A0 C1 G2 T3, position 0 in the
// most significant pair; other bytes get some code) and their '$' flags (position 0 in bit 31)
// NONACGT: the flags mark every byte other than A/C/G/T ('$' included) -- the stops of the class-A
// (ACGT-only) k-mers of a mixed sba, and on an ACGT sba the same bits as the '$' flags
template <bool NONACGT = false>
__device__ __forceinline__ void pack2_word(const uint8_t *p, uint64_t &cw, uint32_t &dw) {
    constexpr uint64_t kOnes = 0x0101010101010101ull;
    const uint4 *s4 = reinterpret_cast<const uint4 *>(p);
    const uint4 ra = s4[0], rb = s4[1];
    const uint64_t x[4] = {((uint64_t)ra.y << 32) | ra.x, ((uint64_t)ra.w << 32) | ra.z,
                           ((uint64_t)rb.y << 32) | rb.x, ((uint64_t)rb.w << 32) | rb.z};
    cw = 0;
    dw = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        cw = (cw << 16) | pack2_8e(x[j]);
        const uint64_t f = NONACGT ? non_acgt_bytes(x[j]) : zero_bytes(x[j] ^ (kOnes * 0x24u));  // ('$')
        dw = (dw << 8) | gather_flags8(f);
    }
}

}  // namespace gkm

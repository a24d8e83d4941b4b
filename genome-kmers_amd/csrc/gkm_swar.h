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

}  // namespace gkm

// gkm_synth.cpp -- the reference's synthetic genome generator, in C++ (host).
//
// profiling.get_random_seq (profiling.py:12-24) draws its bases with
// np.random.choice(["A", "T", "G", "C"], seq_len) after np.random.seed(s): numpy's legacy
// RandomState, i.e. MT19937 seeded by init_genrand(s), and choice -> randint(0, 4) -> a masked
// bounded draw whose mask (3) never rejects, so base i is "ATGC"[genrand_int32() & 3].  The stream
// is chunk-invariant, so the 3.1 Gb C3 genome is exactly what the reference's generator would
// return for the same seed, made here at ~1 ns per base instead of numpy's ~10 ns
// (tests/test_synthetic.py checks it against numpy's RandomState).
#include <stdint.h>

#include "gkm.h"

namespace {
struct Mt19937 {
    static constexpr int N = 624, M = 397;
    uint32_t mt[N];
    explicit Mt19937(uint32_t s) {
        mt[0] = s;
        for (int k = 1; k < N; ++k) mt[k] = 1812433253u * (mt[k - 1] ^ (mt[k - 1] >> 30)) + (uint32_t)k;
    }
    static uint32_t mix(uint32_t a, uint32_t b, uint32_t c) {
        const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
        return c ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    void twist() {
        int k = 0;
        for (; k < N - M; ++k) mt[k] = mix(mt[k], mt[k + 1], mt[k + M]);
        for (; k < N - 1; ++k) mt[k] = mix(mt[k], mt[k + 1], mt[k + M - N]);
        mt[N - 1] = mix(mt[N - 1], mt[0], mt[M - 1]);
    }
    static uint32_t temper(uint32_t y) {
        y ^= y >> 11;
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        return y ^ (y >> 18);
    }
};
}  // namespace

extern "C" int gk_reference_random_bases(uint8_t *out, uint64_t n, uint32_t seed) {
    if (!out && n) return GK_E_ARG;
    static const uint8_t kBases[4] = {'A', 'T', 'G', 'C'};
    Mt19937 g(seed);
    for (uint64_t p = 0; p < n; p += Mt19937::N) {  // one twist per 624 bases
        g.twist();
        const uint64_t m = n - p < (uint64_t)Mt19937::N ? n - p : (uint64_t)Mt19937::N;
        for (uint64_t k = 0; k < m; ++k) out[p + k] = kBases[Mt19937::temper(g.mt[k]) & 3u];
    }
    return GK_OK;
}

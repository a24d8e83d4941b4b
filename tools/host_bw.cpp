// Host memory bandwidth of the GPU box's CPU share (context for gk_set_sequence's packed
// transfer): streaming read and read+quarter-write (the packing's traffic shape) at 1..32 threads.
// Build: g++ -O3 -mavx2 -pthread tools/host_bw.cpp -o /tmp/host_bw ; run: /tmp/host_bw
#include <immintrin.h>
#include <stdint.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

int main() {
    const uint64_t L = 3100000000ull;
    uint8_t *s = (uint8_t *)aligned_alloc(64, L);
    uint8_t *d = (uint8_t *)aligned_alloc(64, L / 4);
    for (uint64_t i = 0; i < L; i += 4096) s[i] = 1;
    for (uint64_t i = 0; i < L / 4; i += 4096) d[i] = 1;
    for (int T : {1, 2, 4, 8, 16, 32}) {
        for (int mode = 0; mode < 2; ++mode) {
            double best = 1e9;
            for (int rep = 0; rep < 2; ++rep) {
                std::vector<uint64_t> acc(T * 8);
                auto t0 = std::chrono::steady_clock::now();
                std::vector<std::thread> th;
                for (int t = 0; t < T; t++)
                    th.emplace_back([&, t] {
                        const uint64_t a = L * t / T / 64 * 64, b = L * (t + 1) / T / 64 * 64;
                        __m256i x = _mm256_setzero_si256();
                        for (uint64_t i = a; i + 64 <= b; i += 64) {
                            const __m256i v = _mm256_xor_si256(_mm256_loadu_si256((const __m256i *)(s + i)),
                                                               _mm256_loadu_si256((const __m256i *)(s + i + 32)));
                            x = _mm256_xor_si256(x, v);
                            if (mode) _mm_storeu_si128((__m128i *)(d + i / 4), _mm256_castsi256_si128(v));
                        }
                        acc[t * 8] = (uint64_t)_mm256_extract_epi64(x, 0);
                    });
                for (auto &t : th) t.join();
                const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                if (dt < best) best = dt;
            }
            printf("threads %2d %-22s %6.1f GB/s (read side)\n", T, mode ? "read + 1/4 write" : "read", L / best / 1e9);
        }
    }
    return 0;
}

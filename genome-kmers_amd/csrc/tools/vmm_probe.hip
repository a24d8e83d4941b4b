// Probe (not product): do hipMemsetAsync / hipMemcpyAsync / kernels see an address range mapped
// from several physical allocations (hipMemCreate + hipMemMap) as one buffer?
//   hipcc --offload-arch=gfx950 -O2 vmm_probe.hip -o vmm_probe && ./vmm_probe [chunk_MiB] [chunks]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s -> %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

static int map_range(void **base, size_t chunk, int n) {
    hipMemAllocationProp prop{};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = 0;
    size_t gran = 0;
    CK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended));
    CK(hipMemAddressReserve(base, chunk * n, gran, nullptr, 0));
    for (int i = 0; i < n; ++i) {
        hipMemGenericAllocationHandle_t h;
        CK(hipMemCreate(&h, chunk, &prop, 0));
        CK(hipMemMap(static_cast<char *>(*base) + i * chunk, chunk, 0, h, 0));
    }
    hipMemAccessDesc d{};
    d.location = prop.location;
    d.flags = hipMemAccessFlagsProtReadWrite;
    CK(hipMemSetAccess(*base, chunk * n, &d, 1));
    return 0;
}

__global__ void fill(unsigned *p, size_t n) {
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) p[i] = (unsigned)(i * 2654435761u);
}

int main(int argc, char **argv) {
    const size_t chunk = (argc > 1 ? std::atoll(argv[1]) : 2) << 20;
    const int n = argc > 2 ? std::atoi(argv[2]) : 5;
    const size_t bytes = chunk * n, words = bytes / 4;
    void *a, *b;
    if (map_range(&a, chunk, n) || map_range(&b, chunk, n)) return 1;
    std::vector<unsigned> h(words);
    hipStream_t s;
    CK(hipStreamCreate(&s));
    // 1. memset over the whole range, from an offset inside the first chunk
    CK(hipMemsetAsync(a, 0, bytes, s));
    CK(hipMemsetAsync(static_cast<char *>(a) + 4096, 0xAB, bytes - 8192, s));
    CK(hipMemcpyAsync(h.data(), a, bytes, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    size_t bad = 0;
    for (size_t i = 0; i < words; ++i) {
        const unsigned want = (i >= 1024 && i < words - 1024) ? 0xABABABABu : 0u;
        bad += h[i] != want;
    }
    std::printf("memset across %d chunks of %zu MiB: %zu bad words of %zu\n", n, chunk >> 20, bad, words);
    // 2. kernel fill, D2D copy across chunks at an odd offset, D2H
    hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, s, (unsigned *)a, words);
    CK(hipMemsetAsync(b, 0, bytes, s));
    CK(hipMemcpyAsync(static_cast<char *>(b) + 12, static_cast<char *>(a) + 12, bytes - 24, hipMemcpyDeviceToDevice, s));
    CK(hipMemcpyAsync(h.data(), b, bytes, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    bad = 0;
    for (size_t i = 0; i < words; ++i) {
        const unsigned want = (i >= 3 && i < words - 3) ? (unsigned)(i * 2654435761u) : 0u;
        bad += h[i] != want;
    }
    std::printf("D2D copy across chunks: %zu bad words of %zu\n", bad, words);
    // 3. H2D from pinned and from pageable host memory into a window that straddles each chunk
    //    boundary (odd byte offsets), as the transfer's raw blocks land in the resident sequence
    const size_t win = std::min<size_t>(chunk, 48u << 20);
    unsigned char *hp = nullptr;
    CK(hipHostMalloc(reinterpret_cast<void **>(&hp), win, hipHostMallocDefault));
    std::vector<unsigned char> pg(win), back(win);
    for (int mode = 0; mode < 2; ++mode) {
        size_t badb = 0;
        for (int j = 1; j < n; ++j) {
            const size_t at = j * chunk - win / 2 + 7;
            unsigned char *src = mode ? pg.data() : hp;
            for (size_t i = 0; i < win; ++i) src[i] = (unsigned char)((i * 131 + j * 7 + mode) & 0xFF);
            CK(hipMemsetAsync(b, 0, bytes, s));
            CK(hipMemcpyAsync(static_cast<char *>(b) + at, src, win - 11, hipMemcpyHostToDevice, s));
            CK(hipMemcpyAsync(back.data(), static_cast<char *>(b) + at, win - 11, hipMemcpyDeviceToHost, s));
            CK(hipStreamSynchronize(s));
            for (size_t i = 0; i < win - 11; ++i) badb += back[i] != src[i];
        }
        std::printf("H2D from %s host across %d boundaries: %zu bad bytes\n", mode ? "pageable" : "pinned", n - 1, badb);
    }
    return 0;
}

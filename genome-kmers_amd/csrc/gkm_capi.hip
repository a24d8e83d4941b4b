// gkm_capi.hip -- the extern "C" boundary of libgkm.so and the sort orchestration.
//
// Sort strategies:
//   direct   max_kmer_len given and the padded key fits 256 bits: encode once, LSD radix sort.
//   doubling max_kmer_len None (suffix order up to '$', the Kmers default) or a very long bound:
//            prefix doubling over every sba position -- seed keys of 29 (ACGT, 2 bits + length) / 16 (IUPAC)
//            symbols, then rounds of (rank[p], rank[p + h]) 64-bit keys, each a stable radix sort --
//            and finally the starts with >= min_kmer_len bases are kept, in order.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>

#include "gkm_internal.h"
#include "gkm_partition.h"

namespace gkm {

// ---------------------------------------------------------------------------------------------
// options (gk_set_option): test and tuning overrides of the GKM_* knobs, process-wide
// ---------------------------------------------------------------------------------------------
namespace {
std::mutex g_opt_mu;
std::map<std::string, std::string> g_opts;
// the operational knobs the environment may still set (transfer, packer, rank fallback, prefetch,
// tracing); everything else needs gk_set_option
const char *const kEnvKnobs[] = {"GKM_RANK_BALLOT", "GKM_PACK_IMPL",       "GKM_PACK_MIN",        "GKM_PACK_BLOCKS",
                                 "GKM_XFER_THREADS", "GKM_XFER_HYBRID",    "GKM_XFER_NUMA",       "GKM_NO_RESIDENT_PACK",
                                 "GKM_PREFETCH_REGIONS", "GKM_MSD_TRACE",   "GKM_VMM_CHUNK_MB"};
}  // namespace

const char *opt(const char *name) {
    {
        std::lock_guard<std::mutex> lk(g_opt_mu);
        auto it = g_opts.find(name);
        if (it != g_opts.end()) return it->second.c_str();  // (stable until the option is set again)
    }
    for (const char *e : kEnvKnobs)
        if (std::strcmp(e, name) == 0) return std::getenv(name);
    return nullptr;
}

// Large device buffers (the k-mer arrays, the sort's scratch): hipMalloc, or -- GKM_VMM_CHUNK_MB=N,
// opt-in -- an address range mapped from physical allocations of N MiB each (hipMemAddressReserve /
// hipMemCreate / hipMemMap).  The scatter passes ran faster on mapped 1-4 GiB chunks: C3 69.8-70.0 ->
// 64.7-64.9 ms with 2 GiB chunks on one box (the L1 pass 18.5 -> 15.3 ms, L2 14.5 -> 13.4-13.7, the
// wave-local one 15.8 -> 15.1), 68.4 -> 64.7-65.4 ms with 1-4 GiB on another; chunks of 2-64 MiB or
// of the whole array were no better than hipMalloc (profiles/r6/ab_vmm_*.txt).  Not the default: a
// full-size C4 sort through the Python API (sort hint, prefetched class-A L0) hit an illegal address
// with it, whose cause is not found.  A failed mapping falls back to hipMalloc.
namespace {
constexpr size_t kVmmMin = 256ull << 20;  // smaller buffers: hipMalloc
struct VmmAlloc {
    size_t size, chunk;
    std::vector<hipMemGenericAllocationHandle_t> h;
};
std::mutex g_vmm_mu;
std::map<void *, VmmAlloc> g_vmm;

void vmm_release(void *base, const VmmAlloc &a) {
    for (size_t i = 0; i < a.h.size(); ++i) {
        (void)hipMemUnmap(static_cast<char *>(base) + i * a.chunk, a.chunk);
        (void)hipMemRelease(a.h[i]);
    }
    (void)hipMemAddressFree(base, a.size);
}

hipError_t vmm_alloc(void **p, size_t bytes, size_t want) {
    int dev = 0;
    hipError_t r = hipGetDevice(&dev);
    if (r != hipSuccess) return r;
    hipMemAllocationProp prop{};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = dev;
    size_t gran = 0;
    r = hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended);
    if (r != hipSuccess) return r;
    if (gran == 0) gran = 2ull << 20;
    const size_t whole = (bytes + gran - 1) / gran * gran;
    const size_t chunk = std::min(std::max(want, gran) / gran * gran, whole);
    VmmAlloc a{(bytes + chunk - 1) / chunk * chunk, chunk, {}};
    void *base = nullptr;
    r = hipMemAddressReserve(&base, a.size, gran, nullptr, 0);
    if (r != hipSuccess) return r;
    for (size_t off = 0; off < a.size && r == hipSuccess; off += chunk) {
        hipMemGenericAllocationHandle_t h{};
        r = hipMemCreate(&h, chunk, &prop, 0);
        if (r != hipSuccess) break;
        a.h.push_back(h);
        r = hipMemMap(static_cast<char *>(base) + off, chunk, 0, h, 0);
        if (r != hipSuccess) {  // (this handle is not mapped: release it alone)
            (void)hipMemRelease(h);
            a.h.pop_back();
        }
    }
    if (r == hipSuccess) {
        hipMemAccessDesc d{};
        d.location = prop.location;
        d.flags = hipMemAccessFlagsProtReadWrite;
        r = hipMemSetAccess(base, a.size, &d, 1);
    }
    // zero-filled, as the driver hands out fresh hipMalloc memory
    if (r == hipSuccess) r = hipMemset(base, 0, a.size);
    if (r != hipSuccess) {
        vmm_release(base, a);
        return r;
    }
    std::lock_guard<std::mutex> g(g_vmm_mu);
    g_vmm[base] = std::move(a);
    *p = base;
    return hipSuccess;
}
}  // namespace

hipError_t dev_alloc(void **p, size_t bytes) {
    const char *e = opt("GKM_VMM_CHUNK_MB");
    const size_t want = e ? (size_t)std::strtoull(e, nullptr, 10) << 20 : 0;
    const char *tm = opt("GKM_TEST_VMM_MIN_KB");  // (tests: mapped buffers at parity-test sizes)
    const size_t vmin = tm ? (size_t)std::strtoull(tm, nullptr, 10) << 10 : kVmmMin;
    if (want == 0 || bytes < vmin) return hipMalloc(p, bytes);
    if (vmm_alloc(p, bytes, want) == hipSuccess) return hipSuccess;
    (void)hipGetLastError();  // (the mapping's error: hipMalloc decides)
    return hipMalloc(p, bytes);
}

hipError_t dev_free(void *p) {
    if (!p) return hipSuccess;
    VmmAlloc a{};
    {
        std::lock_guard<std::mutex> g(g_vmm_mu);
        auto it = g_vmm.find(p);
        if (it == g_vmm.end()) return hipFree(p);
        a = std::move(it->second);
        g_vmm.erase(it);
    }
    (void)hipDeviceSynchronize();  // (hipFree's own semantics: no kernel may still use it)
    vmm_release(p, a);
    return hipSuccess;
}

hipError_t ensure(void **p, uint64_t *cap, uint64_t bytes) {
    if (bytes == 0) bytes = 16;
    if (*p && *cap >= bytes) return hipSuccess;
    if (*p) {
        hipError_t e = dev_free(*p);
        if (e != hipSuccess) return e;
        *p = nullptr;
        *cap = 0;
    }
    hipError_t e = dev_alloc(p, bytes);
    if (e != hipSuccess) {
        *p = nullptr;
        return e;
    }
    *cap = bytes;
    return hipSuccess;
}

int fail(gk_ctx *c, int code, const std::string &msg) {
    if (c) c->err = msg;
    return code;
}

int hip_fail(gk_ctx *c, hipError_t e, const char *where) {
    std::string m = std::string(hipGetErrorString(e)) + " at " + where;
    return fail(c, e == hipErrorOutOfMemory ? GK_E_OOM : GK_E_HIP, m);
}

void timer_begin(gk_ctx *c, const char *name, int *slot) {
    *slot = -1;
    if (!c->profile) return;
    Timer t;
    t.name = name;
    while (c->ev_pool.size() < c->ev_used + 2) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return;
        c->ev_pool.push_back(e);
    }
    t.start = c->ev_pool[c->ev_used++];
    t.stop = c->ev_pool[c->ev_used++];
    hipEventRecord(t.start, c->stream);
    c->timers.push_back(t);
    *slot = (int)c->timers.size() - 1;
}

void timer_end(gk_ctx *c, int slot) {
    if (slot < 0 || !c->profile) return;
    hipEventRecord(c->timers[slot].stop, c->stream);
}

void timer_units(gk_ctx *c, int slot, uint64_t units) {
    if (slot >= 0 && c->profile) c->timers[slot].units = units;
}

// ---------------------------------------------------------------------------------------------
// prefix-doubling kernels
// ---------------------------------------------------------------------------------------------

// R[vals[i]] = gstart[gid[i] - 1] + 1   (rank = 1 + index of the group's first element)
__global__ __launch_bounds__(256) void rank_scatter_kernel(const uint32_t *__restrict__ vals,
                                                           const uint32_t *__restrict__ gid,
                                                           const uint32_t *__restrict__ gstart, uint64_t n,
                                                           uint32_t *__restrict__ R) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        R[vals[i]] = gstart[gid[i] - 1] + 1;
}

// Groups of the current order that may still split: more than one member, and members longer than
// the h symbols the keys hold.  Members of a group share their first h symbols, so a group whose
// first member's suffix (to '$' / the end) is at most h long holds equal k-mers and is final --
// the '$'-terminated tails shared by several contigs, which no doubling round can separate.
__global__ __launch_bounds__(256) void unresolved_groups_kernel(const uint32_t *__restrict__ vals,
                                                                const uint32_t *__restrict__ gstart, uint64_t G,
                                                                uint64_t n, const uint32_t *__restrict__ seg,
                                                                uint32_t nseg, uint64_t L, uint64_t h,
                                                                uint32_t *__restrict__ count) {
    for (uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; g < G; g += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t b = gstart[g], e = g + 1 < G ? gstart[g + 1] : n;
        if (e - b < 2) continue;
        const uint64_t p = vals[b];
        if (seg_end_of(seg, nseg, L, p) - p + 1 > h) atomicAdd(count, 1u);
    }
}

// key = rank[p] << 32 | (p + o <= seg_end(p) ? rank[p + o] : 0)
__global__ __launch_bounds__(256) void pair_keys_kernel(const uint32_t *__restrict__ vals,
                                                        const uint32_t *__restrict__ R,
                                                        const uint32_t *__restrict__ seg, uint32_t nseg, uint64_t L,
                                                        uint64_t o, uint64_t n, int bw,
                                                        uint64_t *__restrict__ keys) {
    // (rank of p, rank of p + o) in 2 bw bits: ranks are <= n < 2^bw
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t p = vals[i];
        const uint64_t q = p + o;
        const uint32_t r2 = (q <= seg_end_of(seg, nseg, L, p)) ? R[q] : 0u;
        keys[i] = ((uint64_t)R[p] << bw) | r2;
    }
}

// Prefix doubling by tied groups (sort_doubling, MSD path): the rank of p + o for the elements
// still tied (flags: 1 starts a group), the others untouched
__global__ __launch_bounds__(256) void member_r2_kernel(const uint8_t *__restrict__ flags,
                                                        const uint32_t *__restrict__ vals,
                                                        const uint32_t *__restrict__ R,
                                                        const uint32_t *__restrict__ seg, uint32_t nseg, uint64_t L,
                                                        uint64_t o, uint64_t n, uint64_t *__restrict__ keys) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        if (flags[i] != 0 && (i + 1 >= n || flags[i + 1] != 0)) continue;  // a group of one: final
        const uint64_t p = vals[i];
        const uint64_t q = p + o;
        keys[i] = (q <= seg_end_of(seg, nseg, L, p)) ? R[q] : 0u;
    }
}

// the groups after a round: a group start stays one, a tied element starts a group where the
// round's sort found its key different from its predecessor's (heads of the sorted groups)
__global__ __launch_bounds__(256) void merge_heads_kernel(const uint8_t *__restrict__ fold,
                                                          const uint8_t *__restrict__ heads, uint64_t n,
                                                          uint8_t *__restrict__ fnew) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        fnew[i] = (fold[i] != 0 || heads[i] != 0) ? 1 : 0;
}

// new ranks (group start + 1) of the elements that were tied before the round; the others keep theirs
__global__ __launch_bounds__(256) void member_rank_kernel(const uint8_t *__restrict__ fold,
                                                          const uint32_t *__restrict__ vals,
                                                          const uint32_t *__restrict__ gid,
                                                          const uint32_t *__restrict__ gstart, uint64_t n,
                                                          uint32_t *__restrict__ R) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        if (fold[i] != 0 && (i + 1 >= n || fold[i + 1] != 0)) continue;
        R[vals[i]] = gstart[gid[i] - 1] + 1;
    }
}

// keep starts with >= m bases before the end of their segment
__global__ __launch_bounds__(256) void len_flags_kernel(const uint32_t *__restrict__ vals,
                                                        const uint32_t *__restrict__ seg, uint32_t nseg, uint64_t L,
                                                        uint64_t m, uint64_t n, uint8_t *__restrict__ flags) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t p = vals[i];
        flags[i] = (p + m - 1 <= seg_end_of(seg, nseg, L, p)) ? 1 : 0;
    }
}

__global__ __launch_bounds__(256) void gather_pairs_kernel(const uint32_t *__restrict__ idx, uint64_t count,
                                                           const uint32_t *__restrict__ vin,
                                                           const uint64_t *__restrict__ kin,
                                                           uint32_t *__restrict__ vout, uint64_t *__restrict__ kout) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < count;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t j = idx[i];
        vout[i] = vin[j];
        kout[i] = kin[j];
    }
}

// keys[i] = R[starts[i]] (final rank of a user-provided start)
__global__ __launch_bounds__(256) void rank_gather_kernel(const uint32_t *__restrict__ starts,
                                                          const uint32_t *__restrict__ R, uint64_t n,
                                                          uint64_t *__restrict__ keys) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        keys[i] = R[starts[i]];
}

__global__ __launch_bounds__(256) void u32_to_key_kernel(const uint32_t *__restrict__ v, uint64_t n,
                                                         uint64_t *__restrict__ keys) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        keys[i] = v[i];
}

__global__ __launch_bounds__(256) void full_key_heads_kernel(const uint64_t *__restrict__ keys, uint64_t n,
                                                             uint8_t *__restrict__ head) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        head[i] = (i == 0 || keys[i] != keys[i - 1]) ? 1 : 0;
}

static int grid_of(uint64_t n, int cap = 8192) {
    uint64_t g = (n + 255) / 256;
    if (g < 1) g = 1;
    return (int)std::min<uint64_t>(g, (uint64_t)cap);
}

hipError_t launch_rank_scatter(gk_ctx *c, const uint32_t *vals, const uint32_t *gid, const uint32_t *gstart,
                               uint64_t n, uint32_t *R) {
    hipLaunchKernelGGL(rank_scatter_kernel, dim3(grid_of(n)), dim3(256), 0, c->stream, vals, gid, gstart, n, R);
    return hipGetLastError();
}

hipError_t read_back(gk_ctx *c, const void *dev, size_t bytes, void *host) {
    if (bytes > 8 * (size_t)kHostPinWords) return hipErrorInvalidValue;
    hipError_t e = hipMemcpyAsync(c->hpin, dev, bytes, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e == hipSuccess) std::memcpy(host, c->hpin, bytes);
    return e;
}

}  // namespace gkm

using namespace gkm;

// ---------------------------------------------------------------------------------------------
// buffers
// ---------------------------------------------------------------------------------------------
int gkm::ensure_elems(gk_ctx *c, uint64_t n, int words) {
    // vals[0] / vals[1] hold data that must survive when only keys grow; grow both together
    if (n > c->elem_cap) {
        uint32_t *nv[2] = {nullptr, nullptr};
        for (int b = 0; b < 2; ++b) GK_TRY_HIP(c, dev_alloc(reinterpret_cast<void **>(&nv[b]), 4 * (n + 64)));
        if (c->have_starts && c->elem_cap > 0)
            GK_TRY_HIP(c, hipMemcpyAsync(nv[c->cur], c->vals[c->cur], 4 * c->n, hipMemcpyDeviceToDevice, c->stream));
        GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
        for (int b = 0; b < 2; ++b) {
            if (c->vals[b]) dev_free(c->vals[b]);
            c->vals[b] = nv[b];
            if (c->keys[b]) dev_free(c->keys[b]);
            c->keys[b] = nullptr;
        }
        c->elem_cap = n;
        c->key_words_cap = 0;
        c->key_words_b[0] = c->key_words_b[1] = 0;
        c->keys_valid = false;
    }
    if (words > c->key_words_cap) {
        for (int b = 0; b < 2; ++b) {
            if (c->key_words_b[b] >= words) continue;
            if (c->keys[b]) dev_free(c->keys[b]);
            c->keys[b] = nullptr;
            GK_TRY_HIP(c, dev_alloc(reinterpret_cast<void **>(&c->keys[b]), 8 * (uint64_t)words * (c->elem_cap + 64)));
            c->key_words_b[b] = words;
        }
        c->key_words_cap = words;
        c->keys_valid = false;
    }
    const uint64_t tiles = (n + kSortTile - 1) / kSortTile + 1;
    if (tiles * 256 > c->status_cap) {
        if (c->status) hipFree(c->status);
        c->status = nullptr;
        GK_TRY_HIP(c, hipMalloc(&c->status, 8 * tiles * 256));
        GK_TRY_HIP(c, hipMemsetAsync(c->status, 0, 8 * tiles * 256, c->stream));
        c->status_cap = tiles * 256;
    }
    return GK_OK;
}

int gkm::grow_key_buffer(gk_ctx *c, int b, int words) {
    if (c->key_words_b[b] >= words) return GK_OK;
    GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
    if (c->keys[b]) dev_free(c->keys[b]);
    c->keys[b] = nullptr;
    GK_TRY_HIP(c, dev_alloc(reinterpret_cast<void **>(&c->keys[b]), 8 * (uint64_t)words * (c->elem_cap + 64)));
    c->key_words_b[b] = words;
    c->key_words_cap = std::min(c->key_words_b[0], c->key_words_b[1]);
    return GK_OK;
}

namespace gkm {
int materialize_starts(gk_ctx *c) {
    if (!c->have_starts || c->starts_materialized) return GK_OK;
    int slot;
    timer_begin(c, "enumerate", &slot);
    GK_TRY_HIP(c, launch_enumerate(c, c->min_k, c->vals[c->cur]));
    timer_end(c, slot);
    c->starts_materialized = true;
    return GK_OK;
}
}  // namespace gkm

// ---------------------------------------------------------------------------------------------
// lifetime
// ---------------------------------------------------------------------------------------------
extern "C" int gk_device_count(int *count) {
    if (!count) return GK_E_ARG;
    hipError_t e = hipGetDeviceCount(count);
    return e == hipSuccess ? GK_OK : GK_E_HIP;
}

// Every partition of the sort ranks an item by one returning LDS atomic (rank_atomic,
// gkm_partition.h): it relies on the LDS applying the same-address lanes of one wave instruction in
// increasing lane order.  That is how gfx950 behaves (tools/lds_rank_probe.hip: no exception in
// 4e10 lane-ranks), not an ISA guarantee, so it is checked once per device and process against a
// ballot-match ground truth over every digit space the partitions rank in -- 2048, 1024, 512, 256,
// 128, 64, 16, 4 and 1 digits (the wide L0's 11 bits, the wave kernels' 10 / 9 / 8, the level
// passes' 8, L0's 7) with per-wave counter arrays of 2048 words, in both counter forms (u32 words,
// and the u16 halves of rank_atomic16), 8 items per trial, lanes sitting out, every CU busy.  Where
// it does not hold, the partitions switch to ballot-match ranking (rank_ballot): the same ranks
// from ballots alone.  The kernel checks that path as well.
__global__ __launch_bounds__(256) void lds_rank_check_kernel(uint32_t trials, unsigned long long *bad) {
    __shared__ uint32_t s_cnt[4][2048];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint32_t *cnt = s_cnt[wave];
    unsigned long long nb = 0;
    for (uint32_t t = 0; t < trials; ++t) {
        constexpr uint32_t kMasks[9] = {2047u, 1023u, 511u, 255u, 127u, 63u, 15u, 3u, 0u};
        const uint32_t dmask = kMasks[t % 9];
        const uint32_t form = (t / 9) & 3;  // 0 atomic u32, 1 ballot u32, 2 atomic u16, 3 ballot u16
        const bool ballot = form & 1;
#pragma unroll
        for (int u = 0; u < 32; ++u) cnt[u * 64 + lane] = 0;
        uint32_t dd[8], got[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            uint32_t x = (blockIdx.x * 0x9E3779B9u) ^ (t * 0x85EBCA6Bu) ^ ((uint32_t)(i * 64 + lane) * 0xC2B2AE35u);
            x ^= x >> 15;
            x *= 0x2C1B3C6Du;
            x ^= x >> 12;
            dd[i] = x & dmask;
            const bool valid = ((x >> 20) & 7u) != 0;  // some lanes sit out
            const uint32_t d = dd[i], sh = (d & 1u) << 4;
            if (form == 0) got[i] = valid ? atomicAdd(&cnt[d], 1u) : 0u;
            else if (form == 1) got[i] = rank_ballot<11, false>(cnt, d, valid);
            else if (form == 2) got[i] = valid ? (atomicAdd(&cnt[d >> 1], 1u << sh) >> sh) & 0xFFFFu : 0u;
            else got[i] = rank_ballot<11, true>(cnt, d, valid);
            if (!valid) got[i] = ~0u;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const bool valid = got[i] != ~0u;
            // ground truth: valid lanes with the same digit below this lane, and in earlier items
            uint32_t want = 0;
            for (int j = 0; j <= i; ++j) {
                uint64_t m = __ballot(got[j] != ~0u);
#pragma unroll
                for (int b = 0; b < 11; ++b) {
                    const uint64_t x = __ballot((dd[j] >> b) & 1u);
                    m &= ((dd[i] >> b) & 1u) ? x : ~x;
                }
                want += (uint32_t)__popcll(j < i ? m : (m & ((1ull << lane) - 1ull)));
            }
            nb += (valid && got[i] != want) ? (ballot ? (1ull << 40) : 1ull) : 0ull;
        }
    }
    if (nb) atomicAdd(bad, nb);
}

namespace {
struct RankState {
    int checked = 0;  // 0 unchecked, 1 lane order holds, -1 it does not
    int forced = 0;   // ballot-match forced by gk_rank_mode (tests)
    int active = 0;   // ranking in use: 0 atomic, 1 ballot-match
};
std::mutex g_rank_mu;
std::map<int, RankState> g_rank;  // per device (hipGetDeviceCount-sized by use)

bool env_force_ballot() {
    const char *v = opt("GKM_RANK_BALLOT");
    return v && *v && std::strcmp(v, "0") != 0;
}

hipError_t set_rank_mode_all(int ballot) {
    hipError_t e = gkm::rank_mode_msd(ballot);
    if (e == hipSuccess) e = gkm::rank_mode_sort(ballot);
    return e;
}
}  // namespace

// the check on the current device (once per process), then its ranking mode
static int lds_rank_check(int device) {
    std::lock_guard<std::mutex> lock(g_rank_mu);
    RankState &st = g_rank[device];
    if (st.checked == 0) {
        unsigned long long *d = nullptr, h = 0;
        if (hipMalloc(&d, 8) != hipSuccess) return GK_E_HIP;
        hipError_t e = hipMemset(d, 0, 8);
        if (e == hipSuccess) {
            hipLaunchKernelGGL(lds_rank_check_kernel, dim3(2048), dim3(256), 0, 0, 72u, d);
            e = hipGetLastError();
        }
        if (e == hipSuccess) e = hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
        hipFree(d);
        if (e != hipSuccess) return GK_E_HIP;
        if (h >> 40) {  // the ballot-match ranking itself is wrong: nothing on this device can sort
            std::fprintf(stderr, "libgkm: device %d: ballot-match ranks differ from their ground truth (%llu)\n",
                         device, h >> 40);
            return GK_E_UNSUPPORTED;
        }
        st.checked = h == 0 ? 1 : -1;
        if (h)
            std::fprintf(stderr, "libgkm: device %d: a returning LDS atomic did not apply same-address lanes in "
                                 "lane order (%llu of ~1.9e8 ranks differ); the partitions rank by ballots instead\n",
                         device, h);
    }
    const int want = (st.checked < 0 || st.forced || env_force_ballot()) ? 1 : 0;
    if (hipError_t e = set_rank_mode_all(want); e != hipSuccess) return GK_E_HIP;
    st.active = want;
    return GK_OK;
}

extern "C" int gk_rank_mode(gk_ctx *c, int mode, int *active) {
    if (!c || mode < -1 || mode > 1) return GK_E_ARG;
    if (hipSetDevice(c->device) != hipSuccess) return GK_E_HIP;
    std::lock_guard<std::mutex> lock(g_rank_mu);
    RankState &st = g_rank[c->device];
    if (mode >= 0) {
        st.forced = mode == 1;
        const int want = (st.forced || st.checked < 0 || env_force_ballot()) ? 1 : 0;
        if (hipStreamSynchronize(c->stream) != hipSuccess) return GK_E_HIP;  // no launch of the old mode in flight
        if (set_rank_mode_all(want) != hipSuccess) return GK_E_HIP;
        st.active = want;
    }
    if (active) *active = st.active;
    return GK_OK;
}

extern "C" int gk_create(gk_ctx **out, int device) {
    if (!out) return GK_E_ARG;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return GK_E_HIP;
    if (device < 0 || device >= ndev) return GK_E_ARG;
    if (hipSetDevice(device) != hipSuccess) return GK_E_HIP;
    if (int rc = lds_rank_check(device)) return rc;
    gk_ctx *c = new gk_ctx();
    c->device = device;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&c->counters, 4 * 64) != hipSuccess || hipMalloc(&c->hist, 4 * 256 * kMaxWords * 8) != hipSuccess ||
        hipMalloc(&c->offsets, 4 * 256 * kMaxWords * 8) != hipSuccess || hipMalloc(&c->scalars, 8 * 64) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void **>(&c->hpin), 8 * kHostPinWords, hipHostMallocDefault) != hipSuccess) {
        gk_destroy(c);
        return GK_E_HIP;
    }
    *out = c;
    return GK_OK;
}

extern "C" void gk_destroy(gk_ctx *c) {
    if (!c) return;
    hipSetDevice(c->device);
    if (c->stream) hipStreamSynchronize(c->stream);
    if (c->pre_stream) hipStreamSynchronize(c->pre_stream);
    xfer_release(c);
    if (c->hpin) hipHostFree(c->hpin);
    for (hipEvent_t e : c->pre_ev) hipEventDestroy(e);
    if (c->pre_done) hipEventDestroy(c->pre_done);
    if (c->pre_stream) hipStreamDestroy(c->pre_stream);
    void *bufs[] = {c->sba, c->seg, c->res_code, c->res_dol, c->vals[0], c->vals[1], c->keys[0], c->keys[1], c->status, c->counters,
                    c->hist, c->offsets, c->flags, c->idx_a, c->idx_b, c->ucount, c->cumk, c->tile_sums, c->scalars,
                    c->dhist, c->mask, c->hmask, c->ranks, c->ym, c->yoff, c->oy, c->ot, c->onum};
    for (void *b : bufs)
        if (b) dev_free(b);
    for (auto &e : c->scratch)
        if (e.second.first) dev_free(e.second.first);
    for (hipEvent_t e : c->ev_pool) hipEventDestroy(e);
    if (c->stream) hipStreamDestroy(c->stream);
    delete c;
}

extern "C" const char *gk_last_error(gk_ctx *c) { return c ? c->err.c_str() : "null context"; }

extern "C" int gk_sync(gk_ctx *c) {
    if (!c) return GK_E_ARG;
    GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
    return GK_OK;
}

extern "C" int gk_stream(gk_ctx *c, void **stream) {
    if (!c || !stream) return GK_E_ARG;
    *stream = (void *)c->stream;
    return GK_OK;
}

// ---------------------------------------------------------------------------------------------
// input
// ---------------------------------------------------------------------------------------------
extern "C" int gk_set_sequence(gk_ctx *c, const uint8_t *sba, uint64_t len, const uint32_t *seg_starts, uint64_t nseg) {
    if (!c) return GK_E_ARG;
    pre_drop(c);  // (the k-mer buffers: a prefetched L0 does not survive)
    if (!sba || len == 0) return fail(c, GK_E_ARG, "sequence byte array is empty");
    if (!seg_starts || nseg == 0) return fail(c, GK_E_ARG, "sequence_collection is empty");
    if (len > 0xFFFFFFFFull) return fail(c, GK_E_LIMIT, "sequence byte array longer than 2^32-1");
    GK_TRY_HIP(c, hipSetDevice(c->device));
    if (seg_starts[0] != 0) return fail(c, GK_E_ARG, "first segment must start at 0");
    uint64_t max_len = 0;
    bool internal = false;
    for (uint64_t s = 0; s < nseg; ++s) {
        const uint64_t b = seg_starts[s];
        const uint64_t e = (s + 1 == nseg) ? len - 1 : (uint64_t)seg_starts[s + 1] - 2;
        if (s + 1 < nseg && ((uint64_t)seg_starts[s + 1] < b + 2 || (uint64_t)seg_starts[s + 1] > len))
            return fail(c, GK_E_ARG, "segment starts are not strictly increasing by >= 2");
        if (s > 0 && sba[b - 1] != GK_DOLLAR) internal = true;  // separator missing
        if (e < b) return fail(c, GK_E_ARG, "empty segment");
        max_len = std::max<uint64_t>(max_len, e - b + 1);
    }
    const uint64_t padded = ((len + kEncodeTile - 1) / kEncodeTile) * kEncodeTile + kSbaPad;
    GK_TRY_HIP(c, ensure(reinterpret_cast<void **>(&c->sba), &c->sba_cap, padded));
    GK_TRY_HIP(c, hipMemsetAsync(c->sba + len, GK_DOLLAR, c->sba_cap - len, c->stream));
    GK_TRY_HIP(c, ensure(reinterpret_cast<void **>(&c->seg), &c->seg_cap, 4 * nseg));
    GK_TRY_HIP(c, hipMemcpyAsync(c->seg, seg_starts, 4 * nseg, hipMemcpyHostToDevice, c->stream));
    c->sba_len = len;
    c->nseg = nseg;
    c->hseg.assign(seg_starts, seg_starts + nseg);
    c->max_seg_len = max_len;
    uint32_t h[2] = {0, 0};  // alphabet classes seen (alphabet_kernel's bits), '$' count
    if (len >= packed_transfer_min()) {
        // 2-bit packed over the link, census on the host, unpacked into the resident sba on the
        // device (gkm_xfer.hip); the stream orders the sort's kernels behind the last unpack, so
        // only the census is waited for
        uint64_t dollars = 0;
        // (A/B: GKM_EARLY_ELEMS=1 -- the k-mer buffers for every position allocated here, before the
        // transfer's staging slots, as the prefetch path does)
        static const bool early = opt("GKM_EARLY_ELEMS") != nullptr;
        if (early)
            if (int rc = ensure_elems(c, len, 1)) return rc;
        // a sort hint (gk_sort_hint): the L0 pass of gk_sort(k) runs as the sequence lands
        L0Prefetch *pf = nullptr;
        if (c->hint_k && !internal)
            if (int rc = prefetch_plan(c, len, &pf)) return rc;
        if (int rc = packed_transfer(c, sba, len, &h[0], &dollars, pf)) return rc;
        h[1] = (uint32_t)dollars;
    } else {
        GK_TRY_HIP(c, hipMemcpyAsync(c->sba, sba, len, hipMemcpyHostToDevice, c->stream));
        uint32_t *d_flags = reinterpret_cast<uint32_t *>(c->scalars + 8);
        GK_TRY_HIP(c, launch_alphabet(c, d_flags));
        GK_TRY_HIP(c, hipMemcpyAsync(h, d_flags, 8, hipMemcpyDeviceToHost, c->stream));
        GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
    }
    c->have_starts = c->sorted = c->keys_valid = c->enumerated = c->unique_valid = c->heads_valid = c->canonical = false;
    c->enum_sorted = false;
    c->pk_fresh = false;
    if (len < packed_transfer_min()) c->res_pk = false;  // (the packed transfer sets it)
    c->n = 0;
    if (h[0] & 4u) return fail(c, GK_E_ALPHABET, "Sequence contains non-allowed characters!");
    c->acgt = (h[0] & 2u) ? 0 : 1;
    c->internal_dollar = internal || (uint64_t)h[1] != nseg - 1;
    return GK_OK;
}

extern "C" int gk_sort_hint(gk_ctx *c, uint32_t k, uint32_t flags) {
    if (!c) return GK_E_ARG;
    if (flags != 0) return fail(c, GK_E_ARG, "gk_sort_hint: flags must be 0 (forward k-mers)");
    c->hint_k = k;
    return GK_OK;
}

extern "C" int gk_copy_sequence(gk_ctx *c, uint8_t *dst, uint64_t len) {
    if (!c) return GK_E_ARG;
    if (!c->sba) return fail(c, GK_E_STATE, "no sequence loaded");
    if (len != c->sba_len) return fail(c, GK_E_ARG, "len differs from the loaded sequence length");
    GK_TRY_HIP(c, hipSetDevice(c->device));
    GK_TRY_HIP(c, hipMemcpyAsync(dst, c->sba, len, hipMemcpyDeviceToHost, c->stream));
    GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
    return GK_OK;
}

extern "C" int gk_alphabet_is_acgt(gk_ctx *c, int *is_acgt) {
    if (!c || !is_acgt) return GK_E_ARG;
    *is_acgt = c->acgt;
    return GK_OK;
}

extern "C" int gk_resident_packed(gk_ctx *c, int *on) {
    if (!c || !on) return GK_E_ARG;
    *on = c->res_pk ? 1 : 0;
    return GK_OK;
}

extern "C" int gk_set_option(const char *name, const char *value) {
    if (!name || std::strncmp(name, "GKM_", 4) != 0) return GK_E_ARG;
    std::lock_guard<std::mutex> lk(g_opt_mu);
    if (value) g_opts[name] = value;
    else g_opts.erase(name);
    return GK_OK;
}

// ---------------------------------------------------------------------------------------------
// enumerate (kmers.py:789-861)
// ---------------------------------------------------------------------------------------------
extern "C" int gk_enumerate(gk_ctx *c, uint32_t min_k, uint64_t *n_out) {
    if (!c) return GK_E_ARG;
    if (!c->sba) return fail(c, GK_E_STATE, "no sequence loaded");
    if (min_k < 1) return fail(c, GK_E_ARG, "min_kmer_len must be greater than zero");
    uint64_t n = 0, shortest = ~0ull;
    for (uint64_t s = 0; s < c->nseg; ++s) {
        const uint64_t e = (s + 1 == c->nseg) ? c->sba_len - 1 : (uint64_t)c->hseg[s + 1] - 2;
        const uint64_t l = e - c->hseg[s] + 1;
        shortest = std::min(shortest, l);
        if (l >= min_k) n += l - min_k + 1;
    }
    if (min_k > shortest) return fail(c, GK_E_ARG, "min_kmer_len must be <= the shortest sequence length");
    if (n > 0xFFFFFFFFull) return fail(c, GK_E_LIMIT, "the size of the required kmers array exceeds the limit set by a uint32");
    GK_TRY_HIP(c, hipSetDevice(c->device));
    if (min_k != c->pre_k) pre_drop(c);  // (a prefetched L0 serves the enumeration of its k only)
    c->have_starts = false;
    int rc = ensure_elems(c, n, 1);
    if (rc != GK_OK) return rc;
    c->n = n;
    c->min_k = min_k;
    c->cur = 0;
    // The enumerate output is a pure function of (seg, min_k): it is materialised lazily by the
    // first reader (materialize_starts); the encoder regenerates positions itself.
    c->have_starts = true;
    c->enumerated = true;
    c->starts_materialized = false;
    c->sorted = c->keys_valid = c->unique_valid = c->heads_valid = c->canonical = c->enum_sorted = false;
    if (n_out) *n_out = n;
    return GK_OK;
}

extern "C" int gk_set_start_indices(gk_ctx *c, const uint32_t *src, uint64_t n, uint32_t min_k) {
    if (!c) return GK_E_ARG;
    pre_drop(c);  // (the k-mer buffers: a prefetched L0 does not survive)
    if (!c->sba) return fail(c, GK_E_STATE, "no sequence loaded");
    if (n > 0 && !src) return fail(c, GK_E_ARG, "null start array");
    GK_TRY_HIP(c, hipSetDevice(c->device));
    c->have_starts = false;
    int rc = ensure_elems(c, std::max<uint64_t>(n, 1), 1);
    if (rc != GK_OK) return rc;
    c->cur = 0;
    if (n) GK_TRY_HIP(c, hipMemcpyAsync(c->vals[0], src, 4 * n, hipMemcpyHostToDevice, c->stream));
    GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
    c->n = n;
    c->min_k = min_k;
    c->have_starts = true;
    c->enumerated = false;
    c->starts_materialized = true;
    c->sorted = c->keys_valid = c->unique_valid = c->heads_valid = c->canonical = c->enum_sorted = false;
    return GK_OK;
}

extern "C" int gk_num_kmers(gk_ctx *c, uint64_t *n) {
    if (!c || !n) return GK_E_ARG;
    *n = c->have_starts ? c->n : 0;
    return GK_OK;
}

// ---------------------------------------------------------------------------------------------
// sort (kmers.py:1624-1731)
// ---------------------------------------------------------------------------------------------
static int bit_width(uint64_t v) {
    int b = 0;
    while (v) {
        ++b;
        v >>= 1;
    }
    return b;
}

// stable pre-sort of arbitrary start indices by value, so ties end in start order
static int presort_by_start(gk_ctx *c) {
    hipLaunchKernelGGL(u32_to_key_kernel, dim3(grid_of(c->n)), dim3(256), 0, c->stream, c->vals[c->cur], c->n,
                       c->keys[c->cur]);
    GK_TRY_HIP(c, hipGetLastError());
    return radix_sort(c, 1, 32, false);
}

int gkm::ensure_keys(gk_ctx *c) {
    if (!c->keys_valid || !c->keys_stale) return GK_OK;
    // the MSD sort runs on one key word; all words are allocated on first use
    if (int rc = ensure_elems(c, c->n, c->spec.words)) return rc;
    int slot;
    timer_begin(c, "reencode_keys", &slot);
    // multi-word keys of a sorted enumeration: through an enumeration-order table in the free key
    // buffer (one aligned row per k-mer instead of a ~70-byte window at a random position)
    static const bool no_table = opt("GKM_NO_KEY_TABLE") != nullptr;  // (A/B)
    const KeySpec &ks = c->spec;
    // (the table path answers hipErrorNotSupported when it does not apply -- e.g. per-contig k-mer
    // counts that do not add up to n -- and the window gather, always correct, runs instead)
    hipError_t te = hipErrorNotSupported;
    if (c->enum_sorted && !no_table && ks.words >= 2 && ks.symbols == ks.min_len && ks.symbols <= 64 &&
        (ks.bits == 2 || ks.bits == 4) && c->n >= 4096 && c->key_words_b[c->cur ^ 1] >= ks.words)
        te = launch_encode_table_gather(c, ks, c->vals[c->cur], c->n, c->keys[c->cur], c->keys[c->cur ^ 1],
                                        8 * (uint64_t)c->key_words_b[c->cur ^ 1] * (c->elem_cap + 64));
    if (te == hipErrorNotSupported)
        GK_TRY_HIP(c, launch_encode_gather(c, c->spec, c->vals[c->cur], c->n, c->keys[c->cur]));
    else
        GK_TRY_HIP(c, te);
    timer_end(c, slot);
    c->keys_valid = true;
    c->keys_stale = false;
    return GK_OK;
}

static int sort_direct(gk_ctx *c, const KeySpec &ks) {
    // fixed-length keys (k <= 64) from the enumerated starts: stable MSD in one-word phases (gkm_msd.hip)
    static const bool force_lsd = opt("GKM_SORT_LSD") != nullptr;
    const bool msd =
        c->enumerated && ks.symbols == ks.min_len && ks.symbols <= 64 && (ks.bits == 2 || ks.bits == 4) && !force_lsd;
    int rc = ensure_elems(c, c->n, msd ? 1 : ks.words);
    if (rc != GK_OK) return rc;
    if (msd) {
        // a mixed sba (N runs, IUPAC letters): ACGT-only k-mers on 2-bit keys, the rest apart
        static const bool no_split = opt("GKM_NO_SPLIT") != nullptr;
        bool split = false;
        if (!c->acgt && !no_split) {
            rc = split_sort(c, ks, &split);
            if (rc != GK_OK) return rc;
        }
        if (!split) rc = prefetch_matches(c, ks) ? msd_sort_prefetched(c, ks) : msd_sort(c, ks);
        pre_drop(c);
        if (rc != GK_OK) return rc;
        c->spec = ks;
        c->keys_valid = true;
        // a one-word MSD sort leaves the sorted keys in keys[0]; the split sort (2-bit class-A keys
        // under a 4-bit key spec) and multi-word phases leave them to ensure_keys
        c->keys_stale = split ? !c->split_keys_final : !c->msd_keys_final;
        c->keys_are_ranks = false;
        return GK_OK;
    }
    bool hist_ready = false;
    if (c->enumerated && ks.canonical) {  // k > 64: canonical keys of the (ascending) starts
        rc = materialize_starts(c);
        if (rc != GK_OK) return rc;
        int slot;
        timer_begin(c, "encode", &slot);
        GK_TRY_HIP(c, launch_encode_gather(c, ks, c->vals[c->cur], c->n, c->keys[c->cur]));
        timer_end(c, slot);
    } else if (c->enumerated) {
        int slot;
        timer_begin(c, "encode", &slot);
        // (no LSD digit histograms when the MSD path sorts the keys)
        hist_ready = !sort_keys_msd(c, c->n, ks.words, ks.total_bits);
        GK_TRY_HIP(c, launch_encode_positions(c, ks, c->keys[c->cur], c->vals[c->cur], hist_ready ? c->hist : nullptr));
        timer_end(c, slot);
    } else {
        rc = presort_by_start(c);
        if (rc != GK_OK) return rc;
        int slot;
        timer_begin(c, "encode", &slot);
        timer_units(c, slot, c->n);
        GK_TRY_HIP(c, launch_encode_gather(c, ks, c->vals[c->cur], c->n, c->keys[c->cur]));
        timer_end(c, slot);
    }
    rc = sort_keys(c, ks.words, ks.total_bits, hist_ready);
    if (rc != GK_OK) return rc;
    c->spec = ks;
    c->keys_valid = true;
    c->keys_stale = false;
    c->keys_are_ranks = false;
    return GK_OK;
}

// Prefix doubling over all non-'$' positions; M = 0 means unbounded (suffix order).
static int sort_doubling(gk_ctx *c, uint32_t M) {
    const uint64_t n_kmers = c->n;
    const bool was_enumerated = c->enumerated;
    const uint32_t m = c->min_k;
    const uint64_t L = c->sba_len;
    uint32_t *user = nullptr;  // user-provided starts survive in a side buffer
    if (!was_enumerated && n_kmers > 0) {
        GK_TRY_HIP(c, hipMalloc(&user, 4 * n_kmers));
        GK_TRY_HIP(c, hipMemcpyAsync(user, c->vals[c->cur], 4 * n_kmers, hipMemcpyDeviceToDevice, c->stream));
    }
    // universe: every position inside a segment (min length 1)
    uint64_t n1 = L - (c->nseg - 1);
    int rc = ensure_elems(c, std::max(n1, n_kmers), 1);
    if (rc != GK_OK) return rc;
    GK_TRY_HIP(c, ensure(reinterpret_cast<void **>(&c->flags), &c->flags_cap, n1 + 64));
    GK_TRY_HIP(c, ensure(reinterpret_cast<void **>(&c->idx_a), &c->idx_cap, 4 * (n1 + 64)));
    GK_TRY_HIP(c, ensure(reinterpret_cast<void **>(&c->idx_b), &c->idx_b_cap, 4 * (n1 + 64)));
    GK_TRY_HIP(c, ensure(reinterpret_cast<void **>(&c->ranks), &c->ranks_cap, 4 * (L + 64)));

    // seed keys: ACGT data as 29 symbols of 2 bits + a 5-bit length field (the (padded, length)
    // keys of the bounded sort: the same order as '$'-terminated 3-bit codes, 29 symbols instead of
    // 21, and every key bit carries information for the MSD levels; GKM_SEED3=1 keeps the 3-bit
    // seeds); other data as 16 symbols of 4 bits
    static const bool seed3 = opt("GKM_SEED3") != nullptr;
    KeySpec seed{};
    seed.bits = c->acgt ? (seed3 ? 3 : 2) : 4;
    seed.symbols = c->acgt ? (seed3 ? 21 : 29) : 16;
    seed.lenbits = seed.bits == 2 ? bit_width((uint64_t)seed.symbols) : 0;
    seed.min_len = 1;
    seed.words = 1;
    seed.total_bits = seed.bits * seed.symbols + seed.lenbits;
    c->n = n1;
    c->cur = 0;
    int slot;
    // large universes: the rounds sort only the groups still tied (MSD, msd_sort_groups); small ones
    // re-sort the whole array by rank pairs each round (LSD)
    const bool by_groups = sort_keys_msd(c, n1, 1, 64) && opt("GKM_DOUBLING_FULL") == nullptr;
    timer_begin(c, "encode", &slot);
    timer_units(c, slot, n1);
    const bool seed_hist = !sort_keys_msd(c, n1, 1, seed.total_bits);
    GK_TRY_HIP(c, launch_encode_positions(c, seed, c->keys[0], c->vals[0], seed_hist ? c->hist : nullptr));
    timer_end(c, slot);
    rc = sort_keys(c, 1, seed.total_bits, seed_hist);
    if (rc != GK_OK) return rc;

    uint64_t h = (uint64_t)seed.symbols;
    const bool bounded = M != 0;
    bool done = bounded && h >= M;  // (direct path covers M <= capacity; keep for safety)
    if (by_groups && c->cur == 0) {
        // flags of the current groups (fa), the next round's (fb); ranks of every position in R from
        // the second round on (scattered once, then only for the elements a round re-sorts)
        uint8_t *fa = c->flags, *fb;
        GK_TRY_HIP(c, scratch(c, "dbl_flags", n1 + 64, &fb));
        hipLaunchKernelGGL(full_key_heads_kernel, dim3(grid_of(n1)), dim3(256), 0, c->stream, c->keys[0], n1, fa);
        GK_TRY_HIP(c, hipGetLastError());
        uint64_t G = 0;
        GK_TRY_HIP(c, select_flags(c, fa, n1, c->idx_b, &G));
        GK_TRY_HIP(c, scan_flags_inclusive(c, fa, n1, c->idx_a));
        const int bw = std::max(1, bit_width(n1));  // ranks: group start + 1 <= n1 (0: past the segment's end)
        bool ranks_ready = false;  // every position ranked (from the second round on)
        for (int round = 0; !done; ++round) {
            if (G == n1) break;                          // all distinct
            if (!bounded && h >= c->max_seg_len) break;  // every suffix ends within h symbols
            {  // every tied group already holds equal k-mers (shared contig tails): done
                uint32_t *d_cnt = reinterpret_cast<uint32_t *>(c->scalars + 20), cnt = 0;
                GK_TRY_HIP(c, hipMemsetAsync(d_cnt, 0, 4, c->stream));
                hipLaunchKernelGGL(unresolved_groups_kernel, dim3(grid_of(G)), dim3(256), 0, c->stream, c->vals[0],
                                   c->idx_b, G, n1, c->seg, (uint32_t)c->nseg, L, h, d_cnt);
                GK_TRY_HIP(c, hipGetLastError());
                GK_TRY_HIP(c, hipMemcpyAsync(&cnt, d_cnt, 4, hipMemcpyDeviceToHost, c->stream));
                GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
                if (cnt == 0) break;
            }
            const uint64_t o = bounded ? std::min<uint64_t>(h, M - h) : h;
            int bkey = bw;
            if (round == 0) {
                // the rank of p + o after the seed sort (h = seed.symbols) orders like the seed key
                // of p + o, whatever o is: the tied elements read it from their windows, and no
                // position needs ranking yet
                GK_TRY_HIP(c, launch_member_seed_keys(c, seed, fa, c->vals[0], o, n1, c->keys[0]));
                bkey = seed.total_bits;
            } else {
                if (!ranks_ready) {  // every position ranked by the order so far, once
                    GK_TRY_HIP(c, hipMemsetAsync(c->ranks, 0, 4 * (L + 64), c->stream));
                    GK_TRY_HIP(c, launch_rank_scatter(c, c->vals[0], c->idx_a, c->idx_b, n1, c->ranks));
                    ranks_ready = true;
                }
                hipLaunchKernelGGL(member_r2_kernel, dim3(grid_of(n1)), dim3(256), 0, c->stream, fa, c->vals[0],
                                   c->ranks, c->seg, (uint32_t)c->nseg, L, o, n1, c->keys[0]);
                GK_TRY_HIP(c, hipGetLastError());
            }
            rc = msd_sort_groups(c, fa, bkey);
            if (rc != GK_OK) return rc;
            hipLaunchKernelGGL(merge_heads_kernel, dim3(grid_of(n1)), dim3(256), 0, c->stream, fa, c->heads, n1, fb);
            GK_TRY_HIP(c, hipGetLastError());
            GK_TRY_HIP(c, select_flags(c, fb, n1, c->idx_b, &G));
            GK_TRY_HIP(c, scan_flags_inclusive(c, fb, n1, c->idx_a));
            if (ranks_ready) {  // (else ranked from the current order when a round needs it)
                hipLaunchKernelGGL(member_rank_kernel, dim3(grid_of(n1)), dim3(256), 0, c->stream, fa, c->vals[0],
                                   c->idx_a, c->idx_b, n1, c->ranks);
                GK_TRY_HIP(c, hipGetLastError());
            }
            std::swap(fa, fb);
            h += o;
            if (bounded && h >= M) done = true;
        }
        // the keys: dense group numbers (equal iff the k-mers are equal, ascending with the order)
        hipLaunchKernelGGL(u32_to_key_kernel, dim3(grid_of(n1)), dim3(256), 0, c->stream, c->idx_a, n1, c->keys[0]);
        GK_TRY_HIP(c, hipGetLastError());
        done = true;
    }
    while (!done) {
        // groups of equal keys
        hipLaunchKernelGGL(full_key_heads_kernel, dim3(grid_of(n1)), dim3(256), 0, c->stream, c->keys[c->cur], n1,
                           c->flags);
        GK_TRY_HIP(c, hipGetLastError());
        uint64_t G = 0;
        GK_TRY_HIP(c, select_flags(c, c->flags, n1, c->idx_b, &G));
        if (G == n1) break;                          // all distinct
        if (!bounded && h >= c->max_seg_len) break;  // every suffix ends within h symbols
        {  // every tied group already holds equal k-mers (shared contig tails): done
            uint32_t *d_cnt = reinterpret_cast<uint32_t *>(c->scalars + 20), cnt = 0;
            GK_TRY_HIP(c, hipMemsetAsync(d_cnt, 0, 4, c->stream));
            hipLaunchKernelGGL(unresolved_groups_kernel, dim3(grid_of(G)), dim3(256), 0, c->stream, c->vals[c->cur],
                               c->idx_b, G, n1, c->seg, (uint32_t)c->nseg, L, h, d_cnt);
            GK_TRY_HIP(c, hipGetLastError());
            GK_TRY_HIP(c, hipMemcpyAsync(&cnt, d_cnt, 4, hipMemcpyDeviceToHost, c->stream));
            GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
            if (cnt == 0) break;
        }
        GK_TRY_HIP(c, scan_flags_inclusive(c, c->flags, n1, c->idx_a));
        GK_TRY_HIP(c, hipMemsetAsync(c->ranks, 0, 4 * (L + 64), c->stream));
        GK_TRY_HIP(c, launch_rank_scatter(c, c->vals[c->cur], c->idx_a, c->idx_b, n1, c->ranks));
        const uint64_t o = bounded ? std::min<uint64_t>(h, M - h) : h;
        const int bw = std::max(1, bit_width(n1));  // ranks: group start + 1 <= n1 (0: past the segment's end)
        hipLaunchKernelGGL(pair_keys_kernel, dim3(grid_of(n1)), dim3(256), 0, c->stream, c->vals[c->cur], c->ranks,
                           c->seg, (uint32_t)c->nseg, L, o, n1, bw, c->keys[c->cur]);
        GK_TRY_HIP(c, hipGetLastError());
        rc = sort_keys(c, 1, 2 * bw, false);
        if (rc != GK_OK) return rc;
        h += o;
        if (bounded && h >= M) done = true;
    }

    if (was_enumerated && n_kmers == n1) {
        // every position of the universe has >= m bases (m = 1, or no shorter tails): the order is
        // already the k-mers' order, in place
        c->n = n1;
    } else if (was_enumerated) {
        // keep starts with >= m bases, in order
        hipLaunchKernelGGL(len_flags_kernel, dim3(grid_of(n1)), dim3(256), 0, c->stream, c->vals[c->cur], c->seg,
                           (uint32_t)c->nseg, L, (uint64_t)m, n1, c->flags);
        GK_TRY_HIP(c, hipGetLastError());
        uint64_t cnt = 0;
        GK_TRY_HIP(c, select_flags(c, c->flags, n1, c->idx_a, &cnt));
        if (cnt != n_kmers) return fail(c, GK_E_HIP, "doubling: k-mer count mismatch after filtering");
        const int o = c->cur ^ 1;
        hipLaunchKernelGGL(gather_pairs_kernel, dim3(grid_of(cnt)), dim3(256), 0, c->stream, c->idx_a, cnt,
                           c->vals[c->cur], c->keys[c->cur], c->vals[o], c->keys[o]);
        GK_TRY_HIP(c, hipGetLastError());
        c->cur = o;
        c->n = cnt;
    } else {
        // final dense rank of every position, then sort the user's starts by it
        hipLaunchKernelGGL(full_key_heads_kernel, dim3(grid_of(n1)), dim3(256), 0, c->stream, c->keys[c->cur], n1,
                           c->flags);
        GK_TRY_HIP(c, hipGetLastError());
        uint64_t G = 0;
        GK_TRY_HIP(c, select_flags(c, c->flags, n1, c->idx_b, &G));
        GK_TRY_HIP(c, scan_flags_inclusive(c, c->flags, n1, c->idx_a));
        GK_TRY_HIP(c, hipMemsetAsync(c->ranks, 0, 4 * (L + 64), c->stream));
        GK_TRY_HIP(c, launch_rank_scatter(c, c->vals[c->cur], c->idx_a, c->idx_b, n1, c->ranks));
        c->n = n_kmers;
        c->cur = 0;
        if (n_kmers) GK_TRY_HIP(c, hipMemcpyAsync(c->vals[0], user, 4 * n_kmers, hipMemcpyDeviceToDevice, c->stream));
        rc = presort_by_start(c);
        if (rc != GK_OK) return rc;
        hipLaunchKernelGGL(rank_gather_kernel, dim3(grid_of(n_kmers)), dim3(256), 0, c->stream, c->vals[c->cur],
                           c->ranks, n_kmers, c->keys[c->cur]);
        GK_TRY_HIP(c, hipGetLastError());
        rc = radix_sort(c, 1, 32, false);
        if (rc != GK_OK) return rc;
        GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
        hipFree(user);
    }
    c->spec = KeySpec{0, 0, 0, (int)m, 1, 64};
    c->keys_valid = true;
    c->keys_stale = false;
    c->keys_are_ranks = true;
    return GK_OK;
}

namespace gkm {
int quicksort_by_rank(uint64_t *A, uint64_t n);  // gkm_qsort.cpp

// GK_SORT_QUICKSORT_ORDER helpers: the dense group rank of sorted element i is the last group
// whose first sorted index is <= i (binary search over the G group starts), scattered to its start
__global__ __launch_bounds__(256) void qs_rank_scatter_kernel(const uint32_t *__restrict__ S, uint64_t n,
                                                              const uint32_t *__restrict__ gs, uint64_t G,
                                                              uint32_t *__restrict__ rank_of_pos) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t lo = 0, hi = G;  // the last g with gs[g] <= i (gs[0] == 0)
        while (hi - lo > 1) {
            const uint64_t mid = (lo + hi) >> 1;
            if (gs[mid] <= i) lo = mid;
            else hi = mid;
        }
        rank_of_pos[S[i]] = (uint32_t)lo;
    }
}

// one word per original start, in the original order: rank << 32 | start
__global__ __launch_bounds__(256) void qs_pack_kernel(const uint32_t *__restrict__ orig, uint64_t n,
                                                      const uint32_t *__restrict__ rank_of_pos,
                                                      uint64_t *__restrict__ out) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t s = orig[i];
        out[i] = ((uint64_t)rank_of_pos[s] << 32) | s;
    }
}
}  // namespace gkm

// GK_SORT_QUICKSORT_ORDER, after the device sort: every start's dense group rank from the device's
// group pass, packed on the device with the start in the ORIGINAL start order `orig` (a device
// copy taken before the sort), then numba's quicksort on the host over those words with rank
// comparisons (gkm_qsort.cpp); the result replaces the sorted starts.  Only members of a group
// change places, so keys, head flags and unique counts stay valid.  Host memory: 8 B per k-mer.
static int apply_quicksort_order(gk_ctx *c, std::vector<uint32_t> &orig_host) {
    const uint64_t n = c->n;
    uint64_t G = 0;
    if (int rc = gk_unique_counts(c, &G)) return rc;
    if (int rc = materialize_starts(c)) return rc;
    // the one-off buffers below (4 B per position + 12 B per k-mer) are released on every return
    struct Release {
        gk_ctx *c;
        ~Release() {
            scratch_release(c, "qs_orig");
            scratch_release(c, "qs_rank");
            scratch_release(c, "qs_words");
        }
    } release{c};
    uint32_t *orig, *rank_of_pos;
    uint64_t *words;
    GK_TRY_HIP(c, scratch(c, "qs_orig", n, &orig));
    GK_TRY_HIP(c, hipMemcpyAsync(orig, orig_host.data(), 4 * n, hipMemcpyHostToDevice, c->stream));
    GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
    std::vector<uint32_t>().swap(orig_host);  // (host peak: the 8 B per k-mer below)
    GK_TRY_HIP(c, scratch(c, "qs_rank", c->sba_len + 1, &rank_of_pos));
    GK_TRY_HIP(c, scratch(c, "qs_words", n, &words));
    hipLaunchKernelGGL(qs_rank_scatter_kernel, dim3(grid_of(n)), dim3(256), 0, c->stream, c->vals[c->cur], n, c->idx_b,
                       G, rank_of_pos);
    GK_TRY_HIP(c, hipGetLastError());
    hipLaunchKernelGGL(qs_pack_kernel, dim3(grid_of(n)), dim3(256), 0, c->stream, orig, n, rank_of_pos, words);
    GK_TRY_HIP(c, hipGetLastError());
    std::vector<uint64_t> A(n);
    GK_TRY_HIP(c, hipMemcpyAsync(A.data(), words, 8 * n, hipMemcpyDeviceToHost, c->stream));
    GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
    if (quicksort_by_rank(A.data(), n) != 0)
        return fail(c, GK_E_UNSUPPORTED, "numba quicksort stack limit (MAX_STACK = 100) exceeded");
    // the starts (low halves) packed in place into the first 4 n bytes of A: element i is read
    // before bytes [4 i, 4 i + 4) are written, and those lie inside elements already read
    unsigned char *S = reinterpret_cast<unsigned char *>(A.data());
    for (uint64_t i = 0; i < n; ++i) {
        const uint32_t s = (uint32_t)A[i];
        std::memcpy(S + 4 * i, &s, 4);
    }
    GK_TRY_HIP(c, hipMemcpyAsync(c->vals[c->cur], S, 4 * n, hipMemcpyHostToDevice, c->stream));
    GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
    return GK_OK;
}

extern "C" int gk_sort(gk_ctx *c, uint32_t max_kmer_len, uint32_t flags) {
    if (!c) return GK_E_ARG;
    if (flags & ~(GK_SORT_CANONICAL | GK_SORT_QUICKSORT_ORDER)) return fail(c, GK_E_ARG, "unknown gk_sort flags");
    const bool canonical = (flags & GK_SORT_CANONICAL) != 0;
    const bool qorder = (flags & GK_SORT_QUICKSORT_ORDER) != 0;
    if (qorder && canonical)
        return fail(c, GK_E_ARG, "the reference's quicksort tie order exists for forward k-mers only (no canonical sort)");
    if (!c->have_starts) return fail(c, GK_E_STATE, "no k-mers: call gk_enumerate first");
    GK_TRY_HIP(c, hipSetDevice(c->device));
    if (max_kmer_len != 0 && max_kmer_len < c->min_k) return fail(c, GK_E_ARG, "max_kmer_len is less than min_kmer_len");
    if (canonical && max_kmer_len != c->min_k)
        return fail(c, GK_E_ARG, "canonical k-mers need a fixed length (max_kmer_len == min_kmer_len)");
    if (canonical && (c->acgt ? 2u : 4u) * max_kmer_len > 64u * kMaxWords)
        return fail(c, GK_E_UNSUPPORTED, "canonical k-mers are limited to 256-bit keys");
    if (c->internal_dollar)
        return fail(c, GK_E_NO_BASES, "kmers compared were less than min_kmer_len: the sba holds a '$' inside a segment");
    if (!c->enumerated && c->n > 0) {
        uint32_t *d_bad = reinterpret_cast<uint32_t *>(c->scalars + 12);
        GK_TRY_HIP(c, launch_validate_starts(c, c->vals[c->cur], c->n, c->min_k, d_bad));
        uint32_t bad = 0;
        GK_TRY_HIP(c, hipMemcpyAsync(&bad, d_bad, 4, hipMemcpyDeviceToHost, c->stream));
        GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
        if (bad) return fail(c, GK_E_NO_BASES, "kmers compared were less than min_kmer_len");
    }
    c->unique_valid = c->heads_valid = false;
    c->enum_sorted = false;
    const bool from_enum = c->enumerated;
    // only the fixed-length forward sort of the whole enumeration uses a prefetched L0 (sort_direct)
    if (canonical || qorder || max_kmer_len != c->min_k || !from_enum) pre_drop(c);
    int rc;
    // the start order the reference's quicksort starts from: a host copy (4 B per k-mer), so the
    // device sort's memory peak is not raised by it
    std::vector<uint32_t> orig;
    if (qorder && c->n >= 2) {
        if ((rc = materialize_starts(c))) return rc;
        orig.resize(c->n);
        GK_TRY_HIP(c, hipMemcpyAsync(orig.data(), c->vals[c->cur], 4 * c->n, hipMemcpyDeviceToHost, c->stream));
        GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
    }
    if (c->n < 2) {
        rc = materialize_starts(c);
        if (rc != GK_OK) return rc;
        // nothing to order; the group pass compares bytes
        c->sorted = true;
        c->sort_len = max_kmer_len;
        c->keys_valid = false;
        c->canonical = canonical;
        return GK_OK;
    }
    // direct key?
    KeySpec ks{};
    bool direct = false;
    if (max_kmer_len != 0) {
        ks.bits = c->acgt ? 2 : 4;
        ks.symbols = (int)max_kmer_len;
        ks.min_len = (int)c->min_k;
        const bool bounded = max_kmer_len != c->min_k;
        ks.lenbits = (bounded && ks.bits == 2) ? bit_width(max_kmer_len) : 0;
        ks.canonical = canonical ? 1 : 0;
        const uint64_t tb = (uint64_t)ks.bits * max_kmer_len + ks.lenbits;
        if (tb <= 64ull * kMaxWords) {
            ks.total_bits = (int)tb;
            ks.words = (int)((tb + 63) / 64);
            direct = true;
        }
    }
    // bounded keys of two or more words (ACGT, min < max, 2 max + bit_width(max) > 64: max >= 30)
    // over a large array that covers most positions: prefix doubling capped at max -- the seed
    // keys, then only the groups still tied -- instead of one LSD pass per 8 bits of the 2-word
    // keys (13 passes, 21 ms for the reference's max-50 workload).  The doubling ranks every
    // position of the sequence, so a subset of user-given starts (n well below the positions)
    // keeps the direct keys (GKM_BOUNDED_DIRECT=1 keeps them always).  The sort's keys are then
    // ranks; the key contract stays the direct one: they are re-encoded from the sorted starts
    // when asked for (keys_stale)
    const bool reroute = direct && ks.words >= 2 && !canonical && max_kmer_len != c->min_k && c->acgt &&
                         (from_enum || 2 * c->n >= c->sba_len) && sort_keys_msd(c, c->n, 1, 64) &&
                         opt("GKM_BOUNDED_DIRECT") == nullptr;
    if (reroute) direct = false;
    rc = direct ? sort_direct(c, ks) : sort_doubling(c, max_kmer_len);
    if (rc != GK_OK) return rc;
    if (reroute) {  // ranks in keys[cur]: the encoded keys are re-derived on demand (ensure_keys)
        c->spec = ks;
        c->keys_valid = true;
        c->keys_stale = true;
        c->keys_are_ranks = false;
    }
    c->enum_sorted = from_enum && direct && ks.symbols == ks.min_len;
    c->starts_materialized = true;
    c->sorted = true;
    c->enumerated = false;
    c->sort_len = max_kmer_len;
    c->canonical = canonical;
    if (qorder && c->n >= 2) {
        if ((rc = apply_quicksort_order(c, orig)) != GK_OK) {
            c->sorted = false;  // the starts are not in the order asked for
            c->unique_valid = c->heads_valid = false;
            return rc;
        }
    }
    return GK_OK;
}

extern "C" int gk_copy_strands(gk_ctx *c, uint8_t *dst, uint64_t n) {
    if (!c) return GK_E_ARG;
    pre_drop(c);  // (the k-mer buffers: a prefetched L0 does not survive)
    if (!c->sorted || !c->canonical) return fail(c, GK_E_STATE, "strands need a canonical sort (GK_SORT_CANONICAL)");
    if (n != c->n) return fail(c, GK_E_ARG, "n differs from the k-mer count");
    if (n == 0) return GK_OK;
    GK_TRY_HIP(c, hipSetDevice(c->device));
    if (int rc = materialize_starts(c)) return rc;
    KeySpec ks{};
    ks.bits = c->acgt ? 2 : 4;
    ks.symbols = (int)c->sort_len;
    uint8_t *d;
    GK_TRY_HIP(c, scratch(c, "strands", n, &d));
    GK_TRY_HIP(c, launch_canon_strands(c, ks, c->vals[c->cur], n, d));
    GK_TRY_HIP(c, hipMemcpyAsync(dst, d, n, hipMemcpyDeviceToHost, c->stream));
    GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
    return GK_OK;
}

extern "C" int gk_copy_start_indices(gk_ctx *c, uint32_t *dst, uint64_t n) {
    if (!c) return GK_E_ARG;
    if (!c->have_starts) return fail(c, GK_E_STATE, "no k-mers");
    if (int rc = materialize_starts(c)) return rc;
    if (n != c->n) return fail(c, GK_E_ARG, "n differs from the k-mer count");
    if (n == 0) return GK_OK;
    GK_TRY_HIP(c, hipMemcpyAsync(dst, c->vals[c->cur], 4 * n, hipMemcpyDeviceToHost, c->stream));
    GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
    return GK_OK;
}

extern "C" int gk_copy_start_range(gk_ctx *c, uint64_t offset, uint32_t *dst, uint64_t count) {
    if (!c) return GK_E_ARG;
    if (!c->have_starts) return fail(c, GK_E_STATE, "no k-mers");
    if (int rc = materialize_starts(c)) return rc;
    if (offset > c->n || count > c->n - offset) return fail(c, GK_E_ARG, "range outside the k-mer array");
    if (count == 0) return GK_OK;
    GK_TRY_HIP(c, hipMemcpyAsync(dst, c->vals[c->cur] + offset, 4 * count, hipMemcpyDeviceToHost, c->stream));
    GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
    return GK_OK;
}

// start index and segment of selected k-mers: starts[kmer_num[i]] and bisect_right(seg, start) - 1
// (sequence_collection.py:76-97), one thread per k-mer, binary search over the resident seg_starts
__global__ __launch_bounds__(256) void locate_kernel(const uint32_t *__restrict__ starts, uint64_t n,
                                                     const uint32_t *__restrict__ seg, uint32_t nseg,
                                                     const uint64_t *__restrict__ nums, uint64_t m,
                                                     uint32_t *__restrict__ sba_idx, uint32_t *__restrict__ seg_of) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= m) return;
    const uint64_t k = nums[i];
    const uint32_t s = k < n ? starts[k] : 0xFFFFFFFFu;
    uint32_t lo = 0, hi = nseg;  // first segment start > s
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (seg[mid] <= s) lo = mid + 1;
        else hi = mid;
    }
    sba_idx[i] = s;
    seg_of[i] = lo - 1;  // nseg >= 1 and seg[0] == 0, so lo >= 1 for every valid start
}

extern "C" int gk_locate(gk_ctx *c, const uint64_t *kmer_nums, uint64_t m, uint32_t *sba_idx, uint32_t *seg) {
    if (!c) return GK_E_ARG;
    pre_drop(c);  // (the k-mer buffers: a prefetched L0 does not survive)
    if (!c->have_starts) return fail(c, GK_E_STATE, "no k-mers");
    if (m == 0) return GK_OK;
    if (!kmer_nums || !sba_idx || !seg) return fail(c, GK_E_ARG, "null array");
    if (int rc = materialize_starts(c)) return rc;
    for (uint64_t i = 0; i < m; ++i)
        if (kmer_nums[i] >= c->n) return fail(c, GK_E_ARG, "kmer_num out of range");
    uint64_t *d_nums;
    uint32_t *d_out;
    GK_TRY_HIP(c, scratch(c, "locate_nums", m, &d_nums));
    GK_TRY_HIP(c, scratch(c, "locate_out", 2 * m, &d_out));
    GK_TRY_HIP(c, hipMemcpyAsync(d_nums, kmer_nums, 8 * m, hipMemcpyHostToDevice, c->stream));
    hipLaunchKernelGGL(locate_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, c->stream, c->vals[c->cur], c->n,
                       c->seg, (uint32_t)c->nseg, d_nums, m, d_out, d_out + m);
    GK_TRY_HIP(c, hipGetLastError());
    GK_TRY_HIP(c, hipMemcpyAsync(sba_idx, d_out, 4 * m, hipMemcpyDeviceToHost, c->stream));
    GK_TRY_HIP(c, hipMemcpyAsync(seg, d_out + m, 4 * m, hipMemcpyDeviceToHost, c->stream));
    GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
    return GK_OK;
}

extern "C" int gk_key_layout(gk_ctx *c, uint32_t *words, uint32_t *bits, uint32_t *symbols) {
    if (!c) return GK_E_ARG;
    if (!c->keys_valid) return fail(c, GK_E_STATE, "no encoded keys: sort first");
    if (words) *words = (uint32_t)c->spec.words;
    if (bits) *bits = c->keys_are_ranks ? 0u : (uint32_t)c->spec.bits;
    if (symbols) *symbols = c->keys_are_ranks ? 0u : (uint32_t)c->spec.symbols;
    return GK_OK;
}

extern "C" int gk_copy_keys(gk_ctx *c, uint64_t *dst, uint64_t n_words) {
    if (!c) return GK_E_ARG;
    pre_drop(c);  // (the k-mer buffers: a prefetched L0 does not survive)
    if (!c->keys_valid) return fail(c, GK_E_STATE, "no encoded keys: sort first");
    if (int rc = ensure_keys(c)) return rc;
    const uint64_t W = (uint64_t)c->spec.words;
    if (n_words != W * c->n) return fail(c, GK_E_ARG, "n_words differs from words_per_key * n");
    if (!n_words) return GK_OK;
    // device SoA (word-major) -> host AoS (key-major)
    std::vector<uint64_t> tmp(n_words);
    GK_TRY_HIP(c, hipMemcpyAsync(tmp.data(), c->keys[c->cur], 8 * n_words, hipMemcpyDeviceToHost, c->stream));
    GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
    if (W == 1) {
        std::memcpy(dst, tmp.data(), 8 * n_words);
    } else {
        for (uint64_t i = 0; i < c->n; ++i)
            for (uint64_t w = 0; w < W; ++w) dst[i * W + w] = tmp[w * c->n + i];
    }
    return GK_OK;
}

extern "C" int gk_set_filter_mask(gk_ctx *c, const uint8_t *mask, uint64_t n) {
    if (!c) return GK_E_ARG;
    pre_drop(c);  // (the k-mer buffers: a prefetched L0 does not survive)
    GK_TRY_HIP(c, ensure(reinterpret_cast<void **>(&c->mask), &c->mask_cap, n + 64));
    if (n) GK_TRY_HIP(c, hipMemcpyAsync(c->mask, mask, n, hipMemcpyHostToDevice, c->stream));
    GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
    c->mask_n = n;
    return GK_OK;
}

extern "C" int gk_set_group_heads(gk_ctx *c, const uint8_t *heads, uint64_t n) {
    if (!c) return GK_E_ARG;
    pre_drop(c);  // (the k-mer buffers: a prefetched L0 does not survive)
    GK_TRY_HIP(c, ensure(reinterpret_cast<void **>(&c->hmask), &c->hmask_cap, n + 64));
    if (n) GK_TRY_HIP(c, hipMemcpyAsync(c->hmask, heads, n, hipMemcpyHostToDevice, c->stream));
    GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
    c->hmask_n = n;
    return GK_OK;
}

extern "C" int gk_device_views(gk_ctx *c, void **starts, void **keys, uint64_t *n, uint32_t *words) {
    if (!c) return GK_E_ARG;
    pre_drop(c);  // (the k-mer buffers: a prefetched L0 does not survive)
    if (int rc = materialize_starts(c)) return rc;
    if (keys && c->keys_valid)
        if (int rc = ensure_keys(c)) return rc;
    if (starts) *starts = c->vals[c->cur];
    if (keys) *keys = c->keys[c->cur];
    if (n) *n = c->n;
    if (words) *words = (uint32_t)c->spec.words;
    return GK_OK;
}

// ---------------------------------------------------------------------------------------------
// profiling
// ---------------------------------------------------------------------------------------------
extern "C" int gk_profile_enable(gk_ctx *c, int on) {
    if (!c) return GK_E_ARG;
    hipStreamSynchronize(c->stream);
    c->timers.clear();
    c->ev_used = 0;
    c->profile = on != 0;
    // pre-create the events of a few hundred timed stages (a step uses tens): a timed step then
    // only records events
    while (c->profile && c->ev_pool.size() < 16384) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) break;
        c->ev_pool.push_back(e);
    }
    return GK_OK;
}

extern "C" int gk_profile_report(gk_ctx *c, char *buf, uint64_t buflen) {
    if (!c || !buf || buflen == 0) return GK_E_ARG;
    GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
    struct Agg {
        uint64_t count = 0, units = 0;
        double ms = 0;
    };
    std::map<std::string, Agg> agg;
    for (auto &t : c->timers) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, t.start, t.stop) == hipSuccess) {
            auto &a = agg[t.name];
            a.count += 1;
            a.ms += ms;
            a.units += t.units;
        }
    }
    std::string s = "{";
    bool first = true;
    for (auto &kv : agg) {
        char tmp[320];
        std::snprintf(tmp, sizeof tmp, "%s\"%s\": {\"count\": %llu, \"total_ms\": %.6f, \"units\": %llu}",
                      first ? "" : ", ", kv.first.c_str(), (unsigned long long)kv.second.count, kv.second.ms,
                      (unsigned long long)kv.second.units);
        s += tmp;
        first = false;
    }
    s += "}";
    std::snprintf(buf, (size_t)buflen, "%s", s.c_str());
    return s.size() < buflen ? GK_OK : GK_E_ARG;
}

// ---------------------------------------------------------------------------------------------
// multi-GPU shards
// ---------------------------------------------------------------------------------------------
static int shard_spec(gk_ctx *c, uint32_t k, uint32_t flags, KeySpec *ks) {
    if (flags & ~(GK_SORT_CANONICAL | GK_SHARD_STARTS_ONLY)) return fail(c, GK_E_ARG, "unknown shard flags");
    if ((flags & GK_SHARD_STARTS_ONLY) && ((flags & GK_SORT_CANONICAL) || !c->acgt || k > 32))
        return fail(c, GK_E_UNSUPPORTED, "starts-only shards: forward keys of an A/C/G/T sba with k <= 32");
    const int bits = c->acgt ? 2 : 4;
    if (k == 0 || k > 64) return fail(c, GK_E_ARG, "shard k-mers must have 1 <= k <= 64");
    *ks = KeySpec{};
    ks->bits = bits;
    ks->symbols = (int)k;
    ks->min_len = (int)k;
    ks->lenbits = 0;
    ks->total_bits = bits * (int)k;
    ks->words = (ks->total_bits + 63) / 64;  // exchanged: the first word; the rest re-encoded from the sba
    ks->canonical = (flags & GK_SORT_CANONICAL) ? 1 : 0;
    return GK_OK;
}

extern "C" int gk_shard_bucket_bits(void) { return gkm::msd_radix_bits(); }

extern "C" int gk_shard_partition(gk_ctx *c, uint64_t lo, uint64_t hi, uint32_t k, uint32_t flags, uint64_t *d_keys,
                                  uint32_t *d_starts, uint64_t cap, uint64_t *h_hist, uint64_t *n_out) {
    const bool starts_only = (flags & GK_SHARD_STARTS_ONLY) != 0;
    if (!c || (!d_keys && !starts_only) || !d_starts || !h_hist || !n_out) return GK_E_ARG;
    pre_drop(c);  // (the k-mer buffers: a prefetched L0 does not survive)
    GK_TRY_HIP(c, hipSetDevice(c->device));
    if (lo % 32) return fail(c, GK_E_ARG, "shard lo must be a multiple of 32");
    if (hi > c->sba_len) hi = c->sba_len;
    if (c->internal_dollar) return fail(c, GK_E_NO_BASES, "the sba holds a '$' inside a segment");
    KeySpec ks;
    int rc = shard_spec(c, k, flags, &ks);
    if (rc != GK_OK) return rc;
    return msd_shard_partition(c, ks, lo, std::max(hi, lo), starts_only ? nullptr : d_keys, d_starts, cap, h_hist,
                               n_out);
}

// Key-range shards of a mixed sba (N runs, IUPAC letters; k >= 4): the ranges are top-7-bit
// digits of the ACGT-only k-mers' 2-bit keys (split_sort with a SplitRange); other k-mers follow
// the byte-order interval those digits bound.  k < 4: plain 4-bit digits.
static bool range_split(gk_ctx *c, const KeySpec &ks) { return !c->acgt && ks.bits == 4 && ks.symbols >= 4; }

static KeySpec acgt_spec(KeySpec ks) {
    ks.bits = 2;
    ks.total_bits = 2 * ks.symbols;
    ks.words = (ks.total_bits + 63) / 64;
    ks.acgt_only = 1;
    return ks;
}

// the 4-bit code of the first ceil(ob / 2) symbols of the smallest ACGT k-mer with top-ob-bit
// digit d (an odd width ends in a half symbol: A or G by the digit's low bit); a range from digit
// 0 has no lower bound, a range to digit 1 << ob no upper one
static uint32_t range_prefix(uint32_t d, bool lower, int ob) {
    const int ns = (ob + 1) / 2;
    if (lower && d == 0) return 0;
    if (d >= (1u << ob)) return 1u << (4 * ns);
    static const uint32_t c4[4] = {1, 3, 5, 12};  // A C G T among '$' A B C D G H K M N R S T V W Y
    const uint32_t dd = (ob & 1) ? d << 1 : d;
    uint32_t v = 0;
    for (int j = 0; j < ns; ++j) v = (v << 4) | c4[(dd >> (2 * (ns - 1 - j))) & 3];
    return v;
}

extern "C" int gk_shard_histogram(gk_ctx *c, uint64_t lo, uint64_t hi, uint32_t k, uint32_t flags, uint64_t *h_hist,
                                  uint32_t *bits) {
    if (!c || !h_hist || !bits) return GK_E_ARG;
    pre_drop(c);  // (the k-mer buffers: a prefetched L0 does not survive)
    GK_TRY_HIP(c, hipSetDevice(c->device));
    if (lo % 32) return fail(c, GK_E_ARG, "shard lo must be a multiple of 32");
    if (hi > c->sba_len) hi = c->sba_len;
    if (c->internal_dollar) return fail(c, GK_E_NO_BASES, "the sba holds a '$' inside a segment");
    KeySpec ks;
    int rc = shard_spec(c, k, flags, &ks);
    if (rc != GK_OK) return rc;
    if (range_split(c, ks)) ks = acgt_spec(ks);  // mixed sba: digits of the ACGT-only k-mers
    for (int i = 0; i < 4096; ++i) h_hist[i] = 0;
    int b = 0;
    rc = msd_l0_histogram(c, ks, lo, std::max(hi, lo), h_hist, &b);
    *bits = (uint32_t)b;
    return rc;
}

// the weight of a homopolymer k-mer in the ownership histogram, in 16ths of a sorted k-mer: it
// skips the MSD sort, but is expanded, grouped, keyed and merged (fitted to
// the C4 emulation: 11/16 balances the rank that owns the N runs with the others)
constexpr uint32_t kHomoWeight16 = 11;

extern "C" int gk_shard_class_b(gk_ctx *c, uint64_t lo, uint64_t hi, uint32_t k, uint32_t flags, uint64_t *h_hist,
                                uint64_t *n_rest, uint64_t *n_runs) {
    if (!c || !h_hist || !n_rest || !n_runs) return GK_E_ARG;
    pre_drop(c);  // (the k-mer buffers: a prefetched L0 does not survive)
    GK_TRY_HIP(c, hipSetDevice(c->device));
    *n_rest = *n_runs = 0;
    c->shard_rest.clear();
    c->shard_runs.clear();
    if (c->internal_dollar) return fail(c, GK_E_NO_BASES, "the sba holds a '$' inside a segment");
    KeySpec ks;
    int rc = shard_spec(c, k, flags, &ks);
    if (rc != GK_OK) return rc;
    if (!range_split(c, ks)) return GK_OK;  // no class B: ACGT-only sba, or k < 4
    const int ob = range_own_bits(acgt_spec(ks));
    std::vector<uint32_t> bins(1u << ob);
    for (uint32_t d = 0; d < bins.size(); ++d) bins[d] = range_prefix(d, true, ob);
    rc = split_shard_class_b(c, ks, lo, hi, bins, (ob + 1) / 2, kHomoWeight16, h_hist, &c->shard_rest, &c->shard_runs);
    if (rc != GK_OK) return rc;
    *n_rest = c->shard_rest.size();
    *n_runs = c->shard_runs.size() / 3;
    return GK_OK;
}

extern "C" int gk_shard_class_b_copy(gk_ctx *c, uint32_t *rest, uint64_t n_rest, uint32_t *runs, uint64_t n_runs) {
    if (!c) return GK_E_ARG;
    pre_drop(c);  // (the k-mer buffers: a prefetched L0 does not survive)
    if (n_rest != c->shard_rest.size() || 3 * n_runs != c->shard_runs.size())
        return fail(c, GK_E_ARG, "gk_shard_class_b_copy: sizes differ from gk_shard_class_b's");
    if ((n_rest && !rest) || (n_runs && !runs)) return GK_E_ARG;
    if (n_rest) std::memcpy(rest, c->shard_rest.data(), 4 * n_rest);
    if (n_runs) std::memcpy(runs, c->shard_runs.data(), 12 * n_runs);
    return GK_OK;
}

static int shard_sort_range_impl(gk_ctx *c, uint32_t k, uint32_t flags, uint32_t digit_lo, uint32_t digit_hi,
                                 const uint32_t *rest, uint64_t n_rest, const uint32_t *runs, uint64_t n_runs,
                                 bool given, uint64_t *n_kept);

extern "C" int gk_shard_sort_range_b(gk_ctx *c, uint32_t k, uint32_t flags, uint32_t digit_lo, uint32_t digit_hi,
                                     const uint32_t *rest, uint64_t n_rest, const uint32_t *runs, uint64_t n_runs,
                                     uint64_t *n_kept) {
    if ((n_rest && !rest) || (n_runs && !runs)) return GK_E_ARG;
    return shard_sort_range_impl(c, k, flags, digit_lo, digit_hi, rest, n_rest, runs, n_runs, true, n_kept);
}

extern "C" int gk_shard_sort_range(gk_ctx *c, uint32_t k, uint32_t flags, uint32_t digit_lo, uint32_t digit_hi,
                                   uint64_t *n_kept) {
    return shard_sort_range_impl(c, k, flags, digit_lo, digit_hi, nullptr, 0, nullptr, 0, false, n_kept);
}

static int shard_sort_range_impl(gk_ctx *c, uint32_t k, uint32_t flags, uint32_t digit_lo, uint32_t digit_hi,
                                 const uint32_t *rest, uint64_t n_rest, const uint32_t *runs, uint64_t n_runs,
                                 bool given, uint64_t *n_kept) {
    if (!c || !n_kept) return GK_E_ARG;
    pre_drop(c);
    GK_TRY_HIP(c, hipSetDevice(c->device));
    if (c->internal_dollar) return fail(c, GK_E_NO_BASES, "the sba holds a '$' inside a segment");
    if (digit_lo > digit_hi || digit_hi > 4096u) return fail(c, GK_E_ARG, "digit range outside [0, 4096]");
    KeySpec ks;
    int rc = shard_spec(c, k, flags, &ks);
    if (rc != GK_OK) return rc;
    c->min_k = k;
    c->have_starts = true;
    c->enumerated = false;
    c->starts_materialized = true;
    c->sorted = c->keys_valid = c->unique_valid = c->heads_valid = c->canonical = c->enum_sorted = false;
    if (range_split(c, ks)) {  // mixed sba: ACGT-only k-mers by 2-bit digit, the rest by prefix
        const int ob = range_own_bits(acgt_spec(ks));
        SplitRange rg{digit_lo, digit_hi, range_prefix(digit_lo, true, ob), range_prefix(digit_hi, false, ob), (ob + 1) / 2};
        rg.given = given;
        rg.rest = rest;
        rg.n_rest = n_rest;
        rg.runs = runs;
        rg.n_runs = n_runs;
        bool used = false;
        rc = split_sort(c, ks, &used, &rg);
        if (rc == GK_OK && !used) rc = fail(c, GK_E_HIP, "key-range split sort not applicable");
        *n_kept = c->n;
    } else {
        rc = msd_sort_range(c, ks, digit_lo, digit_hi, n_kept);
    }
    if (rc != GK_OK) return rc;
    c->spec = ks;
    c->keys_valid = true;
    c->keys_stale = c->n > 0 && (range_split(c, ks) ? !c->split_keys_final : !c->msd_keys_final);  // see sort_direct
    c->keys_are_ranks = false;
    c->sorted = true;
    c->sort_len = k;
    c->canonical = ks.canonical != 0;
    return GK_OK;
}

extern "C" int gk_shard_sort(gk_ctx *c, const uint64_t *d_keys, const uint32_t *d_starts, uint64_t n, uint32_t k,
                             uint32_t flags, const uint64_t *h_piece_off, const uint64_t *h_piece_len,
                             const uint32_t *h_piece_bucket, uint32_t npieces) {
    const bool starts_only = (flags & GK_SHARD_STARTS_ONLY) != 0;
    if (!c || (n && ((!d_keys && !starts_only) || !d_starts || !h_piece_off || !h_piece_len || !h_piece_bucket)))
        return GK_E_ARG;
    pre_drop(c);  // (the k-mer buffers: a prefetched L0 does not survive)
    GK_TRY_HIP(c, hipSetDevice(c->device));
    if (n > 0xFFFFFFFFull) return fail(c, GK_E_ARG, "more k-mers than uint32 start indices can address");
    KeySpec ks;
    int rc = shard_spec(c, k, flags, &ks);
    if (rc != GK_OK) return rc;
    for (uint32_t i = 1; i < npieces; ++i)
        if (h_piece_bucket[i] < h_piece_bucket[i - 1]) return fail(c, GK_E_ARG, "pieces must be in bucket order");
    rc = ensure_elems(c, std::max<uint64_t>(n, 1), 1);
    if (rc != GK_OK) return rc;
    c->n = n;
    c->min_k = k;
    c->have_starts = true;
    c->enumerated = false;
    c->starts_materialized = true;
    c->sorted = c->keys_valid = c->unique_valid = c->heads_valid = c->canonical = c->enum_sorted = false;
    if (n > 0) {
        rc = msd_shard_sort(c, ks, starts_only ? nullptr : d_keys, d_starts, h_piece_off, h_piece_len, h_piece_bucket,
                            npieces);
        if (rc != GK_OK) return rc;
    } else {
        c->cur = 0;
    }
    c->spec = ks;
    c->keys_valid = true;
    c->keys_stale = n > 0 && !c->msd_keys_final;  // see sort_direct
    c->keys_are_ranks = false;
    c->sorted = true;
    c->sort_len = k;
    c->canonical = ks.canonical != 0;
    return GK_OK;
}

// gkm_xfer.hip -- host -> device transfer of the sequence byte array, 2-bit packed (gk_set_sequence).
//
// The reference hands the hot path a uint8 ASCII sba (sequence_collection.py:531-576, 663-726):
// 1 byte per base, 3.1 GB for a human-sized genome, ~56 ms over PCIe at 55 GB/s -- 40 % of the
// end-to-end time of a C3 sort.  Nearly every base is A, C, G or T, so the transfer ships 2 bits
// per base where it can:
//   host    the sba is cut into 64 KiB blocks and chunks of kBlocksPerChunk blocks.  Worker threads
//           (up to 16) take chunks in order and write each into a pinned staging slot: a header
//           (per block: payload offset | raw flag), then per block either the 16 KiB of 2-bit
//           codes (every byte A/C/G/T: AVX2 compare + pack, 64 bases per step; AVX-512 on request) or the raw bytes
//           (anything else: '$' separators, N runs, IUPAC letters).  The same pass takes the
//           alphabet census the reference's check needs (sequence_collection.py:441-458, 694-697):
//           classes seen and '$' count -- no device pass over the sba afterwards.
//   link    the caller's thread copies each finished chunk H2D on a copy stream, in chunk order,
//           header + payload only (C3: 0.78 GB instead of 3.1 GB).
//   device  unpack_chunk_kernel expands the chunk into the resident ASCII sba (LDS table, 16-B
//           loads, 64-B stores) on the context's stream; the sort kernels read the sba as before.
// Packing, copies and unpacking overlap: slots are recycled once the device has unpacked them.
// Inputs below GKM_PACK_MIN bytes (default 16 MiB) are copied as they are (gkm_capi.hip).
#include <immintrin.h>
#include <pthread.h>
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <cstdio>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "gkm_internal.h"
#include "gkm_swar.h"

namespace gkm {

constexpr uint64_t kXBlock = 64 * 1024;  // bytes of sba per block
constexpr uint32_t kRawFlag = 0x80000000u;
constexpr uint64_t kHeaderBytes = 1024;  // per slot: uint32 per block (<= 256 blocks)
constexpr int kRawDepth = 4;             // raw chunk copies in flight (pinned sources)

// ---------------------------------------------------------------------------------------------
// device
// ---------------------------------------------------------------------------------------------
// packed byte b (bases 4j..4j+3 at bits 2i) -> 4 ASCII bytes, A0 C1 G2 T3
// pkc / pkd (null: none): the chunk's words of the 2-bit packed copy (pack2_kernel layout, 32
// positions per word): a packed block's codes are its own bytes with the base order of each
// 32-base half reversed (rev_pairs), no stops; a raw block is packed from its bytes, its stops the
// bytes other than A/C/G/T (pack2_word<true>).
// Words of a partial last block are left to the caller (the tail pack after the transfer).
__global__ __launch_bounds__(256) void unpack_chunk_kernel(const uint8_t *__restrict__ slot,
                                                           uint8_t *__restrict__ dst, uint64_t chunk_len,
                                                           uint64_t *__restrict__ pkc = nullptr,
                                                           uint32_t *__restrict__ pkd = nullptr) {
    __shared__ uint32_t s_lut[256];
    const int t = threadIdx.x;
    {
        constexpr uint32_t kAscii = 0x54474341u;  // "ACGT" little-endian
        uint32_t w = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) w |= ((kAscii >> (8 * ((t >> (2 * i)) & 3))) & 0xFFu) << (8 * i);
        s_lut[t] = w;
    }
    __syncthreads();
    const uint64_t b0 = (uint64_t)blockIdx.x * kXBlock;
    const uint64_t blen = chunk_len - b0 < kXBlock ? chunk_len - b0 : kXBlock;
    const uint32_t hdr = reinterpret_cast<const uint32_t *>(slot)[blockIdx.x];
    const uint8_t *src = slot + (hdr & ~kRawFlag);
    uint8_t *out = dst + b0;
    if (hdr & kRawFlag) {  // raw bytes: a straight copy, 16 B per lane where whole
        const uint64_t q = blen / 16;
        for (uint64_t i = t; i < q; i += 256)
            reinterpret_cast<uint4 *>(out)[i] = reinterpret_cast<const uint4 *>(src)[i];
        for (uint64_t i = q * 16 + t; i < blen; i += 256) out[i] = src[i];
        if (pkc) {
            for (uint64_t u = t; u < blen / 32; u += 256) {
                uint64_t cw;
                uint32_t dw;
                pack2_word<true>(src + 32 * u, cw, dw);
                pkc[b0 / 32 + u] = cw;
                pkd[b0 / 32 + u] = dw;
            }
        }
        return;
    }
    // 16 packed bytes -> 64 bases per lane step
    const uint64_t groups = (blen + 63) / 64;
    for (uint64_t g = t; g < groups; g += 256) {
        const uint4 p = reinterpret_cast<const uint4 *>(src)[g];
        const uint32_t pw[4] = {p.x, p.y, p.z, p.w};
        uint32_t o[16];
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int j = 0; j < 4; ++j) o[4 * k + j] = s_lut[(pw[k] >> (8 * j)) & 0xFFu];
        if ((g + 1) * 64 <= blen) {
            uint4 *q = reinterpret_cast<uint4 *>(out + g * 64);
#pragma unroll
            for (int k = 0; k < 4; ++k) q[k] = make_uint4(o[4 * k], o[4 * k + 1], o[4 * k + 2], o[4 * k + 3]);
            if (pkc) {
                const uint64_t w = (b0 + g * 64) / 32;
                const uint64_t c0 = rev_pairs(((uint64_t)p.y << 32) | p.x), c1 = rev_pairs(((uint64_t)p.w << 32) | p.z);
                reinterpret_cast<uint4 *>(pkc + w)[0] =
                    make_uint4((uint32_t)c0, (uint32_t)(c0 >> 32), (uint32_t)c1, (uint32_t)(c1 >> 32));
                reinterpret_cast<uint2 *>(pkd + w)[0] = make_uint2(0, 0);
            }
        } else {  // the sba's last, partial group
            for (uint64_t i = g * 64; i < blen; ++i) out[i] = (uint8_t)(o[(i - g * 64) >> 2] >> (8 * (i & 3)));
        }
    }
}

// ---------------------------------------------------------------------------------------------
// host packing
// ---------------------------------------------------------------------------------------------
namespace {

// reference alphabet classes, as the device check (gkm_encode.hip c_class): 0 A/C/G/T/'$',
// 1 other IUPAC letter, 2 not allowed
struct ClassTable {
    uint8_t c[256];
    ClassTable() {
        for (int i = 0; i < 256; ++i) c[i] = 2;
        for (const char *p = "ABCDGHKMNRSTVWY"; *p; ++p) c[(uint8_t)*p] = 1;
        c['A'] = c['C'] = c['G'] = c['T'] = c[GK_DOLLAR] = 0;
    }
};
const ClassTable kClass;

struct Census {
    uint32_t cls_or = 0;
    uint64_t dollars = 0;
};

inline uint32_t code_of(uint8_t c) { return ((c >> 1) ^ (c >> 2)) & 3u; }

// scalar: 2-bit codes of n bases (n % 4 == 0 except at the sba's end), false at the first non-ACGT
bool pack_scalar(const uint8_t *s, uint64_t n, uint8_t *d) {
    for (uint64_t i = 0; i < n; i += 4) {
        uint32_t v = 0;
        for (int j = 0; j < 4; ++j) {
            const uint8_t c = i + j < n ? s[i + j] : 'A';
            if (c != 'A' && c != 'C' && c != 'G' && c != 'T') return false;
            v |= code_of(c) << (2 * j);
        }
        d[i / 4] = (uint8_t)v;
    }
    return true;
}

// AVX2: 64 bases -> 16 bytes per step.  Alphabet: four compares per 32 bytes; code =
// ((c ^ c >> 1) >> 1) & 3 (A0 C1 G2 T3); two multiply-adds fold 4 codes into the low byte of a
// dword, two saturating packs and one dword permute put the 16 bytes in order, one 16-byte store
// (the staging slots are pinned memory: whole 16-byte stores).
__attribute__((target("avx2"))) static inline __m256i avx2_codes(__m256i v) {
    const __m256i x = _mm256_xor_si256(v, _mm256_srli_epi16(v, 1));
    return _mm256_and_si256(_mm256_srli_epi16(x, 1), _mm256_set1_epi8(3));
}

__attribute__((target("avx2"))) static inline uint32_t avx2_acgt_mask(__m256i v) {
    const __m256i ok = _mm256_or_si256(
        _mm256_or_si256(_mm256_cmpeq_epi8(v, _mm256_set1_epi8('A')), _mm256_cmpeq_epi8(v, _mm256_set1_epi8('C'))),
        _mm256_or_si256(_mm256_cmpeq_epi8(v, _mm256_set1_epi8('G')), _mm256_cmpeq_epi8(v, _mm256_set1_epi8('T'))));
    return (uint32_t)_mm256_movemask_epi8(ok);
}

__attribute__((target("avx2"))) bool pack_avx2(const uint8_t *s, uint64_t n, uint8_t *d) {
    const __m256i w1 = _mm256_set1_epi16(0x0401);      // bytes (1, 4): c0 + 4 c1
    const __m256i w2 = _mm256_set1_epi32(0x00100001);  // words (1, 16): (c0 + 4 c1) + 16 (c2 + 4 c3)
    const __m256i order = _mm256_setr_epi32(0, 4, 1, 5, 2, 6, 3, 7);
    uint64_t i = 0;
    for (; i + 64 <= n; i += 64) {
        const __m256i v0 = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(s + i));
        const __m256i v1 = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(s + i + 32));
        if ((avx2_acgt_mask(v0) & avx2_acgt_mask(v1)) != 0xFFFFFFFFu) return false;
        const __m256i q0 = _mm256_madd_epi16(_mm256_maddubs_epi16(avx2_codes(v0), w1), w2);
        const __m256i q1 = _mm256_madd_epi16(_mm256_maddubs_epi16(avx2_codes(v1), w1), w2);
        // per 128-bit lane: packus_epi32 -> (q0 lane, q1 lane) words; packus_epi16 -> their bytes
        // (twice); dwords 0, 4, 1, 5 are then q0[0..3], q0[4..7], q1[0..3], q1[4..7]
        const __m256i b = _mm256_packus_epi16(_mm256_packus_epi32(q0, q1), _mm256_setzero_si256());
        const __m256i o = _mm256_permutevar8x32_epi32(b, order);
        // d is 16-byte aligned (slot payloads start at multiples of 16): a streaming store, the
        // staging slot is written once here and next read by the DMA engine, not by this core
        _mm_stream_si128(reinterpret_cast<__m128i *>(d + i / 4), _mm256_castsi256_si128(o));
    }
    return pack_scalar(s + i, n - i, d + i / 4);
}

// AVX-512 (BW): 64 bases -> 16 bytes per step with a quarter of the AVX2 path's instructions --
// four byte compares into mask registers for the alphabet, the same code arithmetic, two
// multiply-adds, one dword -> byte narrowing (vpmovdb) straight to the 16 output bytes
__attribute__((target("avx512f,avx512bw"))) bool pack_avx512(const uint8_t *s, uint64_t n, uint8_t *d) {
    const __m512i w1 = _mm512_set1_epi16(0x0401);
    const __m512i w2 = _mm512_set1_epi32(0x00100001);
    const __m512i three = _mm512_set1_epi8(3);
    const __m512i cA = _mm512_set1_epi8('A'), cC = _mm512_set1_epi8('C'), cG = _mm512_set1_epi8('G'),
                  cT = _mm512_set1_epi8('T');
    uint64_t i = 0;
    for (; i + 64 <= n; i += 64) {
        const __m512i v = _mm512_loadu_si512(reinterpret_cast<const void *>(s + i));
        const __mmask64 ok = _mm512_cmpeq_epi8_mask(v, cA) | _mm512_cmpeq_epi8_mask(v, cC) |
                             _mm512_cmpeq_epi8_mask(v, cG) | _mm512_cmpeq_epi8_mask(v, cT);
        if (ok != ~0ull) return false;
        const __m512i x = _mm512_xor_si512(v, _mm512_srli_epi16(v, 1));
        const __m512i codes = _mm512_and_si512(_mm512_srli_epi16(x, 1), three);
        const __m512i q = _mm512_madd_epi16(_mm512_maddubs_epi16(codes, w1), w2);
        _mm_stream_si128(reinterpret_cast<__m128i *>(d + i / 4), _mm512_cvtepi32_epi8(q));
    }
    return pack_scalar(s + i, n - i, d + i / 4);
}

bool have_avx2() {
    static const bool v = __builtin_cpu_supports("avx2");
    return v;
}

// GKM_PACK_IMPL=scalar / avx2 / avx512 (A/B and tests); default AVX2: on the GPU box's EPYC 9575F
// the AVX-512 packer moved 3.1 Gb in 25-29 ms against 22 ms for AVX2, 16 threads, medians of 7
// (profiles/r5/xfer_probe.txt) -- the packing is bound by host memory, not by instructions
int pack_impl() {
    static const int v = [] {
        const char *e = opt("GKM_PACK_IMPL");
        const bool a512 = __builtin_cpu_supports("avx512bw") && __builtin_cpu_supports("avx512f");
        if (e && !std::strcmp(e, "scalar")) return 0;
        if (e && !std::strcmp(e, "avx512")) return a512 ? 2 : have_avx2() ? 1 : 0;
        return have_avx2() ? 1 : 0;
    }();
    return v;
}

// one chunk into a staging slot; returns the bytes used (header + payloads)
uint64_t pack_chunk(const uint8_t *src, uint64_t len, uint8_t *slot, Census &cen, bool *all_packed) {
    const uint32_t nb = (uint32_t)((len + kXBlock - 1) / kXBlock);
    uint32_t *hdr = reinterpret_cast<uint32_t *>(slot);
    uint64_t off = kHeaderBytes;
    const int impl = pack_impl();
    *all_packed = true;
    for (uint32_t b = 0; b < nb; ++b) {
        const uint8_t *s = src + (uint64_t)b * kXBlock;
        const uint64_t blen = std::min<uint64_t>(kXBlock, len - (uint64_t)b * kXBlock);
        uint8_t *d = slot + off;
        if (impl == 2 ? pack_avx512(s, blen, d) : impl == 1 ? pack_avx2(s, blen, d) : pack_scalar(s, blen, d)) {
            hdr[b] = (uint32_t)off;
            off += ((blen + 63) / 64) * 16;  // whole 16-byte groups (the unpack reads uint4)
            cen.cls_or |= 1u;
            continue;
        }
        std::memcpy(d, s, blen);
        *all_packed = false;
        for (uint64_t i = 0; i < blen; ++i) {
            cen.cls_or |= 1u << kClass.c[s[i]];
            cen.dollars += s[i] == GK_DOLLAR;
        }
        hdr[b] = (uint32_t)off | kRawFlag;
        off += (blen + 15) & ~15ull;
    }
    return off;
}

// CPUs of the calling thread's NUMA node (within the process's affinity mask), for pinning the
// packing threads next to the memory they read (GKM_XFER_NUMA=1); empty when unknown
// the CPUs (within this process's affinity) of NUMA node `want`, or of the node holding CPU `cpu`
// when want < 0
static std::vector<int> node_cpus(int want, int cpu) {
    std::vector<int> out;
    cpu_set_t allowed;
    CPU_ZERO(&allowed);
    if (sched_getaffinity(0, sizeof allowed, &allowed) != 0) return out;
    for (int node = 0; node < 64; ++node) {
        char path[96];
        std::snprintf(path, sizeof path, "/sys/devices/system/node/node%d/cpulist", node);
        FILE *f = std::fopen(path, "r");
        if (!f) continue;
        char buf[4096] = {0};
        const size_t got = std::fread(buf, 1, sizeof buf - 1, f);
        std::fclose(f);
        buf[got] = 0;
        std::vector<int> cpus;
        for (char *q = buf; *q;) {  // "a-b,c,d-e"
            char *end;
            const long a = std::strtol(q, &end, 10);
            if (end == q) break;
            long b = a;
            if (*end == '-') b = std::strtol(end + 1, &end, 10);
            for (long x = a; x <= b && x < CPU_SETSIZE; ++x)
                if (CPU_ISSET((int)x, &allowed)) cpus.push_back((int)x);
            q = end;
            while (*q == ',' || *q == '\n') ++q;
        }
        if (want >= 0 ? node == want : std::find(cpus.begin(), cpus.end(), cpu) != cpus.end()) return cpus;
    }
    return out;
}

std::vector<int> caller_node_cpus() {
    const int cpu = sched_getcpu();
    return cpu < 0 ? std::vector<int>{} : node_cpus(-1, cpu);
}

// NUMA node of the page holding p (get_mempolicy with MPOL_F_NODE | MPOL_F_ADDR), -1 if unknown
static int page_node(const void *p) {
    int node = -1;
    if (syscall(SYS_get_mempolicy, &node, nullptr, 0UL, const_cast<void *>(p), 3UL) != 0) return -1;
    return node;
}

// the node holding most of [p, p + len) (17 sampled pages), -1 if unknown
static int buffer_node(const uint8_t *p, uint64_t len) {
    int votes[64] = {0};
    for (int i = 0; i <= 16; ++i) {
        const int nd = page_node(p + (len ? (len - 1) * i / 16 : 0));
        if (nd >= 0 && nd < 64) ++votes[nd];
    }
    int best = -1;
    for (int nd = 0; nd < 64; ++nd)
        if (votes[nd] && (best < 0 || votes[nd] > votes[best])) best = nd;
    return best;
}

uint64_t env_u64(const char *name, uint64_t dflt) {
    const char *v = opt(name);
    return (v && *v) ? std::strtoull(v, nullptr, 10) : dflt;
}

}  // namespace

uint64_t packed_transfer_min() { return env_u64("GKM_PACK_MIN", 16ull << 20); }

// staging slots of the context (pinned host + device), grown on demand and kept for later calls
static hipError_t xfer_slots(gk_ctx *c, int slots, uint64_t slot_bytes) {
    if (c->xfer_slots >= slots && c->xfer_slot_bytes >= slot_bytes) return hipSuccess;
    xfer_release(c);
    hipError_t e = hipHostMalloc(reinterpret_cast<void **>(&c->xfer_host), (size_t)slots * slot_bytes, hipHostMallocDefault);
    if (e != hipSuccess) return e;
    e = hipMalloc(&c->xfer_dev, (size_t)slots * slot_bytes);
    if (e != hipSuccess) return e;
    if ((e = hipStreamCreateWithFlags(&c->xfer_stream, hipStreamNonBlocking)) != hipSuccess) return e;
    if ((e = hipStreamCreateWithFlags(&c->xfer_raw_stream, hipStreamNonBlocking)) != hipSuccess) return e;
    // per slot: copy landed, slot unpacked; then kRawDepth raw-copy events
    c->xfer_ev.resize(2 * slots + kRawDepth);
    for (auto &ev : c->xfer_ev)
        if ((e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) return e;
    c->xfer_slots = slots;
    c->xfer_slot_bytes = slot_bytes;
    return hipSuccess;
}

void xfer_release(gk_ctx *c) {
    if (c->unpack_stream) {
        hipStreamSynchronize(c->unpack_stream);
        hipStreamDestroy(c->unpack_stream);
        hipEventDestroy(c->unpack_done);
        c->unpack_stream = nullptr;
        c->unpack_done = nullptr;
    }
    if (c->xfer_stream) hipStreamSynchronize(c->xfer_stream);
    if (c->xfer_raw_stream) hipStreamSynchronize(c->xfer_raw_stream);
    for (auto &ev : c->xfer_ev)
        if (ev) hipEventDestroy(ev);
    c->xfer_ev.clear();
    if (c->xfer_stream) hipStreamDestroy(c->xfer_stream);
    if (c->xfer_raw_stream) hipStreamDestroy(c->xfer_raw_stream);
    if (c->xfer_host) hipHostFree(c->xfer_host);
    if (c->xfer_dev) hipFree(c->xfer_dev);
    c->xfer_stream = c->xfer_raw_stream = nullptr;
    c->xfer_host = nullptr;
    c->xfer_dev = nullptr;
    c->xfer_slots = 0;
    c->xfer_slot_bytes = 0;
}

// is p (page-locked) host memory the DMA engines can read directly?
static bool host_pinned(const void *p) {
    hipPointerAttribute_t at{};
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();  // a pageable pointer reports an error on some runtimes: clear it
        return false;
    }
    return at.type == hipMemoryTypeHost;
}

// sba[0, len) -> c->sba.  Chunks are independent (each writes its own range of the resident sba),
// so they are issued in whatever order they are ready:
//   packed  worker threads claim chunks from the front, pack each into a free staging slot and
//           queue it; the caller's thread copies queued slots H2D (xfer_stream) and unpacks them on
//           the context's stream, and recycles a slot once its unpack has run;
//   raw     when the caller's buffer is pinned, the caller's thread also claims chunks from the
//           back and DMAs them as they are, straight into the resident sba (xfer_raw_stream, at
//           most kRawDepth in flight) -- the link carries raw bytes while the CPUs pack, and the
//           two ends meet where packing and copying balance; raw chunks get their alphabet census
//           on the device (launch_alphabet_range).
// *cls_or / *dollars: the census (host part + device part).
//   prefetch (pf, a sort hint: gkm_msd.hip L0Prefetch) the regions of the sort's L0 pass are launched
//           as the in-order prefix of unpacked chunks covers them; a chunk with a raw block (not
//           ACGT) drops the prefetch.
int packed_transfer(gk_ctx *c, const uint8_t *sba, uint64_t len, uint32_t *cls_or, uint64_t *dollars,
                    L0Prefetch *pf) {
    const uint64_t bpc = std::max<uint64_t>(1, std::min<uint64_t>(env_u64("GKM_PACK_BLOCKS", 128), 256));
    const uint64_t chunk = bpc * kXBlock;
    const uint64_t C = (len + chunk - 1) / chunk;
    unsigned hw = std::thread::hardware_concurrency();
    const int T = (int)std::max<uint64_t>(1, std::min<uint64_t>(env_u64("GKM_XFER_THREADS", std::min(16u, hw ? hw : 1u)), C));
    const int S = (int)std::min<uint64_t>(C, std::max(2, 2 * T));
    // raw DMA from the back of a pinned source (GKM_XFER_HYBRID=1): measured slower than packing
    // alone (3.1 Gb from pinned memory: 24.8-27.4 against 21.0-21.6 ms, profiles/r4/xfer_threads_numa.txt)
    // -- the packing is bound by host memory bandwidth, which the DMA reads share
    const bool hybrid = env_u64("GKM_XFER_HYBRID", 0) != 0 && host_pinned(sba);
    if (hybrid && pf) {  // (raw chunks from the back: no in-order prefix to prefetch behind)
        if (int rc = prefetch_finish(c, pf, false)) return rc;
        pf = nullptr;
    }
    // the copy streams write the resident sba and the staging slots outside the context's stream:
    // everything queued before (an earlier sort reading the sba, an earlier transfer's unpacks,
    // which read the slots xfer_slots may free and reallocate) has to be done first
    GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
    GK_TRY_HIP(c, xfer_slots(c, S, kHeaderBytes + chunk + 16));
    if (!c->unpack_stream) {
        int least = 0, greatest = 0;
        GK_TRY_HIP(c, hipDeviceGetStreamPriorityRange(&least, &greatest));
        GK_TRY_HIP(c, hipStreamCreateWithPriority(&c->unpack_stream, hipStreamNonBlocking, greatest));
        GK_TRY_HIP(c, hipEventCreateWithFlags(&c->unpack_done, hipEventDisableTiming));
    }
    hipStream_t us = c->unpack_stream;  // (everything before on c->stream is done: synchronised above)
    // the packed copy of the sequence beside it (c->res_code / res_dol, valid once the transfer is
    // complete: gk_set_sequence); the raw DMA of the hybrid mode skips the unpack, so not there.
    // GKM_NO_RESIDENT_PACK=1: none (the L0 passes pack the bytes per tile)
    c->res_pk = false;
    const bool res = !hybrid && !opt("GKM_NO_RESIDENT_PACK");
    const uint64_t res_words = c->sba_cap / 32;
    if (res) {
        GK_TRY_HIP(c, ensure(reinterpret_cast<void **>(&c->res_code), &c->res_code_cap, 8 * res_words + 64));
        GK_TRY_HIP(c, ensure(reinterpret_cast<void **>(&c->res_dol), &c->res_dol_cap, 4 * res_words + 64));
    }
    hipEvent_t *ev_copy = c->xfer_ev.data(), *ev_done = c->xfer_ev.data() + S;
    hipEvent_t *ev_raw = c->xfer_ev.data() + 2 * S;
    uint32_t *d_census = reinterpret_cast<uint32_t *>(c->scalars + 24);
    if (hybrid) {
        GK_TRY_HIP(c, hipMemsetAsync(d_census, 0, 8, c->stream));
        GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
    }

    std::mutex mu;
    std::condition_variable cv;
    uint64_t front = 0, back = C;            // unclaimed chunks: [front, back)
    std::vector<int> free_slots;             // slots ready to be packed into
    std::vector<std::pair<uint64_t, int>> ready;  // (chunk, slot) packed, not yet issued
    std::vector<uint64_t> used(S, 0);        // bytes of the packed chunk in each slot
    std::vector<char> all_packed(C, 0);      // chunk k had no raw block (prefetch)
    std::vector<char> chunk_issued(C, 0);    // chunk k's unpack is enqueued
    uint64_t prefix = 0;                     // chunks [0, prefix) issued
    bool pf_ok = pf != nullptr;
    int pf_rc = GK_OK;
    bool abort = false;
    for (int i = 0; i < S; ++i) free_slots.push_back(i);
    std::atomic<uint32_t> cls{0};
    std::atomic<uint64_t> dol{0};

    auto worker = [&]() {
        Census cen;
        for (;;) {
            uint64_t k;
            int slot;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return abort || front >= back || !free_slots.empty(); });
                if (abort || front >= back) break;
                k = front++;
                slot = free_slots.back();
                free_slots.pop_back();
            }
            const uint64_t at = k * chunk, m = std::min(chunk, len - at);
            bool whole = false;
            const uint64_t u = pack_chunk(sba + at, m, c->xfer_host + (uint64_t)slot * c->xfer_slot_bytes, cen, &whole);
            _mm_sfence();  // the chunk's streaming stores are globally visible before it is queued
            {
                std::lock_guard<std::mutex> lk(mu);
                used[slot] = u;
                all_packed[k] = whole ? 1 : 0;
                ready.emplace_back(k, slot);
            }
            cv.notify_all();
        }
        cls.fetch_or(cen.cls_or);
        dol.fetch_add(cen.dollars);
    };
    std::vector<std::thread> pool;
    // GKM_XFER_NUMA: 1 = the packing threads on the caller's node, 2 = on the node holding the source
    const uint64_t numa = env_u64("GKM_XFER_NUMA", 0);
    const std::vector<int> near = numa == 1   ? caller_node_cpus()
                                  : numa == 2 ? [&] {
                                        const int nd = buffer_node(sba, len);
                                        return nd < 0 ? std::vector<int>{} : node_cpus(nd, -1);
                                    }()
                                              : std::vector<int>{};
    for (int i = 0; i < T; ++i) {
        pool.emplace_back(worker);
        if (!near.empty()) {  // the packing threads next to the caller (and the sba it allocated)
            cpu_set_t set;
            CPU_ZERO(&set);
            for (int x : near) CPU_SET(x, &set);
            pthread_setaffinity_np(pool.back().native_handle(), sizeof set, &set);
        }
    }

    hipError_t err = hipSuccess;
    std::vector<int> inflight;           // slots issued, unpack not yet known to have run
    std::vector<char> raw_busy(kRawDepth, 0);
    uint64_t issued = 0, raw_chunks = 0;  // chunks handed to the device (packed + raw)
    while (err == hipSuccess && issued < C) {
        bool progress = false;
        std::vector<std::pair<uint64_t, int>> batch;
        {
            std::lock_guard<std::mutex> lk(mu);
            batch.swap(ready);
        }
        for (auto &kr : batch) {  // packed chunks: copy, then unpack on the context's stream
            const uint64_t k = kr.first;
            const int s = kr.second;
            const uint64_t m = std::min(chunk, len - k * chunk);
            uint8_t *ds = c->xfer_dev + (uint64_t)s * c->xfer_slot_bytes;
            err = hipMemcpyAsync(ds, c->xfer_host + (uint64_t)s * c->xfer_slot_bytes, (size_t)used[s],
                                 hipMemcpyHostToDevice, c->xfer_stream);
            if (err == hipSuccess) err = hipEventRecord(ev_copy[s], c->xfer_stream);
            if (err == hipSuccess) err = hipStreamWaitEvent(us, ev_copy[s], 0);
            if (err == hipSuccess) {
                hipLaunchKernelGGL(unpack_chunk_kernel, dim3((unsigned)((m + kXBlock - 1) / kXBlock)), dim3(256), 0,
                                   us, ds, c->sba + k * chunk, m, res ? c->res_code + k * chunk / 32 : nullptr,
                                   res ? c->res_dol + k * chunk / 32 : nullptr);
                err = hipGetLastError();
            }
            if (err == hipSuccess) err = hipEventRecord(ev_done[s], us);
            if (err != hipSuccess) break;
            inflight.push_back(s);
            ++issued;
            progress = true;
            chunk_issued[k] = 1;
        }
        // prefetch: the in-order prefix of enqueued unpacks has grown -- launch the L0 regions it covers
        // (chunks with raw blocks -- '$' separators, N runs, IUPAC letters -- are unpacked on the same
        // stream; the region passes stop k-mers at every non-ACGT byte: a mixed sba's class A)
        if (pf_ok && err == hipSuccess && prefix < C && chunk_issued[prefix]) {
            {
                std::lock_guard<std::mutex> lk(mu);
                for (; prefix < C && chunk_issued[prefix]; ++prefix) {
                }
            }
            if (int rc = prefetch_launch(c, pf, std::min(prefix * chunk, len))) {
                pf_ok = false;
                pf_rc = rc;
                err = hipErrorUnknown;
            }
        }
        // recycle slots whose unpack has run
        for (size_t i = 0; i < inflight.size() && err == hipSuccess;) {
            const hipError_t q = hipEventQuery(ev_done[inflight[i]]);
            if (q == hipSuccess) {
                {
                    std::lock_guard<std::mutex> lk(mu);
                    free_slots.push_back(inflight[i]);
                }
                cv.notify_all();
                inflight[i] = inflight.back();
                inflight.pop_back();
                progress = true;
            } else if (q == hipErrorNotReady) {
                ++i;
            } else {
                err = q;
            }
        }
        // raw chunks from the back while the raw copy queue has room
        for (int r = 0; hybrid && r < kRawDepth && err == hipSuccess; ++r) {
            if (raw_busy[r]) {
                const hipError_t q = hipEventQuery(ev_raw[r]);
                if (q == hipErrorNotReady) continue;
                if (q != hipSuccess) {
                    err = q;
                    break;
                }
                raw_busy[r] = 0;
            }
            uint64_t k;
            {
                std::lock_guard<std::mutex> lk(mu);
                if (front >= back) break;
                k = --back;
            }
            const uint64_t at = k * chunk, m = std::min(chunk, len - at);
            err = hipMemcpyAsync(c->sba + at, sba + at, (size_t)m, hipMemcpyHostToDevice, c->xfer_raw_stream);
            if (err == hipSuccess) err = hipEventRecord(ev_raw[r], c->xfer_raw_stream);
            if (err == hipSuccess) err = hipStreamWaitEvent(c->stream, ev_raw[r], 0);
            if (err == hipSuccess) err = launch_alphabet_range(c, c->sba + at, m, d_census);
            raw_busy[r] = 1;
            ++issued;
            ++raw_chunks;
            progress = true;
        }
        if (!progress && issued < C) {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait_for(lk, std::chrono::microseconds(50), [&] { return !ready.empty(); });
        }
    }
    {
        std::lock_guard<std::mutex> lk(mu);
        if (err != hipSuccess) abort = true;
    }
    cv.notify_all();
    for (auto &th : pool) th.join();
    // the context's stream (the sort's kernels, the census copy) after every unpack
    if (err == hipSuccess) err = hipEventRecord(c->unpack_done, us);
    if (err == hipSuccess) err = hipStreamWaitEvent(c->stream, c->unpack_done, 0);
    if (err != hipSuccess) {
        // an error leaves unpack (and prefetch) kernels in flight that still read the staging slots
        // and write the sba and the packed copy: drain both streams before the slots can be reused
        (void)hipStreamSynchronize(us);
        if (c->pre_stream) (void)hipStreamSynchronize(c->pre_stream);
    }
    // the packed copy's last words -- the sequence's partial last 32 bytes and the '$' pad -- from
    // the unpacked bytes
    if (err == hipSuccess && res) {
        const uint64_t w0 = (len & ~63ull) / 32;  // (from the last partial group of 64: the unpack skips it)
        err = launch_pack2(c->sba + 32 * w0, res_words - w0, c->res_code + w0, c->res_dol + w0, c->stream);
        if (err == hipSuccess) c->res_pk = true;  // (gk_set_sequence keeps it for an ACGT census)
    }
    if (pf) {
        const int rc = prefetch_finish(c, pf, pf_ok && err == hipSuccess && prefix == C);
        if (err == hipSuccess && rc != GK_OK) return rc;
    }
    if (pf_rc != GK_OK) return pf_rc;  // (prefetch_launch's own error; it set the message)
    if (err != hipSuccess) return hip_fail(c, err, "packed sba transfer");
    uint32_t cen[2] = {0, 0};
    if (hybrid && raw_chunks) {  // the device census of the raw chunks (waits for them to land)
        GK_TRY_HIP(c, hipMemcpyAsync(cen, d_census, 8, hipMemcpyDeviceToHost, c->stream));
        GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
    }
    *cls_or = cls.load() | cen[0];
    *dollars = dol.load() + cen[1];
    return GK_OK;
}

}  // namespace gkm

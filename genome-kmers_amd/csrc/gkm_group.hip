// gkm_group.hip -- group pass over the sorted k-mers (gfx950): filters, group boundaries,
// group-size histogram, generator members, unique k-mers + multiplicities.
//
// Restates kmer_info_by_group_generator (kmers.py:523-648) as data-parallel steps:
//   1. valid[i]   = kmer_filter_func(sba, strand, starts[i])          (filters: kmers.py:14-259)
//   2. cidx       = indices of valid k-mers, in order                  (stream compaction)
//   3. head[q]    = q == 0 || compare(prev valid, this, kmer_len) != 0  (kmers.py:597-601)
//   4. gstart     = indices of heads; size[g] = gstart[g+1] - gstart[g]
//   5. hist[min(size, max_bin)] += 1, total += size for min <= size <= max  (kmers.py:454-520)
// A generator "yield" is one of the first yield_first_n members of a qualifying group.
#include <algorithm>
#include <cstdlib>

#include "gkm_internal.h"

namespace gkm {

// ---------------------------------------------------------------------------------------------
// block scan helpers
// ---------------------------------------------------------------------------------------------
template <int NT>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *s_tmp, uint32_t *block_total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t incl = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(incl, off);
        if (lane >= off) incl += y;
    }
    if (lane == 63) s_tmp[wave] = incl;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) {
        const uint32_t x = s_tmp[w];
        pre += (w < wave) ? x : 0u;
        tot += x;
    }
    __syncthreads();
    *block_total = tot;
    return pre + incl - v;
}

// ---------------------------------------------------------------------------------------------
// scans over u8 flags and u32 values; tile = 256 threads x 16 consecutive elements
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void load16_flags(const uint8_t *__restrict__ f, uint64_t n, uint64_t at, uint8_t (&v)[16]) {
    if (at + 16 <= n) {
        uint4 x = *reinterpret_cast<const uint4 *>(f + at);
        const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
    } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = (at + k < n) ? f[at + k] : 0;
    }
}

__global__ __launch_bounds__(kScanThreads) void flag_count_kernel(const uint8_t *__restrict__ f, uint64_t n,
                                                                  uint32_t *__restrict__ tile_sums) {
    __shared__ uint32_t s_tmp[kScanThreads / 64];
    const uint64_t at = (uint64_t)blockIdx.x * kScanTile + threadIdx.x * 16;
    uint8_t v[16];
    load16_flags(f, n, at, v);
    uint32_t cnt = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) cnt += v[k] != 0;
    uint32_t tot;
    block_excl_scan<kScanThreads>(cnt, s_tmp, &tot);
    if (threadIdx.x == 0) tile_sums[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kScanThreads) void u32_count_kernel(const uint32_t *__restrict__ in, uint64_t n,
                                                                 uint32_t *__restrict__ tile_sums) {
    __shared__ uint32_t s_tmp[kScanThreads / 64];
    const uint64_t at = (uint64_t)blockIdx.x * kScanTile + threadIdx.x * 16;
    uint32_t cnt = 0;
    for (int k = 0; k < 16; ++k)
        if (at + k < n) cnt += in[at + k];
    uint32_t tot;
    block_excl_scan<kScanThreads>(cnt, s_tmp, &tot);
    if (threadIdx.x == 0) tile_sums[blockIdx.x] = tot;
}

// exclusive scan of the tile sums in place (one 1024-thread block); grand total -> *total
__global__ __launch_bounds__(1024) void scan_tiles_kernel(uint32_t *__restrict__ sums, uint64_t ntiles,
                                                          uint64_t *__restrict__ total) {
    __shared__ uint32_t s_tmp[16];
    uint64_t carry = 0;
    for (uint64_t b = 0; b < ntiles; b += 1024) {
        const uint64_t i = b + threadIdx.x;
        const uint32_t v = i < ntiles ? sums[i] : 0;
        uint32_t tot;
        const uint32_t ex = block_excl_scan<1024>(v, s_tmp, &tot);
        if (i < ntiles) sums[i] = (uint32_t)(carry + ex);
        carry += tot;
    }
    if (threadIdx.x == 0) *total = carry;
}

// Many tile sums (a 3.1e9-element selection has 757 k): the single-block scan above walks them in
// 740 sequential steps (~0.7 ms); instead chunks of 16384 are scanned in parallel, the chunk
// totals by one block, and the chunk offsets added back.
constexpr int kScanChunk = 16384;  // multiple of 1024 (GKM_TEST_SCAN_CHUNK overrides: tests only)

__global__ __launch_bounds__(1024) void chunk_scan_kernel(uint32_t *__restrict__ sums, uint64_t ntiles, uint32_t chunk,
                                                          uint32_t *__restrict__ chunk_tot) {
    __shared__ uint32_t s_tmp[16];
    const uint64_t b0 = (uint64_t)blockIdx.x * chunk;
    uint32_t carry = 0;
    for (uint32_t j = 0; j < chunk; j += 1024) {
        const uint64_t i = b0 + j + threadIdx.x;
        const uint32_t v = i < ntiles ? sums[i] : 0;
        uint32_t tot;
        const uint32_t ex = block_excl_scan<1024>(v, s_tmp, &tot);
        if (i < ntiles) sums[i] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) chunk_tot[blockIdx.x] = carry;
}

__global__ __launch_bounds__(256) void chunk_add_kernel(uint32_t *__restrict__ sums, uint64_t ntiles, uint32_t chunk,
                                                        const uint32_t *__restrict__ chunk_off) {
    const uint32_t add = chunk_off[blockIdx.x];
    const uint64_t b0 = (uint64_t)blockIdx.x * chunk;
    for (uint32_t j = threadIdx.x; j < chunk; j += 256)
        if (b0 + j < ntiles) sums[b0 + j] += add;
}

// scan chunk: kScanChunk, or (test-only) a smaller multiple of 1024 so that the parity tests reach
// the chunked branch, which otherwise runs only above 65536 tiles (about 268 M elements)
static uint32_t scan_chunk() {
    if (const char *e = opt("GKM_TEST_SCAN_CHUNK")) {
        const int v = std::atoi(e);
        if (v >= 1024) return (uint32_t)(v / 1024 * 1024);
    }
    return kScanChunk;
}

// exclusive scan of ntiles tile sums in place, grand total -> *total (device)
static void scan_tile_sums(gk_ctx *c, uint32_t *sums, uint64_t ntiles, uint64_t *total) {
    const uint32_t chunk = scan_chunk();
    const bool test = chunk != (uint32_t)kScanChunk;
    if (test ? ntiles <= chunk : ntiles <= (uint64_t)4 * kScanChunk) {
        hipLaunchKernelGGL(scan_tiles_kernel, dim3(1), dim3(1024), 0, c->stream, sums, ntiles, total);
        return;
    }
    const uint64_t nch = (ntiles + chunk - 1) / chunk;
    uint32_t *chunk_tot = sums + ntiles + 16;  // ensure_tile_sums leaves room for the chunk totals
    hipLaunchKernelGGL(chunk_scan_kernel, dim3((unsigned)nch), dim3(1024), 0, c->stream, sums, ntiles, chunk, chunk_tot);
    hipLaunchKernelGGL(scan_tiles_kernel, dim3(1), dim3(1024), 0, c->stream, chunk_tot, nch, total);
    hipLaunchKernelGGL(chunk_add_kernel, dim3((unsigned)nch), dim3(256), 0, c->stream, sums, ntiles, chunk, chunk_tot);
}

// Thread t loads the 16 flags of positions 16t..16t+15 (one 16-B load), writes its selected
// positions to LDS after a block scan, and the tile's list is then copied out as one contiguous
// run.  The LDS index is XOR-swizzled within 32-word rows: dense flags (every k-mer distinct)
// would otherwise put 32 lanes of one store on two banks.
__device__ __forceinline__ uint32_t sel_swz(uint32_t o) { return (o & ~31u) | ((o ^ (o >> 5)) & 31u); }

__global__ __launch_bounds__(kScanThreads) void flag_select_kernel(const uint8_t *__restrict__ f, uint64_t n,
                                                                   const uint32_t *__restrict__ tile_off,
                                                                   uint32_t *__restrict__ out) {
    __shared__ uint32_t s_tmp[kScanThreads / 64];
    __shared__ uint32_t s_idx[kScanTile];
    const uint64_t at = (uint64_t)blockIdx.x * kScanTile + threadIdx.x * 16;
    uint8_t v[16];
    load16_flags(f, n, at, v);
    uint32_t cnt = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) cnt += v[k] != 0;
    uint32_t tot;
    uint32_t o = block_excl_scan<kScanThreads>(cnt, s_tmp, &tot);
#pragma unroll
    for (int k = 0; k < 16; ++k)
        if (v[k]) s_idx[sel_swz(o++)] = (uint32_t)(at + k);
    __syncthreads();
    uint32_t *dst = out + tile_off[blockIdx.x];
    for (uint32_t j = threadIdx.x; j < tot; j += kScanThreads) dst[j] = s_idx[sel_swz(j)];
}

// Group starts and multiplicities in one pass (the unique/count output): entry j of a tile also
// gets its count s_idx[j + 1] - s_idx[j]; the tile's last entry needs the next tile's first start
// and is completed by tile_last_count_kernel once every tile has stored its starts.
// A tile's staged heads (s_idx, sel_swz order) to the output at entry `base`: 16-byte groups
// aligned to the output (4 starts and their 4 multiplicities per pair of stores); the groups at the
// tile's edges go per entry, and the tile's last multiplicity is tile_last_count_kernel's.  out and
// out_cnt share their 16-byte phase (checked by the host).
__device__ __forceinline__ void emit_tile_counts(const uint32_t *s_idx, uint32_t tot, uint64_t base,
                                                 uint32_t *__restrict__ out, uint32_t *__restrict__ out_cnt) {
    const uint32_t a0 = (uint32_t)((((uintptr_t)out >> 2) + base) & 3);
    const uint32_t ng = (tot + a0 + 3) >> 2;
    for (uint32_t q = threadIdx.x; q < ng; q += kScanThreads) {
        const int32_t j0 = (int32_t)(4 * q) - (int32_t)a0;
        if (j0 >= 0 && j0 + 4 < (int32_t)tot) {
            uint32_t g[5];
#pragma unroll
            for (int u = 0; u < 5; ++u) g[u] = s_idx[sel_swz(j0 + u)];
            *reinterpret_cast<uint4 *>(out + base + j0) = make_uint4(g[0], g[1], g[2], g[3]);
            *reinterpret_cast<uint4 *>(out_cnt + base + j0) =
                make_uint4(g[1] - g[0], g[2] - g[1], g[3] - g[2], g[4] - g[3]);
        } else {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int32_t j = j0 + u;
                if (j < 0 || j >= (int32_t)tot) continue;
                const uint32_t g0 = s_idx[sel_swz(j)];
                out[base + j] = g0;
                if (j + 1 < (int32_t)tot) out_cnt[base + j] = s_idx[sel_swz(j + 1)] - g0;
            }
        }
    }
}

__global__ __launch_bounds__(kScanThreads) void flag_select_counts_kernel(const uint8_t *__restrict__ f, uint64_t n,
                                                                          const uint32_t *__restrict__ tile_off,
                                                                          uint32_t *__restrict__ out,
                                                                          uint32_t *__restrict__ out_cnt) {
    __shared__ uint32_t s_tmp[kScanThreads / 64];
    __shared__ uint32_t s_idx[kScanTile + 1];
    const uint64_t at = (uint64_t)blockIdx.x * kScanTile + threadIdx.x * 16;
    uint8_t v[16];
    load16_flags(f, n, at, v);
    uint32_t cnt = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) cnt += v[k] != 0;
    uint32_t tot;
    uint32_t o = block_excl_scan<kScanThreads>(cnt, s_tmp, &tot);
#pragma unroll
    for (int k = 0; k < 16; ++k)
        if (v[k]) s_idx[sel_swz(o++)] = (uint32_t)(at + k);
    __syncthreads();
    emit_tile_counts(s_idx, tot, tile_off[blockIdx.x], out, out_cnt);
}

__global__ __launch_bounds__(256) void tile_last_count_kernel(const uint32_t *__restrict__ tile_off, uint64_t ntiles,
                                                              const uint64_t *__restrict__ total,
                                                              const uint32_t *__restrict__ gstart, uint64_t n,
                                                              uint32_t *__restrict__ out_cnt) {
    const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= ntiles) return;
    const uint64_t G = *total;
    const uint64_t end = t + 1 < ntiles ? tile_off[t + 1] : G;
    if (end == tile_off[t]) return;
    const uint64_t g = end - 1;
    const uint64_t next = end < G ? gstart[end] : n;
    out_cnt[g] = (uint32_t)(next - gstart[g]);
}

// a tile's 16-per-thread results staged in LDS (padded: element e at e + e / 16, so the per-thread
// writes of stride 16 and the per-item reads of stride 1 are both conflict-free) and stored by
// consecutive threads: each store instruction covers 1 KB of contiguous output (per-thread runs of
// 16 scattered the stores 64 B apart, 4.4x slower at 1e8 elements)
constexpr int kScanPad = kScanTile + kScanTile / 16;
__device__ __forceinline__ void store_tile_u32(uint32_t *s_o, uint64_t tile0, uint64_t n, uint32_t *__restrict__ out) {
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        const uint32_t e = k * kScanThreads + threadIdx.x;
        if (tile0 + e < n) out[tile0 + e] = s_o[e + e / 16];
    }
}

__global__ __launch_bounds__(kScanThreads) void flag_scan_incl_kernel(const uint8_t *__restrict__ f, uint64_t n,
                                                                      const uint32_t *__restrict__ tile_off,
                                                                      uint32_t *__restrict__ out) {
    __shared__ uint32_t s_tmp[kScanThreads / 64];
    __shared__ uint32_t s_o[kScanPad];
    const uint64_t tile0 = (uint64_t)blockIdx.x * kScanTile;
    const uint64_t at = tile0 + threadIdx.x * 16;
    uint8_t v[16];
    load16_flags(f, n, at, v);
    uint32_t cnt = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) cnt += v[k] != 0;
    uint32_t tot;
    uint32_t o = tile_off[blockIdx.x] + block_excl_scan<kScanThreads>(cnt, s_tmp, &tot);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        o += v[k] != 0;
        s_o[threadIdx.x * 17 + k] = o;
    }
    store_tile_u32(s_o, tile0, n, out);
}

__global__ __launch_bounds__(kScanThreads) void u32_scan_apply_kernel(const uint32_t *__restrict__ in, uint64_t n,
                                                                      const uint32_t *__restrict__ tile_off,
                                                                      uint32_t *__restrict__ out) {
    __shared__ uint32_t s_tmp[kScanThreads / 64];
    __shared__ uint32_t s_o[kScanPad];
    const uint64_t tile0 = (uint64_t)blockIdx.x * kScanTile;
    // coalesced loads into the padded layout, then each thread's run of 16
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        const uint32_t e = k * kScanThreads + threadIdx.x;
        s_o[e + e / 16] = tile0 + e < n ? in[tile0 + e] : 0;
    }
    __syncthreads();
    uint32_t v[16];
    uint32_t cnt = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        v[k] = s_o[threadIdx.x * 17 + k];
        cnt += v[k];
    }
    uint32_t tot;
    uint32_t o = tile_off[blockIdx.x] + block_excl_scan<kScanThreads>(cnt, s_tmp, &tot);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        s_o[threadIdx.x * 17 + k] = o;
        o += v[k];
    }
    store_tile_u32(s_o, tile0, n, out);
}

static hipError_t ensure_tile_sums(gk_ctx *c, uint64_t ntiles) {
    // + the chunk totals of scan_tile_sums
    return ensure(reinterpret_cast<void **>(&c->tile_sums), &c->tile_sums_cap,
                  4 * (ntiles + 16 + ntiles / 1024 + 16));
}

static hipError_t read_total(gk_ctx *c, uint64_t *count) { return read_back(c, c->scalars, 8, count); }

hipError_t select_flags(gk_ctx *c, const uint8_t *flags, uint64_t n, uint32_t *out_idx, uint64_t *count) {
    const uint64_t ntiles = (n + kScanTile - 1) / kScanTile;
    if (n == 0) { *count = 0; return hipSuccess; }
    hipError_t e = ensure_tile_sums(c, ntiles);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(flag_count_kernel, dim3((unsigned)ntiles), dim3(kScanThreads), 0, c->stream, flags, n,
                       c->tile_sums);
    scan_tile_sums(c, c->tile_sums, ntiles, c->scalars);
    hipLaunchKernelGGL(flag_select_kernel, dim3((unsigned)ntiles), dim3(kScanThreads), 0, c->stream, flags, n,
                       c->tile_sums, out_idx);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    return read_total(c, count);
}

// select_flags + the multiplicity of every selected entry (distance to the next one, or to n).
// Two passes over the flags (count, select) measured faster at C3 than a one-pass decoupled
// look-back (5.3 vs 6.1 ms: the look-back chain across XCDs costs more than re-reading 1 byte/k-mer)
hipError_t select_flags_counts(gk_ctx *c, const uint8_t *flags, uint64_t n, uint32_t *out_idx, uint32_t *out_cnt,
                               uint64_t *count) {
    const uint64_t ntiles = (n + kScanTile - 1) / kScanTile;
    if (n == 0) { *count = 0; return hipSuccess; }
    // emit_tile_counts' 16-byte groups: both outputs 4-byte aligned, in the same 16-byte phase
    if (((uintptr_t)out_idx & 3) || (((uintptr_t)out_idx ^ (uintptr_t)out_cnt) & 15)) return hipErrorInvalidValue;
    hipError_t e = ensure_tile_sums(c, ntiles);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(flag_count_kernel, dim3((unsigned)ntiles), dim3(kScanThreads), 0, c->stream, flags, n,
                       c->tile_sums);
    scan_tile_sums(c, c->tile_sums, ntiles, c->scalars);
    hipLaunchKernelGGL(flag_select_counts_kernel, dim3((unsigned)ntiles), dim3(kScanThreads), 0, c->stream, flags, n,
                       c->tile_sums, out_idx, out_cnt);
    hipLaunchKernelGGL(tile_last_count_kernel, dim3((unsigned)((ntiles + 255) / 256)), dim3(256), 0, c->stream,
                       c->tile_sums, ntiles, c->scalars, out_idx, n, out_cnt);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    return read_total(c, count);
}

hipError_t scan_flags_inclusive(gk_ctx *c, const uint8_t *flags, uint64_t n, uint32_t *out) {
    const uint64_t ntiles = (n + kScanTile - 1) / kScanTile;
    if (n == 0) return hipSuccess;
    hipError_t e = ensure_tile_sums(c, ntiles);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(flag_count_kernel, dim3((unsigned)ntiles), dim3(kScanThreads), 0, c->stream, flags, n,
                       c->tile_sums);
    scan_tile_sums(c, c->tile_sums, ntiles, c->scalars);
    hipLaunchKernelGGL(flag_scan_incl_kernel, dim3((unsigned)ntiles), dim3(kScanThreads), 0, c->stream, flags, n,
                       c->tile_sums, out);
    return hipGetLastError();
}

// the exclusive scan's launches; its total is left in c->scalars[0] (n > 0)
static hipError_t scan_u32_exclusive_launch(gk_ctx *c, const uint32_t *in, uint64_t n, uint32_t *out) {
    const uint64_t ntiles = (n + kScanTile - 1) / kScanTile;
    hipError_t e = ensure_tile_sums(c, ntiles);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(u32_count_kernel, dim3((unsigned)ntiles), dim3(kScanThreads), 0, c->stream, in, n,
                       c->tile_sums);
    scan_tile_sums(c, c->tile_sums, ntiles, c->scalars);
    hipLaunchKernelGGL(u32_scan_apply_kernel, dim3((unsigned)ntiles), dim3(kScanThreads), 0, c->stream, in, n,
                       c->tile_sums, out);
    return hipGetLastError();
}

static hipError_t scan_u32_exclusive(gk_ctx *c, const uint32_t *in, uint64_t n, uint32_t *out, uint64_t *total) {
    if (n == 0) { *total = 0; return hipSuccess; }
    hipError_t e = scan_u32_exclusive_launch(c, in, n, out);
    if (e != hipSuccess) return e;
    return read_total(c, total);
}

// ---------------------------------------------------------------------------------------------
// built-in filters on the device (kmers.py:14-259); returns 1 pass, 0 fail, -code raised
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ int dev_filter(const uint8_t *__restrict__ sba, uint64_t L, int kind, int64_t p0,
                                          int64_t p1, int64_t p2, uint64_t idx, const uint8_t *__restrict__ mask,
                                          uint64_t i) {
    switch (kind) {
    case GK_FILTER_KEEP_ALL:
        return 1;
    case GK_FILTER_LENGTH:  // kmer_has_required_len (kmers.py:262-282)
        for (int64_t t = 0; t < p0; ++t)
            if (idx + t >= L || sba[idx + t] == GK_DOLLAR) return 0;
        return 1;
    case GK_FILTER_HOMOPOLYMER: {  // kmers.py:63-98
        const int64_t maxh = p0, k = p1;
        if ((int64_t)idx + k - 1 >= (int64_t)L) return -GK_FERR_HOMO_LEN;
        if (k < maxh) return 1;
        int64_t h = 1;
        for (int64_t t = 1; t < k; ++t) {
            const uint8_t b = sba[idx + t], pb = sba[idx + t - 1];
            if (b == GK_DOLLAR) return -GK_FERR_HOMO_LEN;
            if (b == pb) {
                if (++h > maxh) return 0;
            } else {
                h = 1;
            }
        }
        return 1;
    }
    case GK_FILTER_GC: {  // kmers.py:150-190
        const int64_t minc = p0, maxc = p1, k = p2;
        if (maxc < minc) return 0;
        int64_t gc = 0;
        for (int64_t t = 0; t < k; ++t) {
            if (idx + t >= L) return -GK_FERR_GC_OOB;
            const uint8_t b = sba[idx + t];
            if (b == GK_DOLLAR) return -GK_FERR_GC_LEN;
            if (b == 'G' || b == 'C') {
                if (++gc > maxc) return 0;
            }
        }
        return (minc <= gc && gc <= maxc) ? 1 : 0;
    }
    case GK_FILTER_NO_AMBIGUOUS: {  // kmers.py:209-227
        const int64_t k = p0;
        if ((int64_t)idx + k > (int64_t)L) return -GK_FERR_AMBIG_LEN;
        for (int64_t t = 0; t < k; ++t) {
            const uint8_t b = sba[idx + t];
            if (b == GK_DOLLAR) return -GK_FERR_AMBIG_SEG;
            if (b != 'A' && b != 'T' && b != 'G' && b != 'C') return 0;
        }
        return 1;
    }
    case GK_FILTER_CRISPR_NGG:  // kmers.py:232-259
        if (idx + 23 > L) return -GK_FERR_CRISPR_LEN;
        return (sba[idx + 21] == 'G' && sba[idx + 22] == 'G') ? 1 : 0;
    case GK_FILTER_MASK:
        return mask[i] ? 1 : 0;
    }
    return 0;
}

__global__ __launch_bounds__(256) void filter_flags_kernel(const uint8_t *__restrict__ sba, uint64_t L,
                                                           const uint32_t *__restrict__ starts, uint64_t n, int kind,
                                                           int64_t p0, int64_t p1, int64_t p2,
                                                           const uint8_t *__restrict__ mask, uint8_t *__restrict__ flags,
                                                           unsigned long long *__restrict__ err) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const int r = dev_filter(sba, L, kind, p0, p1, p2, starts[i], mask, i);
        flags[i] = r > 0;
        if (r < 0) atomicMin(err, ((unsigned long long)i << 8) | (unsigned long long)(-r));
    }
}

// The built-in filters depend on the sba window at a start only, so they are evaluated once per
// POSITION, streaming the sba (neighbouring threads read overlapping windows from the caches), into
// 2 bits per position: word w covers positions 32 w .. 32 w + 31, bit j = passes, bit 32 + j =
// raises.  The sorted-order flags then gather one bit pair per k-mer from L / 4 bytes (a GRCh38-size
// table mostly held by the Infinity Cache) instead of a random ~31-byte window per k-mer: ~100x
// fewer HBM line fetches.  A raising k-mer re-runs dev_filter for its code, so the error (the
// lowest raising sorted index) is the one filter_flags_kernel reports.
__global__ __launch_bounds__(256) void filter_pos_kernel(const uint8_t *__restrict__ sba, uint64_t L, int kind,
                                                         int64_t p0, int64_t p1, int64_t p2,
                                                         uint64_t *__restrict__ words) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t step = (uint64_t)gridDim.x * 256;
    for (uint64_t base = blockIdx.x * 256ull + (threadIdx.x & ~63u); base < L; base += step) {  // wave-uniform
        const uint64_t p = base + lane;
        const int r = p < L ? dev_filter(sba, L, kind, p0, p1, p2, p, nullptr, 0) : 0;
        const uint64_t pass = __ballot(r > 0), raise = __ballot(r < 0);
        if (lane < 2) {
            const uint32_t sh = 32 * lane;
            words[(base >> 5) + lane] = ((pass >> sh) & 0xFFFFFFFFull) | (((raise >> sh) & 0xFFFFFFFFull) << 32);
        }
    }
}

__global__ __launch_bounds__(256) void filter_gather_kernel(const uint64_t *__restrict__ words,
                                                            const uint32_t *__restrict__ starts, uint64_t n,
                                                            const uint8_t *__restrict__ sba, uint64_t L, int kind,
                                                            int64_t p0, int64_t p1, int64_t p2,
                                                            uint8_t *__restrict__ flags,
                                                            unsigned long long *__restrict__ err) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t s = starts[i];
        const uint64_t w = words[s >> 5];
        const uint32_t b = s & 31;
        flags[i] = (uint8_t)((w >> b) & 1);
        if ((w >> (32 + b)) & 1) {
            const int r = dev_filter(sba, L, kind, p0, p1, p2, s, nullptr, i);
            atomicMin(err, ((unsigned long long)i << 8) | (unsigned long long)(-r));
        }
    }
}

// ---------------------------------------------------------------------------------------------
// group heads: q == 0 || k-mer(q-1) != k-mer(q) under compare_sba_kmers_lexicographically(kmer_len)
// ---------------------------------------------------------------------------------------------
struct KeyMasks {
    uint64_t m[kMaxWords];
};

// byte compare (kmers.py:306-397); returns true if equal; kmer_len < 0 = None
__device__ __forceinline__ bool sba_equal(const uint8_t *__restrict__ sba, uint64_t a, uint64_t b, int64_t kmer_len) {
    for (int64_t t = 0;; ++t) {
        const uint8_t x = sba[a + t], y = sba[b + t];  // pad after L reads '$'
        const bool oa = x == GK_DOLLAR, ob = y == GK_DOLLAR;
        if (oa || ob) return oa && ob;
        if (x != y) return false;
        if (kmer_len >= 0 && t == kmer_len - 1) return true;
    }
}

template <int MODE, int W>  // MODE 0: masked key compare, 1: sba byte compare
__global__ __launch_bounds__(256) void head_flags_kernel(const uint8_t *__restrict__ sba,
                                                         const uint32_t *__restrict__ starts,
                                                         const uint64_t *__restrict__ keys, uint64_t nkeys,
                                                         const uint32_t *__restrict__ cidx, uint64_t count,
                                                         int64_t kmer_len, KeyMasks km, uint8_t *__restrict__ head) {
    for (uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; q < count;
         q += (uint64_t)gridDim.x * blockDim.x) {
        if (q == 0) {
            head[q] = 1;
            continue;
        }
        const uint64_t i = cidx ? cidx[q] : q;
        const uint64_t h = cidx ? cidx[q - 1] : q - 1;
        bool eq;
        if (MODE == 0) {
            eq = true;
#pragma unroll
            for (int w = 0; w < W; ++w) eq &= ((keys[(uint64_t)w * nkeys + i] ^ keys[(uint64_t)w * nkeys + h]) & km.m[w]) == 0;
        } else {
            eq = sba_equal(sba, starts[h], starts[i], kmer_len);
        }
        head[q] = !eq;
    }
}

// ---------------------------------------------------------------------------------------------
// group sizes -> histogram / totals / generator members
// ---------------------------------------------------------------------------------------------
constexpr int kLdsBins = 2048;

__device__ __forceinline__ uint64_t group_size(const uint32_t *__restrict__ gstart, uint64_t G, uint64_t count,
                                               uint64_t g) {
    return (g + 1 < G ? (uint64_t)gstart[g + 1] : count) - gstart[g];
}

__global__ __launch_bounds__(256) void group_hist_kernel(const uint32_t *__restrict__ gstart, uint64_t G,
                                                         uint64_t count, int64_t min_g, int64_t max_g, int64_t max_bin,
                                                         unsigned long long *__restrict__ hist,
                                                         unsigned long long *__restrict__ total) {
    __shared__ uint32_t s_hist[kLdsBins];
    __shared__ unsigned long long s_total;
    const int64_t lds_bins = max_bin + 1 < kLdsBins ? max_bin + 1 : kLdsBins;
    for (int i = threadIdx.x; i < lds_bins; i += 256) s_hist[i] = 0;
    if (threadIdx.x == 0) s_total = 0;
    __syncthreads();
    unsigned long long my_total = 0;
    for (uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; g < G; g += (uint64_t)gridDim.x * blockDim.x) {
        const int64_t size = (int64_t)group_size(gstart, G, count, g);
        if (size < min_g || (max_g >= 0 && size > max_g)) continue;
        const int64_t bin = size < max_bin ? size : max_bin;
        if (bin < lds_bins) atomicAdd(&s_hist[bin], 1u);
        else atomicAdd(&hist[bin], 1ull);
        my_total += (unsigned long long)size;
    }
    for (int off = 32; off > 0; off >>= 1) my_total += __shfl_xor(my_total, off);
    if ((threadIdx.x & 63) == 0 && my_total) atomicAdd(&s_total, my_total);
    __syncthreads();
    for (int i = threadIdx.x; i < lds_bins; i += 256)
        if (s_hist[i]) atomicAdd(&hist[i], (unsigned long long)s_hist[i]);
    if (threadIdx.x == 0 && s_total) atomicAdd(total, s_total);
}

__global__ __launch_bounds__(256) void group_yield_count_kernel(const uint32_t *__restrict__ gstart, uint64_t G,
                                                                uint64_t count, int64_t min_g, int64_t max_g,
                                                                int64_t yfn, uint32_t *__restrict__ m) {
    for (uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; g < G; g += (uint64_t)gridDim.x * blockDim.x) {
        const int64_t size = (int64_t)group_size(gstart, G, count, g);
        const bool ok = size >= min_g && (max_g < 0 || size <= max_g);
        m[g] = ok ? (uint32_t)(yfn < 0 ? size : (size < yfn ? size : yfn)) : 0u;
    }
}

__global__ __launch_bounds__(256) void group_yield_write_kernel(const uint32_t *__restrict__ gstart, uint64_t G,
                                                                uint64_t count, const uint32_t *__restrict__ m,
                                                                const uint32_t *__restrict__ off,
                                                                const uint32_t *__restrict__ cidx,
                                                                uint64_t *__restrict__ out_num,
                                                                uint32_t *__restrict__ out_y,
                                                                uint32_t *__restrict__ out_t) {
    for (uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; g < G; g += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t mg = m[g];
        if (!mg) continue;
        const uint32_t size = (uint32_t)group_size(gstart, G, count, g);
        const uint64_t o = off[g];
        for (uint32_t r = 0; r < mg; ++r) {
            const uint64_t q = (uint64_t)gstart[g] + r;
            out_num[o + r] = cidx ? cidx[q] : q;
            out_y[o + r] = mg;
            out_t[o + r] = size;
        }
    }
}

// group heads of the valid k-mers from a host head mask (GK_GROUPS_FROM_HEADS): head of valid
// k-mer q = the mask at its position; the first valid k-mer starts group 0
__global__ __launch_bounds__(256) void heads_from_mask_kernel(const uint8_t *__restrict__ hmask,
                                                              const uint32_t *__restrict__ cidx, uint64_t cnt,
                                                              uint8_t *__restrict__ out) {
    for (uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; q < cnt; q += (uint64_t)gridDim.x * blockDim.x)
        out[q] = q == 0 ? 1 : (hmask[cidx ? cidx[q] : q] != 0);
}

__global__ __launch_bounds__(256) void unique_counts_kernel(const uint32_t *__restrict__ gstart, uint64_t G,
                                                            uint64_t count, uint32_t *__restrict__ counts) {
    for (uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; g < G; g += (uint64_t)gridDim.x * blockDim.x)
        counts[g] = (uint32_t)group_size(gstart, G, count, g);
}

// ---------------------------------------------------------------------------------------------
// host drivers
// ---------------------------------------------------------------------------------------------
static int grid_for(uint64_t n, int cap = 8192) {
    uint64_t g = (n + 255) / 256;
    if (g < 1) g = 1;
    return (int)std::min<uint64_t>(g, (uint64_t)cap);
}

}  // namespace gkm

using namespace gkm;

// Shared front half of gk_group_hist / gk_group_members: filter, compact, heads, group starts.
// On success: *cidx_out (nullptr = identity), *count (valid k-mers), *G, group starts in c->idx_b.
static int group_front(gk_ctx *c, int is_sorted, int64_t kmer_len, const gk_filter *filter, const uint32_t **cidx_out,
                       uint64_t *count, uint64_t *G, int32_t *err_code, uint64_t *err_idx) {
    if (err_code) *err_code = 0;
    if (!c->have_starts) return fail(c, GK_E_STATE, "no k-mers: call gk_enumerate first");
    c->unique_valid = false;  // idx_b (the unique output's group starts) is rewritten below
    if (int rc = materialize_starts(c)) return rc;
    const uint64_t n = c->n;
    const uint32_t *starts = c->vals[c->cur];
    GK_TRY_HIP(c, ensure(reinterpret_cast<void **>(&c->flags), &c->flags_cap, n + 64));
    GK_TRY_HIP(c, ensure(reinterpret_cast<void **>(&c->idx_a), &c->idx_cap, 4 * (n + 64)));
    GK_TRY_HIP(c, ensure(reinterpret_cast<void **>(&c->idx_b), &c->idx_b_cap, 4 * (n + 64)));
    const int kind = filter ? filter->kind : GK_FILTER_KEEP_ALL;
    if (kind == GK_FILTER_MASK && c->mask_n != n) return fail(c, GK_E_ARG, "filter mask length differs from the k-mer count");
    if (kind < 0 || kind > GK_FILTER_MASK) return fail(c, GK_E_ARG, "unknown filter kind");

    // 1-2. filter + compaction
    const uint32_t *cidx = nullptr;
    uint64_t cnt = n;
    if (kind != GK_FILTER_KEEP_ALL) {
        unsigned long long init = ~0ull;
        GK_TRY_HIP(c, hipMemcpyAsync(c->scalars + 1, &init, 8, hipMemcpyHostToDevice, c->stream));
        int slot;
        timer_begin(c, "filter", &slot);
        // per position, then gathered (filter_pos_kernel); a mask is per sorted index, and
        // GKM_FILTER_PER_KMER=1 (A/B) evaluates every k-mer's window in sorted order
        // The per-position pass costs O(sba_len) whatever n is: used when the k-mers are a sizeable
        // share of the positions (a full enumeration), not for a small user-assigned start subset
        static const bool per_kmer = opt("GKM_FILTER_PER_KMER") != nullptr;
        if (kind != GK_FILTER_MASK && !per_kmer && c->sba_len > 0 && n * 8 >= c->sba_len) {
            uint64_t *words;
            GK_TRY_HIP(c, scratch(c, "filter_pos", (c->sba_len + 63) / 64 * 2, &words));
            hipLaunchKernelGGL(filter_pos_kernel, dim3(grid_for((c->sba_len + 255) / 256 * 256, 16384)), dim3(256), 0,
                               c->stream, c->sba, c->sba_len, kind, filter->p0, filter->p1, filter->p2, words);
            hipLaunchKernelGGL(filter_gather_kernel, dim3(grid_for(n)), dim3(256), 0, c->stream, words, starts, n,
                               c->sba, c->sba_len, kind, filter->p0, filter->p1, filter->p2, c->flags,
                               reinterpret_cast<unsigned long long *>(c->scalars + 1));
        } else {
            hipLaunchKernelGGL(filter_flags_kernel, dim3(grid_for(n)), dim3(256), 0, c->stream, c->sba, c->sba_len,
                               starts, n, kind, filter->p0, filter->p1, filter->p2, c->mask, c->flags,
                               reinterpret_cast<unsigned long long *>(c->scalars + 1));
        }
        GK_TRY_HIP(c, hipGetLastError());
        timer_end(c, slot);
        unsigned long long err = 0;
        GK_TRY_HIP(c, hipMemcpyAsync(&err, c->scalars + 1, 8, hipMemcpyDeviceToHost, c->stream));
        GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
        if (err != ~0ull) {
            const uint64_t i = err >> 8;
            uint32_t s = 0;
            GK_TRY_HIP(c, hipMemcpy(&s, starts + i, 4, hipMemcpyDeviceToHost));
            if (err_code) *err_code = (int32_t)(err & 0xFF);
            if (err_idx) *err_idx = s;
            return fail(c, GK_E_FILTER, "k-mer filter raised");
        }
        GK_TRY_HIP(c, select_flags(c, c->flags, n, c->idx_a, &cnt));
        cidx = c->idx_a;
    }
    *cidx_out = cidx;
    *count = cnt;
    if (cnt == 0) {
        *G = 0;
        return GK_OK;
    }

    // groups a caller's comparison decided (a custom kmer_comparison_func)
    if (is_sorted == GK_GROUPS_FROM_HEADS) {
        if (c->hmask_n != n) return fail(c, GK_E_ARG, "group head mask length differs from the k-mer count");
        hipLaunchKernelGGL(heads_from_mask_kernel, dim3(grid_for(cnt)), dim3(256), 0, c->stream, c->hmask, cidx, cnt,
                           c->flags);
        GK_TRY_HIP(c, hipGetLastError());
        uint64_t g = 0;
        GK_TRY_HIP(c, select_flags(c, c->flags, cnt, c->idx_b, &g));
        *G = g;
        return GK_OK;
    }
    // canonical k-mers have no prefixes: groups exist at the sort length only
    if (is_sorted && c->canonical && (kmer_len < 0 || (uint64_t)kmer_len != c->sort_len))
        return fail(c, GK_E_UNSUPPORTED, "canonical k-mers are grouped at kmer_len == the sort length only");

    // 3. heads
    const uint8_t *heads = c->flags;
    if (is_sorted && kind == GK_FILTER_KEEP_ALL && c->heads_valid && c->keys_valid && !c->keys_are_ranks &&
        c->spec.lenbits == 0 && kmer_len == c->spec.symbols) {
        heads = c->heads;  // full-key heads written by the MSD sort (gkm_msd.hip)
    } else if (!is_sorted) {
        // compare_sba_kmers_always_less_than: every valid k-mer starts a group (kmers.py:295-303, 957-960)
        GK_TRY_HIP(c, hipMemsetAsync(c->flags, 1, cnt, c->stream));
    } else {
        // decide whether the encoded keys decide equality at kmer_len
        const KeySpec &ks = c->spec;
        bool use_keys = false;
        KeyMasks km{};
        if (c->keys_valid && !c->keys_are_ranks && kmer_len >= 1 && kmer_len <= ks.symbols &&
            (ks.lenbits == 0 || kmer_len == ks.symbols)) {
            // compare the top kmer_len symbols (plus the length field when it is the full key)
            const int top = ks.total_bits;
            const int lowest = (kmer_len == ks.symbols) ? 0 : (top - (int)kmer_len * ks.bits);
            for (int w = 0; w < ks.words; ++w) {
                const int lo = (ks.words - 1 - w) * 64;  // bit index of word w's bit 0
                uint64_t m = 0;
                for (int b = 0; b < 64; ++b) {
                    const int bit = lo + b;
                    if (bit >= lowest && bit < top) m |= 1ull << b;
                }
                km.m[w] = m;
            }
            use_keys = true;
        } else if (c->keys_valid && c->keys_are_ranks && ((kmer_len < 0 && c->sort_len == 0) ||
                                                          (kmer_len >= 0 && (uint64_t)kmer_len == c->sort_len))) {
            for (int w = 0; w < ks.words; ++w) km.m[w] = ~0ull;
            use_keys = true;
        }
        if (use_keys)
            if (int rc = ensure_keys(c)) return rc;
        int slot;
        timer_begin(c, "group_heads", &slot);
        const uint64_t *keys = c->keys[c->cur];
        if (use_keys) {
            switch (ks.words) {
            case 1: hipLaunchKernelGGL((head_flags_kernel<0, 1>), dim3(grid_for(cnt)), dim3(256), 0, c->stream, c->sba, starts, keys, n, cidx, cnt, kmer_len, km, c->flags); break;
            case 2: hipLaunchKernelGGL((head_flags_kernel<0, 2>), dim3(grid_for(cnt)), dim3(256), 0, c->stream, c->sba, starts, keys, n, cidx, cnt, kmer_len, km, c->flags); break;
            case 3: hipLaunchKernelGGL((head_flags_kernel<0, 3>), dim3(grid_for(cnt)), dim3(256), 0, c->stream, c->sba, starts, keys, n, cidx, cnt, kmer_len, km, c->flags); break;
            default: hipLaunchKernelGGL((head_flags_kernel<0, 4>), dim3(grid_for(cnt)), dim3(256), 0, c->stream, c->sba, starts, keys, n, cidx, cnt, kmer_len, km, c->flags); break;
            }
        } else {
            hipLaunchKernelGGL((head_flags_kernel<1, 1>), dim3(grid_for(cnt)), dim3(256), 0, c->stream, c->sba, starts,
                               keys, n, cidx, cnt, kmer_len, km, c->flags);
        }
        GK_TRY_HIP(c, hipGetLastError());
        timer_end(c, slot);
    }
    // 4. group starts
    uint64_t g = 0;
    GK_TRY_HIP(c, select_flags(c, heads, cnt, c->idx_b, &g));
    *G = g;
    return GK_OK;
}

extern "C" int gk_group_hist(gk_ctx *c, int is_sorted, int64_t kmer_len, const gk_filter *filter,
                             int64_t min_group_size, int64_t max_group_size, int64_t max_counts_bin, int64_t *hist,
                             int64_t *total, int32_t *err_code, uint64_t *err_idx) {
    if (!c) return GK_E_ARG;
    pre_drop(c);  // (the k-mer buffers: a prefetched L0 does not survive)
    if (max_counts_bin <= 0) return fail(c, GK_E_ARG, "max_counts_bin must be >= 1");
    if (min_group_size < 1) return fail(c, GK_E_ARG, "min_group_size must be >= 1");
    const uint32_t *cidx;
    uint64_t count, G;
    int rc = group_front(c, is_sorted, kmer_len, filter, &cidx, &count, &G, err_code, err_idx);
    if (rc != GK_OK) return rc;
    const uint64_t bins = (uint64_t)max_counts_bin + 1;
    GK_TRY_HIP(c, ensure(reinterpret_cast<void **>(&c->dhist), &c->dhist_cap, 8 * bins));
    GK_TRY_HIP(c, hipMemsetAsync(c->dhist, 0, 8 * bins, c->stream));
    GK_TRY_HIP(c, hipMemsetAsync(c->scalars + 2, 0, 8, c->stream));
    if (G > 0) {
        int slot;
        timer_begin(c, "group_hist", &slot);
        hipLaunchKernelGGL(group_hist_kernel, dim3(grid_for(G, 4096)), dim3(256), 0, c->stream, c->idx_b, G, count,
                           min_group_size, max_group_size, max_counts_bin,
                           reinterpret_cast<unsigned long long *>(c->dhist),
                           reinterpret_cast<unsigned long long *>(c->scalars + 2));
        GK_TRY_HIP(c, hipGetLastError());
        timer_end(c, slot);
    }
    if (hist) GK_TRY_HIP(c, hipMemcpyAsync(hist, c->dhist, 8 * bins, hipMemcpyDeviceToHost, c->stream));
    uint64_t tot = 0;
    GK_TRY_HIP(c, hipMemcpyAsync(&tot, c->scalars + 2, 8, hipMemcpyDeviceToHost, c->stream));
    GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
    if (total) *total = (int64_t)tot;
    return GK_OK;
}

extern "C" int gk_group_members(gk_ctx *c, int is_sorted, int64_t kmer_len, const gk_filter *filter,
                                int64_t min_group_size, int64_t max_group_size, int64_t yield_first_n,
                                uint64_t *kmer_num, uint32_t *size_yielded, uint32_t *size_total, uint64_t capacity,
                                uint64_t *n_out, int32_t *err_code, uint64_t *err_idx) {
    if (!c) return GK_E_ARG;
    pre_drop(c);  // (the k-mer buffers: a prefetched L0 does not survive)
    if (min_group_size < 1) return fail(c, GK_E_ARG, "min_group_size must be >= 1");
    const uint32_t *cidx;
    uint64_t count, G;
    int rc = group_front(c, is_sorted, kmer_len, filter, &cidx, &count, &G, err_code, err_idx);
    if (rc != GK_OK) return rc;
    if (G == 0) {
        if (n_out) *n_out = 0;
        return GK_OK;
    }
    // per-group yield counts and their offsets
    GK_TRY_HIP(c, ensure(reinterpret_cast<void **>(&c->ym), &c->ym_cap, 4 * (G + 16)));
    GK_TRY_HIP(c, ensure(reinterpret_cast<void **>(&c->yoff), &c->yoff_cap, 4 * (G + 16)));
    hipLaunchKernelGGL(group_yield_count_kernel, dim3(grid_for(G)), dim3(256), 0, c->stream, c->idx_b, G, count,
                       min_group_size, max_group_size, yield_first_n, c->ym);
    GK_TRY_HIP(c, hipGetLastError());
    uint64_t M = 0;
    GK_TRY_HIP(c, scan_u32_exclusive(c, c->ym, G, c->yoff, &M));
    if (kmer_num && M > 0) {
        if (capacity < M) return fail(c, GK_E_ARG, "capacity smaller than the number of yields");
        GK_TRY_HIP(c, ensure(reinterpret_cast<void **>(&c->onum), &c->onum_cap, 8 * M));
        GK_TRY_HIP(c, ensure(reinterpret_cast<void **>(&c->oy), &c->oy_cap, 4 * M));
        GK_TRY_HIP(c, ensure(reinterpret_cast<void **>(&c->ot), &c->ot_cap, 4 * M));
        hipLaunchKernelGGL(group_yield_write_kernel, dim3(grid_for(G)), dim3(256), 0, c->stream, c->idx_b, G, count,
                           c->ym, c->yoff, cidx, c->onum, c->oy, c->ot);
        GK_TRY_HIP(c, hipGetLastError());
        GK_TRY_HIP(c, hipMemcpyAsync(kmer_num, c->onum, 8 * M, hipMemcpyDeviceToHost, c->stream));
        if (size_yielded) GK_TRY_HIP(c, hipMemcpyAsync(size_yielded, c->oy, 4 * M, hipMemcpyDeviceToHost, c->stream));
        if (size_total) GK_TRY_HIP(c, hipMemcpyAsync(size_total, c->ot, 4 * M, hipMemcpyDeviceToHost, c->stream));
        GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
    }
    if (n_out) *n_out = M;
    return GK_OK;
}

// The unique/count output (sorted k-mers -> distinct k-mers + multiplicities), resident in HBM:
// group starts in idx_b (u32, index of each distinct k-mer's first sorted element) and counts in
// ucount (u32); with the sorted keys (keys[cur]) and starts (vals[cur]) this is the full product.
extern "C" int gk_unique_counts(gk_ctx *c, uint64_t *n_unique) {
    if (!c) return GK_E_ARG;
    pre_drop(c);  // (the k-mer buffers: a prefetched L0 does not survive)
    if (!c->sorted || !c->keys_valid) return fail(c, GK_E_STATE, "unique counts need a sorted k-mer set");
    const int64_t kl = c->sort_len == 0 ? -1 : (int64_t)c->sort_len;
    uint64_t G = 0;
    if (c->heads_valid && !c->keys_are_ranks && c->spec.lenbits == 0 && kl == c->spec.symbols) {
        // heads written by the MSD sort: group starts and counts in one selection pass
        if (int rc = materialize_starts(c)) return rc;
        GK_TRY_HIP(c, ensure(reinterpret_cast<void **>(&c->idx_b), &c->idx_b_cap, 4 * (c->n + 64)));
        GK_TRY_HIP(c, ensure(reinterpret_cast<void **>(&c->ucount), &c->ucount_cap, 4 * (c->n + 64)));
        c->unique_valid = false;
        int slot;
        timer_begin(c, "unique_counts", &slot);
        GK_TRY_HIP(c, select_flags_counts(c, c->heads, c->n, c->idx_b, c->ucount, &G));
        timer_end(c, slot);
    } else {
        const uint32_t *cidx;
        uint64_t count;
        int rc = group_front(c, 1, kl, nullptr, &cidx, &count, &G, nullptr, nullptr);
        if (rc != GK_OK) return rc;
        GK_TRY_HIP(c, ensure(reinterpret_cast<void **>(&c->ucount), &c->ucount_cap, 4 * (G + 64)));
        if (G) {
            hipLaunchKernelGGL(unique_counts_kernel, dim3(grid_for(G)), dim3(256), 0, c->stream, c->idx_b, G, c->n,
                               c->ucount);
            GK_TRY_HIP(c, hipGetLastError());
        }
    }
    c->n_unique = G;
    c->unique_valid = true;
    if (n_unique) *n_unique = G;
    return GK_OK;
}

extern "C" int gk_copy_unique(gk_ctx *c, uint64_t *group_start, uint32_t *count, uint64_t n) {
    if (!c) return GK_E_ARG;
    pre_drop(c);  // (the k-mer buffers: a prefetched L0 does not survive)
    if (!c->unique_valid) return fail(c, GK_E_STATE, "call gk_unique_counts first");
    if (n != c->n_unique) return fail(c, GK_E_ARG, "n differs from the unique k-mer count");
    if (n == 0) return GK_OK;
    if (count) GK_TRY_HIP(c, hipMemcpyAsync(count, c->ucount, 4 * n, hipMemcpyDeviceToHost, c->stream));
    if (group_start) {
        std::vector<uint32_t> tmp(n);
        GK_TRY_HIP(c, hipMemcpyAsync(tmp.data(), c->idx_b, 4 * n, hipMemcpyDeviceToHost, c->stream));
        GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
        for (uint64_t i = 0; i < n; ++i) group_start[i] = tmp[i];
    }
    GK_TRY_HIP(c, hipStreamSynchronize(c->stream));
    return GK_OK;
}

extern "C" int gk_device_unique(gk_ctx *c, void **group_start, void **count, uint64_t *n_unique) {
    if (!c) return GK_E_ARG;
    pre_drop(c);  // (the k-mer buffers: a prefetched L0 does not survive)
    if (!c->unique_valid) return fail(c, GK_E_STATE, "call gk_unique_counts first");
    if (group_start) *group_start = c->idx_b;
    if (count) *count = c->ucount;
    if (n_unique) *n_unique = c->n_unique;
    return GK_OK;
}

namespace gkm {
hipError_t scan_u32_exclusive_pub(gk_ctx *c, const uint32_t *in, uint64_t n, uint32_t *out, uint64_t *total) {
    return scan_u32_exclusive(c, in, n, out, total);
}

// two exclusive scans of n entries, no read-back (the caller knows the totals)
hipError_t scan_u32_exclusive_pair_launch(gk_ctx *c, const uint32_t *in1, uint32_t *out1, const uint32_t *in2,
                                          uint32_t *out2, uint64_t n) {
    if (n == 0) return hipSuccess;
    hipError_t e = scan_u32_exclusive_launch(c, in1, n, out1);
    return e == hipSuccess ? scan_u32_exclusive_launch(c, in2, n, out2) : e;
}

// two exclusive scans of n entries with one host round trip for both totals (scalars[62..63])
hipError_t scan_u32_exclusive_pair(gk_ctx *c, const uint32_t *in1, uint32_t *out1, const uint32_t *in2,
                                   uint32_t *out2, uint64_t n, uint64_t *total1, uint64_t *total2) {
    if (n == 0) {
        *total1 = *total2 = 0;
        return hipSuccess;
    }
    hipError_t e = scan_u32_exclusive_launch(c, in1, n, out1);
    if (e == hipSuccess) e = hipMemcpyAsync(c->scalars + 63, c->scalars, 8, hipMemcpyDeviceToDevice, c->stream);
    if (e == hipSuccess) e = scan_u32_exclusive_launch(c, in2, n, out2);
    if (e == hipSuccess) e = hipMemcpyAsync(c->scalars + 62, c->scalars, 8, hipMemcpyDeviceToDevice, c->stream);
    uint64_t t[2] = {0, 0};
    if (e == hipSuccess) e = read_back(c, c->scalars + 62, 16, t);
    *total1 = t[1];
    *total2 = t[0];
    return e;
}
}  // namespace gkm

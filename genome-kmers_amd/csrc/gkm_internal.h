// gkm_internal.h -- shared declarations of the libgkm HIP engine (gfx950 / CDNA4 only).
//
// Data layout in HBM:
//   sba      uint8[L + pad]     ASCII bases, '$'-joined contigs; the pad after L is '$' so every
//                               window read is in bounds and an out-of-array byte reads as '$'.
//   seg      uint32[nseg]       contig start offsets (SequenceCollection._forward_sba_seg_starts)
//   vals[2]  uint32[n]          start indices (ping-pong buffers of the radix sort)
//   keys[2]  uint64[W][n]       encoded k-mers, structure-of-arrays, word 0 most significant
//   status   uint64[tiles*256]  decoupled look-back state of the radix passes (epoch-tagged)
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>
#include <map>
#include <string>
#include <utility>
#include <vector>

#include "gkm.h"

#define GK_DOLLAR 36

namespace gkm {

constexpr int kRadixBits = 8;
constexpr int kRadixBins = 256;
constexpr int kMaxWords = 4;          // direct keys up to 256 bits

constexpr int kEncodeTile = 4096;     // positions per encode tile
constexpr int kSbaPad = 32768;        // '$' bytes after the sba (>= largest tile + max symbols)
constexpr int kSortThreads = 256;     // radix pass workgroup
constexpr int kSortItems = 16;        // keys per thread per radix tile
constexpr int kSortTile = kSortThreads * kSortItems;
constexpr int kScanThreads = 256;
constexpr int kScanItems = 16;
constexpr int kScanTile = kScanThreads * kScanItems;

// How a k-mer is turned into an order-preserving integer key:
//   bits   2: A,C,G,T -> 0..3 (sba holds only ACGT)
//          3: '$'/end -> 0, A,C,G,T -> 1..4 (doubling seeds on ACGT data under GKM_SEED3=1)
//          4: '$'/end -> 0, A B C D G H K M N R S T V W Y -> 1..15 (IUPAC data)
//   symbols  number of leading symbols encoded (= max_kmer_len for direct keys)
//   lenbits  2-bit keys of variable length append min(len, symbols) in the low lenbits bits
struct KeySpec {
    int bits;
    int symbols;
    int lenbits;
    int min_len;      // validity: a start needs min_len bases before '$'
    int words;        // W
    int total_bits;
    int canonical;    // 1: key of min(k-mer, reverse complement) (gkm_canon.h; fixed length only)
    int acgt_only;    // MSD of a mixed sba's ACGT-only k-mers (2-bit keys; the rest sorted apart, gkm_split.hip)
    int digits() const { return (total_bits + kRadixBits - 1) / kRadixBits; }
};

struct Timer {
    std::string name;
    hipEvent_t start, stop;
    uint64_t units = 0;  // work items the timed launch processed (k-mers), 0 = not recorded
};

}  // namespace gkm

struct gk_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;

    // input
    uint8_t *sba = nullptr;
    uint64_t sba_len = 0, sba_cap = 0;
    uint32_t *seg = nullptr;
    uint64_t nseg = 0, seg_cap = 0;
    uint64_t max_seg_len = 0;
    int acgt = 1;
    // the 2-bit packed copy of the sequence (pack2_kernel layout) that the packed transfer writes
    // beside the resident sba; res_pk: it is complete and current (the last gk_set_sequence went
    // through the packed transfer, every chunk unpacked on the device)
    uint64_t *res_code = nullptr;
    uint32_t *res_dol = nullptr;
    uint64_t res_code_cap = 0, res_dol_cap = 0;
    bool res_pk = false;
    bool pk_fresh = false;  // the packed sequence (scratch "pk_code" / "pk_dol") is current for
                            // the next gk_shard_sort_range (set by gk_shard_histogram)

    // k-mers
    uint64_t n = 0;
    uint32_t min_k = 0;
    bool have_starts = false;
    bool enumerated = false;   // vals == canonical enumerate output (ascending)
    bool starts_materialized = true;  // false: enumerated starts not yet written to vals[cur]
    bool sorted = false;
    uint32_t sort_len = 0;     // max_kmer_len of the last sort (0 = None)
    bool canonical = false;    // the last sort ordered canonical k-mers (GK_SORT_CANONICAL)
    bool keys_valid = false;   // keys[cur] encode the k-mers of vals[cur] (sort order)
    bool msd_keys_final = false;  // the last MSD sort wrote its (one-word) keys in sorted order
    bool msd_force_keys = false;  // split_sort: the class-A MSD (acgt_only) writes its final keys too
    bool split_keys_final = false;  // the last split sort wrote the final (4-bit) keys in sorted order
    bool keys_stale = false;   // ... once re-encoded from vals[cur]: the MSD sort does not keep them (ensure_keys)
    bool enum_sorted = false;  // vals = gk_sort's order of ALL enumerated k-mers (fixed length): ensure_keys
                               // may gather the keys through a table in enumeration order
    bool keys_are_ranks = false;
    gkm::KeySpec spec{};

    uint32_t *vals[2] = {nullptr, nullptr};
    uint64_t *keys[2] = {nullptr, nullptr};
    uint64_t elem_cap = 0;     // capacity (elements) of vals/keys buffers
    int key_words_cap = 0;     // key words both key buffers hold (the smaller of key_words_b)
    int key_words_b[2] = {0, 0};
    int cur = 0;

    // radix pass state
    uint64_t *status = nullptr;
    uint64_t status_cap = 0;   // words
    uint32_t epoch = 0;
    uint32_t *counters = nullptr;   // tile-id counters [64]
    uint32_t *hist = nullptr;       // [kMaxWords*8][256]
    uint32_t *offsets = nullptr;    // [kMaxWords*8][256]

    // group / scan scratch
    uint8_t *flags = nullptr;
    uint64_t flags_cap = 0;
    uint32_t *idx_a = nullptr, *idx_b = nullptr;
    uint64_t idx_cap = 0, idx_b_cap = 0;
    uint32_t *ucount = nullptr;  // multiplicities of the unique output (gk_unique_counts)
    uint64_t ucount_cap = 0;
    uint64_t *cumk = nullptr;       // enumerate: cumulative k-mers per segment
    uint64_t cumk_cap = 0;
    std::vector<uint32_t> hseg;     // host copy of the segment table
    bool internal_dollar = false;   // a '$' that is not a segment separator
    uint32_t *tile_sums = nullptr;
    uint64_t tile_sums_cap = 0;
    uint64_t *scalars = nullptr;    // small device scratch [64]
    // pinned host words [kHostPinWords] for the sort's small read-backs (list counters, scan totals):
    // a copy into pageable memory goes through a staging buffer and costs a second blit
    uint64_t *hpin = nullptr;
    int64_t *dhist = nullptr;
    uint64_t dhist_cap = 0;
    uint8_t *mask = nullptr;
    uint64_t mask_cap = 0, mask_n = 0;
    std::vector<uint32_t> shard_rest, shard_runs;  // gk_shard_class_b's lists (host)
    uint8_t *hmask = nullptr;  // gk_set_group_heads
    uint64_t hmask_cap = 0, hmask_n = 0;
    uint32_t *ranks = nullptr;      // doubling: rank per sba position
    uint64_t ranks_cap = 0;
    uint32_t *ym = nullptr, *yoff = nullptr, *oy = nullptr, *ot = nullptr;  // generator yields
    uint64_t *onum = nullptr;
    uint64_t ym_cap = 0, yoff_cap = 0, oy_cap = 0, ot_cap = 0, onum_cap = 0;

    // full-key group heads of the sorted order (1 = key differs from its predecessor), written
    // by the MSD sort as it finishes buckets; valid until the k-mer set or its order changes
    uint8_t *heads = nullptr;
    bool heads_valid = false;

    // unique view
    uint64_t n_unique = 0;
    bool unique_valid = false;

    // named, grow-only scratch buffers (MSD sort tables etc.)
    std::map<std::string, std::pair<void *, uint64_t>> scratch;

    // packed sba transfer (gkm_xfer.hip): pinned host + device staging slots, copy stream, events
    uint8_t *xfer_host = nullptr, *xfer_dev = nullptr;
    hipStream_t xfer_stream = nullptr, xfer_raw_stream = nullptr;
    // the device unpacks of the packed chunks: a stream of the highest priority, so that they are
    // dispatched ahead of a prefetched L0 pass running at the same time (gkm_msd.hip L0Prefetch)
    hipStream_t unpack_stream = nullptr;
    hipEvent_t unpack_done = nullptr;
    std::vector<hipEvent_t> xfer_ev;
    int xfer_slots = 0;
    uint64_t xfer_slot_bytes = 0;

    // sort hint (gk_sort_hint): gk_set_sequence also runs the L0 pass of gk_sort(hint_k) over
    // regions of the sequence as its packed transfer lands them, on pre_stream (gkm_msd.hip,
    // L0Prefetch); the next gk_sort(hint_k) of the enumeration starts from the regions' buckets
    // (pre_valid).  Any other use of the k-mer buffers drops it (pre_drop).
    uint32_t hint_k = 0;
    hipStream_t pre_stream = nullptr;
    hipEvent_t pre_done = nullptr;
    std::vector<hipEvent_t> pre_ev;  // per region: its bytes unpacked on `stream`
    bool pre_valid = false;          // keys[1] / vals[1] / scratch "msd_nd" + "pre_pieces" hold it
    uint32_t pre_k = 0, pre_regions = 0;
    int pre_w0 = 0, pre_w1 = 0;
    int pre_p88_shi = 0;             // != 0: the regions wrote the packed L0 form (gkm_msd.hip P88)

    // profiling
    bool profile = false;
    std::vector<gkm::Timer> timers;
    std::vector<hipEvent_t> ev_pool;  // timing events, created when profiling is switched on and
    size_t ev_used = 0;               // reused (no hipEventCreate inside a timed step)
};

// ---------------------------------------------------------------------------------------------
// launchers (implemented in gkm_encode.hip / gkm_sort.hip / gkm_group.hip)
// ---------------------------------------------------------------------------------------------
namespace gkm {

// Test and tuning overrides (GKM_* names, gkm_capi.hip): the value gk_set_option gave `name`, else
// -- for the few operational knobs listed in gkm_capi.hip (transfer threads and chunking, the
// packer, the rank fallback, prefetch regions, tracing) -- the environment variable; nullptr when
// unset.  Every other knob (alternative sort paths, test-only chunk sizes and forced formats) is
// reachable only through gk_set_option, so no user environment can change the sort path silently.
const char *opt(const char *name);
// timing experiments that write wrong output on purpose (GKM_EXP_*, GKM_L0_PROF): only in builds
// with -DGKM_EXPERIMENTS (tools/build_variant.sh), never in the product library
#ifdef GKM_EXPERIMENTS
inline const char *exp_opt(const char *name) { return std::getenv(name); }
#else
inline const char *exp_opt(const char *) { return nullptr; }
#endif

hipError_t ensure(void **p, uint64_t *cap, uint64_t bytes);
// large device buffers (gkm_capi.hip): hipMalloc, or an address range mapped from physical
// allocations (GKM_VMM_CHUNK_MB); dev_free releases either
hipError_t dev_alloc(void **p, size_t bytes);
hipError_t dev_free(void *p);
constexpr int kHostPinWords = 64;
// copy `bytes` (<= 8 * kHostPinWords) from device memory to `host` through the context's pinned
// words, after everything enqueued on c->stream before it (synchronises the stream)
hipError_t read_back(gk_ctx *c, const void *dev, size_t bytes, void *host);
// pack2_kernel (gkm_msd.hip) over nwords words of 32 bytes from `from`
hipError_t launch_pack2(const uint8_t *from, uint64_t nwords, uint64_t *code, uint32_t *dol, hipStream_t s);
// grow-only named device scratch buffer of at least `bytes` (contents not preserved on growth)
template <typename T>
inline hipError_t scratch(gk_ctx *c, const char *name, uint64_t count, T **out) {
    auto &e = c->scratch[name];
    hipError_t r = ensure(&e.first, &e.second, sizeof(T) * (count + 16));
    *out = static_cast<T *>(e.first);
    return r;
}
// frees a named scratch buffer (one-off large buffers that must not stay for the context's life)
inline void scratch_release(gk_ctx *c, const char *name) {
    auto it = c->scratch.find(name);
    if (it == c->scratch.end()) return;
    if (it->second.first) (void)dev_free(it->second.first);
    c->scratch.erase(it);
}
// re-encode keys[cur] from vals[cur] when the sort left them stale (gk_ctx::keys_stale)
int ensure_keys(gk_ctx *c);
// MSD sort of fixed-length keys from the enumerated positions (gkm_msd.hip)
int msd_sort(gk_ctx *c, const KeySpec &ks);
// fixed-length sort of a mixed-alphabet sba: ACGT-only k-mers by the 2-bit MSD, the others by
// 4-bit keys, merged (gkm_split.hip); *used = false when the split does not pay (caller falls back)
// key-range shards of a mixed sba (gk_shard_sort_range): ACGT-only k-mers whose 2-bit top-7-bit
// digit is in [d_lo, d_hi), other k-mers whose (canonical) first four 4-bit symbols are in
// [p4_lo, p4_hi) -- the same byte-order interval
struct SplitRange {
    uint32_t d_lo, d_hi, p4_lo, p4_hi;
    int pns = 4;  // symbols of the (4-bit) prefixes p4_lo / p4_hi (no upper bound: 1 << 4 pns)
    // given: the class-B k-mers of the whole sba, selected per position share and gathered
    // (gk_shard_class_b), instead of a whole-sequence scan: non-homopolymer starts and
    // homopolymer runs (first start, count, canonical letter), host memory, in start order
    bool given = false;
    const uint32_t *rest = nullptr, *runs = nullptr;
    uint64_t n_rest = 0, n_runs = 0;
};
int split_sort(gk_ctx *c, const KeySpec &ks, bool *used, const SplitRange *rg = nullptr);
int split_shard_class_b(gk_ctx *c, const KeySpec &ks, uint64_t lo, uint64_t hi, const std::vector<uint32_t> &bins,
                        int pns, uint32_t homo_w16, uint64_t *hist, std::vector<uint32_t> *rest,
                        std::vector<uint32_t> *runs);
// multi-GPU shards (gkm_msd.hip): send-side partition of the k-mers starting in [lo, hi) by the
// top msd_radix_bits() key bits; receive-side sort of buckets given as pieces
int msd_shard_partition(gk_ctx *c, const KeySpec &ks, uint64_t lo, uint64_t hi, uint64_t *kout, uint32_t *vout,
                        uint64_t cap, uint64_t *hist, uint64_t *count);
int msd_shard_sort(gk_ctx *c, const KeySpec &ks, const uint64_t *kin, const uint32_t *vin, const uint64_t *poff,
                   const uint64_t *plen, const uint32_t *pbucket, uint32_t np);
int msd_radix_bits();
// key-range shards (gkm_msd.hip): the L0 digit histogram (*bits = digit width) of the k-mers
// starting in [lo, hi); the sort of the k-mers of the whole sba whose L0 digit is in
// [digit_lo, digit_hi) into keys[0] / vals[0] (c->n = *n_kept)
int msd_l0_histogram(gk_ctx *c, const KeySpec &ks, uint64_t lo, uint64_t hi, uint64_t *hist, int *bits);
int msd_sort_range(gk_ctx *c, const KeySpec &ks, uint32_t digit_lo, uint32_t digit_hi, uint64_t *n_kept);
// width of the key-range ownership digits (gk_shard_histogram's bins: 1 << width)
int range_own_bits(const KeySpec &ks);
// partition ranking of each code object: lane-ordered LDS atomics (0) or ballot-match (1), set
// by gk_create from lds_rank_check (gkm_partition.h: g_rank_ballot)
hipError_t rank_mode_msd(int ballot);
hipError_t rank_mode_sort(int ballot);
// key / start buffers for n elements and `words` key words (gkm_capi.hip)
int ensure_elems(gk_ctx *c, uint64_t n, int words);
// key buffer b alone grown to `words` key words of elem_cap elements (contents not kept)
int grow_key_buffer(gk_ctx *c, int b, int words);
void timer_begin(gk_ctx *c, const char *name, int *slot);
void timer_end(gk_ctx *c, int slot);
void timer_units(gk_ctx *c, int slot, uint64_t units);
int fail(gk_ctx *c, int code, const std::string &msg);
int hip_fail(gk_ctx *c, hipError_t e, const char *where);

// packed sba transfer (gkm_xfer.hip): inputs of >= packed_transfer_min() bytes go 2-bit packed;
// the alphabet census (class bits as alphabet_kernel's, '$' count) is taken on the host
uint64_t packed_transfer_min();
struct L0Prefetch;  // gkm_msd.hip
int packed_transfer(gk_ctx *c, const uint8_t *sba, uint64_t len, uint32_t *cls_or, uint64_t *dollars,
                    L0Prefetch *pf = nullptr);
void xfer_release(gk_ctx *c);
// prefetched L0 of a sort hint (gkm_msd.hip): plan the regions of a single-contig sba of len bytes
// (*out = nullptr when the hint does not apply), launch every region whose bytes lie below `landed`
// (the transfer's in-order unpacked prefix, enqueued on c->stream), then finish (ok: the whole
// sequence was ACGT and landed; else the prefetch is dropped)
int prefetch_plan(gk_ctx *c, uint64_t len, L0Prefetch **out);
int prefetch_launch(gk_ctx *c, L0Prefetch *pf, uint64_t landed);
int prefetch_finish(gk_ctx *c, L0Prefetch *pf, bool ok);
// gk_sort(k) of the whole enumeration when the prefetched L0 is valid for its key spec
bool prefetch_matches(const gk_ctx *c, const KeySpec &ks);
int msd_sort_prefetched(gk_ctx *c, const KeySpec &ks);
inline void pre_drop(gk_ctx *c) { c->pre_valid = false; }

// encode
hipError_t launch_alphabet(gk_ctx *c, uint32_t *d_flags);
// the same census over [p, p + len) of the resident sba, accumulated into d_flags (not zeroed)
hipError_t launch_alphabet_range(gk_ctx *c, const uint8_t *p, uint64_t len, uint32_t *d_flags);
hipError_t launch_enumerate(gk_ctx *c, uint32_t min_k, uint32_t *out);
hipError_t launch_validate_starts(gk_ctx *c, const uint32_t *starts, uint64_t n, uint32_t min_k, uint32_t *d_bad);
hipError_t launch_encode_positions(gk_ctx *c, const KeySpec &ks, uint64_t *keys, uint32_t *vals, uint32_t *hist);
hipError_t launch_encode_gather(gk_ctx *c, const KeySpec &ks, const uint32_t *starts, uint64_t n, uint64_t *keys);
// keys of sorted starts that are a permutation of the whole enumeration (c->enum_sorted): every
// k-mer's key into `table` (table_bytes long), then one aligned row gather per sorted start: 2-bit
// rows per sba position (k <= 63), else W-word rows in enumeration order (gkm_encode.hip)
hipError_t launch_encode_table_gather(gk_ctx *c, const KeySpec &ks, const uint32_t *starts, uint64_t n,
                                      uint64_t *keys, uint64_t *table, uint64_t table_bytes);
// strand of each canonical k-mer: 1 if its reverse complement is the smaller (the key), else 0
hipError_t launch_canon_strands(gk_ctx *c, const KeySpec &ks, const uint32_t *starts, uint64_t n, uint8_t *out);

// sort
hipError_t launch_histogram(gk_ctx *c, const uint64_t *keys, uint64_t n, int words, int digits, uint32_t *hist);
int radix_sort(gk_ctx *c, int words, int total_bits, bool hist_ready);
// MSD over one-word keys in memory (gkm_msd.hip), radix_sort's contract; sort_keys picks it for
// one-word arrays of >= kMsdKeysMin keys (gkm_sort.hip)
int msd_sort_keys(gk_ctx *c, int total_bits);
int sort_keys(gk_ctx *c, int words, int total_bits, bool hist_ready);
bool sort_keys_msd(const gk_ctx *c, uint64_t n, int words, int total_bits);  // sort_keys takes the MSD path
// prefix doubling: the tied groups (flags: 1 starts a group) of keys[0] / vals[0] sorted by bkey-bit keys
int msd_sort_groups(gk_ctx *c, const uint8_t *flags, int bkey);
// prefix doubling's first round: the seed key (`seed`, as launch_encode_positions) of position
// vals[i] + o for the elements still tied (flags: 1 starts a group), 0 past the segment's end
hipError_t launch_member_seed_keys(gk_ctx *c, const KeySpec &seed, const uint8_t *flags, const uint32_t *vals,
                                   uint64_t o, uint64_t n, uint64_t *keys);

// last position of the segment holding p (seg: segment starts, '$' between segments)
__device__ __forceinline__ uint64_t seg_end_of(const uint32_t *__restrict__ seg, uint32_t nseg, uint64_t L,
                                               uint64_t p) {
    uint32_t lo = 0, hi = nseg;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if ((uint64_t)seg[mid] <= p) lo = mid; else hi = mid;
    }
    return (lo + 1 == nseg) ? L - 1 : (uint64_t)seg[lo + 1] - 2;
}
constexpr uint64_t kMsdKeysMin = 1ull << 20;

// group / scan
hipError_t select_flags(gk_ctx *c, const uint8_t *flags, uint64_t n, uint32_t *out_idx, uint64_t *count);
hipError_t select_flags_counts(gk_ctx *c, const uint8_t *flags, uint64_t n, uint32_t *out_idx, uint32_t *out_cnt,
                               uint64_t *count);
hipError_t scan_flags_inclusive(gk_ctx *c, const uint8_t *flags, uint64_t n, uint32_t *out);

// write the lazily enumerated starts into vals[cur] if a reader needs them (gkm_capi.hip)
int materialize_starts(gk_ctx *c);

// prefix doubling (gkm_capi.hip)
hipError_t launch_rank_scatter(gk_ctx *c, const uint32_t *vals, const uint32_t *gid, const uint32_t *gstart, uint64_t n, uint32_t *R);

}  // namespace gkm

#define GK_TRY_HIP(c, expr)                                        \
    do {                                                           \
        hipError_t _e = (expr);                                    \
        if (_e != hipSuccess) return gkm::hip_fail((c), _e, #expr); \
    } while (0)

/*
 * gkm.h -- C ABI of libgkm.so, the MI355X (gfx950) k-mer engine.
 *
 * The reference (mrperkett/genome-kmers v1.0.1) is pure Python + numba and has no FFI; its
 * drop-in boundary is the Kmers / SequenceCollection class surface.  Each entry point below
 * replaces one reference routine (paths relative to the reference's src/genome_kmers/) and is what
 * a ctypes binding inside that class surface binds:
 *
 *   gk_set_sequence        SequenceCollection.forward_sba / _forward_sba_seg_starts as the input
 *                          contract (sequence_collection.py:531-576, 663-726, 155-187); H2D copy.
 *   gk_enumerate           Kmers._initialize_single_pass / _get_unfiltered_kmer_count (kmers.py:789-861)
 *   gk_sort                Kmers.sort + get_is_less_than_func (kmers.py:1624-1731), numba quicksort
 *   gk_copy_start_indices  Kmers.kmer_sba_start_indices read-back (kmers.py:811, 1648)
 *   gk_set_start_indices   assigning Kmers.kmer_sba_start_indices (kmers.py:724, 1462, 1522)
 *   gk_group_hist          get_kmer_group_size_hist (kmers.py:454-520) behind Kmers.get_kmer_count
 *                          (kmers.py:994-1083) and Kmers.get_kmer_group_counts (kmers.py:1085-1178)
 *   gk_group_members       kmer_info_by_group_generator (kmers.py:523-648) behind Kmers.get_kmers
 *                          (kmers.py:869-992)
 *   gk_unique_counts       the (unique k-mer, multiplicity) view of the sorted groups (kmers.py:597-625)
 *   gk_copy_keys           encoded k-mers (no reference counterpart: the reference compares bytes)
 *   gk_locate              the start / record lookups behind get_kmer_info (kmers.py:1180-1264)
 *   gk_shard_partition,    one GPU's share of Kmers.sort under torch.distributed (no reference
 *   gk_shard_sort          counterpart: the reference is single-process, kmers.py:1644-1648)
 *   gk_fasta_open,         SequenceCollection._get_fasta_stats + _load_forward_sba_from_fasta
 *   gk_fasta_fill          (sequence_collection.py:476-576): FASTA -> sba on the host, multithreaded
 *
 * Conventions: every function returns GK_OK (0) or a negative gk_status; gk_last_error(ctx)
 * describes the last failure.  Host pointers are borrowed for the duration of the call only.
 * Device memory is owned by the context and freed by gk_destroy.  A context is bound to one HIP
 * device and one stream; it is not thread-safe.  Work is stream-ordered: functions that return
 * data to the host synchronise the stream, others may return before the device finishes
 * (gk_sync waits).
 */
#ifndef GKM_H
#define GKM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct gk_ctx gk_ctx;
typedef struct gk_fasta gk_fasta;

enum gk_status {
    GK_OK = 0,
    GK_E_ARG = -1,          /* invalid argument                                             */
    GK_E_HIP = -2,          /* HIP runtime error                                             */
    GK_E_OOM = -3,          /* device allocation failed                                      */
    GK_E_UNSUPPORTED = -4,  /* configuration not supported by the device path                */
    GK_E_ALPHABET = -5,     /* byte outside {A,B,C,D,G,H,K,M,N,R,S,T,V,W,Y,$}                */
    GK_E_STATE = -6,        /* call out of order (e.g. sort before set_sequence)             */
    GK_E_FILTER = -7,       /* a built-in filter raised (see gk_filter_error)                */
    GK_E_LIMIT = -8,        /* more than 2^32-1 k-mers (kmers.py:805-808)                     */
    GK_E_NO_BASES = -9,     /* comparator found no valid base (kmers.py:368-369)             */
    GK_E_IO = -10,          /* a file could not be opened / mapped                           */
    GK_E_FASTA_NAME = -11,  /* a header line with no name token (IndexError in the reference) */
    GK_E_FASTA_LAYOUT = -12,/* the sba would not be exactly full (sequence_collection.py:565)   */
};

/* built-in k-mer filters (kmers.py:14-259); evaluated on the device */
enum gk_filter_kind {
    GK_FILTER_KEEP_ALL = 0,      /* kmer_filter_keep_all                       kmers.py:14-16   */
    GK_FILTER_LENGTH = 1,        /* gen_kmer_length_filter_func(p0=min_len)    kmers.py:19-34   */
    GK_FILTER_HOMOPOLYMER = 2,   /* gen_kmer_homopolymer_filter_func(p0=max_h, p1=kmer_len)  :37-100 */
    GK_FILTER_GC = 3,            /* gen_kmer_gc_content_filter_func(p0=min_count, p1=max_count, p2=kmer_len) :103-192 */
    GK_FILTER_NO_AMBIGUOUS = 4,  /* gen_no_ambiguous_bases_filter(p0=kmer_len) kmers.py:195-229 */
    GK_FILTER_CRISPR_NGG = 5,    /* crispr_ngg_pam_filter                      kmers.py:232-259 */
    GK_FILTER_MASK = 6,          /* per-sorted-position byte mask from gk_set_filter_mask      */
};

/* filter error codes reported through gk_filter_error (match the reference's raise sites) */
enum gk_filter_error {
    GK_FERR_NONE = 0,
    GK_FERR_HOMO_LEN = 1,    /* kmers.py:66-69 / 83-86  "The kmer_len (..) requested is too large for kmer_sba_start_idx (..)" */
    GK_FERR_GC_LEN = 2,      /* kmers.py:176-179        "... too larger for kmer_sba_start_idx (..)"                        */
    GK_FERR_GC_OOB = 3,      /* read past the end of the sba (undefined behaviour in numba)                                */
    GK_FERR_AMBIG_LEN = 4,   /* kmers.py:212-213        "kmer_len (..) is invalid. It extends beyond len(sba)"              */
    GK_FERR_AMBIG_SEG = 5,   /* kmers.py:220-221        "end of segment was reached. kmer_len (..) invalid."                */
    GK_FERR_CRISPR_LEN = 6,  /* kmers.py:252-253        "The guide defined at this start index extends beyond the sba"      */
};

typedef struct gk_filter {
    int32_t kind;          /* gk_filter_kind */
    int32_t pad;
    int64_t p0, p1, p2;
} gk_filter;

/* gk_sort flags */
#define GK_SORT_DEFAULT 0u
/* Canonical k-mers (C5; this build's extension -- the reference defines none, kmers.py:689-696):
 * sort by min(k-mer, reverse complement) under the reference's byte order, with the reference's
 * IUPAC complement (sequence_collection.py:402-433).  Fixed length only (min_kmer_len ==
 * max_kmer_len); groups, counts and keys then refer to the canonical k-mers. */
#define GK_SORT_CANONICAL 1u
/* The reference's default tie order (Kmers.sort: numba quicksort, break_ties=False,
 * kmers.py:1624-1652): the device sorts, then numba's quicksort runs on the host over the original
 * start order comparing the device's group ranks (gkm_qsort.cpp) -- bit-exact with the reference,
 * equal k-mers included.  Host-bound (8 B of host memory per k-mer: the device hands the host
 * rank << 32 | start per start); not with GK_SORT_CANONICAL. */
#define GK_SORT_QUICKSORT_ORDER 2u

/* ---- lifetime ------------------------------------------------------------------------------ */
int gk_create(gk_ctx **out, int device);
void gk_destroy(gk_ctx *ctx);
const char *gk_last_error(gk_ctx *ctx);
int gk_sync(gk_ctx *ctx);
int gk_device_count(int *count);
/* Partition ranking of the sort on ctx's device.  Every stable partition ranks an item by one
 * returning LDS atomic, which relies on gfx950 applying same-address lanes in lane order;
 * gk_create checks that on every device it opens and, where it does not hold (or GKM_RANK_BALLOT=1
 * is set), switches to a ballot-match ranking: the same order, slower.  mode: -1 = query only,
 * 0 = the device's checked default, 1 = ballot-match forced (tests).  *active (may be NULL):
 * 1 if ballot-match ranking is in use afterwards, else 0. */
int gk_rank_mode(gk_ctx *ctx, int mode, int *active);

/* ---- input contract ------------------------------------------------------------------------- */
/* sba: ASCII bases, contigs joined by '$' (36), no trailing '$'; seg_starts: ascending uint32. */
int gk_set_sequence(gk_ctx *ctx, const uint8_t *sba, uint64_t len, const uint32_t *seg_starts, uint64_t nseg);
/* The transfer: inputs of >= 16 MiB (GKM_PACK_MIN) cross the link 2-bit packed wherever a 64 KiB
 * block is pure A/C/G/T and raw elsewhere, packed by up to 16 host threads (AVX2) and unpacked
 * into the resident ASCII sba on the device (gkm_xfer.hip); the alphabet check runs on the host
 * during the packing.  gk_copy_sequence reads the resident sba back (len = the loaded length). */
int gk_copy_sequence(gk_ctx *ctx, uint8_t *dst, uint64_t len);
/* Sort hint (no reference counterpart: the reference has no transfer; Kmers(sc, k, k) followed by
 * Kmers.sort(), kmers.py:656-760, 1624-1652, is the call pattern it serves).  While k != 0, every
 * later gk_set_sequence that crosses the link packed (>= GKM_PACK_MIN bytes, any number of contigs)
 * also runs the first pass of gk_sort(k) -- the L0 partition of the A/C/G/T-only k-mers by their top
 * key bits -- over regions of the sequence as they land, on a stream of its own; the next
 * gk_enumerate(k) + gk_sort(k, 0) of the whole enumeration then starts from its buckets (same
 * result, less time after the transfer): on an A/C/G/T sba they are the sort's own L0, on a mixed
 * one (N runs, IUPAC letters) the L0 of the split sort's A/C/G/T-only class.
 * Any other call that uses the k-mer buffers drops the prefetched pass.  k = 0 clears the hint;
 * flags must be 0.  Hints outside 8 <= k <= 32 are ignored. */
int gk_sort_hint(gk_ctx *ctx, uint32_t k, uint32_t flags);
/* 1 if the loaded sba holds only {A,C,G,T,$} (2-bit keys), 0 otherwise (4-bit keys) */
int gk_alphabet_is_acgt(gk_ctx *ctx, int *is_acgt);
/* 1 if the last gk_set_sequence left the 2-bit packed copy of the sequence resident beside the sba
 * (the packed transfer: the L0 passes of the sort read it, 0.375 B per position), else 0.  No
 * reference counterpart (the reference has no transfer). */
int gk_resident_packed(gk_ctx *ctx, int *on);
/* Test and tuning overrides of the library's GKM_* knobs, process-wide (no reference counterpart):
 * value NULL clears the override.  Only the operational knobs (GKM_XFER_THREADS, GKM_XFER_NUMA,
 * GKM_XFER_HYBRID, GKM_PACK_IMPL, GKM_PACK_MIN, GKM_PACK_BLOCKS, GKM_NO_RESIDENT_PACK,
 * GKM_RANK_BALLOT, GKM_PREFETCH_REGIONS, GKM_MSD_TRACE; and GKM_FASTA_CHUNK of the FASTA parser)
 * are also read from the environment; every other knob -- alternative sort paths, forced formats,
 * test-only chunk sizes -- is reachable only through this call. */
int gk_set_option(const char *name, const char *value);

/* ---- enumerate / sort ------------------------------------------------------------------------ */
/* every start with >= min_kmer_len bases before '$' / end, contig by contig, ascending */
int gk_enumerate(gk_ctx *ctx, uint32_t min_kmer_len, uint64_t *n_out);
/* replace the start indices with host-provided ones (any order, each must be a valid start) */
int gk_set_start_indices(gk_ctx *ctx, const uint32_t *src, uint64_t n, uint32_t min_kmer_len);
/*
 * Sort the start indices by the k-mer at each start, compared as compare_sba_kmers_lexicographically
 * with max_kmer_len (0 = None: compare up to the '$' that ends the contig).  Equal k-mers are
 * ordered by start index (the reference's break_ties=True order, kmers.py:1710-1711).
 */
int gk_sort(gk_ctx *ctx, uint32_t max_kmer_len, uint32_t flags);
int gk_num_kmers(gk_ctx *ctx, uint64_t *n);
int gk_copy_start_indices(gk_ctx *ctx, uint32_t *dst, uint64_t n);
/* start indices [offset, offset + count) of the current order (Kmers.get_kmer_str, kmers.py:1604) */
int gk_copy_start_range(gk_ctx *ctx, uint64_t offset, uint32_t *dst, uint64_t count);
/* encoded keys of the sorted k-mers: words_per_key uint64 words per k-mer, most significant first */
int gk_key_layout(gk_ctx *ctx, uint32_t *words_per_key, uint32_t *bits_per_symbol, uint32_t *symbols);
int gk_copy_keys(gk_ctx *ctx, uint64_t *dst, uint64_t n_words);
/* after a GK_SORT_CANONICAL sort: dst[i] = 1 if the reverse complement of sorted k-mer i is its
 * canonical form (strictly smaller than the k-mer), else 0 (the k-mer itself, or a palindrome) */
int gk_copy_strands(gk_ctx *ctx, uint8_t *dst, uint64_t n);

/* ---- groups ---------------------------------------------------------------------------------- */
/* mask for GK_FILTER_MASK: one byte per position of the current start-index order */
int gk_set_filter_mask(gk_ctx *ctx, const uint8_t *mask, uint64_t n);
/* Group boundaries decided by a caller's comparison (a custom kmer_comparison_func the device cannot
 * run, kmers.py:285-303, 597-601): heads[i] = 1 if the k-mer at position i of the current order
 * differs from the previous VALID k-mer (passing the filter), 0 if it is equal; read at valid
 * positions only, the first valid k-mer always starts a group.  Used by gk_group_hist /
 * gk_group_members called with is_sorted = GK_GROUPS_FROM_HEADS. */
int gk_set_group_heads(gk_ctx *ctx, const uint8_t *heads, uint64_t n);
#define GK_GROUPS_FROM_HEADS 2
/*
 * Histogram of group sizes over k-mers passing `filter`; groups are runs of equal k-mers under
 * compare_sba_kmers_lexicographically(kmer_len) (kmer_len < 0 = None) when is_sorted, else every
 * k-mer is its own group (compare_sba_kmers_always_less_than); is_sorted = GK_GROUPS_FROM_HEADS: the
 * groups gk_set_group_heads described.  max_group_size < 0 = None.
 * hist has max_counts_bin + 1 entries.  On GK_E_FILTER, *err_code / *err_idx name the failing
 * filter check and the SBA index of the first (in start-index order) k-mer that raised.
 */
int gk_group_hist(gk_ctx *ctx, int is_sorted, int64_t kmer_len, const gk_filter *filter, int64_t min_group_size,
                  int64_t max_group_size, int64_t max_counts_bin, int64_t *hist, int64_t *total,
                  int32_t *err_code, uint64_t *err_idx);
/*
 * The first yield_first_n (< 0 = None) members of every qualifying group, in generator order:
 * (kmer_num, group_size_yielded, group_size_total).  Two calls: with kmer_num == NULL only
 * *n_out is set; then call again with arrays of at least *n_out entries.
 */
int gk_group_members(gk_ctx *ctx, int is_sorted, int64_t kmer_len, const gk_filter *filter, int64_t min_group_size,
                     int64_t max_group_size, int64_t yield_first_n, uint64_t *kmer_num, uint32_t *size_yielded,
                     uint32_t *size_total, uint64_t capacity, uint64_t *n_out, int32_t *err_code, uint64_t *err_idx);
/* distinct k-mers of the sorted order (kmer_len = sort length): first sorted index and multiplicity
 * of each, computed and kept in HBM (after a one-word sort, one selection pass over the sort's
 * group heads writes both); gk_copy_unique copies them out, gk_device_unique exposes them.
 * Together with the sorted starts and keys (gk_device_views) this is the unique/count product. */
int gk_unique_counts(gk_ctx *ctx, uint64_t *n_unique);
int gk_copy_unique(gk_ctx *ctx, uint64_t *group_start, uint32_t *count, uint64_t n);
/* device pointers of the unique output: group_start uint32[n_unique], count uint32[n_unique] */
int gk_device_unique(gk_ctx *ctx, void **group_start, void **count, uint64_t *n_unique);

/* ---- device views / timing (bench + multi-GPU orchestration) --------------------------------- */
/* device pointers of the current sorted start indices and keys (valid until the next call); with
 * keys != NULL the keys are materialised first if the sort left them stale (multi-word keys, mixed
 * alphabets: a re-encode from the sorted starts); a one-word sort writes them in sorted order */
int gk_device_views(gk_ctx *ctx, void **starts, void **keys, uint64_t *n, uint32_t *words_per_key);
/* enable per-kernel HIP-event timing; gk_profile_report writes a JSON object to buf */
int gk_profile_enable(gk_ctx *ctx, int on);
int gk_profile_report(gk_ctx *ctx, char *buf, uint64_t buflen);
/* stream handle of the context (hipStream_t), for interop */
int gk_stream(gk_ctx *ctx, void **stream);

/* ---- multi-GPU shards (one process per GPU; the exchange is the caller's all-to-all) --------- */
/* number of top key bits the shard buckets are cut on (buckets = 1 << bits) */
int gk_shard_bucket_bits(void);
/*
 * Send side: encode the fixed-length k-mers (length k <= 64, no '$') that start in sequence
 * positions [lo, hi) (lo a multiple of 32) and partition them stably by their top
 * gk_shard_bucket_bits() key bits into the caller's DEVICE buffers d_keys / d_starts (capacity
 * cap >= count + 1), in ascending bucket order.  d_keys holds each k-mer's FIRST key word (the
 * first 64 / bits symbols); later words are re-encoded from the sba by the receiver.  flags:
 * 0 or GK_SORT_CANONICAL (the same on every rank and in gk_shard_sort).  h_hist[1 << bits] receives the bucket sizes, *n_out the count.
 * Returns after the device work is complete (the buffers can go straight to another stream).
 */
int gk_shard_partition(gk_ctx *ctx, uint64_t lo, uint64_t hi, uint32_t k, uint32_t flags, uint64_t *d_keys,
                       uint32_t *d_starts, uint64_t cap, uint64_t *h_hist, uint64_t *n_out);
/* Shard flag (round 6): only the start indices cross the exchange -- 4 B per k-mer instead of 12.
 * gk_shard_partition writes d_starts only (d_keys may be NULL); gk_shard_sort ignores d_keys and
 * re-derives every received k-mer's key from its own resident copy of the sequence (every rank holds
 * the whole sba, as the key-range shards do).  Forward keys of an A/C/G/T sba with k <= 32 only
 * (GK_E_UNSUPPORTED otherwise); the same flag on every rank. */
#define GK_SHARD_STARTS_ONLY 4u
/*
 * Receive side: sort n received (key, start) pairs in DEVICE buffers, given as npieces pieces
 * (offset, length, bucket) listed in ascending bucket order; the pieces of one bucket are listed
 * in ascending start order (source rank order).  The context then holds the sorted k-mers as if
 * gk_sort(k) had run on them: starts, keys, unique counts and group passes work as usual.
 * The buffers must be complete when the call is made (work queued on another stream must have
 * been synchronised by the caller).
 */
int gk_shard_sort(gk_ctx *ctx, const uint64_t *d_keys, const uint32_t *d_starts, uint64_t n, uint32_t k,
                  uint32_t flags, const uint64_t *h_piece_off, const uint64_t *h_piece_len, const uint32_t *h_piece_bucket,
                  uint32_t npieces);

/*
 * Key-range shards: multi-GPU with NO data exchange.  Every rank holds the whole sba (as in the
 * all-to-all scheme above); rank r keeps the k-mers whose top key digit lies in its digit range and
 * sorts them, so the ranks' outputs concatenated in rank order are the single-GPU gk_sort order
 * (kmers.py:1624-1652 with break_ties=True, kmers.py:1710-1711).  Replaces the same reference call
 * as gk_sort; the reference has no multi-process path.
 * gk_shard_histogram: histogram of the ownership digits -- the top *bits key bits, 12 for 2-bit
 * keys (k >= 6), 8 for 4-bit keys -- (h_hist[4096], entries >= 1 << *bits are 0) of the
 * fixed-length k-mers starting in [lo, hi) (lo a multiple of 32); on a mixed sba the digits of
 * the ACGT-only k-mers.  Each rank counts its position share, the caller sums the histograms over
 * ranks (an all-reduce of 1 << *bits counts, 32 KiB as int64) and cuts the digits into contiguous
 * ranges of about n / N k-mers: 4096 digits let a hot digit of a skewed genome be split finely.
 * gk_shard_sort_range: sort every k-mer of the sba whose ownership digit d has digit_lo <= d < digit_hi;
 * *n_kept receives their number and the context then holds them as after gk_sort(k).
 */
int gk_shard_histogram(gk_ctx *ctx, uint64_t lo, uint64_t hi, uint32_t k, uint32_t flags, uint64_t *h_hist,
                       uint32_t *bits);
int gk_shard_sort_range(gk_ctx *ctx, uint32_t k, uint32_t flags, uint32_t digit_lo, uint32_t digit_hi,
                        uint64_t *n_kept);
/* Key-range shards of a mixed sba (N runs, IUPAC letters) without a whole-sequence class-B scan
 * per rank:
 * gk_shard_class_b: the class-B k-mers (some non-ACGT letter) STARTING in [lo, hi) -- the rank's
 *   position share -- kept in the context as host lists in start order: n_rest non-homopolymer
 *   starts and n_runs homopolymer runs (first start, count, canonical letter: three uint32 each);
 *   their ownership digits are ADDED to h_hist (gk_shard_histogram's bins; a homopolymer k-mer
 *   weighs 11/16), so the all-reduced histogram balances them too.  An ACGT-only sba gives 0, 0.
 * gk_shard_class_b_copy: the two lists out (sizes as returned).
 * gk_shard_sort_range_b: gk_shard_sort_range with the class-B k-mers of the WHOLE sba given as the
 *   concatenation, in rank order, of every rank's lists (all-gathered): the rank keeps those in its
 *   interval instead of scanning the sequence for them. */
int gk_shard_class_b(gk_ctx *ctx, uint64_t lo, uint64_t hi, uint32_t k, uint32_t flags, uint64_t *h_hist,
                     uint64_t *n_rest, uint64_t *n_runs);
int gk_shard_class_b_copy(gk_ctx *ctx, uint32_t *rest, uint64_t n_rest, uint32_t *runs, uint64_t n_runs);
int gk_shard_sort_range_b(gk_ctx *ctx, uint32_t k, uint32_t flags, uint32_t digit_lo, uint32_t digit_hi,
                          const uint32_t *rest, uint64_t n_rest, const uint32_t *runs, uint64_t n_runs,
                          uint64_t *n_kept);

/* Location of selected k-mers for Kmers.get_kmers(kmer_info_to_yield="full") (kmers.py:1180-1264):
 * sba_idx[i] = kmer_sba_start_indices[kmer_nums[i]] and seg[i] = the segment holding it
 * (bisect_right over the segment starts, sequence_collection.py:76-97), computed on the device
 * against the resident starts -- the host never needs the whole start array. */
int gk_locate(gk_ctx *ctx, const uint64_t *kmer_nums, uint64_t m, uint32_t *sba_idx, uint32_t *seg);

/* ---- FASTA ingest (host; no context, no device) ------------------------------------------
 * gk_fasta_open maps `path` and scans it once with n_threads threads (<= 0: up to 16): the
 * number of records ('>' lines), the sequence bytes left after each line's strip(), and the bytes
 * of the record names (each NUL-terminated) -- _get_fasta_stats (sequence_collection.py:476-515).
 * The caller allocates sba[total_seq_len + num_records - 1], seg_starts[num_records] and
 * names[names_bytes]; gk_fasta_fill writes them as _load_forward_sba_from_fasta does (:517-566):
 * upper-cased bytes, '$' between records, segment starts, names in record order.  bad_bytes[256]
 * (optional, zeroed by the caller) flags every sequence byte outside ACGTRYSWKMBDHVN$, for the
 * reference's alphabet error (:571-574).  GK_E_FASTA_NAME: a header without a name;
 * GK_E_FASTA_LAYOUT: the bytes do not fill sba exactly.  gk_fasta_close unmaps. */
int gk_fasta_open(const char *path, int n_threads, gk_fasta **out, uint64_t *num_records, uint64_t *total_seq_len,
                  uint64_t *names_bytes);
int gk_fasta_fill(gk_fasta *f, uint8_t *sba, uint64_t sba_len, uint32_t *seg_starts, char *names,
                  uint8_t *bad_bytes);
void gk_fasta_close(gk_fasta *f);

/* ---- synthetic genomes (host) --------------------------------------------------------------
 * The reference's profiling genome: profiling.get_random_seq(n) after np.random.seed(seed)
 * (profiling.py:12-24) -- MT19937 init_genrand(seed), base i = "ATGC"[genrand_int32() & 3] --
 * written as n ASCII bytes. */
int gk_reference_random_bases(uint8_t *out, uint64_t n, uint32_t seed);

#ifdef __cplusplus
}
#endif
#endif /* GKM_H */

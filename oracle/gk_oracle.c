/*
 * gk_oracle.c -- CPU restatement of the genome-kmers hot path (TEST INFRASTRUCTURE ONLY).
 *
 * This file is the parity oracle.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg load it; the product (libgkm.so, genome_kmers/) never links or calls it.
 *
 * Every function restates one reference function (mrperkett/genome-kmers v1.0.1, paths relative to
 * the reference's src/genome_kmers/):
 *   gko_compare             kmers.py:306-397  compare_sba_kmers_lexicographically
 *   gko_has_required_len    kmers.py:262-282  kmer_has_required_len
 *   gko_kmer_count /        kmers.py:789-861  _initialize_single_pass / _get_unfiltered_kmer_count
 *     gko_enumerate           (segment ends from sequence_collection.py:155-187)
 *   gko_quicksort           kmers.py:1624-1731 Kmers.sort + get_is_less_than_func, driving the
 *                           third-party numba.misc.quicksort (numba 0.54.1 misc/quicksort.py:
 *                           partition :86-127, insertion_sort :66-84, run_quicksort :164-197;
 *                           SMALL_QUICKSORT = 15, MAX_STACK = 100).  Pinned against the golden
 *                           vectors produced by the reference itself (tests/golden/).
 *   gko_filter              kmers.py:14-259   built-in k-mer filters
 *   gko_group_scan          kmers.py:454-648  kmer_info_by_group_generator + get_kmer_group_size_hist
 *
 * Error reporting: functions return GKO_OK (0) or a negative code; *err_idx receives the SBA index
 * the reference would name in its exception message (the Python wrapper rebuilds the message).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define GKO_OK 0
#define GKO_E_NO_BASES -1        /* AssertionError "There were no valid kmer bases to compare" */
#define GKO_E_TOO_SHORT -2       /* AssertionError "kmers compared were less than min_kmer_len" */
#define GKO_E_STACK -3           /* numba quicksort MAX_STACK assertion */
#define GKO_E_HOMO_LEN -10       /* homopolymer filter: kmer_len too large (kmers.py:66-69, 83-86) */
#define GKO_E_GC_LEN -11         /* gc filter: '$' reached (kmers.py:176-179) */
#define GKO_E_GC_OOB -12         /* gc filter: read past end of sba (undefined in numba) */
#define GKO_E_AMBIG_LEN -13      /* no-ambiguous filter: beyond len(sba) (kmers.py:212-213) */
#define GKO_E_AMBIG_SEG -14      /* no-ambiguous filter: '$' reached (kmers.py:220-221) */
#define GKO_E_CRISPR_LEN -15     /* crispr filter: beyond sba (kmers.py:252-253) */
#define GKO_E_ARG -20

#define DOLLAR 36

/* ------------------------------------------------------------------------------------------ */
/* order definition                                                                            */
/* ------------------------------------------------------------------------------------------ */

/* kmers.py:306-397. max_kmer_len < 0 means None. Returns -1/0/+1 or GKO_E_NO_BASES (as 2). */
int gko_compare(const uint8_t *sba, uint64_t n, uint64_t a, uint64_t b, int64_t max_kmer_len,
                int64_t *last_idx) {
    int64_t t = 0;
    for (;;) {
        uint64_t ia = a + (uint64_t)t, ib = b + (uint64_t)t;
        int oa = ia >= n || sba[ia] == DOLLAR;
        int ob = ib >= n || sba[ib] == DOLLAR;
        if (oa || ob) {
            *last_idx = t - 1;
            if (t == 0) return 2;
            if (oa && !ob) return -1;
            if (ob && !oa) return 1;
            return 0;
        }
        if (sba[ia] < sba[ib]) { *last_idx = t; return -1; }
        if (sba[ia] > sba[ib]) { *last_idx = t; return 1; }
        if (max_kmer_len >= 0 && t == max_kmer_len - 1) { *last_idx = t; return 0; }
        ++t;
    }
}

/* kmers.py:262-282 */
int gko_has_required_len(const uint8_t *sba, uint64_t n, int64_t start, int64_t min_len) {
    for (int64_t i = start; i < start + min_len; ++i) {
        if (i < 0 || (uint64_t)i >= n || sba[i] == DOLLAR) return 0;
    }
    return 1;
}

/* ------------------------------------------------------------------------------------------ */
/* enumerate                                                                                   */
/* ------------------------------------------------------------------------------------------ */

/* segment s covers [starts[s], starts[s+1]-2]; last segment ends at n-1 (sequence_collection.py:180-187) */
static inline uint64_t seg_end(const uint32_t *seg_starts, uint64_t nseg, uint64_t s, uint64_t n) {
    return (s + 1 == nseg) ? n - 1 : (uint64_t)seg_starts[s + 1] - 2;
}

/* kmers.py:837-861 */
int64_t gko_kmer_count(const uint32_t *seg_starts, uint64_t nseg, uint64_t n, int64_t min_k) {
    int64_t total = 0;
    for (uint64_t s = 0; s < nseg; ++s) {
        int64_t len = (int64_t)(seg_end(seg_starts, nseg, s, n) - seg_starts[s] + 1);
        total += len - min_k + 1;
    }
    return total;
}

/* kmers.py:789-835 */
void gko_enumerate(const uint32_t *seg_starts, uint64_t nseg, uint64_t n, int64_t min_k, uint32_t *out) {
    uint64_t o = 0;
    for (uint64_t s = 0; s < nseg; ++s) {
        uint64_t b = seg_starts[s], e = seg_end(seg_starts, nseg, s, n) + 1 - (uint64_t)min_k + 1;
        for (uint64_t p = b; p < e; ++p) out[o++] = (uint32_t)p;
    }
}

/* ------------------------------------------------------------------------------------------ */
/* sort: Kmers.sort -> numba quicksort with is_less_than                                        */
/* ------------------------------------------------------------------------------------------ */

typedef struct {
    const uint8_t *sba;
    uint64_t n;
    int64_t min_k, max_k;
    int break_ties, validate;
    int err;
    uint64_t err_idx;
} lt_ctx;

/* kmers.py:1690-1729 */
static inline int is_less_than(lt_ctx *c, uint32_t a, uint32_t b) {
    int64_t last;
    int cmp = gko_compare(c->sba, c->n, a, b, c->max_k, &last);
    if (cmp == 2) {
        if (!c->err) { c->err = GKO_E_NO_BASES; c->err_idx = a; }
        return 0;
    }
    int lt = cmp < 0 ? 1 : (cmp > 0 ? 0 : (c->break_ties ? a < b : 0));
    if (c->validate) {
        int64_t nb = c->min_k - (last + 1);
        int va = gko_has_required_len(c->sba, c->n, (int64_t)a + last + 1, nb);
        int vb = gko_has_required_len(c->sba, c->n, (int64_t)b + last + 1, nb);
        if ((!va || !vb) && !c->err) { c->err = GKO_E_TOO_SHORT; c->err_idx = a; }
    }
    return lt;
}

#define SWAP(x, y) do { uint32_t _t = A[x]; A[x] = A[y]; A[y] = _t; } while (0)

/* numba misc/quicksort.py:66-84 (inclusive bounds) */
static void insertion_sort(lt_ctx *c, uint32_t *A, int64_t low, int64_t high) {
    if (high <= low) return;
    for (int64_t i = low + 1; i <= high; ++i) {
        uint32_t k = A[i];
        int64_t j = i;
        while (j > low && is_less_than(c, k, A[j - 1])) {
            A[j] = A[j - 1];
            --j;
        }
        A[j] = k;
    }
}

/* numba misc/quicksort.py:86-127: median of three, pivot stashed at high, Hoare sweep */
static int64_t partition(lt_ctx *c, uint32_t *A, int64_t low, int64_t high) {
    int64_t mid = (low + high) >> 1;
    if (is_less_than(c, A[mid], A[low])) SWAP(low, mid);
    if (is_less_than(c, A[high], A[mid])) SWAP(high, mid);
    if (is_less_than(c, A[mid], A[low])) SWAP(low, mid);
    uint32_t pivot = A[mid];
    SWAP(high, mid);
    int64_t i = low, j = high - 1;
    for (;;) {
        while (i < high && is_less_than(c, A[i], pivot)) ++i;
        while (j >= low && is_less_than(c, pivot, A[j])) --j;
        if (i >= j) break;
        SWAP(i, j);
        ++i;
        --j;
    }
    SWAP(i, high);
    return i;
}

/* numba misc/quicksort.py:164-197 run_quicksort; in place on A (is_argsort=False) */
int gko_quicksort(const uint8_t *sba, uint64_t n, uint32_t *A, uint64_t count, int64_t min_k,
                  int64_t max_k, int break_ties, int validate, uint64_t *err_idx) {
    lt_ctx c = {sba, n, min_k, max_k, break_ties, validate, 0, 0};
    if (count < 2) return GKO_OK;
    int64_t stack_lo[100], stack_hi[100];
    int sp = 0;
    stack_lo[0] = 0;
    stack_hi[0] = (int64_t)count - 1;
    sp = 1;
    while (sp > 0) {
        --sp;
        int64_t low = stack_lo[sp], high = stack_hi[sp];
        while (high - low >= 15) {
            if (sp >= 100) return GKO_E_STACK;
            int64_t i = partition(&c, A, low, high);
            if (high - i > i - low) {
                if (high > i) { stack_lo[sp] = i + 1; stack_hi[sp] = high; ++sp; }
                high = i - 1;
            } else {
                if (i > low) { stack_lo[sp] = low; stack_hi[sp] = i - 1; ++sp; }
                low = i + 1;
            }
        }
        insertion_sort(&c, A, low, high);
        if (c.err) break;
    }
    if (c.err && err_idx) *err_idx = c.err_idx;
    return c.err;
}

/* ------------------------------------------------------------------------------------------ */
/* filters (kmers.py:14-259)                                                                   */
/* ------------------------------------------------------------------------------------------ */

enum { F_KEEP_ALL = 0, F_LENGTH = 1, F_HOMOPOLYMER = 2, F_GC = 3, F_NO_AMBIGUOUS = 4, F_CRISPR_NGG = 5 };

/* p0..p2: LENGTH(min_len) HOMOPOLYMER(max_h, kmer_len) GC(min_count, max_count, kmer_len)
 *         NO_AMBIGUOUS(kmer_len).  Returns 1 pass / 0 fail / negative error. */
int gko_filter(const uint8_t *sba, uint64_t n, int kind, int64_t p0, int64_t p1, int64_t p2, uint64_t idx) {
    switch (kind) {
    case F_KEEP_ALL:
        return 1;
    case F_LENGTH:
        return gko_has_required_len(sba, n, (int64_t)idx, p0);
    case F_HOMOPOLYMER: { /* kmers.py:63-98 */
        int64_t maxh = p0, k = p1;
        if ((int64_t)idx + k - 1 >= (int64_t)n) return GKO_E_HOMO_LEN;
        if (k < maxh) return 1;
        int64_t h = 1;
        for (int64_t t = 1; t < k; ++t) {
            uint8_t base = sba[idx + t], prev = sba[idx + t - 1];
            if (base == DOLLAR) return GKO_E_HOMO_LEN;
            if (base == prev) {
                if (++h > maxh) return 0;
            } else {
                h = 1;
            }
        }
        return 1;
    }
    case F_GC: { /* kmers.py:150-190 */
        int64_t minc = p0, maxc = p1, k = p2, gc = 0;
        if (maxc < minc) return 0;
        for (int64_t t = 0; t < k; ++t) {
            if (idx + t >= n) return GKO_E_GC_OOB;
            uint8_t base = sba[idx + t];
            if (base == DOLLAR) return GKO_E_GC_LEN;
            if (base == 'G' || base == 'C') {
                if (++gc > maxc) return 0;
            }
        }
        return (minc <= gc && gc <= maxc) ? 1 : 0;
    }
    case F_NO_AMBIGUOUS: { /* kmers.py:209-227 */
        int64_t k = p0;
        if ((int64_t)idx + k > (int64_t)n) return GKO_E_AMBIG_LEN;
        for (int64_t t = 0; t < k; ++t) {
            uint8_t base = sba[idx + t];
            if (base == DOLLAR) return GKO_E_AMBIG_SEG;
            if (base != 'A' && base != 'T' && base != 'G' && base != 'C') return 0;
        }
        return 1;
    }
    case F_CRISPR_NGG: /* kmers.py:232-259 */
        if (idx + 23 > n) return GKO_E_CRISPR_LEN;
        return (sba[idx + 21] == 'G' && sba[idx + 22] == 'G') ? 1 : 0;
    }
    return GKO_E_ARG;
}

/* ------------------------------------------------------------------------------------------ */
/* group scan: kmer_info_by_group_generator (kmers.py:523-648) + hist (kmers.py:454-520)        */
/* ------------------------------------------------------------------------------------------ */

typedef struct {
    int64_t *hist;      /* [max_bin + 1] or NULL */
    int64_t max_bin;
    int64_t total;
    /* per-yield outputs (kmer_num, size_yielded, size_total), or NULL */
    int64_t *y_num, *y_yielded, *y_total;
    int64_t y_cap, y_count;
} scan_out;

static void emit_group(scan_out *o, const int64_t *members, int64_t nm, int64_t size, int64_t min_g, int64_t max_g) {
    if (size < min_g) return;
    if (max_g >= 0 && size > max_g) return;
    if (o->hist) {
        o->hist[size < o->max_bin ? size : o->max_bin] += 1;
        o->total += size;
    }
    if (o->y_num) {
        for (int64_t i = 0; i < nm; ++i) {
            if (o->y_count < o->y_cap) {
                o->y_num[o->y_count] = members[i];
                o->y_yielded[o->y_count] = nm;
                o->y_total[o->y_count] = size;
            }
            o->y_count++;
        }
    }
}

/*
 * sorted_mode = 1: compare neighbours with compare_sba_kmers_lexicographically(kmer_len)
 * sorted_mode = 0: compare_sba_kmers_always_less_than (every valid k-mer its own group)
 * kmer_len < 0 = None; max_g < 0 = None; yield_first_n < 0 = None.
 * hist mode: pass hist != NULL (yield_first_n forced to 1 as in kmers.py:495-496).
 */
int gko_group_scan(const uint8_t *sba, uint64_t n, const uint32_t *starts, uint64_t count, int sorted_mode,
                   int64_t kmer_len, int fkind, int64_t f0, int64_t f1, int64_t f2, int64_t min_g, int64_t max_g,
                   int64_t yield_first_n, int64_t *hist, int64_t max_bin, int64_t *total, int64_t *y_num,
                   int64_t *y_yielded, int64_t *y_total, int64_t y_cap, int64_t *y_count, uint64_t *err_idx) {
    scan_out o = {hist, max_bin, 0, y_num, y_yielded, y_total, y_cap, 0};
    if (hist) {
        memset(hist, 0, sizeof(int64_t) * (size_t)(max_bin + 1));
        yield_first_n = 1;
    }
    int64_t cap = yield_first_n < 0 ? (int64_t)count + 1 : yield_first_n;
    int64_t *members = (int64_t *)malloc(sizeof(int64_t) * (size_t)(cap > 0 ? cap : 1));
    int64_t nm = 0, size = 0;
    int have_prev = 0;
    uint64_t prev = 0;
    int rc = GKO_OK;
    for (uint64_t j = 0; j < count; ++j) {
        uint64_t idx = starts[j];
        int pass = gko_filter(sba, n, fkind, f0, f1, f2, idx);
        if (pass < 0) { rc = pass; if (err_idx) *err_idx = idx; goto done; }
        if (!pass) continue;
        int same;
        if (!have_prev) {
            have_prev = 1;
            same = 1;
        } else {
            if (sorted_mode) {
                int64_t last;
                int c = gko_compare(sba, n, prev, idx, kmer_len, &last);
                if (c == 2) { rc = GKO_E_NO_BASES; if (err_idx) *err_idx = prev; goto done; }
                same = (c == 0);
            } else {
                same = 0;
            }
        }
        prev = idx;
        if (same) {
            size++;
            if (yield_first_n < 0 || nm < yield_first_n) members[nm++] = (int64_t)j;
        } else {
            emit_group(&o, members, nm, size, min_g, max_g);
            size = 1;
            members[0] = (int64_t)j;
            nm = 1;
        }
    }
    emit_group(&o, members, nm, size, min_g, max_g);
done:
    free(members);
    if (total) *total = o.total;
    if (y_count) *y_count = o.y_count;
    return rc;
}

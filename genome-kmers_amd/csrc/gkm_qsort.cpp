// gkm_qsort.cpp -- the reference's default tie order (gk_sort flag GK_SORT_QUICKSORT_ORDER), host C++.
//
// Kmers.sort() (kmers.py:1624-1652) runs numba's quicksort (numba.misc.quicksort, pinned ^0.59.1:
// run_quicksort / partition / insertion_sort; SMALL_QUICKSORT = 15, MAX_STACK = 100) in place over
// the uint32 start indices with is_less_than(break_ties=False) (kmers.py:1654-1731).  Equal k-mers
// keep whatever order that quicksort's swaps leave them in, which no parallel sort reproduces.
//
// Product path (not the oracle): the device sorts first (stable order) and its group pass gives
// every start the dense rank of its k-mer group; the device hands the host, in the ORIGINAL start
// order, one word per start: rank << 32 | start.  The quicksort below then runs on the host over
// those words with LT(a, b) = rank(a) < rank(b) -- O(n) host memory, and no random lookups.  That comparator returns exactly what
// the reference's byte comparator returns for every pair (ranks are order-isomorphic to the k-mers
// under compare_sba_kmers_lexicographically, equal exactly when the k-mers are equal up to
// max_kmer_len), so every swap, and the result, is the reference's -- at O(1) per comparison
// instead of a byte loop over two random sba windows.  The validation inside is_less_than never
// fires here: gk_sort has already checked every start's length (launch_validate_starts).
#include <stdint.h>

#include <utility>

namespace gkm {

namespace {
struct RankLess {  // words rank << 32 | start: compare the ranks only
    bool operator()(uint64_t a, uint64_t b) const { return (a >> 32) < (b >> 32); }
};

// insertion sort of A[low..high] (inclusive), numba misc/quicksort.py insertion_sort
void insertion_sort(uint64_t *A, int64_t low, int64_t high, RankLess lt) {
    if (high <= low) return;
    for (int64_t i = low + 1; i <= high; ++i) {
        const uint64_t k = A[i];
        int64_t j = i;
        while (j > low && lt(k, A[j - 1])) {
            A[j] = A[j - 1];
            --j;
        }
        A[j] = k;
    }
}

// numba misc/quicksort.py partition: median of {low, mid, high} by three compare-swaps, the pivot
// parked at high, a two-sided sweep, the pivot swapped into place
int64_t partition(uint64_t *A, int64_t low, int64_t high, RankLess lt) {
    const int64_t mid = (low + high) >> 1;
    if (lt(A[mid], A[low])) std::swap(A[low], A[mid]);
    if (lt(A[high], A[mid])) std::swap(A[high], A[mid]);
    if (lt(A[mid], A[low])) std::swap(A[low], A[mid]);
    const uint64_t pivot = A[mid];
    std::swap(A[high], A[mid]);
    int64_t i = low, j = high - 1;
    for (;;) {
        while (i < high && lt(A[i], pivot)) ++i;
        while (j >= low && lt(pivot, A[j])) --j;
        if (i >= j) break;
        std::swap(A[i], A[j]);
        ++i;
        --j;
    }
    std::swap(A[i], A[high]);
    return i;
}
}  // namespace

// numba misc/quicksort.py run_quicksort (is_argsort=False): in place on A[0..n) (words rank << 32 |
// start; the starts leave in the reference's order in the low halves).  Returns 0, or -1 where
// numba's `assert n < MAX_STACK` would fail (the reference raises AssertionError there).
int quicksort_by_rank(uint64_t *A, uint64_t n) {
    constexpr int kSmall = 15, kMaxStack = 100;
    if (n < 2) return 0;
    const RankLess lt{};
    int64_t lo_st[kMaxStack], hi_st[kMaxStack];
    lo_st[0] = 0;
    hi_st[0] = (int64_t)n - 1;
    int sp = 1;
    while (sp > 0) {
        --sp;
        int64_t low = lo_st[sp], high = hi_st[sp];
        while (high - low >= kSmall) {
            if (sp >= kMaxStack) return -1;
            const int64_t i = partition(A, low, high, lt);
            if (high - i > i - low) {  // push the larger side, continue with the smaller
                if (high > i) {
                    lo_st[sp] = i + 1;
                    hi_st[sp] = high;
                    ++sp;
                }
                high = i - 1;
            } else {
                if (i > low) {
                    lo_st[sp] = low;
                    hi_st[sp] = i - 1;
                    ++sp;
                }
                low = i + 1;
            }
        }
        insertion_sort(A, low, high, lt);
    }
    return 0;
}

}  // namespace gkm

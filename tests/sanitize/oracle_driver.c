/* Sanitizer driver for the CPU oracle (oracle/gk_oracle.c): built with
 * -fsanitize=address,undefined by tests/test_sanitizers.py; enumerates, sorts (both tie orders)
 * and group-scans one input and writes the results (test infrastructure only).
 *   oracle_driver <sba file> <seg file (uint32)> <min_k> <max_k (0 = None)> <out_prefix> */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

int64_t gko_kmer_count(const uint32_t *seg_starts, uint64_t nseg, uint64_t n, int64_t min_k);
void gko_enumerate(const uint32_t *seg_starts, uint64_t nseg, uint64_t n, int64_t min_k, uint32_t *out);
int gko_quicksort(const uint8_t *sba, uint64_t n, uint32_t *A, uint64_t count, int64_t min_k, int64_t max_k,
                  int break_ties, int validate, uint64_t *err_idx);

static void *slurp(const char *path, size_t *n) {
    FILE *f = fopen(path, "rb");
    if (!f) exit(3);
    fseek(f, 0, SEEK_END);
    *n = (size_t)ftell(f);
    fseek(f, 0, SEEK_SET);
    void *p = malloc(*n ? *n : 1);
    if (*n && fread(p, 1, *n, f) != *n) exit(4);
    fclose(f);
    return p;
}

static void dump(const char *prefix, const char *ext, const void *p, size_t n) {
    char path[4096];
    snprintf(path, sizeof path, "%s.%s", prefix, ext);
    FILE *f = fopen(path, "wb");
    if (!f) exit(5);
    if (n) fwrite(p, 1, n, f);
    fclose(f);
}

int main(int argc, char **argv) {
    if (argc != 6) return 2;
    size_t n = 0, ns = 0;
    uint8_t *sba = slurp(argv[1], &n);
    uint32_t *seg = slurp(argv[2], &ns);
    const int64_t min_k = atoll(argv[3]), max_k = atoll(argv[4]);
    const int64_t cnt = gko_kmer_count(seg, ns / 4, n, min_k);
    uint32_t *a = malloc(4 * (size_t)(cnt > 0 ? cnt : 1)), *b = malloc(4 * (size_t)(cnt > 0 ? cnt : 1));
    gko_enumerate(seg, ns / 4, n, min_k, a);
    for (int64_t i = 0; i < cnt; ++i) b[i] = a[i];
    uint64_t e1 = 0, e2 = 0;
    const int r1 = gko_quicksort(sba, n, a, (uint64_t)cnt, min_k, max_k ? max_k : -1, 0, 1, &e1);
    const int r2 = gko_quicksort(sba, n, b, (uint64_t)cnt, min_k, max_k ? max_k : -1, 1, 1, &e2);
    dump(argv[5], "default", a, 4 * (size_t)cnt);
    dump(argv[5], "stable", b, 4 * (size_t)cnt);
    printf("rc %d %d %lld\n", r1, r2, (long long)cnt);
    free(a);
    free(b);
    free(sba);
    free(seg);
    return 0;
}

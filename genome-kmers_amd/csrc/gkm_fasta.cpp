// gkm_fasta.cpp -- FASTA -> sequence byte array, host side, multithreaded.
//
// Replaces the reference's two per-line Python passes, SequenceCollection._get_fasta_stats
// (sequence_collection.py:476-515) and _load_forward_sba_from_fasta (:517-576), with the same
// result byte for byte:
//   - lines end at '\n', '\r\n' or '\r' (Python text mode, universal newlines);
//   - a line whose first byte is '>' is a record header; its name is the first whitespace-separated
//     token after the '>' (line[1:].strip().split()[0]);
//   - any other line contributes line.strip().upper(): Python's whitespace set (space, \t, \n, \r,
//     \v, \f, \x1c-\x1f) is trimmed at both ends and a-z are upper-cased;
//   - records are joined by one '$' (36); the '$' is skipped while no sequence byte has been
//     written (`if at != 0`), so the first record starts at 0 and there is no trailing '$'.
// The file is memory-mapped and cut into chunks at line starts.  gk_fasta_open scans every chunk
// once (records, sequence bytes, name bytes, headers before the chunk's first sequence byte);
// gk_fasta_fill then writes each chunk's bytes at its own offset in parallel.
#include <errno.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "gkm.h"

namespace {

inline bool py_space(uint8_t c) {  // str.isspace() for ASCII
    return c == ' ' || (c >= '\t' && c <= '\r') || (c >= 0x1c && c <= 0x1f);
}

struct Chunk {
    uint64_t begin = 0, end = 0;  // lines starting in [begin, end)
    // scan results
    uint64_t headers = 0, seq_bytes = 0, name_bytes = 0;
    uint64_t lead_headers = 0;  // headers before the chunk's first sequence byte
    bool bad_name = false;
    // placement
    uint64_t at0 = 0, rec0 = 0, name0 = 0;
};

}  // namespace

struct gk_fasta {
    int fd = -1;
    const uint8_t *map = nullptr;
    uint64_t size = 0;
    int threads = 1;
    std::vector<Chunk> chunks;
    uint64_t records = 0, seq_bytes = 0, name_bytes = 0;
    uint64_t no_dollar = 0;  // headers met while nothing was written (at == 0): no '$'
};

namespace {

// p is a line start: first byte, or after '\n', or after a '\r' not followed by '\n'
inline bool line_start(const uint8_t *b, uint64_t size, uint64_t p) {
    if (p == 0) return true;
    if (p >= size) return false;
    return b[p - 1] == '\n' || (b[p - 1] == '\r' && b[p] != '\n');
}

// calls fn(line_begin, line_end_excl_terminator) for every line starting in [c.begin, c.end)
template <typename F>
void for_lines(const uint8_t *b, uint64_t size, uint64_t begin, uint64_t end, F &&fn) {
    uint64_t p = begin;
    while (p < size && !line_start(b, size, p)) ++p;
    while (p < end && p < size) {
        // line end: the first '\n' or '\r' (memchr scans 16+ bytes per step)
        const void *nl = std::memchr(b + p, '\n', size - p);
        uint64_t q = nl ? (uint64_t)(static_cast<const uint8_t *>(nl) - b) : size;
        if (const void *cr = std::memchr(b + p, '\r', q - p)) q = (uint64_t)(static_cast<const uint8_t *>(cr) - b);
        fn(p, q);
        if (q >= size) break;
        p = q + ((b[q] == '\r' && q + 1 < size && b[q + 1] == '\n') ? 2 : 1);
    }
}

inline void trim(const uint8_t *b, uint64_t &s, uint64_t &e) {
    while (s < e && py_space(b[s])) ++s;
    while (e > s && py_space(b[e - 1])) --e;
}

// the header's name token: [s, e) of line[1:].strip().split()[0]; false if there is none
inline bool name_token(const uint8_t *b, uint64_t p, uint64_t q, uint64_t &s, uint64_t &e) {
    s = p + 1;
    while (s < q && py_space(b[s])) ++s;
    e = s;
    while (e < q && !py_space(b[e])) ++e;
    return e > s;
}

void scan_chunk(const uint8_t *b, uint64_t size, Chunk &c) {
    for_lines(b, size, c.begin, c.end, [&](uint64_t p, uint64_t q) {
        if (b[p] == '>' && p < q) {
            uint64_t s, e;
            if (!name_token(b, p, q, s, e)) c.bad_name = true;
            c.name_bytes += (e - s) + 1;
            if (c.seq_bytes == 0) ++c.lead_headers;
            ++c.headers;
        } else {
            uint64_t s = p, e = q;
            trim(b, s, e);
            c.seq_bytes += e - s;
        }
    });
}

const uint8_t *allowed_lut() {
    static uint8_t lut[256] = {0};
    static bool init = false;
    if (!init) {
        for (const char *a = "ACGTRYSWKMBDHVN$"; *a; ++a) lut[(uint8_t)*a] = 1;
        init = true;
    }
    return lut;
}

template <typename F>
void parallel_for(int threads, size_t n, F &&fn) {
    std::vector<std::thread> pool;
    const int t = (int)std::min<size_t>((size_t)std::max(threads, 1), n);
    for (int i = 0; i < t; ++i)
        pool.emplace_back([&, i] {
            for (size_t j = (size_t)i; j < n; j += (size_t)t) fn(j);
        });
    for (auto &th : pool) th.join();
}

}  // namespace

extern "C" int gk_fasta_open(const char *path, int n_threads, gk_fasta **out, uint64_t *num_records,
                             uint64_t *total_seq_len, uint64_t *names_bytes) {
    if (!path || !out) return GK_E_ARG;
    *out = nullptr;
    const int fd = ::open(path, O_RDONLY);
    if (fd < 0) return GK_E_IO;
    struct stat st;
    if (fstat(fd, &st) != 0) {
        ::close(fd);
        return GK_E_IO;
    }
    gk_fasta *f = new gk_fasta();
    f->fd = fd;
    f->size = (uint64_t)st.st_size;
    if (f->size) {
        void *m = mmap(nullptr, f->size, PROT_READ, MAP_PRIVATE, fd, 0);
        if (m == MAP_FAILED) {
            ::close(fd);
            delete f;
            return GK_E_IO;
        }
        madvise(m, f->size, MADV_SEQUENTIAL);
        f->map = static_cast<const uint8_t *>(m);
    }
    unsigned hw = std::thread::hardware_concurrency();
    f->threads = n_threads > 0 ? n_threads : (int)std::min(16u, std::max(1u, hw));
    uint64_t target = std::max<uint64_t>(64ull << 20, f->size / (uint64_t)(4 * f->threads) + 1);
    if (const char *e = std::getenv("GKM_FASTA_CHUNK")) target = std::max<uint64_t>(1, std::strtoull(e, nullptr, 10));  // tests
    for (uint64_t b = 0; b < f->size || f->chunks.empty(); b += target) {
        Chunk c;
        c.begin = b;
        c.end = std::min(f->size, b + target);
        f->chunks.push_back(c);
        if (f->size == 0) break;
    }
    parallel_for(f->threads, f->chunks.size(), [&](size_t i) { scan_chunk(f->map, f->size, f->chunks[i]); });
    // placement: records, names, sequence bytes and '$' before each chunk.  A header writes no
    // '$' while at == 0, i.e. before the file's first sequence byte.
    uint64_t at = 0, rec = 0, nb = 0;
    for (auto &c : f->chunks) {
        c.at0 = at;
        c.rec0 = rec;
        c.name0 = nb;
        const uint64_t skip = at == 0 ? (c.seq_bytes ? c.lead_headers : c.headers) : 0;
        f->no_dollar += skip;
        at += c.seq_bytes + c.headers - skip;
        rec += c.headers;
        nb += c.name_bytes;
    }
    for (auto &c : f->chunks) {
        f->records += c.headers;
        f->seq_bytes += c.seq_bytes;
        f->name_bytes += c.name_bytes;
    }
    if (num_records) *num_records = f->records;
    if (total_seq_len) *total_seq_len = f->seq_bytes;
    if (names_bytes) *names_bytes = f->name_bytes;
    *out = f;
    return GK_OK;
}

extern "C" int gk_fasta_fill(gk_fasta *f, uint8_t *sba, uint64_t sba_len, uint32_t *seg_starts, char *names,
                             uint8_t *bad_bytes) {
    if (!f) return GK_E_ARG;
    for (const auto &c : f->chunks)
        if (c.bad_name) return GK_E_FASTA_NAME;
    const uint8_t *b = f->map;
    const uint8_t *lut = allowed_lut();
    std::vector<std::vector<uint8_t>> bad(f->chunks.size(), std::vector<uint8_t>(256, 0));
    std::vector<uint8_t> overflow(f->chunks.size(), 0);
    parallel_for(f->threads, f->chunks.size(), [&](size_t i) {
        const Chunk &c = f->chunks[i];
        uint64_t at = c.at0, rec = c.rec0, nb = c.name0;
        uint8_t *badc = bad[i].data();
        for_lines(b, f->size, c.begin, c.end, [&](uint64_t p, uint64_t q) {
            if (overflow[i]) return;
            if (b[p] == '>' && p < q) {
                if (at != 0) {
                    if (at >= sba_len) {
                        overflow[i] = 1;
                        return;
                    }
                    sba[at++] = '$';
                }
                if (seg_starts) seg_starts[rec] = (uint32_t)at;
                ++rec;
                uint64_t s, e;
                name_token(b, p, q, s, e);
                if (names) {
                    std::memcpy(names + nb, b + s, e - s);
                    names[nb + (e - s)] = 0;
                }
                nb += (e - s) + 1;
            } else {
                uint64_t s = p, e = q;
                trim(b, s, e);
                if (at + (e - s) > sba_len) {
                    overflow[i] = 1;
                    return;
                }
                // upper-case copy (vectorised); the common all-ACGTN line skips the table check
                uint8_t *dst = sba + at;
                const uint8_t *src = b + s;
                const uint64_t len = e - s;
                uint8_t odd = 0;
                for (uint64_t j = 0; j < len; ++j) {
                    uint8_t ch = src[j];
                    ch = (uint8_t)(ch - (((uint8_t)(ch - 'a') < 26) ? 32 : 0));
                    dst[j] = ch;
                    odd |= (uint8_t)!(ch == 'A' || ch == 'C' || ch == 'G' || ch == 'T' || ch == 'N');
                }
                if (odd)
                    for (uint64_t j = 0; j < len; ++j) badc[dst[j]] |= (uint8_t)!lut[dst[j]];
                at += len;
            }
        });
    });
    for (size_t i = 0; i < f->chunks.size(); ++i) {
        if (overflow[i]) return GK_E_FASTA_LAYOUT;
        if (bad_bytes)
            for (int k = 0; k < 256; ++k) bad_bytes[k] |= bad[i][k];
    }
    // the reference's `assert at == sba_len` (sequence_collection.py:565-566)
    const uint64_t written = f->seq_bytes + f->records - f->no_dollar;
    if (written != sba_len) return GK_E_FASTA_LAYOUT;
    return GK_OK;
}

extern "C" void gk_fasta_close(gk_fasta *f) {
    if (!f) return;
    if (f->map) munmap(const_cast<uint8_t *>(f->map), f->size);
    if (f->fd >= 0) ::close(f->fd);
    delete f;
}

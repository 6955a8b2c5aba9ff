// Streaming FASTA reader and writer for the top-genes step (host code).
//
// Replaces the two Bio.SeqIO passes of TopGeneSelector
// (select_top_genes.py:108-127) and the Bio.SeqIO.write of
// select_top_and_save (select_top_genes_all.py:12-46). Transcript-ID parsing
// stays in Python (user regex, transcripts.py:69-126); this file only splits
// records, cleans sequences and copies the selected ones into the flat arrays
// rc_add_sample takes.
//
// Record semantics follow Bio.SeqIO's "fasta" parser: content before the first
// '>' line is ignored; the title is the header line without '>' and trailing
// whitespace; the id is the title's first whitespace-separated token; the
// sequence is the concatenation of the record's lines, each right-stripped,
// with ' ' and '\r' removed.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rcgpu.h"

int rcg_fail(int code, const std::string &msg);   // engine.hip

struct rc_fasta {
    const char *data = nullptr;
    size_t size = 0;
    std::vector<uint64_t> title_off;   // [n] title start in data
    std::vector<uint32_t> title_len;   // [n]
    std::vector<uint64_t> body_off;    // [n + 1] body byte range in data
    std::vector<uint64_t> seq_len;     // [n] cleaned sequence length
};

namespace {

inline bool is_ws(char c)
{
    return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f';
}

// end of the right-stripped line [b, e)
inline const char *rstrip(const char *b, const char *e)
{
    while (e > b && is_ws(e[-1])) e--;
    return e;
}

// Walk the body [b, e) line by line, calling f(ptr, n) for every run of kept
// sequence characters.
template <class F>
void body_runs(const char *b, const char *e, F &&f)
{
    while (b < e) {
        const char *nl = static_cast<const char *>(memchr(b, '\n', (size_t)(e - b)));
        const char *le = nl ? nl : e;
        const char *re = rstrip(b, le);
        const char *p = b;
        while (p < re) {
            const char *q = p;
            while (q < re && *q != ' ' && *q != '\r') q++;
            if (q > p) f(p, (size_t)(q - p));
            p = q + 1;
        }
        b = nl ? nl + 1 : e;
    }
}

// body i: [body_off[i], the '>' of record i + 1)
inline uint64_t body_end(const rc_fasta *f, size_t i)
{
    return i + 1 < f->title_off.size() ? f->title_off[i + 1] - 1 : (uint64_t)f->size;
}

}  // namespace

extern "C" {

int rc_fasta_open(const char *path, rc_fasta **out)
{
    if (!path || !out) return rcg_fail(RC_E_ARG, "null argument");
    *out = nullptr;
    const int fd = open(path, O_RDONLY);
    if (fd < 0) return rcg_fail(RC_E_ARG, std::string("cannot open ") + path);
    struct stat stt;
    if (fstat(fd, &stt) != 0) {
        close(fd);
        return rcg_fail(RC_E_ARG, std::string("cannot stat ") + path);
    }
    rc_fasta *f = new rc_fasta;
    f->size = (size_t)stt.st_size;
    if (f->size) {
        void *m = mmap(nullptr, f->size, PROT_READ, MAP_PRIVATE, fd, 0);
        if (m == MAP_FAILED) {
            close(fd);
            delete f;
            return rcg_fail(RC_E_NOMEM, std::string("cannot map ") + path);
        }
        madvise(m, f->size, MADV_SEQUENTIAL);
        f->data = static_cast<const char *>(m);
    }
    close(fd);
    const char *d = f->data, *end = f->data + f->size;
    // record starts: '>' at the beginning of a line
    const char *p = d;
    while (p < end) {
        const char *nl = static_cast<const char *>(memchr(p, '\n', (size_t)(end - p)));
        const char *le = nl ? nl : end;
        if (*p == '>') {
            f->title_off.push_back((uint64_t)(p + 1 - d));
            f->title_len.push_back((uint32_t)(rstrip(p + 1, le) - (p + 1)));
            f->body_off.push_back((uint64_t)((nl ? nl + 1 : end) - d));
        }
        p = nl ? nl + 1 : end;
    }
    const size_t n = f->title_off.size();
    f->body_off.push_back((uint64_t)f->size);
    f->seq_len.assign(n, 0);
    for (size_t i = 0; i < n; i++) {
        uint64_t L = 0;
        body_runs(d + f->body_off[i], d + body_end(f, i), [&](const char *, size_t k) { L += k; });
        f->seq_len[i] = L;
    }
    *out = f;
    return RC_OK;
}

int rc_fasta_close(rc_fasta *f)
{
    if (!f) return RC_OK;
    if (f->data) munmap(const_cast<char *>(f->data), f->size);
    delete f;
    return RC_OK;
}

int rc_fasta_info(const rc_fasta *f, uint64_t *n_records, uint64_t *n_bases, uint64_t *title_bytes)
{
    if (!f) return rcg_fail(RC_E_ARG, "null fasta handle");
    uint64_t nb = 0, tb = 0;
    for (size_t i = 0; i < f->seq_len.size(); i++) {
        nb += f->seq_len[i];
        tb += f->title_len[i];
    }
    if (n_records) *n_records = f->seq_len.size();
    if (n_bases) *n_bases = nb;
    if (title_bytes) *title_bytes = tb;
    return RC_OK;
}

int rc_fasta_titles(const rc_fasta *f, char *buf, uint64_t *offsets, uint64_t *seq_lens)
{
    if (!f || !buf || !offsets) return rcg_fail(RC_E_ARG, "null argument");
    uint64_t w = 0;
    const size_t n = f->seq_len.size();
    for (size_t i = 0; i < n; i++) {
        offsets[i] = w;
        memcpy(buf + w, f->data + f->title_off[i], f->title_len[i]);
        w += f->title_len[i];
        if (seq_lens) seq_lens[i] = f->seq_len[i];
    }
    offsets[n] = w;
    return RC_OK;
}

int rc_fasta_select(const rc_fasta *f, const uint8_t *keep, uint8_t *seq, uint64_t *tx_offsets)
{
    if (!f || !seq || !tx_offsets) return rcg_fail(RC_E_ARG, "null argument");
    uint64_t w = 0, k = 0;
    for (size_t i = 0; i < f->seq_len.size(); i++) {
        if (keep && !keep[i]) continue;
        tx_offsets[k++] = w;
        body_runs(f->data + f->body_off[i], f->data + body_end(f, i), [&](const char *p, size_t m) {
            memcpy(seq + w, p, m);
            w += m;
        });
    }
    tx_offsets[k] = w;
    return RC_OK;
}

int rc_fasta_write(const rc_fasta *f, const uint8_t *keep, const char *path, int32_t width)
{
    if (!f || !path) return rcg_fail(RC_E_ARG, "null argument");
    if (width <= 0) return rcg_fail(RC_E_ARG, "line width must be positive");
    FILE *o = fopen(path, "wb");
    if (!o) return rcg_fail(RC_E_ARG, std::string("cannot create ") + path);
    std::vector<char> buf(1 << 20);
    setvbuf(o, buf.data(), _IOFBF, buf.size());
    bool ok = true;
    for (size_t i = 0; i < f->seq_len.size() && ok; i++) {
        if (keep && !keep[i]) continue;
        ok &= fputc('>', o) != EOF;
        ok &= fwrite(f->data + f->title_off[i], 1, f->title_len[i], o) == f->title_len[i];
        ok &= fputc('\n', o) != EOF;
        int col = 0;
        body_runs(f->data + f->body_off[i], f->data + body_end(f, i), [&](const char *p, size_t m) {
            while (m) {
                const size_t take = std::min<size_t>(m, (size_t)(width - col));
                ok &= fwrite(p, 1, take, o) == take;
                p += take;
                m -= take;
                col += (int)take;
                if (col == width) {
                    ok &= fputc('\n', o) != EOF;
                    col = 0;
                }
            }
        });
        if (col) ok &= fputc('\n', o) != EOF;
    }
    ok &= fclose(o) == 0;
    if (!ok) return rcg_fail(RC_E_ARG, std::string("write failed: ") + path);
    return RC_OK;
}

}  // extern "C"

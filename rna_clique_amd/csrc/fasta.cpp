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
    std::vector<char> clean;           // every record's cleaned sequence, back to back
    std::vector<uint64_t> seq_off;     // [n + 1] record i's sequence in clean
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
        const size_t n = (size_t)(re - b);
        // the usual line holds neither ' ' nor '\r': one run
        if (n && !memchr(b, ' ', n) && !memchr(b, '\r', n)) {
            f(b, n);
            b = nl ? nl + 1 : e;
            continue;
        }
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
    // clean every sequence once; select and write copy from here
    f->seq_len.assign(n, 0);
    f->seq_off.assign(n + 1, 0);
    f->clean.resize(f->size);
    char *c = f->clean.data();
    uint64_t w = 0;
    for (size_t i = 0; i < n; i++) {
        f->seq_off[i] = w;
        body_runs(d + f->body_off[i], d + body_end(f, i), [&](const char *q, size_t k) {
            memcpy(c + w, q, k);
            w += k;
        });
        f->seq_len[i] = w - f->seq_off[i];
    }
    f->seq_off[n] = w;
    f->clean.resize(w);
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

// rnaSPAdes ids under the default pattern of transcripts.py (the reference's
// default_gene_re, transcripts.py:8): re.search(r"^.*cov_([0-9]+(?:\.[0-9]+))
// _g([0-9]+)_i([0-9]+)", id) on the record id (the title's first whitespace
// token). The greedy ".*" makes the match the LAST position where the tail
// pattern matches; its digit runs are maximal (each is followed by a fixed
// non-digit or, for the isoform, by nothing). Coverage goes through strtod
// (correctly rounded, as Python's float()). A record this cannot decide --
// a non-ASCII title (Python splits ids on Unicode whitespace too), no match,
// a gene or isoform beyond 18 digits -- counts in *n_undecided and gets
// zeros; the caller then parses every id with the regex instead.
int rc_fasta_parse_rnaspades(const rc_fasta *f, double *cov, int64_t *gene, int64_t *iso, uint64_t *n_undecided)
{
    if (!f || !cov || !gene || !iso || !n_undecided) return rcg_fail(RC_E_ARG, "null argument");
    const size_t n = f->seq_len.size();
    uint64_t bad = 0;
    auto digits = [](const char *p, const char *e) {
        const char *q = p;
        while (q < e && *q >= '0' && *q <= '9') q++;
        return q;
    };
    for (size_t i = 0; i < n; i++) {
        const char *t = f->data + f->title_off[i];
        const char *const te = t + f->title_len[i];
        bool ascii = true;
        for (const char *p = t; p < te; p++)
            if ((unsigned char)*p >= 0x80) ascii = false;
        auto split_ws = [](char c) { return is_ws(c) || (c >= '\x1c' && c <= '\x1f'); };
        while (t < te && split_ws(*t)) t++;   // str.split() drops leading whitespace
        const char *e = t;
        while (e < te && !split_ws(*e)) e++;
        cov[i] = 0;
        gene[i] = iso[i] = 0;
        bool ok = false;
        if (ascii) {
            for (ptrdiff_t jo = (e - t) - 4; jo >= 0 && !ok; jo--) {
                const char *j = t + jo;
                if (memcmp(j, "cov_", 4) != 0) continue;
                const char *c0 = j + 4, *c1 = digits(c0, e);
                if (c1 == c0 || c1 >= e || *c1 != '.') continue;
                const char *c2 = digits(c1 + 1, e);
                if (c2 == c1 + 1 || e - c2 < 2 || c2[0] != '_' || c2[1] != 'g') continue;
                const char *g0 = c2 + 2, *g1 = digits(g0, e);
                if (g1 == g0 || e - g1 < 2 || g1[0] != '_' || g1[1] != 'i') continue;
                const char *i0 = g1 + 2, *i1 = digits(i0, e);
                if (i1 == i0) continue;
                if (g1 - g0 > 18 || i1 - i0 > 18) break;   // undecided
                const std::string cs(c0, c2);
                cov[i] = strtod(cs.c_str(), nullptr);
                int64_t gv = 0, iv = 0;
                for (const char *p = g0; p < g1; p++) gv = gv * 10 + (*p - '0');
                for (const char *p = i0; p < i1; p++) iv = iv * 10 + (*p - '0');
                gene[i] = gv;
                iso[i] = iv;
                ok = true;
            }
        }
        if (!ok) bad++;
    }
    *n_undecided = bad;
    return RC_OK;
}

int rc_fasta_select(const rc_fasta *f, const uint8_t *keep, uint8_t *seq, uint64_t *tx_offsets)
{
    if (!f || !seq || !tx_offsets) return rcg_fail(RC_E_ARG, "null argument");
    const size_t n = f->seq_len.size();
    const char *c = f->clean.data();
    if (!keep) {
        if (n) memcpy(seq, c, f->seq_off[n]);
        for (size_t i = 0; i <= n; i++) tx_offsets[i] = f->seq_off[i];
        return RC_OK;
    }
    uint64_t w = 0, k = 0;
    for (size_t i = 0; i < n; i++) {
        if (!keep[i]) continue;
        tx_offsets[k++] = w;
        memcpy(seq + w, c + f->seq_off[i], f->seq_len[i]);
        w += f->seq_len[i];
    }
    tx_offsets[k] = w;
    return RC_OK;
}

int rc_fasta_write(const rc_fasta *f, const uint8_t *keep, const char *path, int32_t width)
{
    if (!f || !path) return rcg_fail(RC_E_ARG, "null argument");
    if (width <= 0) return rcg_fail(RC_E_ARG, "line width must be positive");
    // the whole file in one buffer, one write
    const size_t n = f->seq_len.size();
    uint64_t bytes = 0;
    for (size_t i = 0; i < n; i++) {
        if (keep && !keep[i]) continue;
        const uint64_t L = f->seq_len[i];
        bytes += 2 + f->title_len[i] + L + (L + (uint64_t)width - 1) / (uint64_t)width;
    }
    std::vector<char> out(bytes);
    char *o = out.data();
    const char *c = f->clean.data();
    for (size_t i = 0; i < n; i++) {
        if (keep && !keep[i]) continue;
        *o++ = '>';
        memcpy(o, f->data + f->title_off[i], f->title_len[i]);
        o += f->title_len[i];
        *o++ = '\n';
        const char *p = c + f->seq_off[i];
        for (uint64_t L = f->seq_len[i]; L;) {
            const uint64_t take = std::min<uint64_t>(L, (uint64_t)width);
            memcpy(o, p, take);
            o += take;
            *o++ = '\n';
            p += take;
            L -= take;
        }
    }
    FILE *fo = fopen(path, "wb");
    if (!fo) return rcg_fail(RC_E_ARG, std::string("cannot create ") + path);
    bool ok = fwrite(out.data(), 1, (size_t)(o - out.data()), fo) == (size_t)(o - out.data());
    ok &= fclose(fo) == 0;
    if (!ok) return rcg_fail(RC_E_ARG, std::string("write failed: ") + path);
    return RC_OK;
}

}  // extern "C"

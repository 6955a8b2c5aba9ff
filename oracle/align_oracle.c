/*
 * CPU oracle for the alignment stage (the NCBI BLAST+ `blastn` replacement).
 * TEST INFRASTRUCTURE ONLY: loaded by tests/, by __graft_entry__.smoke() and by
 * bench.py's cpu_baseline leg, as the checker. The product never links it.
 *
 * PARITY STATUS: BLAST+ is absent from this image and simple_blast's flags are
 * not visible in /root/reference, so this file restates the
 * *published* megablast algorithm as an exact specification ("RC-megablast v1")
 * that the HIP kernel must reproduce bit for bit. Against BLAST itself the
 * alignment stage is "parity unpinned"; see DESIGN.md §Oracle.
 *
 * Reference call sites this replaces:
 *   TabularBlastnSearch(query=path2, subject=path1, evalue, additional_columns=
 *   ["gaps","nident","sstrand"])                      find_homologs.py:124,209
 *   BlastDBCache.makedb                              find_all_pairs.py:120-132
 *
 * Spec (one directed search: query sample Q against subject sample T):
 *  1. Words. w = 16 (index word), W = word_size (28 = megablast default),
 *     stride s = W - w + 1. Query positions p with p % s == 0 on the oriented
 *     query (plus strand = q, minus strand = revcomp(q)); subject positions at
 *     every offset. A query word is usable unless its window holds a non-ACGT
 *     base or a DUST-masked base (1b).
 * 1b. DUST (blastn's default query filter, -dust 20 64 1, applied as a soft
 *     mask: it removes query words, extension runs through masked bases).
 *     Symmetric DUST (Morgulis et al. 2006) on the forward transcript, each
 *     maximal ACGT run on its own: an interval x of 3..window bases with
 *     n >= 3 triplets, r(x) = sum over the 64 triplets of c(c-1)/2, is
 *     *perfect* iff 10 r(x) > level (n - 1) and r(x)/(n-1) >= r(y)/(n_y-1)
 *     for every perfect interval y inside x. Masked bases = the union of the
 *     perfect intervals, plus gaps shorter than `linker` between them. The
 *     minus strand uses the same bases, reversed. (dust_run below evaluates
 *     this with the windowed bookkeeping of the published algorithm.)
 *  2. Seeds. A word hit (p, subject tx t, offset o) lies on a maximal exact run
 *     [x, e) of its diagonal (non-ACGT never matches). It is canonical iff no
 *     usable query word p' with x <= p' < p exists, i.e. p - x < D(p), D(p) =
 *     distance to the previous usable word (s when that word is usable; with
 *     no DUST always s, since a run never covers a non-ACGT base); a canonical
 *     hit with e - x >= W is a seed (x, y = x + o - p, len = e - x). Every exact
 *     match of length >= W holding a usable word yields exactly one seed.
 *  3. Per (query tx, strand, subject tx) seeds are sorted by (x, y). Each seed
 *     not contained in an HSP found so far (box containment) is extended left
 *     and right with the greedy X-drop algorithm below (at most 8 HSPs).
 *  4. Greedy X-drop (Zhang et al. 2000, non-affine, megablast reward 1 /
 *     penalty -2 / linear gap 2.5): in half-score units match +2, mismatch -4,
 *     gap -5, so score(i, j, d) = i + j - 6d. Band of 64 diagonals around the
 *     seed diagonal, X = xdrop_half (108 = 100 bits, BLAST's final x-dropoff).
 * 4b. Canonical roles. The greedy step breaks ties between moves (mismatch,
 *     then insertion, then deletion) and between diagonals (lowest) in the
 *     order of its two sequences, so run with query and subject swapped it can
 *     return a different (equally scored) end point or gap count. Every
 *     extension is therefore evaluated with the LOWER-numbered sample's
 *     sequence in the first role (i, the insertion side), whichever sample is
 *     the query of the directed search; the walk itself (the base pairs it
 *     visits, outward from the seed) is the same in both directions. Then the
 *     extension of a given seed is one geometric result in both directed
 *     searches of a pair, and the GPU can share it between them (DESIGN.md
 *     §4). Each search keeps its own seeds, seed order, containment, MAX_HSP,
 *     purge and e-value cut. BLAST's own tie-breaking is unpinned here
 *     (BLAST+ is absent), so this restates no departure that could be
 *     checked; it fixes the one arbitrary choice the restatement had.
 *  5. Purge HSPs sharing a start or end point (keep higher score, then earlier),
 *     keep HSPs whose e-value <= evalue (Karlin-Altschul, lambda 1.28, K 0.46,
 *     H 0.85, alpha 1.5, beta -2 for 1/-2 linear; BLAST length adjustment).
 *  5b. Symmetry: both directed searches of a sample pair find the same seed set
 *     (every maximal exact run >= W), so candidates are extended once, with the
 *     lower-numbered sample as query; the other direction reports the mirror
 *     images under its own e-value cut. (BLAST runs the two searches
 *     independently; this is where the restatement departs from it.)
 *  6. Bitscore as BLAST prints it (integer-truncated above 99.9) in tenths.
 */
#include <limits.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define W16 16
#define BAND 64
#define BAND_LO (-32)
#define MAX_HSP 8
#define DMAX 4096

typedef struct {
    uint32_t q_tx, s_tx;
    int32_t qstart, qend, sstart, send;
    int32_t length, nident, mismatch, gaps, gapopen, score_half, bits10, strand;
    double evalue;
} orc_hsp;

typedef struct {
    int32_t word_size;
    int32_t xdrop_half;
    double evalue;
    int32_t symmetric;     /* 1: spec 5b (mirror), 0: two independent directed searches */
    int32_t dust_level;    /* symmetric DUST on the query (spec 1b); 0 = off */
    int32_t dust_window;
    int32_t dust_linker;
} orc_params;

/* Karlin-Altschul parameters for reward 1 / penalty -2, linear gaps
 * (BLAST's blastn table entry {0,0,1.28,0.46,0.85,1.5,-2,0.45}). */
static const double KA_LAMBDA = 1.28, KA_K = 0.46, KA_ALPHA = 1.5, KA_BETA = -2.0;

static uint8_t code_of(char c)
{
    switch (c) {
    case 'A': case 'a': return 0;
    case 'C': case 'c': return 1;
    case 'G': case 'g': return 2;
    case 'T': case 't': return 3;
    default: return 4;
    }
}

/* ---------------- statistics (host-side in the product too) ---------------- */

/* BLAST_ComputeLengthAdjustment (restated from the published BLAST+ algorithm). */
static int32_t length_adjustment(double m, double n, double N)
{
    const double logK = log(KA_K), adl = KA_ALPHA / KA_LAMBDA, beta = KA_BETA;
    double ell = 0, ss, ell_min = 0, ell_max, ell_next = 0;
    int converged = 0, i;
    {
        double a = N, mb = m * N + n, c = n * m - (m > n ? m : n) / KA_K;
        if (c < 0) return 0;
        ell_max = 2 * c / (mb + sqrt(mb * mb - 4 * a * c));
    }
    for (i = 1; i <= 20; i++) {
        double ell_bar;
        ell = ell_next;
        ss = (m - ell) * (n - N * ell);
        ell_bar = adl * (logK + log(ss)) + beta;
        if (ell_bar >= ell) {
            ell_min = ell;
            if (ell_bar - ell_min <= 1.0) { converged = 1; break; }
            if (ell_min == ell_max) break;
        } else {
            ell_max = ell;
        }
        if (ell_min <= ell_bar && ell_bar <= ell_max) ell_next = ell_bar;
        else ell_next = (i == 1) ? ell_max : (ell_min + ell_max) / 2;
    }
    if (converged) {
        int32_t adj = (int32_t)ell_min;
        ell = ceil(ell_min);
        if (ell <= ell_max) {
            ss = (m - ell) * (n - N * ell);
            if (adl * (logK + log(ss)) + beta >= ell) adj = (int32_t)ell;
        }
        return adj;
    }
    return (int32_t)ell_min;
}

static double search_space(int64_t qlen, int64_t dblen, int64_t dbn)
{
    int32_t ell = length_adjustment((double)qlen, (double)dblen, (double)dbn);
    double mq = (double)(qlen - ell), nd = (double)(dblen - dbn * (int64_t)ell);
    if (mq < 1) mq = 1;
    if (nd < 1) nd = 1;
    return mq * nd;
}

static double evalue_of(double ss, int32_t score_half)
{
    return ss * KA_K * exp(-KA_LAMBDA * (score_half / 2.0));
}

/* smallest half-unit score whose e-value passes the cutoff */
static int32_t score_threshold(double ss, double cutoff)
{
    int32_t lo = 0, hi = 1 << 26;
    if (evalue_of(ss, hi) > cutoff) return hi;
    while (lo < hi) {
        int32_t mid = lo + (hi - lo) / 2;
        if (evalue_of(ss, mid) <= cutoff) hi = mid; else lo = mid + 1;
    }
    return lo;
}

/* CAlignFormatUtil::GetScoreString bit-score formatting, in tenths */
static int32_t bits10_of(int32_t score_half)
{
    double bits = (KA_LAMBDA * (score_half / 2.0) - log(KA_K)) / log(2.0);
    char buf[64];
    if (bits > 99999) {
        snprintf(buf, sizeof buf, "%5.3le", bits);
        return (int32_t)llround(strtod(buf, NULL) * 10.0);
    } else if (bits > 99.9) {
        return (int32_t)((long)bits) * 10;
    }
    snprintf(buf, sizeof buf, "%4.1lf", bits);
    return (int32_t)llround(strtod(buf, NULL) * 10.0);
}

/* ---------------- sequences ---------------- */

typedef struct {
    const uint8_t *c;   /* codes 0..4 of the whole concatenation */
    const uint64_t *tx_start;
    const int32_t *tx_sample;
    uint32_t n_tx;
} seqdb;

static inline uint8_t qbase(const uint8_t *codes, uint64_t start, int32_t len, int strand, int32_t u)
{
    if (!strand) return codes[start + u];
    uint8_t b = codes[start + (uint64_t)(len - 1 - u)];
    return b < 4 ? (uint8_t)(3 - b) : 4;
}

/* ---------------- DUST (spec 1b) ---------------- */

/* One maximal ACGT run s[0, n): mask[u] = 1 for every base of a perfect
 * interval. Window bookkeeping of the published symmetric DUST: the last
 * `window` bases as a queue of triplets with counts cw (rw = r of the whole
 * window) and, for the longest suffix whose triplet counts all stay <= 2
 * level / 10, counts cv (rv, L triplets; no interval inside that suffix can
 * be perfect). Ending at each base, the suffixes longer than L are tried from
 * shortest to longest against the best ratio of the perfect intervals they
 * contain. Perfect intervals are kept per start (best ratio, furthest end):
 * that is all the containment test and the union need. */
static void dust_run(const uint8_t *s, int32_t n, int T, int W, uint8_t *mask)
{
    int cw[64], cv[64], c[64];
    int q[256], qh = 0, qn = 0;                    /* triplet queue (ring), oldest at qh */
    int sr[256], sl[256], sf[256];                 /* per start (mod W): best ratio r/l, furthest end */
    int rw = 0, rv = 0, L = 0;
    memset(cw, 0, sizeof cw);
    memset(cv, 0, sizeof cv);
    for (int k = 0; k < W; k++) sf[k] = -1;
    for (int32_t i = 2; i <= n; i++) {
        const int32_t wstart = (i < n) ? (i + 1 - W > 0 ? i + 1 - W : 0) : n;
        /* perfect intervals whose start left the window are final: one start
         * leaves per base (wstart - 1), at the end of the run all of them */
        for (int32_t st = wstart - 1; st >= 0 && st >= (i < n ? wstart - 1 : wstart - W); st--) {
            const int k = st % W;
            if (sf[k] < 0) continue;
            for (int32_t u = st; u < sf[k]; u++) mask[u] = 1;
            sf[k] = -1;
        }
        if (i == n) break;
        const int t = s[i - 2] * 16 + s[i - 1] * 4 + s[i];
        if (qn == W - 2) {   /* drop the oldest triplet */
            const int o = q[qh];
            qh = (qh + 1) % 256;
            qn--;
            rw -= --cw[o];
            if (L > qn) { L--; rv -= --cv[o]; }
        }
        q[(qh + qn) % 256] = t;
        qn++;
        L++;
        rw += cw[t]++;
        rv += cv[t]++;
        if (cv[t] * 10 > 2 * T) {   /* shrink the suffix past the previous copy of t */
            int o;
            do {
                o = q[(qh + qn - L) % 256];
                rv -= --cv[o];
                L--;
            } while (o != t);
        }
        if (rw * 10 <= L * T) continue;
        /* suffixes longer than L, shortest first: triplet index j .. qn-1,
         * bases [wstart + j, i + 1) */
        memcpy(c, cv, sizeof c);
        int r = rv, mr = 0, ml = 0;
        for (int32_t st = wstart + qn - L; st <= i; st++) {   /* perfect intervals inside the L-suffix */
            const int k = st % W;
            if (st < n && sf[k] >= 0 && (mr == 0 || sr[k] * ml > mr * sl[k])) { mr = sr[k]; ml = sl[k]; }
        }
        for (int j = qn - L - 1; j >= 0; j--) {
            const int tt = q[(qh + j) % 256];
            r += c[tt]++;
            const int l = qn - j - 1;
            const int32_t st = wstart + j;
            const int k = st % W;
            if (sf[k] >= 0 && (mr == 0 || sr[k] * ml > mr * sl[k])) { mr = sr[k]; ml = sl[k]; }
            if (r * 10 > T * l && (mr == 0 || r * ml >= mr * l)) {
                if (sf[k] < 0 || r * sl[k] > sr[k] * l) { sr[k] = r; sl[k] = l; }
                if (sf[k] < i + 1) sf[k] = i + 1;
                mr = r;
                ml = l;
            }
        }
    }
}

/* mask[0, L) of one transcript (codes c): DUST on every ACGT run, then gaps
 * shorter than `linker` between masked bases filled */
static void dust_tx(const uint8_t *c, int32_t L, int T, int W, int linker, uint8_t *mask)
{
    memset(mask, 0, (size_t)(L > 0 ? L : 1));
    for (int32_t i = 0; i < L;) {
        while (i < L && c[i] > 3) i++;
        const int32_t a = i;
        while (i < L && c[i] <= 3) i++;
        if (i - a >= 3) dust_run(c + a, i - a, T, W, mask + a);
    }
    int32_t last = -1;   /* end of the last masked base run */
    for (int32_t u = 0; u < L; u++) {
        if (!mask[u]) continue;
        if (last >= 0 && u > last && u - last < linker)
            for (int32_t v = last; v < u; v++) mask[v] = 1;
        while (u < L && mask[u]) u++;
        last = u;
    }
}

/* exported for tests: the DUST mask of one code sequence */
void orc_dust(const uint8_t *codes, int32_t L, int32_t level, int32_t window, int32_t linker, uint8_t *mask)
{
    dust_tx(codes, L, level, window, linker, mask);
}

/* ---------------- index of one subject sample ---------------- */

typedef struct { uint32_t key, tx, off; } ientry;

typedef struct { ientry *e; uint64_t n; } sindex;

static void build_index(const seqdb *db, int32_t sample, sindex *ix)
{
    uint64_t cap = 0, n = 0;
    uint32_t t;
    for (t = 0; t < db->n_tx; t++)
        if (db->tx_sample[t] == sample) {
            int64_t L = (int64_t)(db->tx_start[t + 1] - db->tx_start[t]);
            if (L >= W16) cap += (uint64_t)(L - W16 + 1);
        }
    ientry *a = (ientry *)malloc((cap ? cap : 1) * sizeof(ientry));
    ientry *b = (ientry *)malloc((cap ? cap : 1) * sizeof(ientry));
    for (t = 0; t < db->n_tx; t++) {
        if (db->tx_sample[t] != sample) continue;
        uint64_t s0 = db->tx_start[t];
        int64_t L = (int64_t)(db->tx_start[t + 1] - s0);
        for (int64_t o = 0; o + W16 <= L; o++) {
            uint32_t key = 0;
            int ok = 1;
            for (int k = 0; k < W16; k++) {
                uint8_t c = db->c[s0 + o + k];
                if (c > 3) { ok = 0; break; }
                key |= (uint32_t)c << (2 * k);
            }
            if (!ok) continue;
            a[n].key = key; a[n].tx = t; a[n].off = (uint32_t)o; n++;
        }
    }
    /* stable LSD radix sort on key: entries stay in (tx, off) order per key */
    for (int pass = 0; pass < 4; pass++) {
        uint64_t cnt[257];
        memset(cnt, 0, sizeof cnt);
        for (uint64_t i = 0; i < n; i++) cnt[((a[i].key >> (8 * pass)) & 255) + 1]++;
        for (int k = 0; k < 256; k++) cnt[k + 1] += cnt[k];
        for (uint64_t i = 0; i < n; i++) b[cnt[(a[i].key >> (8 * pass)) & 255]++] = a[i];
        ientry *tmp = a; a = b; b = tmp;
    }
    free(b);
    ix->e = a;
    ix->n = n;
}

static uint64_t lower_key(const sindex *ix, uint32_t key)
{
    uint64_t lo = 0, hi = ix->n;
    while (lo < hi) {
        uint64_t mid = (lo + hi) / 2;
        if (ix->e[mid].key < key) lo = mid + 1; else hi = mid;
    }
    return lo;
}

/* ---------------- greedy X-drop extension ---------------- */

typedef struct { int32_t score, i, j, d, g, o; } ext_result;

/* A(u) / B(u): base u of the two extension sequences (u < alen / blen). */
typedef struct {
    const uint8_t *codes;
    uint64_t start;
    int32_t len;
    int strand;    /* oriented transcript: 0 = forward, 1 = revcomp */
    int reverse;   /* walk backwards from `from` */
    int32_t from;  /* first oriented position walked */
} walker;

static inline uint8_t wbase(const walker *w, int32_t u)
{
    int32_t pos = w->reverse ? (w->from - u) : (w->from + u);
    return qbase(w->codes, w->start, w->len, w->strand, pos);
}

static int32_t slide(const walker *A, int32_t ia, const walker *B, int32_t ib, int32_t maxn)
{
    int32_t n = 0;
    while (n < maxn) {
        uint8_t a = wbase(A, ia + n), b = wbase(B, ib + n);
        if (a > 3 || b > 3 || a != b) break;
        n++;
    }
    return n;
}

static ext_result greedy_ext(const walker *A, int32_t alen, const walker *B, int32_t blen, int32_t X)
{
    int32_t R[BAND], G[BAND], O[BAND], E[BAND];
    int32_t Rn[BAND], Gn[BAND], On[BAND], En[BAND];
    int32_t sc[BAND];
    ext_result best;
    int32_t k0 = -BAND_LO;  /* lane of diagonal 0 */
    for (int l = 0; l < BAND; l++) R[l] = -1, G[l] = O[l] = E[l] = 0;
    {
        int32_t m = alen < blen ? alen : blen;
        R[k0] = slide(A, 0, B, 0, m);
    }
    best.score = 2 * R[k0]; best.i = best.j = R[k0]; best.d = best.g = best.o = 0;
    for (int32_t d = 1; d <= DMAX; d++) {
        int any = 0;
        for (int l = 0; l < BAND; l++) {
            int32_t k = l + BAND_LO;
            int32_t ni = -1, ng = 0, no = 0, ne = 0;
            /* mismatch from k */
            if (R[l] >= 0 && R[l] < alen && R[l] - k < blen) {
                ni = R[l] + 1; ng = G[l]; no = O[l]; ne = 0;
            }
            /* insertion (A advances) from k-1 */
            if (l > 0 && R[l - 1] >= 0 && R[l - 1] < alen) {
                int32_t c = R[l - 1] + 1;
                if (c > ni) { ni = c; ng = G[l - 1] + 1; no = O[l - 1] + (E[l - 1] == 1 ? 0 : 1); ne = 1; }
            }
            /* deletion (B advances) from k+1 */
            if (l < BAND - 1 && R[l + 1] >= 0 && R[l + 1] - (k + 1) < blen) {
                int32_t c = R[l + 1];
                if (c > ni) { ni = c; ng = G[l + 1] + 1; no = O[l + 1] + (E[l + 1] == 2 ? 0 : 1); ne = 2; }
            }
            if (ni >= 0 && ni - k >= 0) {
                int32_t ja = ni - k;
                int32_t m = alen - ni < blen - ja ? alen - ni : blen - ja;
                int32_t s = slide(A, ni, B, ja, m);
                if (s > 0) { ni += s; ne = 0; }
                int32_t score = 2 * ni - k - 6 * d;
                if (score < best.score - X) ni = -1;
                sc[l] = score;
            } else {
                ni = -1;
            }
            Rn[l] = ni; Gn[l] = ng; On[l] = no; En[l] = ne;
            if (ni >= 0) any = 1;
        }
        /* best update uses this step's live diagonals; ties -> smallest k */
        {
            int bl = -1;
            for (int l = 0; l < BAND; l++)
                if (Rn[l] >= 0 && (bl < 0 || sc[l] > sc[bl])) bl = l;
            if (bl >= 0 && sc[bl] > best.score) {
                int32_t k = bl + BAND_LO;
                best.score = sc[bl]; best.i = Rn[bl]; best.j = Rn[bl] - k;
                best.d = d; best.g = Gn[bl]; best.o = On[bl];
            }
        }
        memcpy(R, Rn, sizeof R); memcpy(G, Gn, sizeof G); memcpy(O, On, sizeof O); memcpy(E, En, sizeof E);
        if (!any) break;
    }
    return best;
}

/* ---------------- one directed search ---------------- */

typedef struct { uint32_t tx; int32_t x, y, len; } seed;

typedef struct { int32_t qa, qb, sa, sb, score, d, g, o, nident; } hsp_box;

static int seed_cmp(const void *pa, const void *pb)
{
    const seed *a = (const seed *)pa, *b = (const seed *)pb;
    if (a->tx != b->tx) return a->tx < b->tx ? -1 : 1;
    if (a->x != b->x) return a->x < b->x ? -1 : 1;
    if (a->y != b->y) return a->y < b->y ? -1 : 1;
    return 0;
}

typedef struct { orc_hsp *v; uint64_t n, cap; } hsp_vec;

static void push_hsp(hsp_vec *hv, const orc_hsp *h)
{
    if (hv->n == hv->cap) {
        hv->cap = hv->cap ? 2 * hv->cap : 1024;
        hv->v = (orc_hsp *)realloc(hv->v, hv->cap * sizeof(orc_hsp));
    }
    hv->v[hv->n++] = *h;
}

/* A kept (purged) HSP of a candidate, before any e-value cut. */
typedef struct {
    uint32_t qtx, stx;
    int32_t strand, hidx;      /* hidx: index in the candidate's HSP list */
    int32_t qa, qb, sa, sb, score, d, g, o, nident, Lq, Lt;
} core_hsp;

typedef struct { core_hsp *v; uint64_t n, cap; } core_vec;

static void push_core(core_vec *cv, const core_hsp *h)
{
    if (cv->n == cv->cap) {
        cv->cap = cv->cap ? 2 * cv->cap : 1024;
        cv->v = (core_hsp *)realloc(cv->v, cv->cap * sizeof(core_hsp));
    }
    cv->v[cv->n++] = *h;
}

/* spec 4b: the greedy primitive with the lower-numbered sample in the first
 * (diagonal i) role; swap = the query sample is the higher-numbered one */
static ext_result greedy_canon(const walker *Q, int32_t qlen, const walker *T, int32_t tlen, int32_t X, int swap)
{
    if (!swap) return greedy_ext(Q, qlen, T, tlen, X);
    ext_result r = greedy_ext(T, tlen, Q, qlen, X);
    const int32_t t = r.i;
    r.i = r.j;
    r.j = t;
    return r;
}

static void process_candidate(const seqdb *db, uint32_t qtx, int strand, uint32_t stx,
                              const seed *sd, int ns, int32_t X, int swap, core_vec *out)
{
    hsp_box H[MAX_HSP];
    int nh = 0;
    uint64_t qs = db->tx_start[qtx], ts = db->tx_start[stx];
    int32_t Lq = (int32_t)(db->tx_start[qtx + 1] - qs), Lt = (int32_t)(db->tx_start[stx + 1] - ts);
    for (int i = 0; i < ns && nh < MAX_HSP; i++) {
        int32_t x = sd[i].x, y = sd[i].y, len = sd[i].len, c = 0;
        for (int h = 0; h < nh; h++)
            if (H[h].qa <= x && x + len <= H[h].qb && H[h].sa <= y && y + len <= H[h].sb) { c = 1; break; }
        if (c) continue;
        walker qa = {db->c, qs, Lq, strand, 0, x + len};
        walker ta = {db->c, ts, Lt, 0, 0, y + len};
        ext_result r = greedy_canon(&qa, Lq - (x + len), &ta, Lt - (y + len), X, swap);
        walker qb = {db->c, qs, Lq, strand, 1, x - 1};
        walker tb = {db->c, ts, Lt, 0, 1, y - 1};
        ext_result l = greedy_canon(&qb, x, &tb, y, X, swap);
        hsp_box b;
        b.qa = x - l.i; b.qb = x + len + r.i; b.sa = y - l.j; b.sb = y + len + r.j;
        b.score = l.score + 2 * len + r.score;
        b.d = l.d + r.d; b.g = l.g + r.g; b.o = l.o + r.o;
        b.nident = len + (l.i + l.j - 2 * l.d + l.g) / 2 + (r.i + r.j - 2 * r.d + r.g) / 2;
        H[nh++] = b;
    }
    /* purge common endpoints: by (score desc, index asc), keep unless it shares
     * a start or end point with an already kept HSP */
    int order[MAX_HSP], keep[MAX_HSP];
    for (int i = 0; i < nh; i++) order[i] = i, keep[i] = 0;
    for (int i = 1; i < nh; i++)
        for (int j = i; j > 0; j--) {
            int a = order[j - 1], b = order[j];
            if (H[b].score > H[a].score) { order[j - 1] = b; order[j] = a; } else break;
        }
    for (int ii = 0; ii < nh; ii++) {
        int i = order[ii], ok = 1;
        for (int jj = 0; jj < ii; jj++) {
            int j = order[jj];
            if (!keep[j]) continue;
            if ((H[i].qa == H[j].qa && H[i].sa == H[j].sa) || (H[i].qb == H[j].qb && H[i].sb == H[j].sb)) { ok = 0; break; }
        }
        keep[i] = ok;
    }
    for (int i = 0; i < nh; i++) {
        if (!keep[i]) continue;
        core_hsp c;
        c.qtx = qtx; c.stx = stx; c.strand = strand; c.hidx = i;
        c.qa = H[i].qa; c.qb = H[i].qb; c.sa = H[i].sa; c.sb = H[i].sb;
        c.score = H[i].score; c.d = H[i].d; c.g = H[i].g; c.o = H[i].o; c.nident = H[i].nident;
        c.Lq = Lq; c.Lt = Lt;
        push_core(out, &c);
    }
}

/* BLAST-tabular record of a core HSP, from the computing direction's view
 * (mirror = 0) or from the other direction's (mirror = 1: query and subject
 * swap; on the minus strand the subject coordinates run backwards). */
static orc_hsp to_record(const core_hsp *c, int mirror)
{
    orc_hsp o;
    int32_t qs, qe, ss, se;
    memset(&o, 0, sizeof o);
    if (!c->strand) {
        qs = c->qa + 1; qe = c->qb; ss = c->sa + 1; se = c->sb;
    } else {
        qs = c->Lq - c->qb + 1; qe = c->Lq - c->qa; ss = c->sb; se = c->sa + 1;
    }
    if (!mirror) {
        o.q_tx = c->qtx; o.s_tx = c->stx;
        o.qstart = qs; o.qend = qe; o.sstart = ss; o.send = se;
    } else {
        o.q_tx = c->stx; o.s_tx = c->qtx;
        if (!c->strand) { o.qstart = ss; o.qend = se; o.sstart = qs; o.send = qe; }
        else { o.qstart = se; o.qend = ss; o.sstart = qe; o.send = qs; }
    }
    o.strand = c->strand;
    o.gaps = c->g; o.gapopen = c->o; o.mismatch = c->d - c->g; o.nident = c->nident;
    o.length = o.nident + o.mismatch + o.gaps;
    o.score_half = c->score;
    o.bits10 = bits10_of(c->score);
    return o;
}

/* Core search: every gene of query sample Q (genes in ascending global gene
 * order, isoforms in input order) against subject sample T. Output order:
 * (gene, isoform, strand, subject tx, HSP index). No e-value cut. */
static void core_search(const uint8_t *codes, const uint64_t *tx_start, const int32_t *tx_sample,
                        uint32_t n_tx, const uint32_t *gene_tx_off, const uint32_t *gene_tx,
                        uint32_t n_genes, const int32_t *gene_sample, int32_t qsample,
                        int32_t tsample, const orc_params *P, core_vec *cv)
{
    seqdb db = {codes, tx_start, tx_sample, n_tx};
    sindex ix;
    build_index(&db, tsample, &ix);
    const int32_t s = P->word_size - W16 + 1;
    seed *sd = NULL;
    uint64_t sdcap = 0;
    uint8_t *mask = NULL;
    int32_t mcap = 0;
    for (uint32_t g = 0; g < n_genes; g++) {
        if (gene_sample[g] != qsample) continue;
        for (uint32_t ii = gene_tx_off[g]; ii < gene_tx_off[g + 1]; ii++) {
            uint32_t q = gene_tx[ii];
            uint64_t qs = tx_start[q];
            int32_t Lq = (int32_t)(tx_start[q + 1] - qs);
            if (P->dust_level > 0) {
                if (Lq + 1 > mcap) {
                    mcap = 2 * Lq + 1;
                    mask = (uint8_t *)realloc(mask, (size_t)mcap);
                }
                dust_tx(codes + qs, Lq, P->dust_level, P->dust_window, P->dust_linker, mask);
            }
            for (int strand = 0; strand < 2; strand++) {
                uint64_t nsd = 0;
                int32_t prev_usable = INT32_MIN / 2;   /* previous usable word (spec 2: D(p)) */
                for (int32_t p = 0; p + W16 <= Lq; p += s) {
                    uint32_t key = 0;
                    int ok = 1;
                    for (int k = 0; k < W16; k++) {
                        uint8_t c = qbase(codes, qs, Lq, strand, p + k);
                        if (c > 3) { ok = 0; break; }
                        key |= (uint32_t)c << (2 * k);
                    }
                    if (ok && P->dust_level > 0)   /* forward bases of the oriented window */
                        for (int k = 0; k < W16 && ok; k++)
                            if (mask[strand ? Lq - 1 - (p + k) : p + k]) ok = 0;
                    if (!ok) continue;
                    const int32_t D = p - prev_usable;
                    prev_usable = p;
                    for (uint64_t e = lower_key(&ix, key); e < ix.n && ix.e[e].key == key; e++) {
                        uint32_t t = ix.e[e].tx;
                        int32_t o = (int32_t)ix.e[e].off;
                        uint64_t ts = tx_start[t];
                        int32_t Lt = (int32_t)(tx_start[t + 1] - ts);
                        int32_t x = p, y = o;
                        while (x > 0 && y > 0) {
                            uint8_t a = qbase(codes, qs, Lq, strand, x - 1), b = codes[ts + y - 1];
                            if (a > 3 || b > 3 || a != b) break;
                            x--, y--;
                        }
                        if (p - x >= D) continue;  /* not canonical */
                        int32_t e2 = p + W16, f2 = o + W16;
                        while (e2 < Lq && f2 < Lt) {
                            uint8_t a = qbase(codes, qs, Lq, strand, e2), b = codes[ts + f2];
                            if (a > 3 || b > 3 || a != b) break;
                            e2++, f2++;
                        }
                        if (e2 - x < P->word_size) continue;
                        if (nsd == sdcap) {
                            sdcap = sdcap ? 2 * sdcap : 256;
                            sd = (seed *)realloc(sd, sdcap * sizeof(seed));
                        }
                        sd[nsd].tx = t; sd[nsd].x = x; sd[nsd].y = y; sd[nsd].len = e2 - x;
                        nsd++;
                    }
                }
                qsort(sd, nsd, sizeof(seed), seed_cmp);
                for (uint64_t i = 0; i < nsd;) {
                    uint64_t j = i;
                    while (j < nsd && sd[j].tx == sd[i].tx) j++;
                    process_candidate(&db, q, strand, sd[i].tx, sd + i, (int)(j - i), P->xdrop_half, qsample > tsample, cv);
                    i = j;
                }
            }
        }
    }
    free(sd);
    free(mask);
    free(ix.e);
}

/* ordering of mirrored records: (query gene, query isoform position, strand,
 * subject tx, HSP index) */
typedef struct { uint64_t k1, k2; orc_hsp h; } keyed_hsp;

static int keyed_cmp(const void *pa, const void *pb)
{
    const keyed_hsp *a = (const keyed_hsp *)pa, *b = (const keyed_hsp *)pb;
    if (a->k1 != b->k1) return a->k1 < b->k1 ? -1 : 1;
    if (a->k2 != b->k2) return a->k2 < b->k2 ? -1 : 1;
    return 0;
}

/* Directed search (query sample Q, subject sample T). Symmetric spec: the
 * candidates of a sample pair are extended once, with the lower-numbered
 * sample as query; the other direction's HSPs are their mirror images. Each
 * direction applies its own e-value cut (its query length and subject DB).
 * Output order: (query gene, isoform, strand, subject tx, HSP index). */
int orc_align_codes(const uint8_t *codes, const uint64_t *tx_start,
                    const int32_t *tx_sample, uint32_t n_tx,
                    const uint32_t *gene_tx_off, const uint32_t *gene_tx, uint32_t n_genes,
                    const int32_t *gene_sample, int32_t qsample, int32_t tsample,
                    const orc_params *P, orc_hsp **out, uint64_t *n_out)
{
    if (P->word_size < W16 || P->word_size > 64 || qsample == tsample) return -1;
    int64_t dblen = 0, dbn = 0;   /* subject sample of this direction */
    for (uint32_t t = 0; t < n_tx; t++)
        if (tx_sample[t] == tsample) { dblen += (int64_t)(tx_start[t + 1] - tx_start[t]); dbn++; }
    const int mirror = P->symmetric && qsample > tsample;
    core_vec cv = {0, 0, 0};
    core_search(codes, tx_start, tx_sample, n_tx, gene_tx_off, gene_tx, n_genes, gene_sample,
                mirror ? tsample : qsample, mirror ? qsample : tsample, P, &cv);
    hsp_vec hv = {0, 0, 0};
    if (!mirror) {
        for (uint64_t i = 0; i < cv.n; i++) {
            const core_hsp *c = &cv.v[i];
            const double ss = search_space(c->Lq, dblen, dbn);
            if (c->score < score_threshold(ss, P->evalue)) continue;
            orc_hsp o = to_record(c, 0);
            o.evalue = evalue_of(ss, c->score);
            push_hsp(&hv, &o);
        }
    } else {
        /* position of each transcript inside its gene, and its gene */
        uint32_t *tx_gene = (uint32_t *)malloc((n_tx ? n_tx : 1) * sizeof(uint32_t));
        uint32_t *tx_pos = (uint32_t *)malloc((n_tx ? n_tx : 1) * sizeof(uint32_t));
        for (uint32_t g = 0; g < n_genes; g++)
            for (uint32_t ii = gene_tx_off[g]; ii < gene_tx_off[g + 1]; ii++) {
                tx_gene[gene_tx[ii]] = g;
                tx_pos[gene_tx[ii]] = ii - gene_tx_off[g];
            }
        keyed_hsp *kv = (keyed_hsp *)malloc((cv.n ? cv.n : 1) * sizeof(keyed_hsp));
        uint64_t nk = 0;
        for (uint64_t i = 0; i < cv.n; i++) {
            const core_hsp *c = &cv.v[i];
            const double ss = search_space(c->Lt, dblen, dbn);   /* query = c->stx */
            if (c->score < score_threshold(ss, P->evalue)) continue;
            kv[nk].h = to_record(c, 1);
            kv[nk].h.evalue = evalue_of(ss, c->score);
            kv[nk].k1 = ((uint64_t)tx_gene[c->stx] << 32) | ((uint64_t)tx_pos[c->stx] << 1) | (uint64_t)c->strand;
            kv[nk].k2 = ((uint64_t)c->qtx << 8) | (uint64_t)c->hidx;
            nk++;
        }
        qsort(kv, nk, sizeof(keyed_hsp), keyed_cmp);
        for (uint64_t i = 0; i < nk; i++) push_hsp(&hv, &kv[i].h);
        free(kv);
        free(tx_gene);
        free(tx_pos);
    }
    free(cv.v);
    *out = hv.v;
    *n_out = hv.n;
    return 0;
}

/* ASCII entry point: the whole concatenation converted to codes first. */
int orc_align(const char *seq, uint64_t total_len, const uint64_t *tx_start,
              const int32_t *tx_sample, uint32_t n_tx,
              const uint32_t *gene_tx_off, const uint32_t *gene_tx, uint32_t n_genes,
              const int32_t *gene_sample, int32_t qsample, int32_t tsample,
              const orc_params *P, orc_hsp **out, uint64_t *n_out)
{
    uint8_t *codes = (uint8_t *)malloc(total_len ? total_len : 1);
    for (uint64_t i = 0; i < total_len; i++) codes[i] = code_of(seq[i]);
    int rc = orc_align_codes(codes, tx_start, tx_sample, n_tx, gene_tx_off, gene_tx, n_genes, gene_sample,
                             qsample, tsample, P, out, n_out);
    free(codes);
    return rc;
}

void orc_free(void *p) { free(p); }

/* exported helpers so tests can check the statistics tables directly */
int32_t orc_bits10(int32_t score_half) { return bits10_of(score_half); }
int32_t orc_threshold(int64_t qlen, int64_t dblen, int64_t dbn, double cutoff)
{
    return score_threshold(search_space(qlen, dblen, dbn), cutoff);
}
double orc_evalue(int64_t qlen, int64_t dblen, int64_t dbn, int32_t score_half)
{
    return evalue_of(search_space(qlen, dblen, dbn), score_half);
}

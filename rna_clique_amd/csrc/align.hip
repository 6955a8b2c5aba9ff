// Seed-and-extend (the BLAST+ replacement):
//
//   seed_kernel          one workgroup per query gene: 16-mer lookups at
//                        stride W-15 on both strands of every isoform,
//                        canonical maximal exact runs >= W (seeds), sorted per
//                        candidate (query tx, strand, subject tx); candidates
//                        grouped by subject sample.
//   extend_rows_kernel   each candidate's first seed on a sliding 32-lane
//                        sub-band row (two rows per wave), greedy X-drop; the
//                        64-lane instantiation continues what outgrew it.
//   first_finish_kernel  one thread per candidate: a search whose seeds all
//                        lie in the first seed's box is done (cuts, record).
//   later_round_kernel   the other searches, one seed per round: the next
//   later_finish_kernel  seed outside every box goes to the 64-lane rows;
//                        then purge and cuts, one thread per search.
//   extend_kernel        one wave per search (the full band, seeds by
//                        selection, purge, cuts): what the rounds cannot take.
//   group_* / mirror_*   per (query gene, subject sample): HSPs made
//                        contiguous in candidate order (the oracle's order).
//
// Semantics: oracle/align_oracle.c ("RC-megablast v1"), bit for bit.
#include "device.h"

#include <algorithm>
#include <climits>
#include <cstdlib>
#include <type_traits>

namespace rcg {

constexpr int SBLOCK = 256;
// Seed kernel occupancy (r04, profiles/r04_i, C3 seed kernel per step):
// 1024-seed LDS passes at 4 workgroups per CU 79.5 ms; 512-seed passes at 5
// (96 VGPRs, 28 KB LDS) 70.7; 6 (2 hits per lane) 74.7; 256-seed passes at
// 7 or 8: 92 / 98 (more passes halve their subject range). C3v: 103-104 ms
// at 4 and 5 alike.
#ifndef RC_SEED_CAP
#define RC_SEED_CAP 512
#endif
#ifndef RC_SEED_WAVES
#define RC_SEED_WAVES 5
#endif
constexpr int SEED_CAP = RC_SEED_CAP;   // seeds of one pass in LDS (a power of two: the bitonic sort pads to one)
static_assert((SEED_CAP & (SEED_CAP - 1)) == 0, "RC_SEED_CAP must be a power of two");
// Hits per lane per batch of the forward pass (their loads in flight
// together; r05 at C3: 3 / 4 / 6 / 7 -> 59.1 / 58.3 / 56.6 / 71.4 ms, 7 no
// longer fits 5 workgroups' LDS; C3v 86.3 -> 84.6 ms at 6)
#ifndef RC_HBATCH
#define RC_HBATCH 6
#endif
constexpr int HBATCH = RC_HBATCH;
// The reverse pass (REV) keeps no seeds in LDS and finds few hits (the
// near-mask index is small): its own instantiation, without the seed and
// per-sample arrays and with fewer hits per lane, runs more workgroups per CU.
#ifndef RC_SEED_REV_WAVES
#define RC_SEED_REV_WAVES 7
#endif
#ifndef RC_REV_HBATCH
#define RC_REV_HBATCH 2
#endif
#ifndef RC_PASS_SAMPLES
#define RC_PASS_SAMPLES 256
#endif
constexpr int PASS_SAMPLES = RC_PASS_SAMPLES;                // subject samples of one seed pass (per-sample counts in LDS)

constexpr int EBLOCK = 256;
constexpr int EWAVES = EBLOCK / 64;
#ifndef EXT_MIN_WAVES
#define EXT_MIN_WAVES 8
#endif
constexpr int STAGE_BASES = 8192;                 // staged transcript length limit

// wave-uniform copies (SGPR) of values the compiler cannot prove uniform
// (LDS and vector-memory loads at a uniform address)
__device__ __forceinline__ int rfl(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint32_t rfl(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ uint64_t rfl(uint64_t v)
{
    return ((uint64_t)rfl((uint32_t)(v >> 32)) << 32) | rfl((uint32_t)v);
}


// Oriented query geometry. strand 0: q; strand 1: revcomp(q).
struct QGeo {
    uint64_t qs;   // forward start
    int Lq;
};

__device__ __forceinline__ uint64_t qfwd_pos(const QGeo &q, int strand, uint64_t total, int u)
{
    return strand ? (total - q.qs - (uint64_t)q.Lq + (uint64_t)u) : (q.qs + (uint64_t)u);
}
// walk leftwards from oriented position x (x-1, x-2, ...) as a forward walk
__device__ __forceinline__ uint64_t qrev_pos(const QGeo &q, int strand, uint64_t total, int x)
{
    return strand ? (q.qs + (uint64_t)q.Lq - (uint64_t)x) : (total - q.qs - (uint64_t)x);
}

// ------------------------------------------------------------------------
// seeds
// ------------------------------------------------------------------------

// Exclusive scan of one value per thread over a SBLOCK-thread block.
__device__ __forceinline__ uint32_t block_exscan(uint32_t v, uint32_t *wsum, uint32_t &total)
{
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    uint32_t before = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < SBLOCK / 64; i++) {
        const uint32_t w = wsum[i];
        if (i < wid) before += w;
        tot += w;
    }
    __syncthreads();
    total = tot;
    return before + x - v;
}

// last k with pre[k] <= h over an SBLOCK + 1 prefix table (the word a hit belongs to)
__device__ __forceinline__ int run_of(const uint32_t *pre, uint32_t h)
{
    int lo = 0, hi = SBLOCK;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (pre[mid] <= h) lo = mid; else hi = mid;
    }
    return lo;
}

// Query word at oriented position p of a transcript (forward start qs,
// length Lq): usable for seeding unless its 16 bases hold an ambiguous base or
// a DUST-masked one (spec 1, 1b; the mask is over forward positions)
template <bool AMB>
__device__ __forceinline__ bool word_usable(const Db &db, uint64_t qs, int Lq, int strand, int p, uint64_t total)
{
    if (AMB) {
        const QGeo qg = {qs, Lq};
        const uint64_t *QM = strand ? db.ARC : db.AF;
        if (win(QM, qfwd_pos(qg, strand, total, p)) & 0xFFFFFFFFull) return false;
    }
    if (db.dmask) {
        const int64_t f = (int64_t)qs + (strand ? (int64_t)(Lq - p - W16) : (int64_t)p);
        if (win_bits(db.dmask, f) & 0xFFFFull) return false;
    }
    return true;
}

// BIG = false: one workgroup per query gene, the seeds of a pass in LDS; a
// (gene, subject sample) pass that alone overflows LDS is put on P.big_list.
// BIG = true: one workgroup per big_list entry, that single pass with its
// seeds in global scratch (P.big_cap per workgroup); an entry that overflows
// even that goes to P.big_retry (the host doubles big_cap).
// ISOG (with BIG = false): one workgroup per gene of P.iso_list -- the genes
// with more than ISO_LDS isoforms, whose isoform tables are read from HBM; the
// plain launch leaves them to it (so its own code has no such path).
template <bool AMB, bool BIG, bool ISOG, bool REV>
__global__ __launch_bounds__(SBLOCK, REV ? RC_SEED_REV_WAVES : RC_SEED_WAVES) void seed_kernel(Db db, Index ix,
                                                                                          SeedParams P)
{
    static_assert(!(REV && BIG), "the reverse pass has no global-memory passes");
    constexpr int HB = REV ? RC_REV_HBATCH : HBATCH;   // hits per lane per batch
    constexpr bool LSEEDS = !BIG && !REV;             // the pass's seeds in LDS
    const uint64_t big_e = BIG ? P.big_list[blockIdx.x] : 0ull;
    const uint32_t g = BIG ? P.gene_begin + (uint32_t)(big_e >> 16)
                           : (ISOG ? P.iso_list[blockIdx.x] : P.gene_begin + blockIdx.x);
    if (g >= P.gene_end) return;
    const int tid = threadIdx.x;

    using SegIdx = typename std::conditional<BIG, uint32_t, uint16_t>::type;
    __shared__ LSeed seeds_lds[LSEEDS ? SEED_CAP : 1];
    __shared__ SegIdx seg_lds[LSEEDS ? SEED_CAP + 1 : 1];
    __shared__ __attribute__((aligned(16))) uint8_t segT_lds[LSEEDS ? SEED_CAP : 4];
    const uint32_t cap = BIG ? P.big_cap : (REV ? 0u : (uint32_t)SEED_CAP);
    LSeed *const seeds = BIG ? P.big_seeds + (size_t)blockIdx.x * cap : seeds_lds;
    SegIdx *const seg_begin = BIG ? reinterpret_cast<SegIdx *>(P.big_seg + (size_t)blockIdx.x * (cap + 1)) : seg_lds;
    uint8_t *const seg_T = BIG ? P.big_segT + (size_t)blockIdx.x * cap : segT_lds;
    __shared__ uint32_t it_lo[SBLOCK], it_cnt[SBLOCK], it_pre[SBLOCK + 1], it_info[SBLOCK];
    __shared__ uint32_t it_key[SBLOCK];
    __shared__ uint32_t it_d[SBLOCK];   // D(p): distance to the previous usable query word (spec 2)
    __shared__ uint32_t hq_pos[SBLOCK / 64][64 * HB];   // per-wave queue of hits for the full test
    __shared__ uint8_t hq_k[SBLOCK / 64][64 * HB];
    __shared__ uint64_t it_qlw[SBLOCK], it_qlm[AMB ? SBLOCK : 1];
    __shared__ uint64_t iso_start[ISO_LDS];
    __shared__ uint32_t iso_len[ISO_LDS], iso_gtx[ISO_LDS], iso_pre[ISO_LDS + 1];
    __shared__ uint16_t it_iso[SBLOCK];   // isoform of each word item (it_info: p | strand << 24)
    __shared__ uint32_t tcnt[REV ? 1 : PASS_SAMPLES], tpre[REV ? 1 : PASS_SAMPLES + 1];   // by subject sample - T0
    __shared__ uint32_t wsum[SBLOCK / 64];
    __shared__ uint32_t sh_nseed, sh_flags, sh_rs0, sh_rs1;
    __shared__ unsigned long long sh_sbase, sh_cbase, sh_lbase;

    // shared searches: the forward pass finds this query's seeds (its usable
    // words, as its own search does); each seed also records whether the
    // reverse search (query = the subject) has a usable word in it (SEED_R)
    const uint64_t *const dm = P.share ? db.dmask : nullptr;
    const int Q = db.gene_sample[g];
    const uint32_t t0 = db.gene_tx_off[g];
    const uint32_t niso = db.gene_tx_off[g + 1] - t0;
    const int N = db.n_samples;
    const uint64_t total = db.total;
    const int stride = P.stride;
    const uint32_t shard = blockIdx.x % NSHARD;
    const int xb = P.xbits;
    if (niso > P.max_iso) {
        if (tid == 0) atomicOr(P.status, 2u);
        return;
    }
    // a gene's isoform tables: in LDS, or -- more than ISO_LDS isoforms (rare:
    // real assemblies have genes with hundreds) -- read from HBM (transcript
    // table and the host's word-item prefix); a block-uniform branch
    const bool isog = BIG ? niso > (uint32_t)ISO_LDS : ISOG;
    if (!BIG && !ISOG && niso > (uint32_t)ISO_LDS) return;   // the ISOG launch takes this gene
    // subject samples of this query sample in this shard (spec 5b: the
    // higher-numbered ones only, the pair's other direction is the mirror
    // image): its row of tmask; tm holds the bits of the current pass's
    // samples [T0, T0 + PASS_SAMPLES) (pass_mask)
    const uint64_t *const tmrow = P.tmask + (size_t)Q * (size_t)P.tmw;
    __shared__ uint64_t tm[4];   // (in LDS: the kernel's scalar registers already spill)
    auto pass_mask = [&](int T0) {   // the caller synchronises before tm is read
        if (tid < 4) {
            const int b = T0 + 64 * tid, wi = b >> 6, sh = b & 63;
            const uint64_t lo = wi < P.tmw ? tmrow[wi] : 0ull, hi = wi + 1 < P.tmw ? tmrow[wi + 1] : 0ull;
            tm[tid] = (lo >> sh) | ((hi << 1) << (63 - sh));
        }
    };
    auto in_mask = [&](int T, int T0) { return ((tm[(T - T0) >> 6] >> ((T - T0) & 63)) & 1ull) != 0; };
    // passes run over the span [T0, Tr) of the subject samples (a contiguous
    // position range, so hits are filtered by position; the query's own
    // sample, inside the span when both directions are searched, is filtered
    // out by position too), halved [T0, T1) while their seeds overflow the
    // pass capacity; the seed test drops any other sample outside the mask
    int T0, Tr;
    if (BIG) {
        T0 = (int)(big_e & 0xFFFFu);
        Tr = T0 + 1;
    } else {
        T0 = P.trange[2 * Q];
        Tr = P.trange[2 * Q + 1];
        if (P.sym || P.share) T0 = max(T0, Q + 1);
    }
    int T1 = min(Tr, T0 + PASS_SAMPLES);
    pass_mask(T0);
    const uint32_t qpb0 = (uint32_t)db.sample_pos_begin[Q], qpb1 = (uint32_t)db.sample_pos_begin[Q + 1];
    // the reverse pass's seeds of this gene's transcripts: [sh_rs0, sh_rs1) of
    // rs_key (rs_range_kernel), loaded beside the isoform tables
    if (P.rs_n && tid < 2) (tid ? sh_rs1 : sh_rs0) = P.rs_range[2 * (size_t)(g - P.gene_begin) + tid];
    // (the word-item prefix of the gene's isoforms comes from the host's
    // table, P.iso_pre_g: gene g's niso + 1 entries start at t0 + g)
    const uint32_t *const gpre = P.iso_pre_g + t0 + g;
    if (!isog) {
        for (uint32_t i = tid; i <= niso; i += SBLOCK) {
            if (i < niso) {
                const IsoRec r = db.giso[t0 + i];
                iso_gtx[i] = r.gtx;
                iso_start[i] = r.start;
                iso_len[i] = r.len;
            }
            iso_pre[i] = gpre[i];
        }
        __syncthreads();
    }
    auto I_gtx = [&](uint32_t i) -> uint32_t { return isog ? db.giso[t0 + i].gtx : iso_gtx[i]; };
    auto I_start = [&](uint32_t i) -> uint64_t { return isog ? (uint64_t)db.giso[t0 + i].start : iso_start[i]; };
    auto I_len = [&](uint32_t i) -> int { return isog ? (int)db.giso[t0 + i].len : (int)iso_len[i]; };
    auto I_pre = [&](uint32_t i) -> uint32_t { return isog ? gpre[i] : iso_pre[i]; };
    const uint32_t n_items = I_pre(niso);
#ifdef RC_ROW_TIMING
    unsigned long long tph[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long tc = __builtin_readcyclecounter();
    auto tick = [&](int i) {
        const unsigned long long t = __builtin_readcyclecounter();
        tph[i] += t - tc;
        tc = t;
    };
#define SEED_TICK(i) tick(i)
#else
#define SEED_TICK(i) ((void)0)
#endif
    const uint32_t gl = g - P.gene_begin;

    if (P.rs_n) __syncthreads();   // sh_rs0 / sh_rs1
    SEED_TICK(8);
    while (T0 < Tr) {
        if (tid == 0) {
            sh_nseed = 0;
            sh_flags = 0;
        }
        __syncthreads();
        if (P.rs_n && sh_rs1 > sh_rs0) {
            // reverse-only seeds (SEED_R, no usable word of this query inside)
            // with a subject in this pass's samples
            for (uint32_t i = sh_rs0 + (uint32_t)tid; i < sh_rs1; i += SBLOCK) {
                const LSeed sd = P.rs_rec[P.rs_idx[i]];
                const int T = db.tx[key_gtx(sd.k1, xb)].sample;
                if (T < T0 || T >= T1 || !in_mask(T, T0)) continue;
                const uint32_t slot = atomicAdd(&sh_nseed, 1u);
                if (slot < cap) seeds[slot] = sd;
                else atomicOr(&sh_flags, 1u);
            }
            __syncthreads();
        }
        // words p of the oriented query at stride s, one per thread; hits are
        // the entries of the word's bucket with its key and a position in the
        // subject samples [T0, T1) (samples are contiguous in position)
        const uint32_t pb0 = (uint32_t)db.sample_pos_begin[T0], pb1 = (uint32_t)db.sample_pos_begin[T1];
        // canonical pre-test by sequence: a hit whose s bases before it match
        // (inside both transcripts) extends left past p - s: not canonical
        const bool fast = stride <= 32;
        const bool lpre = !AMB && P.pre_mode == 1 && stride >= 1 && stride < W16;
        for (uint32_t ib = 0; ib < n_items; ib += SBLOCK) {
            const uint32_t it = ib + tid;
            uint32_t lo = 0, cnt = 0, info = 0, key = 0;
            uint64_t qlw = 0, qlm = 0;
            bool ok = false;
            int p = 0, strand = 0;
            uint32_t ii = 0;
            // the word's k-mer, the 32 query bases before it (canonical
            // pre-test) and its bucket are loaded together with its DUST
            // usability, in flight across the D(p) barriers below
            if (it < n_items) {
                if (!isog) {
                    while (ii + 1 < niso && iso_pre[ii + 1] <= it) ii++;
                } else {
                    uint32_t lo2 = 0, hi2 = niso;   // last isoform with pre <= it
                    while (hi2 - lo2 > 1) {
                        const uint32_t mid = (lo2 + hi2) >> 1;
                        if (gpre[mid] <= it) lo2 = mid; else hi2 = mid;
                    }
                    ii = lo2;
                }
                const uint32_t pre0 = I_pre(ii);
                const uint32_t rem = it - pre0;
                const uint32_t ns = (I_pre(ii + 1) - pre0) >> 1;
                strand = rem >= ns ? 1 : 0;
                p = (int)(rem - (strand ? ns : 0)) * stride;
                info = (uint32_t)p | ((uint32_t)strand << 24);
                const QGeo qg = {I_start(ii), I_len(ii)};
                const uint64_t qp = qfwd_pos(qg, strand, total, p);
                const uint64_t *QA = strand ? db.RC : db.F;
                key = (uint32_t)win(QA, qp);
                if (fast && p >= stride) {
                    qlw = win_s(QA, (int64_t)qp - 32);
                    if (AMB) qlm = win_s(strand ? db.ARC : db.AF, (int64_t)qp - 32);
                }
                ok = word_usable<AMB>(db, qg.qs, qg.Lq, strand, p, total);
                if (ok) {
                    const uint32_t b = key >> (32 - ix.bits);
                    lo = ix.bucket[b];
                    cnt = ix.bucket[b + 1];
                }
            }
            // D(p): the previous usable word of the same isoform and strand is
            // item it - k (p - k s), in this batch's LDS or looked up again
            it_d[tid] = ok ? 1u : 0u;
            __syncthreads();
            uint32_t D = (uint32_t)p + 1u;   // none: every hit is canonical
            if (ok) {
                for (int k = 1; p - k * stride >= 0; k++) {
                    const bool u = tid - k >= 0 ? it_d[tid - k] != 0
                                                : word_usable<AMB>(db, I_start(ii), I_len(ii), strand,
                                                                   p - k * stride, total);
                    if (u) {
                        D = (uint32_t)(k * stride);
                        break;
                    }
                }
            }
            __syncthreads();
            SEED_TICK(9);
            it_d[tid] = D;
            if (it < n_items) {
                if (ok) {
                    // the bucket of the key's top bits
                    cnt -= lo;
                    // entries are ascending (k-mer, position) and the subject
                    // samples a contiguous position range: two lower bounds in
                    // the bucket (searched together) leave exactly the key's
                    // entries in [pb0, pb1)
                    const uint64_t K0 = ((uint64_t)key << 32) | pb0, K1 = ((uint64_t)key << 32) | pb1;
                    uint32_t b0 = lo, n0 = cnt, b1 = lo, n1 = cnt;
                    while (n0 | n1) {
                        const uint32_t h0 = n0 >> 1, h1 = n1 >> 1;
                        const uint64_t e0 = n0 ? ix.ent[b0 + h0] : 0ull, e1 = n1 ? ix.ent[b1 + h1] : 0ull;
                        if (n0) {
                            if (e0 < K0) { b0 += h0 + 1; n0 -= h0 + 1; } else n0 = h0;
                        }
                        if (n1) {
                            if (e1 < K1) { b1 += h1 + 1; n1 -= h1 + 1; } else n1 = h1;
                        }
                    }
                    lo = b0;
                    cnt = b1 - b0;
                } else {
                    key = 0;
                    qlw = qlm = 0;
                }
            }
            it_lo[tid] = lo;
            it_cnt[tid] = cnt;
            it_info[tid] = info;
            it_iso[tid] = (uint16_t)ii;
            it_key[tid] = key;
            it_qlw[tid] = qlw;
            if (AMB) it_qlm[tid] = qlm;
            uint32_t tot;
            SEED_TICK(0);
            it_pre[tid] = block_exscan(cnt, wsum, tot);
            if (tid == 0) it_pre[SBLOCK] = tot;
            __syncthreads();
            SEED_TICK(1);
            const uint32_t nh = it_pre[SBLOCK];
            const int lane = tid & 63, wid = tid >> 6;
            uint32_t *wqp = hq_pos[wid];
            uint8_t *wqk = hq_k[wid];
            for (uint32_t hb0 = 0; hb0 < nh; hb0 += SBLOCK * HB) {
                // pass A: HB hits per lane with their loads in flight
                // together; drop other keys, other samples and hits the
                // sequence pre-test proves non-canonical (the s bases before
                // them equal and unambiguous, no transcript start in
                // (pos - s, pos]: the full test below would reject them)
                uint32_t hk[HB];
                uint64_t hev[HB], hsw[HB], hsm[HB], hbw[HB];
                bool live[HB];
#pragma unroll
                for (int j = 0; j < HB; j++) {
                    const uint32_t h = hb0 + (uint32_t)j * SBLOCK + (uint32_t)tid;
                    live[j] = h < nh;
                    hk[j] = live[j] ? (uint32_t)run_of(it_pre, h) : 0u;
                    hev[j] = live[j] ? ix.ent[it_lo[hk[j]] + (h - it_pre[hk[j]])] : 0ull;
                }
                // Hit-list pre-test (stride < 16, no ambiguity codes): item k-1
                // is the word at p - s of the same isoform and strand, and its
                // hit list is exactly its k-mer's entries in [pb0, pb1), in
                // position order. The s bases before a hit at pos match (same
                // transcript, no start in (pos - s, pos]) iff pos - s is in that
                // list: the entry's 16-mer covers them and the base at pos.
                // The chunk's positions go to LDS (the queue's space) and each
                // hit binary-searches its previous word's list there; hits whose
                // previous list is not wholly in this chunk take the sequence
                // pre-test.
                constexpr uint32_t HCHUNK = SBLOCK * HB;
                uint32_t *chk = &hq_pos[0][0];
                if (lpre) {
                    __syncthreads();   // the previous chunk's queue is consumed
#pragma unroll
                    for (int j = 0; j < HB; j++)
                        if (live[j]) chk[(uint32_t)j * SBLOCK + (uint32_t)tid] = (uint32_t)hev[j];
                    __syncthreads();
                }
                SEED_TICK(5);
#pragma unroll
                for (int j = 0; j < HB; j++) {
                    const uint32_t pos = (uint32_t)hev[j];
                    live[j] = live[j] && (uint32_t)(hev[j] >> 32) == it_key[hk[j]] && pos >= pb0 && pos < pb1 &&
                              (pos < qpb0 || pos >= qpb1);
                    hsw[j] = hsm[j] = hbw[j] = 0;
                    bool decided = false;
                    if (lpre && live[j] && hk[j] > 0 && it_d[hk[j]] == (uint32_t)stride &&
                        (int)(it_info[hk[j]] & 0xFFFFFFu) >= stride) {
                        const uint32_t a = it_pre[hk[j] - 1], b = it_pre[hk[j]];
                        if (a >= hb0 && b <= hb0 + HCHUNK) {
                            const uint32_t tgt = pos - (uint32_t)stride;
                            uint32_t lo = a - hb0, n = b - a;
                            while (n) {
                                const uint32_t half = n >> 1;
                                if (chk[lo + half] < tgt) {
                                    lo += half + 1;
                                    n -= half + 1;
                                } else {
                                    n = half;
                                }
                            }
                            const bool found = pos >= (uint32_t)stride && lo < b - hb0 && chk[lo] == tgt;
                            hsw[j] = found ? 0ull : ~0ull;
                            decided = true;
                        }
                    }
                    if (decided) {
                    } else if (live[j] && fast && it_d[hk[j]] == (uint32_t)stride &&
                               (int)(it_info[hk[j]] & 0xFFFFFFu) >= stride) {
                        hsw[j] = win_s(db.F, (int64_t)pos - 32) ^ it_qlw[hk[j]];
                        if (AMB) hsm[j] = win_s(db.AF, (int64_t)pos - 32) | it_qlm[hk[j]];
                        hbw[j] = win_bits(db.txstart, (int64_t)pos - 63);
                    } else {
                        hsw[j] = ~0ull;
                    }
                }
                if (lpre) __syncthreads();   // every wave is done with chk before the queue reuses it
                uint32_t qn = 0;
#pragma unroll
                for (int j = 0; j < HB; j++) {
                    if (live[j] && (((hsw[j] | hsm[j]) >> (64 - 2 * stride)) == 0) && ((hbw[j] >> (64 - stride)) == 0))
                        live[j] = false;
                    const uint64_t m = __ballot(live[j]);
                    if (live[j]) {
                        const uint32_t q = qn + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
                        wqp[q] = (uint32_t)hev[j];
                        wqk[q] = (uint8_t)hk[j];
                    }
                    qn += (uint32_t)__popcll(m);
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                SEED_TICK(6);
                // pass B: the full canonical test and the seed of each queued hit
                for (uint32_t q = (uint32_t)lane; q < qn; q += 64) {
                    const uint32_t pos = wqp[q];
                    const int k = wqk[q];
                    const uint32_t inf = it_info[k];
                    const int p = (int)(inf & 0xFFFFFFu);
                    const uint32_t ii = it_iso[k];
                    const int strand = (int)(inf >> 24);
                    QGeo qg = {I_start(ii), I_len(ii)};
                    const uint64_t *QA = strand ? db.RC : db.F;
                    const uint64_t *QAM = strand ? db.ARC : db.AF;
                    const uint64_t qp = qfwd_pos(qg, strand, total, p);
                    // the transcript lookup and the 32-base windows on both sides
                    // of the word (query and subject) are independent: all their
                    // loads go out together, the bounds are applied afterwards
                    TxInfo st;
                    const uint32_t stx = tx_of_pos(db, ix, pos, st);
                    uint64_t xl = 0, xr = 0, xr2 = 0;   // xr2: the next 32 bases right (exact runs are long)
                    if (fast) {
                        xl = win_s(QA, (int64_t)qp - 32) ^ win_s(db.F, (int64_t)pos - 32);
                        xr = win(QA, qp + W16) ^ win(db.F, (uint64_t)pos + W16);
                        xr2 = win(QA, qp + W16 + 32) ^ win(db.F, (uint64_t)pos + W16 + 32);
                        if (AMB) {
                            xl |= win_s(QAM, (int64_t)qp - 32) | win_s(db.AF, (int64_t)pos - 32);
                            xr |= win(QAM, qp + W16) | win(db.AF, (uint64_t)pos + W16);
                            xr2 |= win(QAM, qp + W16 + 32) | win(db.AF, (uint64_t)pos + W16 + 32);
                        }
                    }
                    // (pos in [pb0, pb1): st.sample is in [T0, T1))
                    if (!in_mask(st.sample, T0)) continue;
                    const int off = (int)(pos - (uint32_t)st.start);
                    const int Dp = (int)it_d[k];
                    const int maxl = min(min(p, off), Dp);
                    int l;
                    if (fast && (xl || maxl <= 32)) {
                        // matching bases leftwards from (p - 1, pos - 1): the
                        // highest differing base of the windows ending there
                        l = min(xl ? (int)(__builtin_clzll(xl) >> 1) : 32, maxl);
                    } else {
                        const uint64_t *QL = strand ? db.F : db.RC;
                        const uint64_t *QLM = strand ? db.AF : db.ARC;
                        l = lcp<AMB>(QL, QLM, qrev_pos(qg, strand, total, p), db.RC, db.ARC,
                                     total - st.start - (uint64_t)off, maxl);
                    }
                    if (l >= Dp) continue;   // not canonical: a usable word lies in [x, p)
                    const int maxr = min(qg.Lq - p - W16, (int)st.len - off - W16);
                    int r;
                    if (fast && xr) {
                        r = min((int)(__builtin_ctzll(xr) >> 1), max(maxr, 0));
                    } else if (fast && xr2) {
                        r = min(32 + (int)(__builtin_ctzll(xr2) >> 1), max(maxr, 0));
                    } else {
                        const int r0 = fast ? min(64, max(maxr, 0)) : 0;
                        r = r0 + lcp64<AMB>(QA, QAM, qp + (uint64_t)(W16 + r0), db.F, db.AF,
                                            st.start + (uint64_t)(off + W16 + r0), maxr - r0);
                    }
                    const int len = l + W16 + r;
                    if (len < P.word) continue;
                    if (REV) {
                        // the reverse pass: only runs the forward pass cannot see
                        // go on -- no usable aligned word of the subject (the
                        // forward query, oriented by the strand) inside -- as
                        // SEED_R seeds of the forward candidate (subject tx,
                        // strand, this tx) in its coordinates
                        const int La = (int)st.len, ya = off - l, pb = p - l;
                        const int xa = strand ? La - ya - len : ya;
                        bool fwd = false;
                        for (int u = (xa + stride - 1) / stride * stride; !fwd && u + W16 <= xa + len; u += stride)
                            fwd = word_usable<AMB>(db, st.start, La, strand, u, total);
                        if (fwd) continue;
                        LSeed sd;
                        sd.k1 = seed_key(P.tx_pos[stx], (uint32_t)strand, I_gtx(ii), (uint32_t)xa, xb);
                        sd.y = (uint32_t)(strand ? qg.Lq - pb - len : pb);
                        sd.len = (uint32_t)len | SEED_R;
                        const unsigned long long k = atomicAdd(P.rseed_n, 1ull);
                        if (k < P.rseed_cap) {
                            P.rseeds[k] = sd;
                            P.rseed_gene[k] = db.tx_gene[stx];
                        }
                        continue;
                    }
                    uint32_t dfl = 0u;
                    if (P.share) {
                        // the reverse search (query = the subject, oriented by the
                        // strand): an aligned word of it in the run's span there,
                        // unmasked. Without DUST one always exists (a run of W =
                        // s + 15 bases holds an aligned word). Runs of the reverse
                        // search with no usable word of this query inside come
                        // from the reverse pass (P.rs_*).
                        bool okR = !dm;
                        if (dm) {
                            const int y = off - l, Lt = (int)st.len;
                            const int r0 = strand ? Lt - y - len : y;   // the run in the reverse query's orientation
                            for (int pp = (r0 + stride - 1) / stride * stride; !okR && pp + W16 <= r0 + len;
                                 pp += stride) {
                                const int64_t f = (int64_t)st.start + (strand ? (int64_t)(Lt - pp - W16) : (int64_t)pp);
                                okR = (win_bits(dm, f) & 0xFFFFull) == 0;
                            }
                        }
                        dfl = SEED_F | (okR ? SEED_R : 0u);
                    }
                    const uint32_t slot = atomicAdd(&sh_nseed, 1u);
                    if (slot < cap) {
                        LSeed sd;
                        sd.k1 = seed_key(ii, (uint32_t)strand, stx, (uint32_t)(p - l), xb);
                        sd.y = (uint32_t)(off - l);
                        sd.len = (uint32_t)len | dfl;
                        seeds[slot] = sd;
                    } else {
                        atomicOr(&sh_flags, 1u);
                    }
                }
                __builtin_amdgcn_wave_barrier();
                SEED_TICK(7);
            }
            __syncthreads();
        }
        if (REV) {   // the reverse pass keeps no seeds of its own: on to the next subject samples
            T0 = T1;
            T1 = min(Tr, T0 + PASS_SAMPLES);
            if (T0 < Tr) {
                pass_mask(T0);
                __syncthreads();
            }
            continue;
        }
        if (sh_flags & 1u) {   // too many seeds: fewer subject samples per pass
            if (T1 - T0 == 1) {
                // one subject sample alone overflows: the global-memory pass
                // takes (gene, T0); its groups stay empty here
                if (tid == 0) {
                    const uint64_t e = ((uint64_t)gl << 16) | (uint64_t)T0;
                    const unsigned long long k = atomicAdd(BIG ? P.big_retry_n : P.big_n, 1ull);
                    if (k < P.big_list_cap) (BIG ? P.big_retry : P.big_out)[k] = e;
                    else atomicOr(P.status, 8u);
                }
                T0 = T1;
                T1 = min(Tr, T0 + PASS_SAMPLES);
                pass_mask(T0);
                __syncthreads();
                continue;
            }
            T1 = T0 + (T1 - T0) / 2;
            __syncthreads();
            continue;
        }
        SEED_TICK(2);
        const uint32_t nseed = sh_nseed;
        // the pass's seed and candidate slots are claimed as soon as their
        // counts are known; the atomics' round trips run under the sort and
        // the segment scan (the results are only read by thread 0, later)
        unsigned long long sb_claim = 0, cb_claim = 0;
        if (tid == 0 && nseed) sb_claim = atomicAdd(&P.seed_count[shard], (unsigned long long)nseed);
        // sort by (k1, y). Chunks of SBLOCK seeds: one per thread, bitonic in
        // registers -- partners within the wave by lane exchange, the few
        // stages across waves through the chunk's LDS. Then (LDS pass) merge
        // rounds of sorted runs: each seed's place is its index in its run plus
        // its rank in the partner run (a binary search there), all reads before
        // a barrier, then written in place. Global-memory passes (BIG): one
        // bitonic network over the whole pass instead.
        auto seed_gt = [](const LSeed &a, const LSeed &b) { return (a.k1 > b.k1) || (a.k1 == b.k1 && a.y > b.y); };
        uint32_t np2 = 1;
        if (!BIG || nseed <= SBLOCK) {
            const uint32_t nch = (nseed + SBLOCK - 1) / SBLOCK;
            for (uint32_t c = 0; c < nch; c++) {
                LSeed *cs = seeds + (size_t)c * SBLOCK;
                const uint32_t cn = min(nseed - c * (uint32_t)SBLOCK, (uint32_t)SBLOCK);
                uint32_t cp2 = 1;
                while (cp2 < cn) cp2 <<= 1;
                LSeed v = {~0ull, 0xFFFFFFFFu, 0u};
                if ((uint32_t)tid < cn) v = cs[tid];
                for (uint32_t kk = 2; kk <= cp2; kk <<= 1) {
                    for (uint32_t j = kk >> 1; j > 0; j >>= 1) {
                        LSeed o;
                        if (j >= 64) {
                            __syncthreads();
                            if ((uint32_t)tid < cp2) cs[tid] = v;
                            __syncthreads();
                            o = (uint32_t)tid < cp2 ? cs[tid ^ j] : v;
                        } else {
                            const int jj = (int)j;
                            o.k1 = ((uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)(v.k1 >> 32), jj) << 32) |
                                   (uint32_t)__shfl_xor((int)(uint32_t)v.k1, jj);
                            o.y = (uint32_t)__shfl_xor((int)v.y, jj);
                            o.len = (uint32_t)__shfl_xor((int)v.len, jj);
                        }
                        const bool gt = seed_gt(v, o);
                        const bool want_min = ((tid & j) == 0) == ((tid & kk) == 0);
                        if (gt == want_min) v = o;
                    }
                }
                __syncthreads();
                if ((uint32_t)tid < cn) cs[tid] = v;
            }
            __syncthreads();
            if (!BIG) {
                constexpr int MPT = SEED_CAP / SBLOCK;   // seeds per thread in a merge round
                for (uint32_t w = SBLOCK; w < nseed; w <<= 1) {
                    LSeed mv[MPT];
                    uint32_t mdst[MPT];
#pragma unroll
                    for (int m = 0; m < MPT; m++) {
                        const uint32_t i = (uint32_t)(m * SBLOCK + tid);
                        mdst[m] = ~0u;
                        if (i >= nseed) continue;
                        mv[m] = seeds[i];
                        const uint32_t a0 = i / (2 * w) * (2 * w), b0 = a0 + w;
                        if (b0 >= nseed) {   // a run without a partner stays
                            mdst[m] = i;
                            continue;
                        }
                        const bool inA = i < b0;
                        // partner run [p0, p1): A's seeds go before equal B seeds
                        const uint32_t p0 = inA ? b0 : a0, p1 = inA ? min(b0 + w, nseed) : b0;
                        uint32_t lo = p0, n = p1 - p0;
                        while (n) {
                            const uint32_t h = n >> 1;
                            const LSeed &o = seeds[lo + h];
                            const bool before = inA ? seed_gt(mv[m], o) : !seed_gt(o, mv[m]);
                            if (before) {
                                lo += h + 1;
                                n -= h + 1;
                            } else {
                                n = h;
                            }
                        }
                        mdst[m] = a0 + (i - (inA ? a0 : b0)) + (lo - p0);
                    }
                    __syncthreads();
#pragma unroll
                    for (int m = 0; m < MPT; m++)
                        if (mdst[m] != ~0u) seeds[mdst[m]] = mv[m];
                    __syncthreads();
                }
            }
        } else {
            while (np2 < nseed) np2 <<= 1;
        }
        for (uint32_t i = nseed + tid; i < np2; i += SBLOCK) {
            seeds[i].k1 = ~0ull;
            seeds[i].y = 0xFFFFFFFFu;
        }
        if (np2 > 1) __syncthreads();
        for (uint32_t kk = 2; kk <= np2; kk <<= 1) {
            for (uint32_t j = kk >> 1; j > 0; j >>= 1) {
                for (uint32_t i = tid; i < np2; i += SBLOCK) {
                    const uint32_t ixj = i ^ j;
                    if (ixj > i) {
                        LSeed a = seeds[i], b = seeds[ixj];
                        const bool up = (i & kk) == 0;
                        if (seed_gt(a, b) == up) {
                            seeds[i] = b;
                            seeds[ixj] = a;
                        }
                    }
                }
                __syncthreads();
            }
        }
        SEED_TICK(3);
        // candidates (segments of equal (iso, strand, gtx)), block-parallel
        uint32_t nseg = 0;
        for (uint32_t c0 = 0; c0 < nseed; c0 += SBLOCK) {
            const uint32_t i = c0 + tid;
            const uint32_t f = (i < nseed && (i == 0 || (seeds[i].k1 >> xb) != (seeds[i - 1].k1 >> xb))) ? 1u : 0u;
            uint32_t tot;
            const uint32_t pos = nseg + block_exscan(f, wsum, tot);
            if (f) seg_begin[pos] = (SegIdx)i;
            nseg += tot;
        }
        if (tid == 0) {
            seg_begin[nseg] = (SegIdx)nseed;
            if (nseg) cb_claim = atomicAdd(&P.cand_count[shard], (unsigned long long)nseg);
        }
        const int NT = T1 - T0;   // <= PASS_SAMPLES: counts by T - T0
        for (int T = tid; T < NT; T += SBLOCK) tcnt[T] = 0;
        __syncthreads();
        // the subject transcript of segment tid is kept for the candidate
        // write in the word-item arrays (free after the hits; tile positions
        // are < 2^32)
        for (uint32_t sg = tid; sg < nseg; sg += SBLOCK) {
            const uint32_t gtx = key_gtx(seeds[seg_begin[sg]].k1, xb);
            const TxInfo st = db.tx[gtx];
            if (sg == (uint32_t)tid) {
                it_lo[tid] = (uint32_t)st.start;
                it_cnt[tid] = st.len;
                it_info[tid] = (uint32_t)st.sample;
            }
            const int T = st.sample - T0;
            seg_T[sg] = (uint8_t)T;
            atomicAdd(&tcnt[T], 1u);
        }
        __syncthreads();
        {
            uint32_t tot;
            const uint32_t v = tid < NT ? tcnt[tid] : 0u;
            const uint32_t pre = block_exscan(v, wsum, tot);
            if (tid < NT) tpre[tid] = pre;
        }
        if (tid == 0) {
            sh_sbase = sb_claim;
            sh_cbase = cb_claim;
            if (sb_claim + nseed > P.seed_cap || cb_claim + nseg > P.cand_cap) atomicOr(P.status, 1u);
        }
        __syncthreads();
        const bool room = sh_sbase + nseed <= P.seed_cap && sh_cbase + nseg <= P.cand_cap;
        const uint64_t sbase = (uint64_t)shard * P.seed_cap + sh_sbase;
        const uint64_t cbase = (uint64_t)shard * P.cand_cap + sh_cbase;
        if (room) {
            for (uint32_t i = tid; i < nseed; i += SBLOCK) {
                GSeed gs;
                gs.x = key_x(seeds[i].k1, xb);
                gs.y = seeds[i].y;
                gs.len = seeds[i].len;
                P.seeds[sbase + i] = gs;
            }
            // rounds of SBLOCK candidates (uniform: the list2 append is a block scan)
            for (uint32_t c0 = 0; c0 < nseg; c0 += SBLOCK) {
                const uint32_t sg = c0 + tid;
                uint32_t want = 0;
                uint64_t cslot = 0;
                if (sg < nseg) {
                    const uint32_t b0 = seg_begin[sg], b1 = seg_begin[sg + 1];
                    const uint64_t k1 = seeds[b0].k1;
                    const uint32_t gtx = key_gtx(k1, xb);
                    const int T = seg_T[sg];   // - T0
                    uint32_t rk = 0;   // rank among earlier candidates of the same sample
                    if (T1 - T0 == 1) {
                        rk = sg;
                    } else {
                        // four samples per dword: bytes equal to T are the zero
                        // bytes of w ^ T x 0x01010101
                        const uint32_t pat = 0x01010101u * (uint32_t)T;
                        const uint32_t *const w4 = reinterpret_cast<const uint32_t *>(seg_T);
                        auto zb = [](uint32_t x) {
                            return (uint32_t)__builtin_popcount(~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u);
                        };
                        const uint32_t nf = sg >> 2;
                        for (uint32_t q = 0; q < nf; q++) rk += zb(w4[q] ^ pat);
                        if (sg & 3u) rk += zb((w4[nf] ^ pat) | (0xFFFFFFFFu << (8u * (sg & 3u))));
                    }
                    Cand c;
                    c.seed_off = (uint32_t)(sbase + b0);
                    c.q_gtx = I_gtx(key_iso(k1, xb));
                    c.s_gtx = gtx;
                    c.seed_lo = (uint16_t)(b1 - b0);
                    c.seed_hi = (uint16_t)((b1 - b0) >> 16);
                    c.strand = (uint8_t)key_strand(k1, xb);
                    c.dflags = 1;
                    c.e0 = 0;
                    c.e1 = SEED_NONE;
                    if (P.share) {
                        // each search's first seed: forward (x, y) order is the
                        // sorted order; reverse order is (y, x) on the plus strand,
                        // (y + len, x + len) descending on the minus strand (the
                        // reverse query is the subject's reverse complement there)
                        int fF = -1, fR = -1;
                        uint64_t bk = ~0ull;
                        for (uint32_t i = b0; i < b1; i++) {
                            const uint32_t sl = seeds[i].len;
                            if ((sl & SEED_F) && fF < 0) fF = (int)(i - b0);
                            if (sl & SEED_R) {
                                const uint32_t sx = key_x(seeds[i].k1, xb), sy = seeds[i].y, ln = sl & SEED_LEN;
                                const uint64_t key = c.strand ? ((uint64_t)~(sy + ln) << 32) | (uint32_t)~(sx + ln)
                                                              : ((uint64_t)sy << 32) | sx;
                                if (key < bk) {
                                    bk = key;
                                    fR = (int)(i - b0);
                                }
                            }
                        }
                        // e0 / e1 are 16-bit seed indices (SEED_NONE reserved)
                        if (fF >= (int)SEED_NONE || fR >= (int)SEED_NONE) atomicOr(P.status, 16u);
                        c.dflags = (uint8_t)((fF >= 0 ? 1 : 0) | (fR >= 0 ? 2 : 0));
                        c.e0 = (uint16_t)(fF >= 0 ? fF : fR);
                        c.e1 = (fF >= 0 && fR >= 0 && fR != fF) ? (uint16_t)fR : SEED_NONE;
                        want = c.e1 != SEED_NONE ? 1u : 0u;
                    }
                    const uint32_t qi = key_iso(k1, xb);
                    const uint64_t qstart = I_start(qi);
                    const int qlen = I_len(qi);
                    c.q0 = (uint32_t)(c.strand ? total - qstart - (uint64_t)qlen : qstart);
                    TxInfo st;
                    if (c0 == 0) {
                        st.start = it_lo[tid];
                        st.len = it_cnt[tid];
                        st.sample = (int)it_info[tid];
                    } else {
                        st = db.tx[gtx];
                    }
                    c.s0 = (uint32_t)st.start;
                    c.Lq = (int32_t)qlen;
                    c.Lt = (int32_t)st.len;
                    c.qsam = (uint16_t)Q;
                    c.ssam = (uint16_t)st.sample;
                    c.pad0 = 0;
                    c.pad1 = 0;
                    cslot = cbase + tpre[T] + rk;
                    P.cands[cslot] = c;
                }
                if (P.share) {
                    uint32_t tot;
                    const uint32_t pos = block_exscan(want, wsum, tot);
                    if (tot) {
                        if (tid == 0) sh_lbase = atomicAdd(P.list2_n, (unsigned long long)tot);
                        __syncthreads();
                        if (want) P.list2[sh_lbase + pos] = (uint32_t)cslot;
                        __syncthreads();
                    }
                }
            }
        }
        for (int T = T0 + tid; T < T1; T += SBLOCK) {
            const size_t gi = (size_t)gl * (size_t)N + (size_t)T;
            P.gc_off[gi] = (uint32_t)(cbase + tpre[T - T0]);
            P.gc_cnt[gi] = tcnt[T - T0];
        }
        T0 = T1;
        T1 = min(Tr, T0 + PASS_SAMPLES);
        if (T0 < Tr) {   // (no next pass: no mask to load, nothing to wait for)
            pass_mask(T0);
            __syncthreads();
        }
        SEED_TICK(4);
    }
#ifdef RC_ROW_TIMING
    if (tid == 0 && P.prof)
        for (int i = 0; i < 10; i++) atomicAdd(&P.prof[i], tph[i]);
#endif
#undef SEED_TICK
}

// Reverse-only seeds of each query gene of [g0, g1): the lower bounds of g
// and g + 1 in rs_key (sorted by forward gene), one thread per gene (instead
// of a dependent binary search at the start of every seed workgroup).
__global__ void rs_range_kernel(const uint32_t *__restrict__ rs_key, uint32_t rs_n, uint32_t g0, uint32_t g1,
                                uint32_t *__restrict__ out)
{
    const uint64_t n = (uint64_t)(g1 - g0) * 2;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t key = g0 + (uint32_t)(i >> 1) + (uint32_t)(i & 1);
        uint32_t lo = 0, m = rs_n;
        while (m) {
            const uint32_t h = m >> 1;
            if (rs_key[lo + h] < key) {
                lo += h + 1;
                m -= h + 1;
            } else {
                m = h;
            }
        }
        out[i] = lo;
    }
}

void launch_rs_range(const uint32_t *rs_key, uint32_t rs_n, uint32_t g0, uint32_t g1, uint32_t *out, hipStream_t st)
{
    const uint64_t n = (uint64_t)(g1 - g0) * 2;
    if (!n) return;
    const uint64_t g = std::min<uint64_t>((n + 255) / 256, 65536);
    hipLaunchKernelGGL(rs_range_kernel, dim3((unsigned)g), dim3(256), 0, st, rs_key, rs_n, g0, g1, out);
}

// ------------------------------------------------------------------------
// extension
// ------------------------------------------------------------------------

struct ExtRes {
    int score, i, j, d, g, o;
};

// Max over the wave: DPP inside rows of 16 (xor 1, xor 2, half-row mirror,
// row mirror), then the four row maxima through readlane. No LDS round trips.
__device__ __forceinline__ int wave_max(int v)
{
    v = max(v, __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false));   // quad_perm [1,0,3,2]
    v = max(v, __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false));   // quad_perm [2,3,0,1]
    v = max(v, __builtin_amdgcn_mov_dpp(v, 0x141, 0xF, 0xF, false));  // row_half_mirror
    v = max(v, __builtin_amdgcn_mov_dpp(v, 0x140, 0xF, 0xF, false));  // row_mirror
    const int a = max(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16));
    const int b = max(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48));
    return max(a, b);
}

// lane l <- lane l-1 (lane 0 gets `edge`) / lane l <- lane l+1 (lane 63 gets
// `edge`): gfx9-family DPP wavefront shifts, one VALU op each.
__device__ __forceinline__ int from_lower(int v, int edge)
{
    return __builtin_amdgcn_update_dpp(edge, v, 0x138, 0xF, 0xF, false);   // wave_shr:1
}
__device__ __forceinline__ int from_upper(int v, int edge)
{
    return __builtin_amdgcn_update_dpp(edge, v, 0x130, 0xF, 0xF, false);   // wave_shl:1
}

// 32 bases starting at base p of a packed array viewed as dwords (16 bases
// each): three dword loads and two funnel shifts (v_alignbit_b32).
template <typename PT>
__device__ __forceinline__ uint64_t win3(const uint32_t *__restrict__ a, PT p)
{
    const PT i = p >> 4;
    const uint32_t sh = ((uint32_t)p & 15u) * 2u;
    const uint32_t w0 = a[i], w1 = a[i + 1], w2 = a[i + 2];
    const uint32_t lo = __builtin_amdgcn_alignbit(w1, w0, sh);
    const uint32_t hi = __builtin_amdgcn_alignbit(w2, w1, sh);
    return ((uint64_t)hi << 32) | lo;
}

// Matching bases walking forward from (pa, pb) (BACK = false) or backwards
// from (pa - 1, pb - 1) (BACK = true; the window ending at p is read at p - 32
// and the first mismatch is its highest differing base), at most maxn.
template <bool AMB, bool BACK, typename PT>
__device__ __forceinline__ int slide(const uint32_t *A, const uint32_t *AM, PT pa, const uint32_t *B,
                                     const uint32_t *BM, PT pb, int maxn)
{
    int n = 0;
    while (n < maxn) {
        const PT qa = BACK ? pa - (PT)(n + 32) : pa + (PT)n;
        const PT qb = BACK ? pb - (PT)(n + 32) : pb + (PT)n;
        uint64_t x = win3(A, qa) ^ win3(B, qb);
        if (AMB) x |= win3(AM, qa) | win3(BM, qb);
        if (x == 0) {
            n += 32;
            continue;
        }
        n += (BACK ? __builtin_clzll(x) : __builtin_ctzll(x)) >> 1;
        return n < maxn ? n : maxn;
    }
    return maxn > 0 ? maxn : 0;
}

// Greedy X-drop extension (oracle/align_oracle.c greedy_ext), one diagonal per
// lane of the wave. A / B: oriented query and subject; the walk starts at
// (pa, pb) forward, or at (pa - 1, pb - 1) backwards. Branch-free step; the
// per-lane gap state G | O << 13 | E << 26 travels in one register. Stops as
// soon as no live diagonal can still beat the best score (score + 2 x bases
// left on the shorter side <= best): the result is unchanged.
template <bool AMB, bool BACK, typename PT>
__device__ __forceinline__ ExtRes ext_wave(const uint32_t *A, const uint32_t *AM, PT pa, int alen,
                                           const uint32_t *B, const uint32_t *BM, PT pb, int blen, int X,
                                           int lane, uint32_t &steps, uint32_t &edge)
{
    constexpr int EBIT = 26, OBIT = 13;
    constexpr int GMASK = 8191;
    const int k = lane + BAND_LO;
    int r0 = 0;
    if (lane == -BAND_LO) r0 = slide<AMB, BACK, PT>(A, AM, pa, B, BM, pb, min(alen, blen));
    r0 = __builtin_amdgcn_readlane(r0, -BAND_LO);
    ExtRes best = {2 * r0, r0, r0, 0, 0, 0};
    if (min(alen, blen) - r0 <= 0) return best;
    int R = lane == -BAND_LO ? r0 : -1;
    int goe = 0;
    for (int d = 1; d <= DMAX; ++d) {
        steps++;
        const int Rl = from_lower(R, -1), Rr = from_upper(R, -1);
        const int gl = from_lower(goe, 0), gr = from_upper(goe, 0);
        // candidates; ties prefer mismatch, then insertion, then deletion
        const int cm = (R >= 0 && R < alen && R - k < blen) ? R + 1 : -1;
        const int ci = (Rl >= 0 && Rl < alen) ? Rl + 1 : -1;
        const int cd = (Rr >= 0 && Rr - (k + 1) < blen) ? Rr : -1;
        int ni = max(max(cm, ci), cd);
        const bool fm = ni >= 0 && cm == ni, fi = !fm && ci == ni;
        const int gi = (gl & ~(3 << EBIT)) + 1 + ((((gl >> EBIT) & 3) == 1) ? 0 : (1 << OBIT)) + (1 << EBIT);
        const int gd = (gr & ~(3 << EBIT)) + 1 + ((((gr >> EBIT) & 3) == 2) ? 0 : (1 << OBIT)) + (2 << EBIT);
        int ng = fm ? (goe & ~(3 << EBIT)) : (fi ? gi : gd);
        int score = INT_MIN, bound = INT_MIN;
        if (ni >= 0) {
            const int ja = ni - k;
            const int m = min(alen - ni, blen - ja);
            const int s = slide<AMB, BACK, PT>(A, AM, BACK ? pa - (PT)ni : pa + (PT)ni, B, BM,
                                               BACK ? pb - (PT)ja : pb + (PT)ja, m);
            ni += s;
            if (s > 0) ng &= ~(3 << EBIT);
            score = 2 * ni - k - 6 * d;
            if (score < best.score - X) ni = -1;
            bound = score + 2 * (m - s);
        }
        R = ni;
        goe = ng;
        const bool live = ni >= 0;
        if (!__ballot(live)) break;
        // the 64-diagonal band binds (spec 3): a live diagonal at its edge
        if (__ballot(live && (lane == 0 || lane == BAND - 1))) edge = 1;
        if (__ballot(live && score > best.score)) {
            // (score, lowest lane) as one key: score * 64 + (63 - lane)
            const int mk = wave_max(live ? score * 64 + (63 - lane) : INT_MIN);
            const int bl = 63 - (mk & 63);
            best.score = mk >> 6;
            best.i = __builtin_amdgcn_readlane(R, bl);
            best.j = best.i - (bl + BAND_LO);
            best.d = d;
            const int bg = __builtin_amdgcn_readlane(goe, bl);
            best.g = bg & GMASK;
            best.o = (bg >> OBIT) & GMASK;
        }
        if (!__ballot(live && bound > best.score)) break;
    }
    return best;
}

// Both extensions of one seed (x, y, len): right from its end, left from its
// start. swap (spec 4b): the query is the higher-numbered sample, so the
// greedy primitive runs with the subject in the first role and its end
// point is swapped back.
template <bool AMB, typename PT>
__device__ __forceinline__ void extend_seed(const uint32_t *QO, const uint32_t *QOM, PT qo, const uint32_t *TF,
                                            const uint32_t *TFM, PT tf, int Lq, int Lt, int x, int y, int len, int X,
                                            int lane, uint32_t &steps, uint32_t &eg, bool swap, ExtRes &r, ExtRes &l)
{
    if (!swap) {
        r = ext_wave<AMB, false, PT>(QO, QOM, qo + (PT)(x + len), Lq - (x + len), TF, TFM, tf + (PT)(y + len),
                                     Lt - (y + len), X, lane, steps, eg);
        l = ext_wave<AMB, true, PT>(QO, QOM, qo + (PT)x, x, TF, TFM, tf + (PT)y, y, X, lane, steps, eg);
    } else {
        r = ext_wave<AMB, false, PT>(TF, TFM, tf + (PT)(y + len), Lt - (y + len), QO, QOM, qo + (PT)(x + len),
                                     Lq - (x + len), X, lane, steps, eg);
        l = ext_wave<AMB, true, PT>(TF, TFM, tf + (PT)y, y, QO, QOM, qo + (PT)x, x, X, lane, steps, eg);
        int t = r.i;
        r.i = r.j;
        r.j = t;
        t = l.i;
        l.i = l.j;
        l.j = t;
    }
}

// cand_box record of a first-seed extension: status (0 done, -1 deferred),
// right (score, i, j, d, gap state), left (same)
enum { FX_STATUS = 0, FX_R = 1, FX_L = 6 };

// Shared searches: one directed search of a candidate on one wave, in the
// forward search's coordinates (query = the lower sample, which is also the
// first role of spec 4b). The search's seeds (dbit) are taken in ITS order
// -- forward: (x, y); reverse: (y, x) on the plus strand, (y + len, x + len)
// descending on the minus strand -- by selection: the next seed extended is
// the first in that order outside every box so far (a seed inside a box
// stays inside as boxes are added, so this is the sequential rule of spec 3).
template <bool AMB, typename PT>
__device__ __forceinline__ void process_search(const uint32_t *QO, const uint32_t *QOM, PT qo, const uint32_t *TF,
                                               const uint32_t *TFM, PT tf, int Lq, int Lt, const GSeed *sd, int ns,
                                               int X, int lane, uint32_t dbit, int strand, int &bqa, int &bqb,
                                               int &bsa, int &bsb, int &bsc, int &bd, int &bg, int &bo, int &bni,
                                               int &nh, uint32_t &steps, uint32_t &exts, uint32_t &edges,
                                               uint32_t &capped, bool swap, const int *fx = nullptr, int e = -1)
{
    nh = 0;
    if (fx) {
        // the search's first seed (always extended, spec 3) was extended by
        // the row kernel: its HSP as first_finish_kernel builds it
        constexpr int OBIT = 13, GMASK = 8191;
        const GSeed s0 = sd[e];
        const int x = (int)s0.x, y = (int)s0.y, len = (int)(s0.len & SEED_LEN);
        const int rsc = fx[FX_R], ri = fx[FX_R + 1], rj = fx[FX_R + 2], rd = fx[FX_R + 3], rgo = fx[FX_R + 4];
        const int lsc = fx[FX_L], lI = fx[FX_L + 1], lJ = fx[FX_L + 2], ld = fx[FX_L + 3], lgo = fx[FX_L + 4];
        if (lane == 0) {
            bqa = x - lI; bqb = x + len + ri; bsa = y - lJ; bsb = y + len + rj;
            bsc = lsc + 2 * len + rsc;
            bd = ld + rd; bg = (lgo & GMASK) + (rgo & GMASK); bo = ((lgo >> OBIT) & GMASK) + ((rgo >> OBIT) & GMASK);
            bni = len + (lI + lJ - 2 * ld + (lgo & GMASK)) / 2 + (ri + rj - 2 * rd + (rgo & GMASK)) / 2;
        }
        nh = 1;
    }
    for (;;) {
        unsigned long long bk = ~0ull;
        int bi = 0;
        for (int c0 = 0; c0 < ns; c0 += 64) {
            const int i = c0 + lane;
            if (i >= ns) continue;
            const GSeed g = sd[i];
            if (!(g.len & dbit)) continue;
            const uint32_t x = g.x, y = g.y, len = g.len & SEED_LEN;
            bool in = false;
            for (int h = 0; h < nh; h++) {
                const int qa = __builtin_amdgcn_readlane(bqa, h), qb = __builtin_amdgcn_readlane(bqb, h);
                const int sa = __builtin_amdgcn_readlane(bsa, h), sb = __builtin_amdgcn_readlane(bsb, h);
                in = in || (qa <= (int)x && (int)(x + len) <= qb && sa <= (int)y && (int)(y + len) <= sb);
            }
            if (in) continue;
            const unsigned long long key =
                dbit == SEED_F ? ((unsigned long long)x << 32) | y
                               : (strand ? ((unsigned long long)(uint32_t)~(y + len) << 32) | (uint32_t)~(x + len)
                                         : ((unsigned long long)y << 32) | x);
            if (key < bk) {
                bk = key;
                bi = i;
            }
        }
        unsigned long long m = bk;
        for (int o = 32; o; o >>= 1) {
            const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(m >> 32), o);
            const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)m, o);
            const unsigned long long v = ((unsigned long long)hi << 32) | lo;
            m = v < m ? v : m;
        }
        if (m == ~0ull) break;
        if (nh >= MAX_HSP) {   // MAX_HSP binds (spec 3): a seed outside every box remains
            capped++;
            break;
        }
        const int src = __ffsll((unsigned long long)__ballot(bk == m)) - 1;
        const int si = __shfl(bi, src);
        const GSeed g = sd[si];
        const int x = (int)g.x, y = (int)g.y, len = (int)(g.len & SEED_LEN);
        uint32_t eg = 0;
        ExtRes r, l;
        extend_seed<AMB, PT>(QO, QOM, qo, TF, TFM, tf, Lq, Lt, x, y, len, X, lane, steps, eg, swap, r, l);
        exts += 2;
        edges += eg;
        if (lane == nh) {
            bqa = x - l.i; bqb = x + len + r.i; bsa = y - l.j; bsb = y + len + r.j;
            bsc = l.score + 2 * len + r.score;
            bd = l.d + r.d; bg = l.g + r.g; bo = l.o + r.o;
            bni = len + (l.i + l.j - 2 * l.d + l.g) / 2 + (r.i + r.j - 2 * r.d + r.g) / 2;
        }
        nh++;
    }
}

// One candidate (all its seeds) on one wave. QO: oriented query (its base u at
// qo + u), TF: subject forward (base v at tf + v); right extensions walk
// forward from the seed end, left extensions backwards from the seed start.
template <bool AMB, typename PT>
__device__ __forceinline__ void process_candidate(const uint32_t *QO, const uint32_t *QOM, PT qo, const uint32_t *TF,
                                                  const uint32_t *TFM, PT tf, int Lq, int Lt, const GSeed *sd,
                                                  int ns, int X, int lane, int &bqa, int &bqb, int &bsa, int &bsb,
                                                  int &bsc, int &bd, int &bg, int &bo, int &bni, int &nh,
                                                  uint32_t &steps, uint32_t &exts, uint32_t &edges, uint32_t &capped,
                                                  bool swap)
{
    nh = 0;
    int next = ns;   // the first seed not examined (MAX_HSP reached before it)
    for (int c0 = 0; c0 < ns && next == ns; c0 += 64) {
        // lane i holds seed c0 + i; the loop broadcasts them with readlane
        int sx = 0, sy = 0, sl = 0;
        if (c0 + lane < ns) {
            const GSeed g = sd[c0 + lane];
            sx = (int)g.x;
            sy = (int)g.y;
            sl = (int)(g.len & SEED_LEN);
        }
        const int nc = min(ns - c0, 64);
        for (int si = 0; si < nc; si++) {
            if (nh >= MAX_HSP) {
                next = c0 + si;
                break;
            }
            const int x = __builtin_amdgcn_readlane(sx, si), y = __builtin_amdgcn_readlane(sy, si);
            const int len = __builtin_amdgcn_readlane(sl, si);
            const bool inside = lane < nh && bqa <= x && x + len <= bqb && bsa <= y && y + len <= bsb;
            if (__ballot(inside)) continue;
            uint32_t eg = 0;
            ExtRes r, l;
            extend_seed<AMB, PT>(QO, QOM, qo, TF, TFM, tf, Lq, Lt, x, y, len, X, lane, steps, eg, swap, r, l);
            exts += 2;
            edges += eg;
            if (lane == nh) {
                bqa = x - l.i; bqb = x + len + r.i; bsa = y - l.j; bsb = y + len + r.j;
                bsc = l.score + 2 * len + r.score;
                bd = l.d + r.d; bg = l.g + r.g; bo = l.o + r.o;
                bni = len + (l.i + l.j - 2 * l.d + l.g) / 2 + (r.i + r.j - 2 * r.d + r.g) / 2;
            }
            nh++;
        }
    }
    // MAX_HSP binds (spec 3) when a seed past the cap lies outside every box
    for (int i = next; i < ns; i++) {
        const GSeed g = sd[i];
        const int x = (int)g.x, y = (int)g.y, len = (int)(g.len & SEED_LEN);
        if (!__ballot(lane < nh && bqa <= x && x + len <= bqb && bsa <= y && y + len <= bsb)) {
            capped++;
            break;
        }
    }
}

constexpr int SPAD = 32;                               // front pad of staged sequences (bases)
constexpr int SW2 = (STAGE_BASES + SPAD) / 32 + 3;     // u64 words per staged sequence

// stage bases [pos, pos + L) of a packed global array at LDS base SPAD
__device__ __forceinline__ void stage_seq(uint64_t *dst, const uint64_t *src, uint64_t pos, int L, int lane)
{
    const int nw = (L >> 5) + 3;
    for (int w = lane; w < nw; w += 64) dst[w] = w ? win<uint64_t>(src, pos + 32 * (uint64_t)(w - 1)) : 0ull;
}

template <bool AMB>
__global__ __launch_bounds__(EBLOCK, EXT_MIN_WAVES) void extend_kernel(Db db, ExtParams P)
{
    constexpr int NA = AMB ? 4 : 2;
    __shared__ uint64_t stg[EWAVES][NA][SW2];
    __shared__ unsigned long long sprefix[NSHARD + 1];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int i = threadIdx.x; i <= NSHARD; i += EBLOCK) sprefix[i] = P.shard_prefix[i];
    __syncthreads();
    const uint64_t total = db.total;
    const uint64_t nwaves = (uint64_t)gridDim.x * EWAVES;
    int shard = 0;   // advances monotonically with li
    uint64_t li = (uint64_t)blockIdx.x * EWAVES + wid;
    // list mode (P.defer set): the candidates extend_dual_kernel deferred
    const bool list = P.defer != nullptr;
    const uint64_t n_work = list ? (uint64_t)*P.defer_count : P.n_cand;
    // candidate slots are wave-uniform: keep them (and what is loaded through
    // them) in scalar registers
    auto locate = [&](uint64_t l) -> uint64_t {
        if (list) return rfl((uint64_t)P.defer[l]);
        while (shard + 1 < NSHARD && sprefix[shard + 1] <= l) shard++;
        return rfl((uint64_t)((uint64_t)shard * P.cand_cap + (l - sprefix[shard])));
    };
    const Cand *__restrict__ cands = P.cands;
    const TxInfo *__restrict__ txs = db.tx;
    uint32_t steps = 0, exts = 0, ncands = 0, edges = 0, capped = 0;
    for (; li < n_work; li += nwaves) {
        const uint64_t ci = locate(li);
        const Cand cd = cands[ci];
        const TxInfo qt = txs[cd.q_gtx], st = txs[cd.s_gtx];
        const int Lq = (int)qt.len, Lt = (int)st.len;
        const int strand = cd.strand;
        const int ns = (int)cand_seeds(cd);
        const GSeed *sd = P.seeds + cd.seed_off;
        ncands++;
        int bqa = 0, bqb = 0, bsa = 0, bsb = 0, bsc = 0, bd = 0, bg = 0, bo = 0, bni = 0, nh = 0;
        // oriented query: q (forward array) or revcomp(q) (reverse-complement array)
        const uint64_t *QA = strand ? db.RC : db.F;
        const uint64_t *QAM = strand ? db.ARC : db.AF;
        const uint64_t q0 = strand ? total - qt.start - (uint64_t)Lq : qt.start;
        // spec 4b: the lower-numbered sample in the greedy's first role
        const bool swap = qt.sample > st.sample;
        // shared searches: this work item is one directed search of the candidate
        const uint32_t dbit = P.dir ? SEED_R : SEED_F;
        // its first seed's extension from the row kernel, when that finished
        // (a search deferred for a seed outside the first box, not for a
        // sub-band overflow): the search starts with that HSP
        const int *fx0 = nullptr;
        int e0 = -1;
        if (P.share && P.reuse_first) {
            const bool second = P.dir == 1 && cd.e1 != SEED_NONE;
            const int *fx = (second ? P.cand_box2 : P.cand_box) + ci * BOX_REC;
            if (fx[FX_STATUS] >= 0) {
                fx0 = fx;
                e0 = (int)(second ? cd.e1 : cd.e0);
            }
        }
        if (Lq + SPAD <= STAGE_BASES && Lt + SPAD <= STAGE_BASES) {
            uint64_t *QO = stg[wid][0], *TF = stg[wid][1];
            stage_seq(QO, QA, q0, Lq, lane);
            stage_seq(TF, db.F, st.start, Lt, lane);
            const uint32_t *QOM = nullptr, *TFM = nullptr;
            if (AMB) {
                stage_seq(stg[wid][2], QAM, q0, Lq, lane);
                stage_seq(stg[wid][3], db.AF, st.start, Lt, lane);
                QOM = reinterpret_cast<const uint32_t *>(stg[wid][2]);
                TFM = reinterpret_cast<const uint32_t *>(stg[wid][3]);
            }
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            if (P.share)
                process_search<AMB, uint32_t>(reinterpret_cast<const uint32_t *>(QO), QOM, (uint32_t)SPAD,
                                              reinterpret_cast<const uint32_t *>(TF), TFM, (uint32_t)SPAD, Lq, Lt,
                                              sd, ns, P.xdrop, lane, dbit, strand, bqa, bqb, bsa, bsb, bsc, bd, bg,
                                              bo, bni, nh, steps, exts, edges, capped, swap, fx0, e0);
            else
                process_candidate<AMB, uint32_t>(reinterpret_cast<const uint32_t *>(QO), QOM, (uint32_t)SPAD,
                                                 reinterpret_cast<const uint32_t *>(TF), TFM, (uint32_t)SPAD, Lq, Lt,
                                                 sd, ns, P.xdrop, lane, bqa, bqb, bsa, bsb, bsc, bd, bg, bo, bni, nh,
                                                 steps, exts, edges, capped, swap);
        } else if (P.share) {
            process_search<AMB, int64_t>(reinterpret_cast<const uint32_t *>(QA),
                                         reinterpret_cast<const uint32_t *>(QAM), (int64_t)q0,
                                         reinterpret_cast<const uint32_t *>(db.F),
                                         reinterpret_cast<const uint32_t *>(db.AF), (int64_t)st.start, Lq, Lt, sd,
                                         ns, P.xdrop, lane, dbit, strand, bqa, bqb, bsa, bsb, bsc, bd, bg, bo, bni,
                                         nh, steps, exts, edges, capped, swap, fx0, e0);
        } else {
            // global arrays carry two zero words in front, so backward windows
            // of the first transcript stay in bounds (positions may go to -32)
            process_candidate<AMB, int64_t>(reinterpret_cast<const uint32_t *>(QA),
                                            reinterpret_cast<const uint32_t *>(QAM), (int64_t)q0,
                                            reinterpret_cast<const uint32_t *>(db.F),
                                            reinterpret_cast<const uint32_t *>(db.AF), (int64_t)st.start, Lq, Lt,
                                            sd, ns, P.xdrop, lane, bqa, bqb, bsa, bsb, bsc, bd, bg, bo, bni, nh,
                                            steps, exts, edges, capped, swap);
        }
        // purge HSPs with common endpoints: by (score desc, index asc)
        int rank = 0;
        for (int j = 0; j < nh; j++) {
            const int sj = __builtin_amdgcn_readlane(bsc, j);
            if (lane < nh && (sj > bsc || (sj == bsc && j < lane))) rank++;
        }
        bool kept = false;
        for (int rr = 0; rr < nh; rr++) {
            const uint64_t m = __ballot(lane < nh && rank == rr);
            const int i = __ffsll((unsigned long long)m) - 1;
            const int qa = __builtin_amdgcn_readlane(bqa, i), sa = __builtin_amdgcn_readlane(bsa, i);
            const int qb = __builtin_amdgcn_readlane(bqb, i), sb2 = __builtin_amdgcn_readlane(bsb, i);
            const bool conflict = kept && lane < nh && ((bqa == qa && bsa == sa) || (bqb == qb && bsb == sb2));
            if (!__ballot(conflict) && lane == i) kept = true;
        }
        // e-value cut of each direction: query->subject (query length, subject
        // DB) and the mirrored one (subject length, query sample's DB)
        const int thr_f = P.thr[(size_t)st.sample * (size_t)(P.max_len + 1) + (size_t)Lq];
        const int thr_r = P.thr[(size_t)qt.sample * (size_t)(P.max_len + 1) + (size_t)Lt];
        // shared searches: the forward item applies the forward cut, the
        // reverse item the reverse one (its records go to the _r arrays)
        const bool pf = (!P.share || !P.dir) && bsc >= thr_f, pr = (P.sym || (P.share && P.dir)) && bsc >= thr_r;
        const bool out = kept && (pf || pr);
        const uint64_t om = __ballot(out);
        const int nout = __popcll(om);
        uint32_t obase = 0;
        if (nout > 1 && lane == 0) {
            const unsigned long long b = atomicAdd(P.ovf_count, (unsigned long long)(nout - 1));
            if (b + (nout - 1) > P.ovf_cap) atomicOr(P.status, 1u);
            obase = (uint32_t)b;
        }
        obase = __builtin_amdgcn_readlane(obase, 0);
        if (out) {
            const int rk = __popcll(om & ((1ull << lane) - 1ull));
            DHsp h;
            h.q_tx = cd.q_gtx;
            h.s_tx = cd.s_gtx;
            if (!strand) {
                h.qstart = bqa + 1; h.qend = bqb; h.sstart = bsa + 1; h.send = bsb;
            } else {
                h.qstart = Lq - bqb + 1; h.qend = Lq - bqa; h.sstart = bsb; h.send = bsa + 1;
            }
            h.gaps = bg;
            h.gapopen = bo;
            h.mismatch = bd - bg;
            h.nident = bni;
            h.length = bni + (bd - bg) + bg;
            h.score_half = bsc;
            h.bits10 = P.bits10[bsc];
            h.strand = strand | (pf ? HSP_FWD : 0) | (pr ? HSP_REV : 0) | (lane << HSP_IDX_SHIFT);
            if (rk == 0) (P.share && P.dir ? P.cand_hsp_r : P.cand_hsp)[ci] = h;
            else if ((uint64_t)obase + (rk - 1) < P.ovf_cap) P.ovf[obase + rk - 1] = h;
        }
        if (lane == 0) {
            (P.share && P.dir ? P.cand_nh_r : P.cand_nh)[ci] = (uint8_t)nout;
            (P.share && P.dir ? P.cand_ovf_r : P.cand_ovf)[ci] = obase;
        }
    }
    if (lane == 0 && P.counters) {
        atomicAdd(&P.counters[0], (unsigned long long)steps);
        atomicAdd(&P.counters[1], (unsigned long long)exts);
        atomicAdd(&P.counters[2], (unsigned long long)ncands);
        if (edges) atomicAdd(&P.counters[7], (unsigned long long)edges);     // extensions the band bound
        if (capped) atomicAdd(&P.counters[10], (unsigned long long)capped);  // candidates MAX_HSP bound
    }
}

// ------------------------------------------------------------------------
// extension, four candidates per wave: one 16-lane DPP row per candidate
// ------------------------------------------------------------------------
//
// The greedy frontier of a near-identical transcript pair stays within a few
// diagonals of the seed's, so most of the 64-diagonal band of extend_kernel is
// dead lanes. Here each row of RW lanes (16: one DPP row, 32: half a wave)
// runs its own candidate over the sub-band of diagonals [-RW/2, RW/2 - 1]
// (row lane rl <-> diagonal rl - RW/2). The sub-band computes exactly what the
// full band computes as long as no live diagonal reaches its edge lanes (a
// diagonal outside can only be entered from a live neighbour); the first time
// an edge lane is live while the extension continues, the candidate is handed
// to extend_kernel (list mode) whole. Rows advance independently (their own
// seeds, extensions, candidates): a row that finishes an extension does its
// bookkeeping while the other rows wait one transition, then all rows step
// together. Every extension walks forward: a left extension runs on reversed
// copies of both transcripts staged next to the forward ones.

#ifndef ROW_MIN_WAVES
#define ROW_MIN_WAVES 8   // r05_zn/zo: 8 beats 7 (C3 rows 84.1 -> 82.7 ms, C4 459 -> 450) and 6 (87.5); r02/r04: 7 was best then
#endif

// max over the 16 lanes of each DPP row, in every lane of the row
__device__ __forceinline__ int row_max(int v)
{
    v = max(v, __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false));   // quad_perm [1,0,3,2]
    v = max(v, __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false));   // quad_perm [2,3,0,1]
    v = max(v, __builtin_amdgcn_mov_dpp(v, 0x141, 0xF, 0xF, false));  // row_half_mirror
    v = max(v, __builtin_amdgcn_mov_dpp(v, 0x140, 0xF, 0xF, false));  // row_mirror
    return v;
}

// lane rl <- rl - 1 inside the row (rl 0 gets `edge`). Rows wider than a DPP
// row shift the whole wave: lane 0 keeps `edge` (FIX) or reads 0, and the
// first lane of the upper half-wave reads the last lane of the lower one.
// The frontier (FIX) relies on that lane being dead (-1 = edge) whenever a
// step starts: a live sub-band edge lane ends its row's extension (abort or
// done), every extension starts with only the seed diagonal live, and a row
// without work sets its lanes dead. Values other than the frontier are only
// read where the frontier neighbour is live.
template <int RW, bool FIX>
__device__ __forceinline__ int rw_from_lower(int v, int edge, int rl)
{
    if constexpr (RW == 16) {
        return __builtin_amdgcn_update_dpp(edge, v, 0x111, 0xF, 0xF, false);   // row_shr:1
    } else if constexpr (FIX) {
        return __builtin_amdgcn_update_dpp(edge, v, 0x138, 0xF, 0xF, false);   // wave_shr:1
    } else {
        return __builtin_amdgcn_mov_dpp(v, 0x138, 0xF, 0xF, true);             // edge is 0
    }
}
// lane rl <- rl + 1 inside the row (rl RW - 1 gets `edge`; as above)
template <int RW, bool FIX>
__device__ __forceinline__ int rw_from_upper(int v, int edge, int rl)
{
    if constexpr (RW == 16) {
        return __builtin_amdgcn_update_dpp(edge, v, 0x101, 0xF, 0xF, false);   // row_shl:1
    } else if constexpr (FIX) {
        return __builtin_amdgcn_update_dpp(edge, v, 0x130, 0xF, 0xF, false);   // wave_shl:1
    } else {
        return __builtin_amdgcn_mov_dpp(v, 0x130, 0xF, 0xF, true);             // edge is 0
    }
}
// max over the row, in every lane of the row
template <int RW>
__device__ __forceinline__ int rw_max(int v)
{
    v = row_max(v);
    if constexpr (RW >= 32) {
        const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);   // DPP rows 0<->1, 2<->3
        v = max((int)r[0], (int)r[1]);
    }
    if constexpr (RW == 64) {
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);   // the two halves
        v = max((int)r[0], (int)r[1]);
    }
    return v;
}
// bit r set iff some lane of row r is set in a wave mask (scalar work)
template <int RW>
__device__ __forceinline__ uint32_t rw_bits(uint64_t m)
{
    if constexpr (RW == 16)
        return ((m & 0xFFFFull) ? 1u : 0u) | ((m & 0xFFFF0000ull) ? 2u : 0u) | ((m & 0xFFFF00000000ull) ? 4u : 0u) |
               ((m >> 48) ? 8u : 0u);
    else if constexpr (RW == 32)
        return ((uint32_t)m ? 1u : 0u) | ((m >> 32) ? 2u : 0u);
    else
        return m ? 1u : 0u;
}
// the RW bits of this lane's row in a wave mask
template <int RW>
__device__ __forceinline__ uint32_t rw_mask(uint64_t m, int row)
{
    if constexpr (RW == 64) return (uint32_t)m;   // (callers take the low half only)
    return (uint32_t)(m >> (RW * row)) & (RW == 32 ? 0xFFFFFFFFu : 0xFFFFu);
}

// x != 0 ? ~0 : 0 on a wave-uniform value, kept in scalar registers
__device__ __forceinline__ uint32_t s_nonzero(uint32_t x)
{
    uint32_t r;
    asm volatile("s_cmp_lg_u32 %1, 0\n\ts_cselect_b32 %0, -1, 0" : "=s"(r) : "s"(x) : "scc");
    return r;
}
// lowest set bit of a wave-uniform value (-1 for 0), one scalar instruction
__device__ __forceinline__ int s_ff1(uint32_t x)
{
    int r;
    asm volatile("s_ff1_i32_b32 %0, %1" : "=s"(r) : "s"(x));
    return r;
}
// lane masks of single compares (one v_cmp each, combined in scalar registers)
__device__ __forceinline__ uint64_t m_gt(int a, int b) { return __builtin_amdgcn_ballot_w64(a > b); }
__device__ __forceinline__ uint64_t m_ge(int a, int b) { return __builtin_amdgcn_ballot_w64(a >= b); }
__device__ __forceinline__ uint64_t m_lt(int a, int b) { return __builtin_amdgcn_ballot_w64(a < b); }
__device__ __forceinline__ uint64_t m_eq(int a, int b) { return __builtin_amdgcn_ballot_w64(a == b); }
// lane mask of a condition (the HIP __ballot goes through an int and two extra vector ops)
__device__ __forceinline__ uint64_t ballot(bool b) { return __builtin_amdgcn_ballot_w64(b); }

// spread a wave mask to whole rows: every lane of a row with a set lane (scalar work)
template <int RW>
__device__ __forceinline__ uint64_t rw_spread(uint64_t m)
{
    if constexpr (RW == 32) {   // per 32-bit half, scalar ops (the compiler turns a test of the high half into a vector compare)
        const uint32_t lo = s_nonzero((uint32_t)m), hi = s_nonzero((uint32_t)(m >> 32));
        return (uint64_t)lo | ((uint64_t)hi << 32);
    } else if constexpr (RW == 64) {
        const uint32_t a = s_nonzero((uint32_t)m | (uint32_t)(m >> 32));
        return (uint64_t)a | ((uint64_t)a << 32);
    } else {
        uint64_t r = 0;
        for (int i = 0; i < 4; i++)
            if ((m >> (16 * i)) & 0xFFFFull) r |= 0xFFFFull << (16 * i);
        return r;
    }
}
// lane in mask ? a : b, one v_cndmask with the mask as the SGPR-pair condition
__device__ __forceinline__ int lane_sel(uint64_t m, int a, int b)
{
    int r;
    asm("v_cndmask_b32_e64 %0, %2, %1, %3" : "=v"(r) : "v"(a), "v"(b), "s"(m));
    return r;
}

// 32-base windows of the row kernel's staging at absolute LDS base positions
// (4 bases per byte of LDS address): three dword reads and two v_alignbit
// each. The reads are one asm block so that the address is the position's
// dword and nothing else (through a pointer the compiler adds the staging's
// LDS symbol to every address); the block waits for its own reads.
__device__ __forceinline__ uint64_t lds_join(uint64_t w01, uint32_t w2, uint32_t p)
{
    const uint32_t w0 = (uint32_t)w01, w1 = (uint32_t)(w01 >> 32);
    const uint32_t lo = __builtin_amdgcn_alignbit(w1, w0, p * 2u), hi = __builtin_amdgcn_alignbit(w2, w1, p * 2u);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ void lds_win2(uint32_t pa, uint32_t pb, uint64_t &wa, uint64_t &wb)
{
    const uint32_t aa = (pa >> 2) & ~3u, ab = (pb >> 2) & ~3u;
    uint64_t a01, b01;
    uint32_t a2, b2;
    asm volatile("ds_read2_b32 %0, %4 offset1:1\n\t"
                 "ds_read_b32 %1, %4 offset:8\n\t"
                 "ds_read2_b32 %2, %5 offset1:1\n\t"
                 "ds_read_b32 %3, %5 offset:8\n\t"
                 "s_waitcnt lgkmcnt(0)"
                 : "=&v"(a01), "=&v"(a2), "=&v"(b01), "=&v"(b2)
                 : "v"(aa), "v"(ab));
    wa = lds_join(a01, a2, pa);
    wb = lds_join(b01, b2, pb);
}
__device__ __forceinline__ uint64_t lds_diff(uint32_t pa, uint32_t pb)
{
    uint64_t a, b;
    lds_win2(pa, pb, a, b);
    return a ^ b;
}

// lane in mask ? K : b, K an inline constant (no register for it)
template <int K>
__device__ __forceinline__ int lane_sel_k(uint64_t m, int b)
{
    int r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(b), "i"(K), "s"(m));
    return r;
}

// 32 bases of each side from the dwords at byte addresses a, b holding the
// bases at LDS base positions pa, pb (+ a multiple of 16): three dword reads
// and two funnel shifts per side
__device__ __forceinline__ void lds_pair_at(uint32_t a, uint32_t b, uint32_t pa, uint32_t pb, uint64_t &wa,
                                            uint64_t &wb)
{
    uint64_t a01, b01;
    uint32_t a2, b2;
    asm volatile("ds_read2_b32 %0, %4 offset1:1\n\t"
                 "ds_read_b32 %1, %4 offset:8\n\t"
                 "ds_read2_b32 %2, %5 offset1:1\n\t"
                 "ds_read_b32 %3, %5 offset:8\n\t"
                 "s_waitcnt lgkmcnt(0)"
                 : "=&v"(a01), "=&v"(a2), "=&v"(b01), "=&v"(b2)
                 : "v"(a), "v"(b));
    wa = lds_join(a01, a2, pa);
    wb = lds_join(b01, b2, pb);
}

// Matching bases from (pa, pb) forward, at most maxn (>= 0); positions are
// absolute LDS base positions (lds_win2); masks (AMB) sit `moff` bases
// further on. Reads bases up to pa + max(maxn, 1) + 47 (WIN_MARGIN).
#ifndef RC_SLIDE_UNIFORM
#define RC_SLIDE_UNIFORM 1
#endif
template <bool AMB>
__device__ __forceinline__ int slide_fwd(uint32_t pa, uint32_t pb, int maxn, uint32_t moff)
{
    // the first window outside any loop (a mismatch within 32 bases is the
    // common case); lanes on a run of 32+ matches go on in the loop, whose
    // dword addresses advance by 8 bytes per 32 bases (the shifts stay)
    uint64_t x = lds_diff(pa, pb);
    if (AMB) {
        uint64_t ma, mb;
        lds_win2(pa + moff, pb + moff, ma, mb);
        x |= ma | mb;
    }
    int n = x ? (int)(__builtin_ctzll(x) >> 1) : 32;
#if RC_SLIDE_UNIFORM
    // the loop is wave-uniform (a ballot per round): lanes whose run ended
    // keep their count and stop advancing; no exec-mask bookkeeping per round
    // (the dword addresses follow n: a stopped lane re-reads its last window)
    bool go = n == 32 && maxn > 32;
    if (__builtin_amdgcn_ballot_w64(go)) {
        const uint32_t a0 = ((pa + 32u) >> 2) & ~3u, b0 = ((pb + 32u) >> 2) & ~3u;
        do {
            const uint32_t o = ((uint32_t)(n - 32) >> 2) & ~7u;
            uint64_t wa, wb;
            lds_pair_at(a0 + o, b0 + o, pa, pb, wa, wb);
            x = wa ^ wb;
            if (AMB) {
                lds_pair_at(a0 + o + moff / 4u, b0 + o + moff / 4u, pa, pb, wa, wb);
                x |= wa | wb;
            }
            const int k = x ? (int)(__builtin_ctzll(x) >> 1) : 32;
            n = go ? n + k : n;
            go = go && k == 32 && n < maxn;
        } while (__builtin_amdgcn_ballot_w64(go));
    }
#else
    if (n == 32 && maxn > 32) {
        uint32_t a = ((pa + 32u) >> 2) & ~3u, b = ((pb + 32u) >> 2) & ~3u;
        for (;;) {
            uint64_t wa, wb;
            lds_pair_at(a, b, pa, pb, wa, wb);
            x = wa ^ wb;
            if (AMB) {
                lds_pair_at(a + moff / 4u, b + moff / 4u, pa, pb, wa, wb);
                x |= wa | wb;
            }
            if (x) {
                n += (int)(__builtin_ctzll(x) >> 1);
                break;
            }
            n += 32;
            if (n >= maxn) break;
            a += 8u;
            b += 8u;
        }
    }
#endif
    return min(n, maxn);
}

// per-row bookkeeping in LDS: the candidate record (CAND_DWORDS dwords) and state
enum { RM_REC = 0, RM_CLO = CAND_DWORDS, RM_CHI, RM_QB, RM_TB, RM_X, RM_Y, RM_LEN,
       RM_RSC, RM_RI, RM_RJ, RM_RD, RM_RGO,
       RM_PHASE,                                  // the running extension's done action (A_RDONE / A_LDONE)
       RM_KOF,                                    // the window's diagonal offset (sliding sub-band)
       RM_PWI, RM_PWG, RM_PWD, RM_PK,             // the row's best record parked by a window slide, its diagonal
       RM_N };   // (its size is part of the row kernel's tuning: 3 more fields cost 4 VGPR spills)
// the step count and best score of an extension that outgrew the window, kept
// (SAVE kernel) in record fields the row kernel does not read (the seed
// count's high half, the padding)
enum { RM_AD6 = RM_REC + 9, RM_ABEST = RM_REC + 11 };
// a saved extension (ExtParams::resume, RES_REC ints): the bookkeeping
// RM_RSC .. RM_PK, the step count, the best score, then the window's frontier
// R and gap states
enum { RES_RSC = 0, RES_PHASE = RM_PHASE - RM_RSC, RES_KOF = RM_KOF - RM_RSC, RES_PWI = RM_PWI - RM_RSC,
       RES_PWG = RM_PWG - RM_RSC, RES_PWD = RM_PWD - RM_RSC, RES_PK = RM_PK - RM_RSC, RES_D6 = RES_PK + 1,
       RES_BEST = RES_PK + 2, RES_R = 16, RES_G = 48 };
static_assert(RES_BEST < RES_R && RES_G + 32 <= RES_REC, "resume record layout");
// fields of the record (dword offsets, layout of Cand)
enum { RC_SOFF = 0, RC_QTX = 1, RC_STX = 2, RC_CNT_STRAND = 3, RC_Q0 = 4, RC_S0 = 5, RC_LQ = 6, RC_LT = 7,
       RC_SAMS = 8, RC_SEEDHI = 9, RC_E01 = 10, RC_PAD1 = 11 };
// work cursors of a row
enum { RS_LEND, RS_SHARD, RS_SHN, RS_N };
// row actions (transition actions < A_DONE; extending: A_STEP_R / A_STEP_L = their done action + 4)
enum { A_FETCH, A_SLIDE, A_RDONE, A_LDONE, A_ABORT, A_DONE, A_STEP_R, A_STEP_L };
// bl of a row whose best record is parked in its LDS bookkeeping (a window slide)
constexpr int BL_PARKED = -64;
// The row kernel's arguments, one struct so that the kernarg segment is laid
// out as it.
struct RowArgs {
    Db db;
    ExtParams P;
};
using RowArgsK = const __attribute__((address_space(4))) RowArgs *;
// The kernarg pointer behind an opaque copy: the fields read through it are
// loaded (s_load, scalar cache) where the transitions use them instead of
// being held in SGPRs across the step loop, where ~30 SGPRs of pointers
// spilled into VGPR lanes and cost readlane/writelane pairs every step.
__device__ __forceinline__ RowArgsK row_args()
{
    RowArgsK p = (RowArgsK)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return p;
}

// per-row state that only transitions touch (row kernel LDS)
struct RowLds {
    int meta[RM_N];
    int st[RS_N];
};
// Windowed staging (WIN): a row's four staging slots (0: query forward, 1:
// subject forward, 2: query reverse complement, 3: subject reverse
// complement) hold windows of sw words of the packed tile arrays; the running
// extension walks slot a against slot b. Per row: the global base of the
// extension's start on each side (a: offset ni = 0, b: j = ni - diagonal =
// 0), the side's array (bit 0: 0 = F, 1 = RC) and slot (bits 1-2), the
// window's [lo, lim] in extension offsets, and the first word of each slot.
enum { WM_GA0, WM_GB0, WM_AARR, WM_BARR, WM_ALO, WM_ALIM, WM_BLO, WM_BLIM, WM_W0, WM_N = WM_W0 + 4 };
struct RowWin {
    int w[WM_N];
};
// LDS of a row-kernel block: staging (2 guard words + rows x arrays x sw
// words), shard prefix, rows' bookkeeping (+ window bookkeeping), 8 block counters
__host__ __device__ constexpr size_t row_lds_bytes(int rw, int na, int sw, bool win = false)
{
    return ((size_t)(EBLOCK / rw) * na * sw + 2) * 8 + (NSHARD + 1) * 8 + (size_t)(EBLOCK / rw) * sizeof(RowLds) + 32 +
           (win ? (size_t)(EBLOCK / rw) * sizeof(RowWin) : 0);
}
// windowed slot limits: a slide from offset ni with at most mw bases reads
// bases up to ni + max(mw, 1) + 47 (slide_fwd: three dwords from the dword
// holding the last window's start)
constexpr int WIN_MARGIN = 48;

// Extension of every candidate's FIRST seed (its smallest (x, y): always
// extended, RC-megablast spec 3) to the right and to the left. Anything
// further -- the other seeds' containment, more HSPs, purge, e-values -- is
// first_finish_kernel's; a candidate that needs more than its first seed goes
// to extend_kernel whole.
// Sliding sub-band: a row's RW lanes are the diagonals [kof - RW/2, kof +
// RW/2 - 1] of the spec's 64-diagonal band, kof = 0 when an extension starts.
// When a live lane reaches the window's edge, the window slides so that the
// live diagonals are centred (|kof| <= 31 - RW/2: its edges never meet the
// band's, so the edge lanes stay dead at every step start, as the half-wave
// seam of the frontier shifts needs); the lanes entering it are diagonals no
// live lane has reached (an outside diagonal can only come alive from a live
// edge lane, which slides first), so the extension stays exact. Only a live
// span wider than the window, or one reaching past the band's +-31, goes to
// the one-wave full-band kernel (indels: C3v).
// SAVE (32-lane rows): an extension that outgrows the window is saved for the
// 64-lane pass to continue (a separate instantiation: the save code's
// registers cost the plain kernel 7 % at C3, where nearly nothing overflows).
// WIN: transcripts longer than the staging slot -- each slot holds a window
// of the sequence from the extension's start, refilled from HBM when a
// slide would read past it (or a lane's position lies before it); the
// refill places the window at the lowest position still to be read, so the
// extension is the same as with the whole transcripts staged.
template <bool AMB, int RW, int MINW, bool SAVE = false, bool WIN = false>
__global__ __launch_bounds__(EBLOCK, MINW) void extend_rows_kernel(RowArgs)
{
    constexpr int RROWS = EBLOCK / RW;   // rows per block
    constexpr int RC0 = RW / 2;          // row lane of diagonal 0
    constexpr int NA = AMB ? 8 : 4;      // staged arrays per row: Q, T (raw words), Qrev, Trev (+ masks)
    constexpr int EBIT = 26, OBIT = 13;
    // All of the block's LDS is the dynamic allocation, staging first, so
    // that the staging starts at LDS address 0 and the step loop's window
    // addresses carry no base: [2 guard words][RROWS][NA][sw] staging, then
    // the shard prefix, the rows' bookkeeping and the block counters.
    extern __shared__ uint64_t rstg[];
    const int sw = row_args()->P.dsw;                     // u64 words per staged array
    unsigned long long *const sprefix = reinterpret_cast<unsigned long long *>(rstg + 2 + (size_t)RROWS * NA * sw);
    RowLds *const rows_lds = reinterpret_cast<RowLds *>(sprefix + NSHARD + 1);
    uint32_t *const rcnt = reinterpret_cast<uint32_t *>(rows_lds + RROWS);   // extensions, candidates, overflows
    uint32_t &s_ncand = rcnt[4];
    RowWin *const rows_win = reinterpret_cast<RowWin *>(rcnt + 8);   // (WIN only)
    {
        const RowArgsK K = row_args();
        if (threadIdx.x < 4 || threadIdx.x == 5) rcnt[threadIdx.x] = 0;   // [5]: 6 x row steps
        for (int i = threadIdx.x; i <= NSHARD; i += EBLOCK) sprefix[i] = K->P.shard_prefix[i];
        // list mode: the candidates are P.list[0, *P.list_n) (a previous row
        // kernel's deferrals), else the linear index space over the shards
        if (threadIdx.x == 0) s_ncand = K->P.list ? (uint32_t)*K->P.list_n : (uint32_t)K->P.n_cand;
    }
    __syncthreads();

    const int lane = threadIdx.x & 63, rl = lane & (RW - 1), row = lane / RW;
    const int rs = threadIdx.x / RW;                      // row slot in the block
    const int k = rl - RC0;                               // this lane's diagonal
    // two guard words in front (windows read from a word boundary before a position)
    uint64_t *stg = rstg + 2 + (size_t)rs * NA * sw;      // Q, T, Qr, Tr, [QM, TM, QMr, TMr]
    // absolute LDS base position of the row's Q array (the staging's LDS
    // offset: the low half of its generic address)
    const uint32_t base0 = 4u * (uint32_t)reinterpret_cast<uintptr_t>(rstg) + (uint32_t)(2 + rs * NA * sw) * 32u;
    const uint32_t bqr = base0 + 64u * (uint32_t)sw, btr = bqr + 32u * (uint32_t)sw;
    const uint32_t moff = 128u * (uint32_t)sw;
    RowLds &RL = rows_lds[rs];
    int *meta = RL.meta;
    int *const wm = rows_win[rs].w;   // (WIN only)
    const int X = row_args()->P.xdrop;
    // candidates come in chunks from a global counter (P.chunk >= 1); the
    // record of the next one is prefetched (one dword per lane) while the
    // current one is extended
    auto chunk = []() { return (uint32_t)max(row_args()->P.chunk, 1); };
    uint32_t lnx = 0;
    auto grab = [&]() {
        const uint32_t ncand = s_ncand, ch = chunk();
        unsigned long long b = 0;
        if (rl == 0) b = atomicAdd(row_args()->P.work, (unsigned long long)ch);
        b = (unsigned long long)__shfl((long long)b, RW * row);
        lnx = b < ncand ? (uint32_t)b : ncand;
        if (rl == 0) RL.st[RS_LEND] = (int)(lnx + ch);
    };
    // candidate slot of linear index l; the shard cursor (in LDS) only advances
    auto slot = [&](uint32_t l, int which) -> uint64_t {
        int sh = RL.st[which];
        while (sh + 1 < NSHARD && sprefix[sh + 1] <= l) sh++;
        if (rl == 0) RL.st[which] = sh;
        return (uint64_t)sh * row_args()->P.cand_cap + (l - sprefix[sh]);
    };
    auto cslot = [&](uint32_t l, int which) -> uint64_t {
        const uint32_t *list = row_args()->P.list;
        return list ? (uint64_t)list[l] : slot(l, which);
    };
    auto load_rec = [&](uint32_t l) -> int {
        if (l >= s_ncand || rl >= CAND_DWORDS) return 0;
        return reinterpret_cast<const int *>(row_args()->P.cands + cslot(l, RS_SHN))[rl];
    };
    // this pass's first-seed results (shared searches: pass 1 -> cand_box,
    // pass 2 over list2 -> cand_box2)
    auto box_out = []() {
        const RowArgsK K = row_args();
        return K->P.which ? K->P.cand_box2 : K->P.cand_box;
    };
    // row-uniform; extend_kernel takes the candidate whole -- or, shared
    // searches, a sub-band overflow (wide) the 64-lane pass over P.wide next
    // (returns the wide-list entry, row-uniform; ~0 when not listed)
    auto defer = [&](uint64_t ci, bool wide) -> unsigned long long {
        unsigned long long wi2 = ~0ull;
        if (rl == 0) {
            const RowArgsK K = row_args();
            if (!K->P.share) {   // shared searches: first_finish_kernel lists each search on its own
                const unsigned long long di = atomicAdd(K->P.defer_count, 1ull);
                K->P.defer[di] = (uint32_t)ci;
            } else if (wide && K->P.wide) {
                wi2 = atomicAdd(K->P.wide_n, 1ull);
                K->P.wide[wi2] = (uint32_t)ci;
            }
            box_out()[ci * BOX_REC + FX_STATUS] = -1;
        }
        if constexpr (SAVE) return (unsigned long long)__shfl((long long)wi2, RW * row);
        return wi2;
    };
    if (rl == 0) {
        RL.st[RS_SHARD] = 0;
        RL.st[RS_SHN] = 0;
    }
    grab();
    int recv = load_rec(lnx);

    int act = A_FETCH;
    // extension state: frontier (R, gap state), winner record, row-uniform best
    int R = -1, goe = 0, wi = 0, wg = 0, wd = 0, best = 0, bl = RC0, d6 = 0;   // d6 = 6 x greedy step
    uint32_t pa = 0, pb = 0;
    int alen = 0, blen = 0;
    // per-lane forms the step uses (k folded in once per extension):
    // pb - k (b position of diagonal k at a offset 0), blen + k, -(k + d6)
    uint32_t pbk = 0;
    int blk = 0, nkd = 0;
    int mnk = 0;   // min(alen, blk): a step's room along its diagonal is mnk - ni
    bool swap = false;                                    // spec 4b: query = the higher-numbered sample
    int wlo = 0, wlim = 0;                                // WIN: the lane's window [wlo, wlim] in extension offsets

    // ---- windowed staging (WIN) ----
    using GW = const __attribute__((address_space(1))) uint64_t *;
    // a packed tile array: 0 = F, 1 = RC (mask: their ambiguity masks)
    auto warr = [](int arr, bool mask) -> GW {
        const RowArgsK K = row_args();
        GW f = (GW)(mask ? K->db.AF : K->db.F), r = (GW)(mask ? K->db.ARC : K->db.RC);
        asm volatile("" : "+s"(f), "+s"(r));
        return arr ? r : f;
    };
    // LDS base position of a slot's word 0
    auto slot_base = [&](int slot) -> uint32_t { return base0 + 32u * (uint32_t)sw * (uint32_t)slot; };
    // the window of `slot`: words W .. of array arr, at most through word ew
    // (the last one a read of the side's sequence can reach)
    auto win_load = [&](int slot, int arr, uint32_t W, uint32_t ew) {
        const int n = ew >= W ? (int)min((uint32_t)sw, ew - W + 1u) : 0;
        GW src = warr(arr, false) + W;
        uint64_t *dst = stg + (size_t)slot * sw;
        for (int w = rl; w < n; w += RW) dst[w] = src[w];
        if (AMB) {
            GW msrc = warr(arr, true) + W;
            uint64_t *mdst = stg + (size_t)(4 + slot) * sw;
            for (int w = rl; w < n; w += RW) mdst[w] = msrc[w];
        }
    };
    // global start base of each slot's extension: right (slots 0, 1: the
    // forward arrays from the seed's end), left (2, 3: the reverse
    // complements from the seed's start, walked forward); and its sequence end
    auto slot_g = [&](int slot, uint32_t &g, uint32_t &e) {
        const uint32_t total = (uint32_t)row_args()->db.total;
        const uint32_t q0 = (uint32_t)meta[RM_REC + RC_Q0], s0 = (uint32_t)meta[RM_REC + RC_S0];
        const uint32_t Lq = (uint32_t)meta[RM_REC + RC_LQ], Lt = (uint32_t)meta[RM_REC + RC_LT];
        const uint32_t x = (uint32_t)meta[RM_X], y = (uint32_t)meta[RM_Y], len = (uint32_t)meta[RM_LEN];
        if (slot == 0) { g = q0 + x + len; e = q0 + Lq; }
        else if (slot == 1) { g = s0 + y + len; e = s0 + Lt; }
        else if (slot == 2) { g = total - q0 - x; e = total - q0; }
        else { g = total - s0 - y; e = total - s0; }
    };
    auto slot_arr = [&](int slot) -> int {
        const int strand = (meta[RM_REC + RC_CNT_STRAND] >> 16) & 1;
        return slot == 0 ? strand : (slot == 1 ? 0 : (slot == 2 ? 1 - strand : 1));
    };
    // the lane's window from the row's bookkeeping (diagonal kk = k + kof)
    auto win_lane = [&](int kk) {
        wlo = max(wm[WM_ALO], wm[WM_BLO] + kk);
        wlim = min(wm[WM_ALIM], wm[WM_BLIM] + kk);
    };
    // an extension starts (dir 0 right, 1 left): its sides' slots, start
    // bases and windows (as staged); pa, pbk, wlo, wlim of diagonal k
    auto win_begin = [&](int dir) {
        const int qsl = dir ? 2 : 0, tsl = dir ? 3 : 1;
        const int asl = swap ? tsl : qsl, bsl = swap ? qsl : tsl;
        uint32_t ga, gb, ea, eb;
        slot_g(asl, ga, ea);
        slot_g(bsl, gb, eb);
        const uint32_t Wa = (uint32_t)wm[WM_W0 + asl], Wb = (uint32_t)wm[WM_W0 + bsl];
        const int alo = (int)(32u * Wa - ga), blo = (int)(32u * Wb - gb);
        __builtin_amdgcn_wave_barrier();
        if (rl == 0) {
            wm[WM_GA0] = (int)ga;
            wm[WM_GB0] = (int)gb;
            wm[WM_AARR] = slot_arr(asl) | (asl << 1);
            wm[WM_BARR] = slot_arr(bsl) | (bsl << 1);
            wm[WM_ALO] = alo;
            wm[WM_ALIM] = alo + 32 * sw - WIN_MARGIN;
            wm[WM_BLO] = blo;
            wm[WM_BLIM] = blo + 32 * sw - WIN_MARGIN;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        pa = slot_base(asl) + (ga - 32u * Wa);
        pb = slot_base(bsl) + (gb - 32u * Wb);
        pbk = pb - (uint32_t)k;
        win_lane(k);
    };
    // refill the row's two windows at the lowest positions still to be read
    // (row-uniform amin on side a, bmin on side b)
    auto win_fill = [&](int amin, int bmin) {
        const uint32_t ga = (uint32_t)wm[WM_GA0], gb = (uint32_t)wm[WM_GB0];
        const int aa = wm[WM_AARR], ba = wm[WM_BARR];
        const uint32_t Wa = (ga + (uint32_t)amin) >> 5, Wb = (gb + (uint32_t)bmin) >> 5;
        win_load(aa >> 1, aa & 1, Wa, (ga + (uint32_t)alen + 47u) >> 5);
        win_load(ba >> 1, ba & 1, Wb, (gb + (uint32_t)blen + 47u) >> 5);
        const int alo = (int)(32u * Wa - ga), blo = (int)(32u * Wb - gb);
        __builtin_amdgcn_wave_barrier();
        if (rl == 0) {
            wm[WM_W0 + (aa >> 1)] = (int)Wa;
            wm[WM_W0 + (ba >> 1)] = (int)Wb;
            wm[WM_ALO] = alo;
            wm[WM_ALIM] = alo + 32 * sw - WIN_MARGIN;
            wm[WM_BLO] = blo;
            wm[WM_BLIM] = blo + 32 * sw - WIN_MARGIN;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        const int kk = k + meta[RM_KOF];
        pa = slot_base(aa >> 1) + (ga - 32u * Wa);
        pbk = slot_base(ba >> 1) + (gb - 32u * Wb) - (uint32_t)kk;
        win_lane(kk);
    };
    // finish the slides whose reads left the window (pend): refill the
    // windows of the rows concerned at their lowest pending position, go on
    // sliding; the lowest pending lane always advances (it is inside both
    // new windows), so this ends. Wave-uniform call.
    auto win_resolve = [&](int ni, int &s, int m, bool pend) {
        do {
            const int kk = k + meta[RM_KOF];
            const int c = ni + s;
            const int amin = -rw_max<RW>(pend ? -c : -INT_MAX), bmin = -rw_max<RW>(pend ? -(c - kk) : -INT_MAX);
            if (amin != INT_MAX) win_fill(amin, bmin);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            if (pend) {
                const int c2 = ni + s, mr = m - s;
                const int mw = c2 < wlo ? -1 : min(mr, wlim - c2);
                const int s2 = slide_fwd<AMB>(pa + (uint32_t)c2, pbk + (uint32_t)c2, max(mw, 0), moff);
                pend = mw < mr && s2 >= mw;
                s += s2;
            }
        } while (ballot(pend));
    };

#ifdef RC_ROW_TIMING
    unsigned long long t_ei = 0;   // extension starts (part of the transitions)
#endif
    auto ext_init = [&](int done_act) {
#ifdef RC_ROW_TIMING
        const unsigned long long e0t = __builtin_readcyclecounter();
#endif
        int r0 = 0;
        if constexpr (WIN) {
            win_begin(done_act == A_LDONE ? 1 : 0);
            const int m0 = min(alen, blen);
            bool pend = false;
            if (rl == RC0) {
                const int mw = min(m0, wlim);
                r0 = slide_fwd<AMB>(pa, pb, max(mw, 0), moff);
                pend = mw < m0 && r0 >= mw;
            }
            if (ballot(pend)) win_resolve(0, r0, m0, pend);
        } else {
            if (rl == RC0) r0 = slide_fwd<AMB>(pa, pb, min(alen, blen), moff);
        }
        r0 = __shfl(r0, RW * row + RC0);
        best = 2 * r0;
        bl = RC0;
        if (rl == RC0) {
            wi = r0;
            wg = 0;
            wd = 0;
        }
        R = rl == RC0 ? r0 : -1;
        goe = 0;
        if (rl == 0 && d6) atomicAdd(&rcnt[5], (uint32_t)d6);   // the previous extension's steps
        d6 = 0;
        if constexpr (!WIN) pbk = pb - (uint32_t)k;   // (WIN: win_begin / win_fill set it)
        blk = blen + k;
        mnk = max(min(alen, blk), 0);
        nkd = -k;
        if (rl == 0) {
            atomicAdd(&rcnt[0], 1u);
            meta[RM_PHASE] = done_act;
            meta[RM_KOF] = 0;
        }
        act = (min(alen, blen) - r0 <= 0) ? done_act : done_act + (A_STEP_R - A_RDONE);
#ifdef RC_ROW_TIMING
        t_ei += __builtin_readcyclecounter() - e0t;
#endif
    };

#ifdef RC_ROW_TIMING
    unsigned long long t_tr = 0, t_st = 0, t_fe = 0, t_sl = 0;   // transitions, steps; fetches and window slides (parts of the transitions)
    // what 16-lane rows could take (r06, profiles/r06_row16): a row's steps
    // until its candidate's live span first outgrows a 16-lane window (14
    // diagonals, simulated with its own centring), the candidates that never
    // do, and that window's slides
    unsigned long long n16 = 0, c16 = 0, sl16 = 0;
    bool ov16 = false, had = false;
    int w16 = 0;
#endif
    for (;;) {
#ifdef RC_ROW_TIMING
        const unsigned long long c0t = __builtin_readcyclecounter();
#endif
        // ---------------- transitions ----------------
        while (act < A_DONE) {
            if (act == A_FETCH) {
#ifdef RC_ROW_TIMING
                const unsigned long long f0t = __builtin_readcyclecounter();
#endif
                if (lnx >= s_ncand) {
                    // no work left: the row's lanes go dead for good (the
                    // other row's steps shift this row's edge lanes in)
                    R = -1;
                    act = A_DONE;
                    continue;
                }
                const uint64_t ci = cslot(lnx, RS_SHARD);
#ifdef RC_ROW_TIMING
                if (rl == 0 && had && !ov16) c16++;   // the previous candidate stayed within 14 diagonals
                ov16 = false;
                had = true;
#endif
                if (rl < CAND_DWORDS) meta[RM_REC + rl] = recv;
                if (rl == 0) {
                    meta[RM_CLO] = (int)(uint32_t)ci;
                    meta[RM_CHI] = (int)(uint32_t)(ci >> 32);
                }
                const uint32_t lidx = lnx;   // list index (the 64-lane pass's resume record)
                // prefetch the next record
                if (++lnx >= (uint32_t)RL.st[RS_LEND]) grab();
                recv = load_rec(lnx);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                const int Lq = meta[RM_REC + RC_LQ], Lt = meta[RM_REC + RC_LT];
                const uint64_t q0 = (uint64_t)(uint32_t)meta[RM_REC + RC_Q0];
                const uint64_t s0 = (uint64_t)(uint32_t)meta[RM_REC + RC_S0];
                const int strand = (meta[RM_REC + RC_CNT_STRAND] >> 16) & 1;
                const int nwq = (int)(((q0 & 31) + (uint64_t)Lq) >> 5) + 3;
                const int nwt = (int)(((s0 & 31) + (uint64_t)Lt) >> 5) + 3;
                const RowArgsK K = row_args();
                uint32_t qb = 0, tb = 0;
                if constexpr (WIN) {
                    // the first seed, then each slot's window from its
                    // extension's start (right: the seed's end; left: its start)
                    const uint32_t e01 = (uint32_t)meta[RM_REC + RC_E01];
                    const GSeed g0 =
                        K->P.seeds[(uint32_t)meta[RM_REC + RC_SOFF] + (K->P.which ? e01 >> 16 : e01 & 0xFFFFu)];
                    if (rl == 0) {
                        meta[RM_X] = (int)g0.x;
                        meta[RM_Y] = (int)g0.y;
                        meta[RM_LEN] = (int)(g0.len & SEED_LEN);
                    }
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    for (int sl = 0; sl < 4; sl++) {
                        uint32_t g, e;
                        slot_g(sl, g, e);
                        win_load(sl, slot_arr(sl), g >> 5, (e + 47u) >> 5);
                        if (rl == 0) wm[WM_W0 + sl] = (int)(g >> 5);
                    }
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                } else {
                // the left extensions walk reversed copies: the other
                // orientation's array from the mirrored start (complements on
                // both sides: the same matches), staged like the forward ones
                const uint64_t total = K->db.total;
                const uint64_t rq0 = total - q0 - (uint64_t)Lq, rs0 = total - s0 - (uint64_t)Lt;
                const int nwqr = (int)(((rq0 & 31) + (uint64_t)Lq) >> 5) + 3;
                const int nwtr = (int)(((rs0 & 31) + (uint64_t)Lt) >> 5) + 3;
                if (nwq > sw || nwt > sw || nwqr > sw || nwtr > sw) {
                    if (rl == 0 && row_args()->P.why) atomicAdd(&row_args()->P.why[0], 1ull);
                    defer(ci, false);
                    continue;
                }
                // raw words of query and subject, and the first seed: one round trip
                // both strands' pointers as scalars, selected per lane (an
                // indexed read of the kernarg segment would be a vector load,
                // one more round trip in front of the staging loads)
                GW dF = (GW)K->db.F, dRC = (GW)K->db.RC;
                asm volatile("" : "+s"(dF), "+s"(dRC));
                const GW QA = strand ? dRC : dF, QR = strand ? dF : dRC;
                const GW qw = QA + (q0 >> 5), tw = dF + (s0 >> 5);
                const GW qrw = QR + (rq0 >> 5), trw = dRC + (rs0 >> 5);
                {
                    // the first two words per lane of the four arrays in two
                    // batches (forward with the first seed, then reverse), each
                    // in flight together: the empty asm takes a batch whole, so
                    // the scheduler cannot sink its loads behind the LDS writes
                    // (r05_z: 2 round trips instead of 6, extension -0.5 ms at
                    // C3; one batch of all eight spills 16 VGPRs: +0.5 ms)
                    const uint32_t e01 = (uint32_t)meta[RM_REC + RC_E01];
                    const GSeed g0 =
                        K->P.seeds[(uint32_t)meta[RM_REC + RC_SOFF] + (K->P.which ? e01 >> 16 : e01 & 0xFFFFu)];
                    const uint64_t a0 = rl < nwq ? qw[rl] : 0ull, a1 = rl + RW < nwq ? qw[rl + RW] : 0ull;
                    const uint64_t b0 = rl < nwt ? tw[rl] : 0ull, b1 = rl + RW < nwt ? tw[rl + RW] : 0ull;
                    asm volatile("" ::"v"(a0), "v"(a1), "v"(b0), "v"(b1));
                    if (rl < nwq) stg[rl] = a0;
                    if (rl + RW < nwq) stg[rl + RW] = a1;
                    if (rl < nwt) stg[sw + rl] = b0;
                    if (rl + RW < nwt) stg[sw + rl + RW] = b1;
                    const uint64_t c0 = rl < nwqr ? qrw[rl] : 0ull, c1 = rl + RW < nwqr ? qrw[rl + RW] : 0ull;
                    const uint64_t d0 = rl < nwtr ? trw[rl] : 0ull, d1 = rl + RW < nwtr ? trw[rl + RW] : 0ull;
                    asm volatile("" ::"v"(c0), "v"(c1), "v"(d0), "v"(d1));
                    if (rl < nwqr) stg[2 * sw + rl] = c0;
                    if (rl + RW < nwqr) stg[2 * sw + rl + RW] = c1;
                    if (rl < nwtr) stg[3 * sw + rl] = d0;
                    if (rl + RW < nwtr) stg[3 * sw + rl + RW] = d1;
                    if (rl == 0) {
                        meta[RM_X] = (int)g0.x;
                        meta[RM_Y] = (int)g0.y;
                        meta[RM_LEN] = (int)(g0.len & SEED_LEN);
                    }
                }
                // (transcripts of more than 2 RW words: the rest)
                for (int w = rl + 2 * RW; w < nwq; w += RW) stg[w] = qw[w];
                for (int w = rl + 2 * RW; w < nwt; w += RW) stg[sw + w] = tw[w];
                for (int w = rl + 2 * RW; w < nwqr; w += RW) stg[2 * sw + w] = qrw[w];
                for (int w = rl + 2 * RW; w < nwtr; w += RW) stg[3 * sw + w] = trw[w];
                if (AMB) {
                    GW dAF = (GW)K->db.AF, dARC = (GW)K->db.ARC;
                    asm volatile("" : "+s"(dAF), "+s"(dARC));
                    const GW qm = (strand ? dARC : dAF) + (q0 >> 5), tm = dAF + (s0 >> 5);
                    const GW qrm = (strand ? dAF : dARC) + (rq0 >> 5), trm = dARC + (rs0 >> 5);
                    for (int w = rl; w < nwq; w += RW) stg[4 * sw + w] = qm[w];
                    for (int w = rl; w < nwt; w += RW) stg[5 * sw + w] = tm[w];
                    for (int w = rl; w < nwqr; w += RW) stg[6 * sw + w] = qrm[w];
                    for (int w = rl; w < nwtr; w += RW) stg[7 * sw + w] = trm[w];
                }
                qb = base0 + (uint32_t)(q0 & 31);
                tb = base0 + 32u * (uint32_t)sw + (uint32_t)(s0 & 31);
                if (rl == 0) {
                    meta[RM_QB] = (int)(bqr + (uint32_t)(rq0 & 31));
                    meta[RM_TB] = (int)(btr + (uint32_t)(rs0 & 31));
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                }
                if (rl == 0) atomicAdd(&rcnt[1], 1u);
                // right extension from the seed's end
                const int x = meta[RM_X], y = meta[RM_Y], len = meta[RM_LEN];
                const uint32_t sams = (uint32_t)meta[RM_REC + RC_SAMS];
                swap = (sams & 0xFFFFu) > (sams >> 16);
                pa = qb + (uint32_t)(x + len);
                alen = Lq - (x + len);
                pb = tb + (uint32_t)(y + len);
                blen = Lt - (y + len);
                if (swap) {
                    const uint32_t t = pa; pa = pb; pb = t;
                    const int u = alen; alen = blen; blen = u;
                }
                if constexpr (RW == 64) {
                    // a 32-lane extension that outgrew its window: continue it
                    // from the saved state (the diagonals outside the window
                    // were never reached, so the full band's state is it)
                    if (K->P.resume && K->P.list && lidx < K->P.res_cap) {
                        const int *rec = K->P.resume + (size_t)lidx * RES_REC;
                        const int phase = rec[RES_PHASE], kof = rec[RES_KOF];
                        if (phase == A_LDONE) {
                            if (rl < 5) meta[RM_RSC + rl] = rec[RES_RSC + rl];
                            // left extension: forward from reversed position L - x
                            pa = (uint32_t)meta[RM_QB] + (uint32_t)(Lq - x);
                            alen = x;
                            pb = (uint32_t)meta[RM_TB] + (uint32_t)(Lt - y);
                            blen = y;
                            if (swap) {
                                const uint32_t t = pa; pa = pb; pb = t;
                                const int u = alen; alen = blen; blen = u;
                            }
                        }
                        // the previous extension's steps; the resumed one's steps
                        // before the resume were counted by its first pass
                        if (rl == 0) atomicAdd(&rcnt[5], (uint32_t)(d6 - rec[RES_D6]));
                        d6 = rec[RES_D6];
                        best = rec[RES_BEST];
                        const int kb = rec[RES_PK];
                        bl = kb + RC0;
                        const int w = rl - RC0 - kof + 16;   // this diagonal's lane in the saved window
                        const bool inw = w >= 0 && w < 32;
                        R = inw ? rec[RES_R + (inw ? w : 0)] : -1;
                        goe = inw ? rec[RES_G + (inw ? w : 0)] : 0;
                        if (rl == bl) {
                            wi = rec[RES_PWI];
                            wg = rec[RES_PWG];
                            wd = rec[RES_PWD];
                        }
                        if constexpr (WIN) win_begin(phase == A_LDONE ? 1 : 0); else pbk = pb - (uint32_t)k;
                        blk = blen + k;
                        mnk = max(min(alen, blk), 0);
                        nkd = -(k + d6);
                        if (rl == 0) {
                            atomicAdd(&rcnt[0], 1u);
                            meta[RM_PHASE] = phase;
                            meta[RM_KOF] = 0;
                        }
                        act = phase + (A_STEP_R - A_RDONE);
                        continue;
                    }
                }
                ext_init(A_RDONE);
#ifdef RC_ROW_TIMING
                t_fe += __builtin_readcyclecounter() - f0t;
#endif
            } else if (act == A_SLIDE) {
#ifdef RC_ROW_TIMING
                const unsigned long long s0t = __builtin_readcyclecounter();
#endif
                // a live lane at the window's edge: centre the live diagonals
                const uint32_t livem = rw_mask<RW>(ballot(R >= 0), row);
                const int kof = meta[RM_KOF];
                const int lmin = __builtin_ctz(livem), lmax = 31 - __builtin_clz(livem);
                constexpr int KMAX = 31 - RW / 2;
                const int kn = max(-KMAX, min(KMAX, kof + ((lmin + lmax + 1) >> 1) - RC0));
                const int s = kn - kof;
                if (s == 0 || lmin - s < 1 || lmax - s > RW - 2) {
                    act = A_ABORT;   // wider than the window, or at the band's edge
                    if constexpr (SAVE && RW == 32) {
                        // what the 64-lane pass needs to continue it (A_ABORT
                        // saves it with the frontier): the best record parked
                        // as a slide parks it, the step count, the best score
                        if (bl != BL_PARKED) {
                            const int bsrc = RW * row + bl;
                            const int pwi = __shfl(wi, bsrc), pwg = __shfl(wg, bsrc), pwd = __shfl(wd, bsrc);
                            if (rl == 0) {
                                meta[RM_PWI] = pwi;
                                meta[RM_PWG] = pwg;
                                meta[RM_PWD] = pwd;
                                meta[RM_PK] = bl - RC0 + kof;
                            }
                        }
                        if (rl == 0) {
                            meta[RM_AD6] = d6;
                            meta[RM_ABEST] = best;
                        }
                    }
                    continue;
                }
                if (bl != BL_PARKED) {
                    // the row's best record leaves its lane's hands (that lane may leave the window)
                    const int bsrc = RW * row + bl;
                    const int pwi = __shfl(wi, bsrc), pwg = __shfl(wg, bsrc), pwd = __shfl(wd, bsrc);
                    if (rl == 0) {
                        meta[RM_PWI] = pwi;
                        meta[RM_PWG] = pwg;
                        meta[RM_PWD] = pwd;
                        meta[RM_PK] = bl - RC0 + kof;
                    }
                    bl = BL_PARKED;
                }
                const int from = rl + s;
                const bool in = from >= 0 && from < RW;
                const int nR = __shfl(R, RW * row + (in ? from : rl)), ng = __shfl(goe, RW * row + (in ? from : rl));
                R = in ? nR : -1;
                goe = in ? ng : 0;
                // this lane's diagonal was k + kof and is k + kn: refold it
                // into the per-lane constants (pb and blen are not kept)
                pbk -= (uint32_t)s;
                blk += s;
                mnk = max(min(alen, blk), 0);
                nkd -= s;
                if constexpr (WIN) win_lane(k + kn);
                if (rl == 0) {
                    meta[RM_KOF] = kn;
                    atomicAdd(&rcnt[3], 1u);
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                act = meta[RM_PHASE] + (A_STEP_R - A_RDONE);
#ifdef RC_ROW_TIMING
                t_sl += __builtin_readcyclecounter() - s0t;
#endif
            } else if (act == A_RDONE || act == A_LDONE) {
                int ei, ed, ego, kb;   // the best record and its diagonal
                if (bl == BL_PARKED) {
                    ei = meta[RM_PWI];
                    ed = meta[RM_PWD] / 6;
                    ego = meta[RM_PWG];
                    kb = meta[RM_PK];
                } else {
                    const int src = RW * row + bl;
                    ei = __shfl(wi, src);
                    ed = __shfl(wd, src) / 6;
                    ego = __shfl(wg, src);
                    kb = bl - RC0 + meta[RM_KOF];
                }
                int ej = ei - kb;
                if (swap) {
                    const int t = ei; ei = ej; ej = t;
                }
                if (act == A_RDONE) {
                    if (rl == 0) {
                        meta[RM_RSC] = best;
                        meta[RM_RI] = ei;
                        meta[RM_RJ] = ej;
                        meta[RM_RD] = ed;
                        meta[RM_RGO] = ego;
                    }
                    // left extension: forward from reversed position L - x
                    // (= base x - 1) of the reversed copies
                    const int x = meta[RM_X], y = meta[RM_Y];
                    const int Lq = meta[RM_REC + RC_LQ], Lt = meta[RM_REC + RC_LT];
                    pa = (uint32_t)meta[RM_QB] + (uint32_t)(Lq - x);
                    alen = x;
                    pb = (uint32_t)meta[RM_TB] + (uint32_t)(Lt - y);
                    blen = y;
                    if (swap) {
                        const uint32_t t = pa; pa = pb; pb = t;
                        const int u = alen; alen = blen; blen = u;
                    }
                    ext_init(A_LDONE);
                } else {
                    // both results of the first seed: first_finish_kernel builds the box
                    const uint64_t ci = (uint64_t)(uint32_t)meta[RM_CLO] | ((uint64_t)(uint32_t)meta[RM_CHI] << 32);
                    int v = 0;
                    if (rl >= FX_R && rl < FX_R + 5) v = meta[RM_RSC + (rl - FX_R)];
                    if (rl == FX_L) v = best;
                    if (rl == FX_L + 1) v = ei;
                    if (rl == FX_L + 2) v = ej;
                    if (rl == FX_L + 3) v = ed;
                    if (rl == FX_L + 4) v = ego;
                    if (rl < BOX_REC) box_out()[ci * BOX_REC + rl] = v;
                    act = A_FETCH;
                }
            } else {   // A_ABORT: the sub-band overflowed
                const uint64_t ci = (uint64_t)(uint32_t)meta[RM_CLO] | ((uint64_t)(uint32_t)meta[RM_CHI] << 32);
                const unsigned long long wi2 = defer(ci, true);
                if constexpr (SAVE && RW == 32) {
                    // the wide pass continues from here: the window's frontier
                    // and the header A_SLIDE left in the bookkeeping
                    if (wi2 != ~0ull) {
                        const RowArgsK K = row_args();
                        if (K->P.resume && wi2 < K->P.res_cap) {
                            int *rec = K->P.resume + (size_t)wi2 * RES_REC;
                            rec[RES_R + rl] = R;
                            rec[RES_G + rl] = goe;
                            // the bookkeeping from the right results to the best
                            // record, the step count, the best score
                            if (rl <= RES_PK) rec[rl] = meta[RM_RSC + rl];
                            if (rl == RES_D6) rec[rl] = meta[RM_AD6];
                            if (rl == RES_BEST) rec[rl] = meta[RM_ABEST];
                        }
                    }
                }
                if (rl == 0) atomicAdd(&rcnt[2], 1u);
                act = A_FETCH;
            }
        }
#ifdef RC_ROW_TIMING
        const unsigned long long c1t = __builtin_readcyclecounter();
        t_tr += c1t - c0t;
#endif
        const bool ext = act >= A_STEP_R;
        const uint64_t mext = m_ge(act, A_STEP_R);
        if (!mext) break;
        // ---------------- one greedy step of every extending row ----------------
        if (ext) {
            d6 += 6;
            nkd -= 6;
            const int Rl = rw_from_lower<RW, true>(R, -1, rl), Rr = rw_from_upper<RW, true>(R, -1, rl);
            const int gl = rw_from_lower<RW, false>(goe, 0, rl), gr = rw_from_upper<RW, false>(goe, 0, rl);
            // candidates; ties prefer mismatch, then insertion, then deletion (a
            // frontier value R >= 0 has j = R - k >= 0, so unsigned compares
            // carry the lower bounds)
            // (j = R - k < blen  <=>  R < blk;  j + 1 = Rr - k < blen + 1  <=>  Rr <= blk)
            const int cm = ((uint32_t)R < (uint32_t)mnk) ? R + 1 : -1;
            const int cil = ((uint32_t)Rl < (uint32_t)alen) ? Rl + 1 : -1;
            const int cd = (Rr >= 0 && Rr <= blk) ? Rr : -1;
            int ni = max(max(cm, cil), cd);
            const bool fm = ni >= 0 && cm == ni, fi = !fm && cil == ni;
            // gap state of the chosen move: G | O << 13 | E << 26 (E: 1 insertion, 2 deletion)
            const int src = fm ? goe : (fi ? gl : gr);
            const int e = fm ? 0 : (fi ? 1 : 2);
            const int pe = (src >> EBIT) & 3;
            // (E goes in after the slide: matches after the move clear it)
            const int ngb = (src & ~(3 << EBIT)) + (fm ? 0 : 1 + (pe == e ? 0 : (1 << OBIT)));
            int ee = e;
            // the score of a lane live after the step; its bound (the score
            // if every remaining base matched): 2 (ni + s) - k - d6 + 2 (m - s)
            // = 2 min(alen, blk) + nkd, on every lane (only live lanes' are read)
            int score = 0;
            const int bound = 2 * mnk + nkd;
            if constexpr (WIN) {
                // slides stop at the window; the ones that reached it (or
                // start outside it) are finished after a refill
                int m = 0, s = 0;
                bool pend = false;
                if (ni >= 0) {
                    m = mnk - ni;
                    const int mw = ni < wlo ? -1 : min(m, wlim - ni);
                    s = slide_fwd<AMB>(pa + (uint32_t)ni, pbk + (uint32_t)ni, max(mw, 0), moff);
                    pend = mw < m && s >= mw;
                }
                if (ballot(pend)) win_resolve(ni, s, m, pend);
                if (ni >= 0) {
                    ni += s;
                    if (s > 0) ee = 0;
                    score = 2 * ni + nkd;   // 2 ni - k - d6
                    if (score < best - X) ni = -1;
                }
            } else if (ni >= 0) {
                const int m = mnk - ni;
                const int s = slide_fwd<AMB>(pa + (uint32_t)ni, pbk + (uint32_t)ni, m, moff);
                ni += s;
                if (s > 0) ee = 0;
                score = 2 * ni + nkd;   // 2 ni - k - d6
                if (score < best - X) ni = -1;
            }
            const int ng = ngb + (ee << EBIT);
            R = ni;
            goe = ng;
            const bool live = ni >= 0;
            // row-wide decisions as lane masks (scalar), applied with v_cndmask.
            // A lane X-dropped this step has score < best.
            const uint64_t mlive = m_ge(ni, 0);
#ifdef RC_ROW_TIMING
            if constexpr (RW == 32) {
                const uint32_t lv = rw_mask<RW>(mlive, row);
                if (d6 == 6) w16 = 0;   // an extension's first step: the window starts centred
                if (lv) {
                    const int kofr = meta[RM_KOF];
                    const int dmin = __builtin_ctz(lv) - RC0 + kofr, dmax = (31 - __builtin_clz(lv)) - RC0 + kofr;
                    if (dmax - dmin + 1 > 14 || dmin < w16 - 8 || dmax > w16 + 7) {
                        ov16 = true;
                    } else if (!ov16 && (dmin == w16 - 8 || dmax == w16 + 7)) {
                        const int c = (dmin + dmax + 1) >> 1;
                        if (c < -23 || c > 23) ov16 = true;
                        else {
                            w16 = c;
                            if (rl == 0) sl16++;
                        }
                    }
                }
                if (!ov16 && rl == 0) n16++;
            }
#endif
            const uint64_t mi = m_gt(score, best) & mlive;
            const uint64_t mimp = rw_spread<RW>(mi);
            if (mimp) {
                uint64_t mwin;
                const uint32_t lo = (uint32_t)mi, hi = (uint32_t)(mi >> 32);
                if (RW == 32 && !(lo & (lo - 1)) && !(hi & (hi - 1))) {
                    // at most one improving lane per row (the usual case): it is
                    // the row's new best, read out directly, no row reduction
                    // (a row without an improving lane reads an unused lane)
                    const int a = s_ff1(lo) & 31, b = s_ff1(hi) & 31;
                    const int s0 = __builtin_amdgcn_readlane(score, a), s1 = __builtin_amdgcn_readlane(score, 32 + b);
                    constexpr uint64_t ROW0 = 0xFFFFFFFFull;
                    best = lane_sel(mimp & ROW0, s0, lane_sel(mimp & ~ROW0, s1, best));
                    bl = lane_sel(mimp & ROW0, a, lane_sel(mimp & ~ROW0, b, bl));
                    mwin = mi;
                } else {
                    const int mk = rw_max<RW>(live ? score * RW + (RW - 1 - rl) : INT_MIN);
                    best = lane_sel(mimp, mk >> (RW == 64 ? 6 : (RW == 32 ? 5 : 4)), best);
                    bl = lane_sel(mimp, RW - 1 - (mk & (RW - 1)), bl);
                    mwin = mimp & m_eq(rl, bl);
                }
                wi = lane_sel(mwin, R, wi);
                wg = lane_sel(mwin, goe, wg);
                wd = lane_sel(mwin, d6, wd);
            }
            // bound >= score, so a lane that can still beat best is live
            // a live lane at a sub-band edge: the candidate goes to a wider
            // pass; 64-lane rows are the spec's band itself (no edge abort)
            constexpr uint64_t EDGES = RW == 64 ? 0ull : (RW == 32 ? 0x8000000180000001ull : 0x8001800180018001ull);
            const uint64_t mcont = rw_spread<RW>(mlive & m_gt(bound, best)) & m_lt(d6, 6 * DMAX);
            const uint64_t medge = RW == 64 ? 0ull : rw_spread<RW>(mlive & EDGES);
            act = lane_sel(mcont, lane_sel_k<A_SLIDE>(medge, act), act - (A_STEP_R - A_RDONE));
        }
#ifdef RC_ROW_TIMING
        t_st += __builtin_readcyclecounter() - c1t;
#endif
    }
#ifdef RC_ROW_TIMING
    unsigned long long *const counters = row_args()->P.counters;
    if (lane == 0 && counters) {
        atomicAdd(&counters[8], t_tr);
        atomicAdd(&counters[9], t_st);
        atomicAdd(&counters[27], t_fe);   // (d_count[28], [29]: slots nothing else uses)
        atomicAdd(&counters[28], t_sl);
        atomicAdd(&counters[29], t_ei);
    }
    if (rl == 0 && had && !ov16) c16++;
    if (rl == 0 && counters) {
        atomicAdd(&counters[26], n16);
        atomicAdd(&counters[30], c16);
        atomicAdd(&counters[31], sl16);
    }
#endif
    unsigned long long *const ctr = row_args()->P.counters;
    if (rl == 0 && d6) atomicAdd(&rcnt[5], (uint32_t)d6);   // the last extension's steps
    __syncthreads();
    if (threadIdx.x < 4 && ctr) atomicAdd(&ctr[1 + threadIdx.x], (unsigned long long)rcnt[threadIdx.x]);   // [4]: slides
    if (threadIdx.x == 5 && ctr) atomicAdd(&ctr[0], (unsigned long long)(rcnt[5] / 6u));
}

// The candidates' first-seed extensions -> box; the other seeds of the
// candidate are checked against it (spec 3: a seed inside a found HSP box is
// not extended). All inside: the candidate has this one HSP -- e-value cuts of
// both directions, HSP record. Otherwise extend_kernel redoes the candidate
// whole (the defer list it runs next). One thread per candidate.
__global__ __launch_bounds__(256) void first_finish_kernel(ExtParams P)
{
    constexpr int OBIT = 13, GMASK = 8191;
    for (uint64_t li = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; li < P.n_cand;
         li += (uint64_t)gridDim.x * blockDim.x) {
        int lo = 0, hi = NSHARD;
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (P.shard_prefix[mid] <= li) lo = mid; else hi = mid;
        }
        const uint64_t ci = (uint64_t)lo * P.cand_cap + (li - P.shard_prefix[lo]);
        if (!P.share && P.cand_box[ci * BOX_REC + FX_STATUS] < 0) continue;   // deferred by the row kernel
        const Cand cd = P.cands[ci];
        // shared searches: each directed search of the candidate on its own --
        // its first seed's box (cand_box, or cand_box2 when the reverse
        // search's first seed is another seed), its own seeds, its own cut.
        // Both searches' containment tests share one pass over the seeds.
        const int ndir = P.share ? 2 : 1;
        bool live[2] = {false, false};
        int bqa[2] = {0, 0}, bqb[2] = {0, 0}, bsa[2] = {0, 0}, bsb[2] = {0, 0}, ex[2] = {-1, -1};
        const int *fxd[2] = {nullptr, nullptr};
        // each live search's HSP fields from its box, computed (and the bit
        // score and cut loads issued) before the pass over the seeds, so that
        // they are not round trips of their own after it
        int bsc[2] = {0, 0}, bd[2] = {0, 0}, bg[2] = {0, 0}, bo[2] = {0, 0}, bni[2] = {0, 0}, b10[2] = {0, 0};
        const int thr_f = P.thr[(size_t)cd.ssam * (size_t)(P.max_len + 1) + (size_t)cd.Lq];
        const int thr_r = P.thr[(size_t)cd.qsam * (size_t)(P.max_len + 1) + (size_t)cd.Lt];
        for (int dir = 0; dir < ndir; dir++) {
            if (P.share && !((cd.dflags >> dir) & 1)) {   // this search found no seed here
                (dir ? P.cand_nh_r : P.cand_nh)[ci] = 0;
                (dir ? P.cand_ovf_r : P.cand_ovf)[ci] = 0;
                continue;
            }
            const bool second = dir == 1 && cd.e1 != SEED_NONE;
            fxd[dir] = (second ? P.cand_box2 : P.cand_box) + ci * BOX_REC;
            if (fxd[dir][FX_STATUS] < 0) {   // (shared searches) the row kernel gave it up
                if (P.why) atomicAdd(&P.why[1], 1ull);
                const unsigned long long di = atomicAdd(dir ? P.defer_r_count : P.defer_count, 1ull);
                (dir ? P.defer_r : P.defer)[di] = (uint32_t)ci;
                continue;
            }
            ex[dir] = (int)(second ? cd.e1 : cd.e0);
            const GSeed s0 = P.seeds[cd.seed_off + ex[dir]];
            const int *fx = fxd[dir];
            const int x = (int)s0.x, y = (int)s0.y, len = (int)(s0.len & SEED_LEN);
            bqa[dir] = x - fx[FX_L + 1];
            bqb[dir] = x + len + fx[FX_R + 1];
            bsa[dir] = y - fx[FX_L + 2];
            bsb[dir] = y + len + fx[FX_R + 2];
            live[dir] = true;
            const int rsc = fx[FX_R], ri = fx[FX_R + 1], rj = fx[FX_R + 2], rd = fx[FX_R + 3], rgo = fx[FX_R + 4];
            const int lsc = fx[FX_L], lI = fx[FX_L + 1], lJ = fx[FX_L + 2], ld = fx[FX_L + 3], lgo = fx[FX_L + 4];
            const int lg = lgo & GMASK, lo2 = (lgo >> OBIT) & GMASK, rg = rgo & GMASK, ro = (rgo >> OBIT) & GMASK;
            bsc[dir] = lsc + 2 * len + rsc;
            bd[dir] = ld + rd;
            bg[dir] = lg + rg;
            bo[dir] = lo2 + ro;
            bni[dir] = len + (lI + lJ - 2 * ld + lg) / 2 + (ri + rj - 2 * rd + rg) / 2;
            b10[dir] = P.bits10[bsc[dir]];
        }
        // the other seeds of each live search inside its box? (four seeds'
        // loads in flight at a time)
        bool in0 = live[0], in1 = live[1];
        const GSeed *const sp = P.seeds + cd.seed_off;
        const uint32_t ns = cand_seeds(cd);
        for (uint32_t i0 = 0; i0 < ns && (in0 || in1); i0 += 4) {
            GSeed s4[4];
#pragma unroll
            for (int k = 0; k < 4; k++) s4[k] = i0 + k < ns ? sp[i0 + k] : GSeed{0u, 0u, 0u};
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int i = (int)(i0 + k);
                if (i >= (int)ns) break;
                const int sl = (int)(s4[k].len & SEED_LEN), sx = (int)s4[k].x, sy = (int)s4[k].y;
                // without shared searches every seed is the one search's
                const bool f = !P.share || (s4[k].len & SEED_F), r = P.share && (s4[k].len & SEED_R);
                if (in0 && f && i != ex[0])
                    in0 = bqa[0] <= sx && sx + sl <= bqb[0] && bsa[0] <= sy && sy + sl <= bsb[0];
                if (in1 && r && i != ex[1])
                    in1 = bqa[1] <= sx && sx + sl <= bqb[1] && bsa[1] <= sy && sy + sl <= bsb[1];
            }
        }
        for (int dir = 0; dir < ndir; dir++) {
            if (!live[dir]) continue;
            DHsp *const hsp_out = dir ? P.cand_hsp_r : P.cand_hsp;
            uint8_t *const nh_out = dir ? P.cand_nh_r : P.cand_nh;
            uint32_t *const ovf_out = dir ? P.cand_ovf_r : P.cand_ovf;
            if (!(dir ? in1 : in0)) {
                if (P.why) atomicAdd(&P.why[2], 1ull);
                const unsigned long long di = atomicAdd(dir ? P.defer_r_count : P.defer_count, 1ull);
                (dir ? P.defer_r : P.defer)[di] = (uint32_t)ci;
                continue;
            }
            const bool pf = (!P.share || dir == 0) && bsc[dir] >= thr_f;
            const bool pr = (P.sym || (P.share && dir == 1)) && bsc[dir] >= thr_r;
            if (pf || pr) {
                DHsp h;
                h.q_tx = cd.q_gtx;
                h.s_tx = cd.s_gtx;
                if (!cd.strand) {
                    h.qstart = bqa[dir] + 1; h.qend = bqb[dir]; h.sstart = bsa[dir] + 1; h.send = bsb[dir];
                } else {
                    h.qstart = cd.Lq - bqb[dir] + 1; h.qend = cd.Lq - bqa[dir];
                    h.sstart = bsb[dir]; h.send = bsa[dir] + 1;
                }
                h.gaps = bg[dir];
                h.gapopen = bo[dir];
                h.mismatch = bd[dir] - bg[dir];
                h.nident = bni[dir];
                h.length = bni[dir] + bd[dir];
                h.score_half = bsc[dir];
                h.bits10 = b10[dir];
                h.strand = cd.strand | (pf ? HSP_FWD : 0) | (pr ? HSP_REV : 0);
                hsp_out[ci] = h;
            }
            nh_out[ci] = (uint8_t)((pf || pr) ? 1 : 0);
            ovf_out[ci] = 0;
        }
    }
}

// HSP box of a seed (x, y, len) from its row-kernel results (cand_box
// record): what process_search builds from extend_seed's two results
__device__ __forceinline__ void box_from_fx(const int *fx, int x, int y, int len, int *b)
{
    constexpr int OBIT = 13, GMASK = 8191;
    const int rsc = fx[FX_R], ri = fx[FX_R + 1], rj = fx[FX_R + 2], rd = fx[FX_R + 3], rgo = fx[FX_R + 4];
    const int lsc = fx[FX_L], lI = fx[FX_L + 1], lJ = fx[FX_L + 2], ld = fx[FX_L + 3], lgo = fx[FX_L + 4];
    const int lg = lgo & GMASK, lo = (lgo >> OBIT) & GMASK, rg = rgo & GMASK, ro = (rgo >> OBIT) & GMASK;
    b[LB_QA] = x - lI;
    b[LB_QB] = x + len + ri;
    b[LB_SA] = y - lJ;
    b[LB_SB] = y + len + rj;
    b[LB_SC] = lsc + 2 * len + rsc;
    b[LB_D] = ld + rd;
    b[LB_G] = lg + rg;
    b[LB_O] = lo + ro;
    b[LB_NI] = len + (lI + lJ - 2 * ld + lg) / 2 + (ri + rj - 2 * rd + rg) / 2;
}

// A search the later-seed rounds cannot take: extend_kernel runs it whole
// (from its first seed's HSP, P.reuse_first)
__device__ __forceinline__ void later_full(const LaterParams &L, int dir, uint64_t ci)
{
    const unsigned long long i = atomicAdd(&L.full_n[dir], 1ull);
    (dir ? L.full1 : L.full0)[i] = (uint32_t)ci;
    if (L.counters) atomicAdd(&L.counters[1], 1ull);
}

// One round of the later-seed rounds, one thread per active search: take the
// result of the seed the previous round extended (round 0: the first seed's,
// from cand_box / cand_box2) as the search's next HSP, then pick the next seed
// as process_search does -- the first in the search's order outside every box
// so far -- and list it for the row kernels as a candidate record whose e0 is
// that seed. A search with no such seed is finished; one at MAX_HSP HSPs with
// such a seed is finished and MAX_HSP-bound (spec 3).
__device__ __forceinline__ bool later_step(const ExtParams &P, const LaterParams &L, uint64_t s, uint32_t &bi_out)
{
    const int dir = s >= L.n0 ? 1 : 0;
    const uint64_t ci = dir ? L.defer1[s - L.n0] : L.defer0[s];
    if (s >= L.n_cap) {   // (round 0 only: past the states' capacity)
        later_full(L, dir, ci);
        return false;
    }
    int *const st = L.state + s * LATER_REC;
    const Cand cd = P.cands[ci];
    const GSeed *const sd = P.seeds + cd.seed_off;
    int nh;
    uint32_t last;   // the seed extended last
    if (L.round == 0) {
        const bool second = dir == 1 && cd.e1 != SEED_NONE;
        const int *fx = (second ? P.cand_box2 : P.cand_box) + ci * BOX_REC;
        st[LS_CAPPED] = 0;
        st[LS_PEND] = -1;
        if (fx[FX_STATUS] < 0) {   // the row kernels gave its first seed up
            st[LS_STATE] = LATER_FULL;
            later_full(L, dir, ci);
            return false;
        }
        last = second ? cd.e1 : cd.e0;
        const GSeed g = sd[last];
        box_from_fx(fx, (int)g.x, (int)g.y, (int)(g.len & SEED_LEN), st + LS_BOX);
        nh = 1;
    } else {
        nh = st[LS_STATE];
        const int w = st[LS_PEND];
        const int *fx = L.box_in + (size_t)w * BOX_REC;
        if (fx[FX_STATUS] < 0) {   // the row kernels gave this seed up
            st[LS_STATE] = LATER_FULL;
            later_full(L, dir, ci);
            return false;
        }
        last = L.vc_in[w].e0;
        const GSeed g = sd[last];
        box_from_fx(fx, (int)g.x, (int)g.y, (int)(g.len & SEED_LEN), st + LS_BOX + nh * LB_N);
        nh++;
    }
    // the next seed: the search's own seeds, in its order, outside every box
    // (the boxes in registers; an unused one is empty)
    int qa[MAX_HSP], qb[MAX_HSP], sa[MAX_HSP], sb[MAX_HSP];
#pragma unroll
    for (int h = 0; h < MAX_HSP; h++) {
        const int *b = st + LS_BOX + h * LB_N;
        const bool u = h < nh;
        qa[h] = u ? b[LB_QA] : INT_MAX;
        qb[h] = u ? b[LB_QB] : INT_MIN;
        sa[h] = u ? b[LB_SA] : INT_MAX;
        sb[h] = u ? b[LB_SB] : INT_MIN;
    }
    const uint32_t dbit = dir ? SEED_R : SEED_F;
    const uint32_t ns = cand_seeds(cd);
    unsigned long long bk = ~0ull;
    uint32_t bi = 0;
    // the forward search's order is the seeds' (x, y) order: the seeds before
    // the last one extended were inside a box when it was picked, and boxes
    // only grow, so they still are (the reverse order is another permutation)
    for (uint32_t i = dir ? 0u : last + 1u; i < ns; i++) {
        const GSeed g = sd[i];
        if (!(g.len & dbit)) continue;
        const int x = (int)g.x, y = (int)g.y, len = (int)(g.len & SEED_LEN);
        bool in = false;
#pragma unroll
        for (int h = 0; h < MAX_HSP; h++)
            in = in || (qa[h] <= x && x + len <= qb[h] && sa[h] <= y && y + len <= sb[h]);
        if (in) continue;
        const unsigned long long key =
            !dir ? ((unsigned long long)g.x << 32) | g.y
                 : (cd.strand ? ((unsigned long long)(uint32_t)~(g.y + (uint32_t)len) << 32) |
                                    (uint32_t)~(g.x + (uint32_t)len)
                              : ((unsigned long long)g.y << 32) | g.x);
        if (key < bk) {
            bk = key;
            bi = i;
        }
    }
    st[LS_STATE] = nh;
    if (bk == ~0ull) return false;   // every seed inside a box: finished
    if (nh >= MAX_HSP) {             // MAX_HSP binds
        st[LS_CAPPED] = 1;
        return false;
    }
    if (bi >= SEED_NONE) {           // past the record's 16-bit seed field
        st[LS_STATE] = LATER_FULL;
        later_full(L, dir, ci);
        return false;
    }
    bi_out = bi;   // (its record goes out once the wave has its work slots)
    return true;
}

__global__ __launch_bounds__(256) void later_round_kernel(ExtParams P, LaterParams L)
{
    const uint64_t n = L.round == 0 ? L.n_search : (uint64_t)*L.act_in_n;
    const int lane = threadIdx.x & 63;
    // whole waves iterate together (the work slots are allocated per wave)
    for (uint64_t b0 = blockIdx.x * (uint64_t)blockDim.x; b0 < n; b0 += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t li = b0 + threadIdx.x;
        uint64_t s = 0;
        uint32_t bi = 0;
        bool emit = false;
        if (li < n) {
            s = L.round == 0 ? li : (uint64_t)L.act_in[li];
            emit = later_step(P, L, s, bi);
        }
        const uint64_t m = __ballot(emit);
        if (!m) continue;
        const int cnt = __popcll(m);
        const int leader = __ffsll((unsigned long long)m) - 1;
        unsigned long long wb = 0, ab = 0;
        if (lane == leader) {
            wb = atomicAdd(L.work_n, (unsigned long long)cnt);
            ab = atomicAdd(L.act_out_n, (unsigned long long)cnt);
        }
        wb = (unsigned long long)__shfl((long long)wb, leader);
        ab = (unsigned long long)__shfl((long long)ab, leader);
        if (emit) {
            const int rk = __popcll(m & ((1ull << lane) - 1ull));
            const uint64_t w = wb + rk;
            const int dir = s >= L.n0 ? 1 : 0;
            const uint64_t ci = dir ? L.defer1[s - L.n0] : L.defer0[s];
            Cand v = P.cands[ci];
            v.e0 = (uint16_t)bi;
            v.e1 = SEED_NONE;
            L.vc[w] = v;
            L.list[w] = (uint32_t)w;
            L.state[s * LATER_REC + LS_PEND] = (int)w;
            L.act_out[ab + rk] = (uint32_t)s;
        }
    }
}

// The searches the rounds finished, one thread each: extend_kernel's end of a
// search -- purge of HSPs with a common end point, by (score desc, index
// asc), then the direction's e-value cut -- and its records: the first in
// cand_hsp (_r), the others in the overflow buffer (one atomic per wave).
__global__ __launch_bounds__(256) void later_finish_kernel(ExtParams P, LaterParams L)
{
    const uint64_t n = L.n_search < L.n_cap ? L.n_search : L.n_cap;
    const int lane = threadIdx.x & 63;
    for (uint64_t b0 = blockIdx.x * (uint64_t)blockDim.x; b0 < n; b0 += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t s = b0 + threadIdx.x;
        const int *const st = L.state + s * LATER_REC;
        const int nh = s < n ? st[LS_STATE] : -1;
        const bool live = nh >= 0;
        const int dir = s >= L.n0 ? 1 : 0;
        uint64_t ci = 0;
        Cand cd{};
        int qa[MAX_HSP], qb[MAX_HSP], sa[MAX_HSP], sb[MAX_HSP], sc[MAX_HSP];
        uint32_t outm = 0, pfm = 0, prm = 0;
        bool capped = false;
        if (live) {
            ci = dir ? L.defer1[s - L.n0] : L.defer0[s];
            cd = P.cands[ci];
            capped = st[LS_CAPPED] != 0;
#pragma unroll
            for (int h = 0; h < MAX_HSP; h++) {
                const int *b = st + LS_BOX + h * LB_N;
                const bool u = h < nh;
                qa[h] = u ? b[LB_QA] : 0;
                qb[h] = u ? b[LB_QB] : 0;
                sa[h] = u ? b[LB_SA] : 0;
                sb[h] = u ? b[LB_SB] : 0;
                sc[h] = u ? b[LB_SC] : INT_MIN;
            }
            // purge: in (score desc, index asc) order, an HSP sharing its start
            // or its end point with one kept before it goes
            uint32_t kept = 0, done = 0;
            for (int rr = 0; rr < nh; rr++) {
                int i = -1, bs = INT_MIN;
#pragma unroll
                for (int h = 0; h < MAX_HSP; h++)
                    if (h < nh && !((done >> h) & 1u) && (i < 0 || sc[h] > bs)) {
                        i = h;
                        bs = sc[h];
                    }
                done |= 1u << i;
                bool conflict = false;
#pragma unroll
                for (int h = 0; h < MAX_HSP; h++)
                    conflict = conflict || (((kept >> h) & 1u) && ((qa[h] == qa[i] && sa[h] == sa[i]) ||
                                                                   (qb[h] == qb[i] && sb[h] == sb[i])));
                if (!conflict) kept |= 1u << i;
            }
            const int thr_f = P.thr[(size_t)cd.ssam * (size_t)(P.max_len + 1) + (size_t)cd.Lq];
            const int thr_r = P.thr[(size_t)cd.qsam * (size_t)(P.max_len + 1) + (size_t)cd.Lt];
#pragma unroll
            for (int h = 0; h < MAX_HSP; h++) {
                const bool pf = (!P.share || !dir) && sc[h] >= thr_f;
                const bool pr = (P.sym || (P.share && dir)) && sc[h] >= thr_r;
                if (((kept >> h) & 1u) && (pf || pr)) {
                    outm |= 1u << h;
                    pfm |= (pf ? 1u : 0u) << h;
                    prm |= (pr ? 1u : 0u) << h;
                }
            }
        }
        // overflow slots of HSPs 2.. of the wave's searches: one atomic
        const int nout = __popc(outm);
        const uint32_t need = nout > 1 ? (uint32_t)(nout - 1) : 0u;
        uint32_t incl = need;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t v = (uint32_t)__shfl_up((int)incl, o);
            if (lane >= o) incl += v;
        }
        const uint32_t tot = (uint32_t)__shfl((int)incl, 63);
        unsigned long long wb = 0;
        if (lane == 63 && tot) {
            wb = atomicAdd(P.ovf_count, (unsigned long long)tot);
            if (wb + tot > P.ovf_cap) atomicOr(P.status, 1u);
        }
        wb = (unsigned long long)__shfl((long long)wb, 63);
        if (P.counters) {
            const uint64_t cm = __ballot(capped);
            if (lane == 0 && cm) atomicAdd(&P.counters[10], (unsigned long long)__popcll(cm));
        }
        if (!live) continue;
        const uint32_t obase = need ? (uint32_t)(wb + incl - need) : 0u;
        DHsp *const hsp_out = dir ? P.cand_hsp_r : P.cand_hsp;
        int rk = 0;
        for (int h = 0; h < nh; h++) {
            if (!((outm >> h) & 1u)) continue;
            const int *b = st + LS_BOX + h * LB_N;
            DHsp o;
            o.q_tx = cd.q_gtx;
            o.s_tx = cd.s_gtx;
            if (!cd.strand) {
                o.qstart = b[LB_QA] + 1; o.qend = b[LB_QB]; o.sstart = b[LB_SA] + 1; o.send = b[LB_SB];
            } else {
                o.qstart = cd.Lq - b[LB_QB] + 1; o.qend = cd.Lq - b[LB_QA]; o.sstart = b[LB_SB]; o.send = b[LB_SA] + 1;
            }
            const int bd = b[LB_D], bg = b[LB_G], bni = b[LB_NI];
            o.gaps = bg;
            o.gapopen = b[LB_O];
            o.mismatch = bd - bg;
            o.nident = bni;
            o.length = bni + (bd - bg) + bg;
            o.score_half = b[LB_SC];
            o.bits10 = P.bits10[b[LB_SC]];
            o.strand = cd.strand | (((pfm >> h) & 1u) ? HSP_FWD : 0) | (((prm >> h) & 1u) ? HSP_REV : 0) |
                       (h << HSP_IDX_SHIFT);
            if (rk == 0) hsp_out[ci] = o;
            else if ((uint64_t)obase + (rk - 1) < P.ovf_cap) P.ovf[obase + rk - 1] = o;
            rk++;
        }
        (dir ? P.cand_nh_r : P.cand_nh)[ci] = (uint8_t)nout;
        (dir ? P.cand_ovf_r : P.cand_ovf)[ci] = obase;
    }
}

// ------------------------------------------------------------------------
// (gene, sample) groups
// ------------------------------------------------------------------------

__global__ void group_count_kernel(GroupParams P)
{
    const uint64_t sg = (uint64_t)(P.gene_end - P.gene_begin), n = sg * (uint64_t)P.N;
    // gi: the seed kernel's gene-major (query gene, subject sample) index, read
    // in order; si: sample-major, the order direct groups are placed in
    for (uint64_t gi = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; gi < n;
         gi += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t si = (gi % (uint64_t)P.N) * sg + gi / (uint64_t)P.N;
        const uint32_t o = P.gc_off[gi], c = P.gc_cnt[gi];
        uint32_t s = 0;
        for (uint32_t i = 0; i < c; i++) {
            const uint32_t nh = P.cand_nh[o + i];
            if (!nh) continue;
            s += (P.cand_hsp[o + i].strand & HSP_FWD) ? 1u : 0u;
            const uint32_t ov = P.cand_ovf[o + i];
            for (uint32_t k = 1; k < nh; k++) s += (P.ovf[ov + k - 1].strand & HSP_FWD) ? 1u : 0u;
        }
        P.cnt[si] = s;
    }
}

__global__ void group_write_kernel(GroupParams P)
{
    const uint64_t sg = (uint64_t)(P.gene_end - P.gene_begin), n = sg * (uint64_t)P.N;
    for (uint64_t gi = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; gi < n;
         gi += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t si = (gi % (uint64_t)P.N) * sg + gi / (uint64_t)P.N;
        const uint32_t o = P.gc_off[gi], c = P.gc_cnt[gi];
        uint64_t w = P.base + P.scan[si];
        const uint64_t gg = grp_index(P.gene_begin + (uint32_t)(si % sg), (int)(si / sg), P.n_genes);
        if (P.cnt[si]) {
            P.grp_off[gg] = (uint32_t)w;
            P.grp_cnt[gg] = P.cnt[si];
        }
        for (uint32_t i = 0; i < c; i++) {
            const uint32_t nh = P.cand_nh[o + i];
            if (!nh) continue;
            const DHsp &h0 = P.cand_hsp[o + i];
            if (h0.strand & HSP_FWD) P.out[w++] = h0;
            const uint32_t ov = P.cand_ovf[o + i];
            for (uint32_t k = 1; k < nh; k++)
                if (P.ovf[ov + k - 1].strand & HSP_FWD) P.out[w++] = P.ovf[ov + k - 1];
        }
    }
}

// the mirror image of a query->subject HSP, as the subject->query search reports it
__device__ __forceinline__ DHsp mirror_hsp(const DHsp &h)
{
    DHsp m = h;
    m.q_tx = h.s_tx;
    m.s_tx = h.q_tx;
    if (!(h.strand & 1)) {
        m.qstart = h.sstart; m.qend = h.send; m.sstart = h.qstart; m.send = h.qend;
    } else {
        m.qstart = h.send; m.qend = h.sstart; m.sstart = h.qend; m.send = h.qstart;
    }
    return m;
}

// candidate slot of linear candidate index li
__device__ __forceinline__ uint64_t cand_slot(const GroupParams &P, uint64_t li)
{
    int lo = 0, hi = NSHARD;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (P.shard_prefix[mid] <= li) lo = mid; else hi = mid;
    }
    return (uint64_t)lo * P.cand_cap + (li - P.shard_prefix[lo]);
}

// pass 0: count mirrored HSPs per (gene of the subject tx, query sample),
// one atomic per candidate (its HSPs share the group), whose return -- the
// candidate's first slot in the group -- is kept per candidate; pass 1:
// scatter them from there, no atomics (the order inside a group is fixed
// later by mirror_sort_kernel)
__global__ void mirror_scatter_kernel(GroupParams P, int pass)
{
    for (uint64_t li = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; li < P.n_cand;
         li += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t ci = cand_slot(P, li);
        const uint32_t nh = P.cand_nh[ci];
        if (!nh) continue;
        const uint32_t ov = P.cand_ovf[ci];
        uint64_t gi = 0, slot = 0;
        uint32_t c = 0;
        for (uint32_t k = 0; k < nh; k++) {
            const DHsp &h = k ? P.ovf[ov + k - 1] : P.cand_hsp[ci];
            if (!(h.strand & HSP_REV)) continue;
            // the reverse search's query tx (its gene and isoform position) and subject tx
            const uint32_t rq = h.s_tx, rs = h.q_tx;
            if (c == 0) {
                gi = (uint64_t)(P.tx[rs].sample - P.ms0) * P.mgw + (P.tx_gene[rq] - P.mg0);   // (the tile's window)
                if (pass == 1) slot = P.mbase + P.mscan[gi] + P.mcur[li];
            }
            c++;
            if (pass == 0) continue;
            P.out[slot] = mirror_hsp(h);
            // order: (isoform position, strand) then (subject tx, index)
            P.mkey[2 * (slot - P.mbase)] = ((uint64_t)P.tx_pos[rq] << 1) | (uint64_t)(h.strand & 1);
            P.mkey[2 * (slot - P.mbase) + 1] = ((uint64_t)rs << 8) | (uint64_t)((h.strand >> HSP_IDX_SHIFT) & 7);
            slot++;
        }
        if (pass == 0 && c) P.mcur[li] = atomicAdd(&P.mcnt[gi], c);
    }
}

// sort each mirrored group by its order keys and fill the group table:
// groups of up to MSORT_SMALL entries (nearly all) by one thread's insertion
// sort; larger ones -- an isoform-rich gene against an isoform-rich ortholog
// holds tens of thousands -- go on a list for mirror_sort_big_kernel
constexpr uint32_t MSORT_SMALL = 32;
__global__ void mirror_sort_kernel(GroupParams P)
{
    const uint64_t n = (uint64_t)P.mgw * (uint64_t)P.msn;
    for (uint64_t gi = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; gi < n;
         gi += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t c = P.mcnt[gi];
        if (!c) continue;
        const uint64_t b = P.mscan[gi];
        // the window's (sample, gene) in the whole group table
        const uint64_t gg = grp_index(P.mg0 + (uint32_t)(gi % P.mgw), P.ms0 + (int)(gi / P.mgw), P.n_genes);
        P.grp_off[gg] = (uint32_t)(P.mbase + b);
        P.grp_cnt[gg] = c;
        if (c > MSORT_SMALL) {
            const unsigned long long k = atomicAdd(P.mbig_n, 1ull);
            P.mbig[k] = gi;   // capacity: nm / (MSORT_SMALL + 1) + 1 entries
            continue;
        }
        for (uint32_t i = 1; i < c; i++) {
            const uint64_t k1 = P.mkey[2 * (b + i)], k2 = P.mkey[2 * (b + i) + 1];
            const DHsp h = P.out[P.mbase + b + i];
            uint32_t j = i;
            while (j > 0) {
                const uint64_t p1 = P.mkey[2 * (b + j - 1)], p2 = P.mkey[2 * (b + j - 1) + 1];
                if (p1 < k1 || (p1 == k1 && p2 < k2)) break;
                P.mkey[2 * (b + j)] = p1;
                P.mkey[2 * (b + j) + 1] = p2;
                P.out[P.mbase + b + j] = P.out[P.mbase + b + j - 1];
                j--;
            }
            P.mkey[2 * (b + j)] = k1;
            P.mkey[2 * (b + j) + 1] = k2;
            P.out[P.mbase + b + j] = h;
        }
    }
}

// One workgroup per large mirrored group (persistent over the list): an
// in-place bitonic network over the group's c entries, ascending in every
// merge (the first stage of each merge compares mirrored positions), so the
// virtual +inf padding past c never moves and its comparators are skipped.
// Keys are unique per group: (isoform position, strand, subject tx, index).
__global__ __launch_bounds__(256) void mirror_sort_big_kernel(GroupParams P)
{
    const uint64_t nb = *P.mbig_n;
    for (uint64_t q = blockIdx.x; q < nb; q += gridDim.x) {
        const uint64_t gi = P.mbig[q];
        const uint32_t c = P.mcnt[gi];
        const uint64_t b = P.mscan[gi];
        uint64_t *K = P.mkey + 2 * b;
        DHsp *H = P.out + P.mbase + b;
        uint32_t np2 = 1;
        while (np2 < c) np2 <<= 1;
        auto cmpx = [&](uint32_t i, uint32_t j) {   // i < j: the smaller key to i
            if (j >= c) return;
            const uint64_t a1 = K[2 * i], a2 = K[2 * i + 1], b1 = K[2 * j], b2 = K[2 * j + 1];
            if (a1 > b1 || (a1 == b1 && a2 > b2)) {
                K[2 * i] = b1; K[2 * i + 1] = b2; K[2 * j] = a1; K[2 * j + 1] = a2;
                const DHsp t = H[i];
                H[i] = H[j];
                H[j] = t;
            }
        };
        for (uint32_t kk = 2; kk <= np2; kk <<= 1) {
            // flip stage: i in the lower half of a kk-block against its mirror
            for (uint32_t t = threadIdx.x; t < np2 / 2; t += blockDim.x) {
                const uint32_t blk = t / (kk / 2), off = t % (kk / 2);
                const uint32_t i = blk * kk + off, j = blk * kk + kk - 1 - off;
                cmpx(i, j);
            }
            __syncthreads();
            for (uint32_t j2 = kk / 4; j2 > 0; j2 >>= 1) {   // half-cleaners
                for (uint32_t t = threadIdx.x; t < np2 / 2; t += blockDim.x) {
                    const uint32_t blk = t / j2, off = t % j2;
                    const uint32_t i = blk * 2 * j2 + off;
                    cmpx(i, i + j2);
                }
                __syncthreads();
            }
        }
    }
}

// ------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------

template <bool AMB, bool REV>
static void launch_seed_t(const Db &db, const Index &ix, const SeedParams &P, uint32_t n, hipStream_t st)
{
    hipLaunchKernelGGL((seed_kernel<AMB, false, false, REV>), dim3(n), dim3(SBLOCK), 0, st, db, ix, P);
    if (P.iso_n)   // the run's genes with more than ISO_LDS isoforms
        hipLaunchKernelGGL((seed_kernel<AMB, false, true, REV>), dim3(P.iso_n), dim3(SBLOCK), 0, st, db, ix, P);
}

void launch_seed(bool amb, const Db &db, const Index &ix, const SeedParams &P, hipStream_t st)
{
    const uint32_t n = P.gene_end - P.gene_begin;
    if (n == 0) return;
    if (P.rev)
        (amb ? launch_seed_t<true, true> : launch_seed_t<false, true>)(db, ix, P, n, st);
    else
        (amb ? launch_seed_t<true, false> : launch_seed_t<false, false>)(db, ix, P, n, st);
}

// the global-memory passes of the (gene, sample) entries P.big_list[0, n)
void launch_seed_big(bool amb, const Db &db, const Index &ix, const SeedParams &P, uint32_t n, hipStream_t st)
{
    if (n == 0) return;
    if (amb)
        hipLaunchKernelGGL((seed_kernel<true, true, false, false>), dim3(n), dim3(SBLOCK), 0, st, db, ix, P);
    else
        hipLaunchKernelGGL((seed_kernel<false, true, false, false>), dim3(n), dim3(SBLOCK), 0, st, db, ix, P);
}

void launch_extend(bool amb, const Db &db, const ExtParams &P, hipStream_t st)
{
    if (P.n_cand == 0) return;
    ExtParams W = P;
    W.defer = nullptr;
    const uint64_t blocks = 256ull * 8;
    if (amb)
        hipLaunchKernelGGL(extend_kernel<true>, dim3((unsigned)blocks), dim3(EBLOCK), 0, st, db, W);
    else
        hipLaunchKernelGGL(extend_kernel<false>, dim3((unsigned)blocks), dim3(EBLOCK), 0, st, db, W);
}

// Row kernel over all candidates, then extend_kernel over the ones it deferred
// (sub-band overflow, or transcripts longer than the row staging slot). The
// deferred count stays on the device: the list launch reads it.
// One resident wave per SIMD slot: a grid past the resident capacity leaves a
// partial second round of waves (static per-row work runs at low occupancy).
template <typename K>
static unsigned resident_blocks(K kernel, size_t lds)
{
    int dev = 0, cus = 256, per_cu = 1;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
        cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, EBLOCK, lds) != hipSuccess || per_cu < 1)
        per_cu = 1;
    return (unsigned)(cus * per_cu);
}

// A row-kernel launch: the windowed instantiation when the staging slot is
// shorter than the longest transcript (P.win), one resident round of blocks.
template <bool A, int RWV, bool SV, bool WV>
static void launch_rows_t(const Db &db, const ExtParams &P, hipStream_t st)
{
    auto kern = extend_rows_kernel<A, RWV, ROW_MIN_WAVES, SV, WV>;
    const size_t lds = row_lds_bytes(RWV, A ? 8 : 4, P.dsw, WV);
    hipLaunchKernelGGL(kern, dim3(resident_blocks(kern, lds)), dim3(EBLOCK), lds, st, RowArgs{db, P});
}
template <int RWV, bool SV = false>
static void launch_rows(bool amb, const Db &db, const ExtParams &P, hipStream_t st)
{
    if (amb) {
        if (P.win) launch_rows_t<true, RWV, SV, true>(db, P, st); else launch_rows_t<true, RWV, SV, false>(db, P, st);
    } else {
        if (P.win) launch_rows_t<false, RWV, SV, true>(db, P, st); else launch_rows_t<false, RWV, SV, false>(db, P, st);
    }
}

// Staging slot (u64 words per staged array) the 32-lane row kernel can have
// at ROW_MIN_WAVES waves per SIMD (as many 4-wave blocks per CU in 160 KB of LDS); a longer
// transcript runs on the windowed instantiation.
int row_slot_words_max(bool amb)
{
    const int na = amb ? 8 : 4, rows = EBLOCK / 32;
    const size_t per_block = (size_t)(160 * 1024) / (size_t)ROW_MIN_WAVES;
    const size_t fixed = row_lds_bytes(32, na, 0, true);
    return (int)((per_block - fixed) / ((size_t)rows * na * 8));
}

// Row kernel (first seeds) over all candidates, first_finish_kernel, then
// extend_kernel over the candidates either deferred (sub-band overflow,
// seeds outside the first box; without the windowed kernel transcripts
// longer than the row staging slot). The deferred count stays on the device:
// the list launch reads it.
// extend_kernel over the searches the row kernels left (B.defer, and for
// shared searches the reverse ones, B.defer_r)
static void extend_lists(bool amb, const Db &db, const ExtParams &B, hipStream_t st)
{
    for (int dir = 0; dir < (B.share ? 2 : 1); dir++) {
        ExtParams W3 = B;
        W3.dir = dir;
        if (dir) {
            W3.defer = B.defer_r;
            W3.defer_count = B.defer_r_count;
        }
        if (amb) {
            auto kern = extend_kernel<true>;
            hipLaunchKernelGGL(kern, dim3(resident_blocks(kern, 0)), dim3(EBLOCK), 0, st, db, W3);
        } else {
            auto kern = extend_kernel<false>;
            hipLaunchKernelGGL(kern, dim3(resident_blocks(kern, 0)), dim3(EBLOCK), 0, st, db, W3);
        }
    }
}

// The extend_kernel launches of launch_extend_rows alone: after it ran with
// lists = false, or again after the HSP overflow buffer overflowed (only
// extend_kernel writes it; the row kernels' results, first_finish_kernel's
// and the defer lists stand)
void launch_extend_retry(bool amb, const Db &db, const ExtParams &P, hipStream_t st)
{
    if (P.n_cand == 0) return;
    ExtParams W = P;
    W.list = nullptr;
    W.list_n = nullptr;
    W.resume = nullptr;
    const char *r64 = getenv("RC_ROW64");
    if (!P.share && r64 && atoi(r64)) {
        W.defer = P.defer2;
        W.defer_count = P.defer2_count;
    }
    extend_lists(amb, db, W, st);
}

// Later-seed rounds over the searches first_finish_kernel deferred (shared
// searches; after launch_extend_rows with lists = false): MAX_HSP rounds of
// later_round_kernel, with the row kernels (32-lane, then the 64-lane pass
// over what outgrew the sliding sub-band) over each round's seeds between
// them. Every count stays on the device: an empty round is a few idle
// launches. cnt: LATER_CNT zeroed counters per round; the work buffers
// (vc, list, box) and the active lists alternate between rounds.
void launch_later_rounds(bool amb, const Db &db, const ExtParams &P, const LaterParams &L0, Cand *const vc[2],
                         uint32_t *const list[2], int32_t *const box[2], uint32_t *const act[2],
                         unsigned long long *cnt, hipStream_t st)
{
    if (!L0.n_search) return;
    const char *wv = getenv("RC_WIDE");
    const bool widep = !(wv && atoi(wv) == 0) && P.wide0;
    // later seeds nearly all outgrow the 32-lane window (C3v: 15.3 M of 15.3 M,
    // profiles/r06_later): straight to 64-lane rows (RC_LATER_ROWS=32: the
    // 32-lane pass first)
    const char *rv = getenv("RC_LATER_ROWS");
    const bool rows64 = !(rv && atoi(rv) == 32);
    uint64_t g = (L0.n_search + 255) / 256;
    if (g > 8192) g = 8192;
    for (int r = 0; r < MAX_HSP; r++) {
        unsigned long long *c = cnt + (size_t)r * LATER_CNT;
        LaterParams L = L0;
        L.round = r;
        L.vc = vc[r & 1];
        L.list = list[r & 1];
        L.vc_in = vc[(r + 1) & 1];
        L.box_in = box[(r + 1) & 1];
        L.act_out = act[r & 1];
        L.act_out_n = c + 1;
        L.act_in = act[(r + 1) & 1];
        L.act_in_n = r ? cnt + (size_t)(r - 1) * LATER_CNT + 1 : nullptr;
        L.work_n = c;
        hipLaunchKernelGGL(later_round_kernel, dim3((unsigned)g), dim3(256), 0, st, P, L);
        if (r == MAX_HSP - 1) break;   // (every search has MAX_HSP boxes or none to add)
        ExtParams B = P;
        B.which = 0;
        B.cands = vc[r & 1];
        B.cand_box = box[r & 1];
        B.list = list[r & 1];
        B.list_n = c;
        B.work = c + 2;
        if (rows64) {   // RC_LATER_ROWS=64: straight to the spec's whole band
            B.wide = nullptr;
            B.wide_n = nullptr;
            B.resume = nullptr;
            launch_rows<64>(amb, db, B, st);
            continue;
        }
        B.wide = widep ? P.wide0 : nullptr;
        B.wide_n = c + 3;
        B.resume = widep ? P.resume : nullptr;
        if (B.resume) launch_rows<32, true>(amb, db, B, st); else launch_rows<32>(amb, db, B, st);
        if (widep) {
            ExtParams V = B;
            V.list = P.wide0;
            V.list_n = c + 3;
            V.work = c + 4;
            V.wide = nullptr;
            V.wide_n = nullptr;
            launch_rows<64>(amb, db, V, st);
        }
    }
}

// The searches the later-seed rounds finished: purge, cuts, records (again
// after an HSP overflow-buffer retry: the search states stand)
void launch_later_finish(const ExtParams &P, const LaterParams &L, hipStream_t st)
{
    const uint64_t n = std::min(L.n_search, L.n_cap);
    if (!n) return;
    uint64_t g = (n + 255) / 256;
    if (g > 8192) g = 8192;
    hipLaunchKernelGGL(later_finish_kernel, dim3((unsigned)g), dim3(256), 0, st, P, L);
}

// lists = false: up to first_finish_kernel only (the caller sizes the HSP
// overflow buffer from the defer counts, then launch_extend_retry)
void launch_extend_rows(bool amb, const Db &db, const ExtParams &P, int row_width, hipStream_t st, bool lists)
{
    if (P.n_cand == 0) return;
    (void)row_width;
    ExtParams W = P;
    W.list = nullptr;
    W.list_n = nullptr;
    // saved extension states: only the shared-search 32-lane passes write
    // them and only their 64-lane passes read them
    W.resume = nullptr;
    auto extend_lists = [&](const ExtParams &B) {
        if (lists) rcg::extend_lists(amb, db, B, st);
    };
    uint64_t g = (P.n_cand + 255) / 256;
    if (g > 65536) g = 65536;
    if (P.share) {
        // shared searches: first seeds e0 over every candidate, then e1 over
        // list2 (reverse searches whose first seed is another seed), then each
        // directed search checked (or listed for extend_kernel) on its own
        // each 32-lane pass is followed by a 64-lane pass (the spec's whole
        // band) over the candidates whose live diagonals outgrew the sliding
        // sub-band (RC_WIDE=0: they go to the one-wave kernel whole). Most of
        // them also have seeds outside the first box; extend_kernel starts
        // those searches from the first seed's HSP (P.reuse_first), so the
        // 64-lane pass is not redone: C3v 806 vs 875 ms per step.
        const char *wv = getenv("RC_WIDE");
        const bool widep = !(wv && atoi(wv) == 0) && P.wide0;
        auto wide_pass = [&](const ExtParams &B, uint32_t *lst, unsigned long long *lst_n, unsigned long long *wk) {
            ExtParams V = B;
            V.list = lst;
            V.list_n = lst_n;
            V.work = wk;
            V.wide = nullptr;
            V.wide_n = nullptr;
            launch_rows<64>(amb, db, V, st);
        };
        W.which = 0;
        W.wide = widep ? P.wide0 : nullptr;
        W.wide_n = P.wide0_n;
        W.resume = widep ? P.resume : nullptr;
        auto rows_pass = [&](const ExtParams &B) {
            if (B.resume) launch_rows<32, true>(amb, db, B, st); else launch_rows<32>(amb, db, B, st);
        };
        rows_pass(W);
        if (widep) wide_pass(W, P.wide0, P.wide0_n, P.work_w0);
        ExtParams W2 = W;
        W2.which = 1;
        W2.list = P.list2;
        W2.list_n = P.list2_n;
        W2.work = P.work3;
        W2.wide = widep ? P.wide1 : nullptr;
        W2.wide_n = P.wide1_n;
        rows_pass(W2);
        if (widep) wide_pass(W2, P.wide1, P.wide1_n, P.work_w1);
        W.list = nullptr;
        W.list_n = nullptr;
        hipLaunchKernelGGL(first_finish_kernel, dim3((unsigned)g), dim3(256), 0, st, W);
        extend_lists(W);
        return;
    }
    // independent searches / spec 5b: 32-lane rows over every candidate
    launch_rows<32>(amb, db, W, st);
    // pass 2 (RC_ROW64=1; off by default: at C3 neutral, at C3v 7 % slower,
    // because 40 % of what it finishes still has seeds outside the first box
    // and is redone whole by the one-wave kernel): the candidates whose
    // frontier left the sub-band, on 64-lane rows (the spec's whole band)
    const char *r64 = getenv("RC_ROW64");
    if (!(r64 && atoi(r64))) {
        hipLaunchKernelGGL(first_finish_kernel, dim3((unsigned)g), dim3(256), 0, st, W);
        extend_lists(W);
        return;
    }
    ExtParams W2 = W;
    W2.list = P.defer;
    W2.list_n = P.defer_count;
    W2.defer = P.defer2;
    W2.defer_count = P.defer2_count;
    W2.work = P.work2;
    launch_rows<64>(amb, db, W2, st);
    ExtParams W3 = W;
    W3.defer = P.defer2;
    W3.defer_count = P.defer2_count;
    hipLaunchKernelGGL(first_finish_kernel, dim3((unsigned)g), dim3(256), 0, st, W3);
    extend_lists(W3);
}

void launch_group(const GroupParams &P, int pass, hipStream_t st)
{
    // 0 direct count, 1 direct write, 2 mirror count, 3 mirror scatter, 4 mirror sort
    uint64_t n = (uint64_t)(P.gene_end - P.gene_begin) * (uint64_t)P.N;
    if (pass == 2 || pass == 3) n = P.n_cand;
    if (pass == 4) n = (uint64_t)P.mgw * (uint64_t)P.msn;
    if (!n) return;
    uint64_t g = (n + 255) / 256;
    if (g > 65536) g = 65536;
    if (pass == 0)
        hipLaunchKernelGGL(group_count_kernel, dim3((unsigned)g), dim3(256), 0, st, P);
    else if (pass == 1)
        hipLaunchKernelGGL(group_write_kernel, dim3((unsigned)g), dim3(256), 0, st, P);
    else if (pass == 2 || pass == 3)
        hipLaunchKernelGGL(mirror_scatter_kernel, dim3((unsigned)g), dim3(256), 0, st, P, pass - 2);
    else {
        hipLaunchKernelGGL(mirror_sort_kernel, dim3((unsigned)g), dim3(256), 0, st, P);
        hipLaunchKernelGGL(mirror_sort_big_kernel, dim3(1024), dim3(256), 0, st, P);
    }
}

}  // namespace rcg

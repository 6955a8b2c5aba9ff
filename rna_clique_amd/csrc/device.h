// Shared device-side declarations of the MI355X RNA-clique engine.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rcg {

constexpr int W16 = 16;         // index word (bases) -> 32-bit key
constexpr int BAND = 64;        // greedy band: one diagonal per lane of a wave
constexpr int BAND_LO = -32;    // diagonal of lane 0
constexpr int MAX_HSP = 8;      // HSPs per (query tx, strand, subject tx)
constexpr int DMAX = 4096;      // greedy differences cap
constexpr int ISO_LDS = 128;    // a gene's isoform tables the seed kernel keeps in LDS (more: read from HBM)
constexpr uint64_t MAX_TX = 1ull << 27;   // transcripts per engine (27-bit field of the seed key)
constexpr int MAX_SAMPLES = 65535;         // samples per engine (16-bit fields of Cand and the big-pass list)

// Transcript record (16 B, one load).
struct TxInfo {
    uint64_t start;   // global base offset of the transcript
    uint32_t len;
    int32_t sample;
};

// HSP of a directed search (56 B), BLAST tabular coordinates.
// HSP group table index of (query gene, subject sample): sample-major, so the
// groups of consecutive genes against one sample are adjacent (the RBH items
// of a sample pair walk them in gene order; gene-major put every item on its
// own cache line of the table)
__host__ __device__ __forceinline__ size_t grp_index(uint32_t gene, int sample, uint32_t n_genes)
{
    return (size_t)sample * n_genes + gene;
}

struct DHsp {
    uint32_t q_tx, s_tx;   // global transcript ids
    int32_t qstart, qend, sstart, send;
    int32_t length, nident, mismatch, gaps, gapopen;
    int32_t score_half, bits10;
    int32_t strand;
};

// Distinct gene-graph edge between gene a (sample A = t1) and gene b (sample B = t2).
struct DEdge {
    uint32_t a, b;         // global gene ids (graph nodes)
    uint32_t pair;         // pair index (combination order)
    int32_t nident;        // sum of nident over the edge's table rows
    int32_t den;           // sum of (length - gaps) over the edge's table rows
};

// DEdge.pair flags of imported graphs (SampleSimilarity(graph, tables)): a
// table row whose edge is not in the graph (sums only), and an isolated graph
// node (a == b: it only counts as present)
constexpr uint32_t EDGE_SUM_ONLY = 0x80000000u, NODE_REC = 0x7FFFFFFFu;

// Final gene-matches-table row: index of the HSP + flags.
struct DRow {
    uint32_t hsp;          // index into the top-hit array
    int32_t reverse;
    int32_t label;
    uint32_t pad;
};

// Everything the kernels need to see, passed by value.
// a gene's transcripts in gene_tx order, with their tile records (the seed
// kernel's isoform tables in one load)
struct IsoRec {
    uint32_t start, len, gtx, pad;
};
// One sample of an alignment tile (load_tile -> launch_tile_tables): its
// transcripts [tx0, tx0 + ntx) (global ids) sit at tile position pos; their
// slots in the tile's transcript list (ttx0) and, for an indexed (subject)
// sample, in the index list (itx0, else ~0u) with its first k-mer slot kbase.
// pad_bit: the tile position where its bases end when padding follows (a
// transcript-start bit there stops DUST runs), else ~0.
struct TileSeg {
    uint64_t pos, kbase, pad_bit;
    uint32_t tx0, ntx, ttx0, itx0;
};
struct Db {
    const uint64_t *F, *RC;     // 2-bit packed forward / reverse-complement
    const uint64_t *AF, *ARC;   // ambiguity masks (2 bits per base) or null
    uint64_t total;             // bases
    const TxInfo *tx;
    const uint32_t *tx_gene;    // global gene of each transcript
    const uint32_t *gene_tx_off, *gene_tx;   // CSR: transcripts of each gene
    const IsoRec *giso;                      // per gene_tx entry: its transcript's tile record
    const int32_t *gene_sample;
    const uint32_t *sample_gene_begin;       // n_samples + 1
    const uint32_t *sample_tx_begin;         // n_samples + 1
    const uint64_t *sample_pos_begin;        // n_samples + 1: first base of each sample
    const uint64_t *txstart;                 // bit per base: 1 where a transcript starts (+1 guard word)
    const uint64_t *dmask;                   // bit per base: DUST-masked query bases (+1 guard word), or null
    int32_t n_samples;
};

// 16-mer index: one u64 per indexed position, (k-mer << 32) | global base
// position, sorted by k-mer (stable, so positions ascend inside a k-mer run);
// bucket[b] = first entry whose k-mer has top `bits` bits >= b.
// block of 2^POS_TX_SHIFT positions -> the transcript holding its first base
// (the last one starting at or before it), with that transcript's record, so
// a position inside it resolves in one load
struct PosTx {
    uint32_t t, start, len;
    int32_t sample;
};
struct Index {
    const uint64_t *ent;
    const uint32_t *bucket;     // 2^bits + 1 offsets
    const PosTx *pos_tx;        // per block of POS_TX_SHIFT bases
    int32_t bits;
};
constexpr int POS_TX_SHIFT = 8;

// transcript of a tile position: the block's record, else forward from it
__device__ __forceinline__ uint32_t tx_of_pos(const Db &db, const Index &ix, uint32_t pos, TxInfo &ti)
{
    const PosTx r = ix.pos_tx[pos >> POS_TX_SHIFT];
    uint32_t t = r.t;
    if (pos - r.start < r.len) {
        ti.start = r.start;
        ti.len = r.len;
        ti.sample = r.sample;
        return t;
    }
    ti = db.tx[++t];
    while ((uint64_t)pos >= ti.start + ti.len) ti = db.tx[++t];
    return t;
}

constexpr int NSHARD = 256;    // output allocation shards (spread the atomics)

// Seed (maximal exact run >= W) of one candidate, oriented query coordinates.
struct GSeed {
    uint32_t x, y, len;   // len: bits 0-29; shared searches: SEED_F / SEED_R in bits 30, 31
};
// Shared searches (RC_SHARE): the directed searches a seed belongs to (it
// holds a usable word of that search's query: spec 1, 1b, 2)
constexpr uint32_t SEED_F = 1u << 30, SEED_R = 1u << 31, SEED_LEN = SEED_F - 1u;
constexpr uint16_t SEED_NONE = 0xFFFFu;

// Candidate = (query transcript, strand, subject transcript) with >= 1 seed.
// Self-contained (48 B, 12 dwords): the extension reads one record, no
// transcript table. Positions are tile positions (a tile has < 2^32 bases).
struct Cand {
    uint32_t seed_off;     // absolute index of its first seed (sorted by (x, y))
    uint32_t q_gtx, s_gtx;
    uint16_t seed_lo;      // seed count, low 16 bits (cand_seeds())
    uint8_t strand;
    uint8_t dflags;        // shared searches: bit 0 the forward search has seeds, bit 1 the reverse one
    uint32_t q0;           // first base of the oriented query: in F (strand 0) or RC (strand 1)
    uint32_t s0;           // first base of the subject in F
    int32_t Lq, Lt;        // transcript lengths
    uint16_t qsam, ssam;   // samples of query and subject
    uint16_t seed_hi;      // seed count, high 16 bits
    uint16_t pad0;
    // seeds (indices in the candidate) the row kernel extends first: e0 into
    // cand_box (the forward search's first seed, or the reverse one's when the
    // forward search has none), e1 into cand_box2 (the reverse search's first
    // seed when it is another seed; SEED_NONE otherwise)
    uint16_t e0, e1;
    uint32_t pad1;
};
__host__ __device__ __forceinline__ uint32_t cand_seeds(const Cand &c) { return c.seed_lo | ((uint32_t)c.seed_hi << 16); }
constexpr int CAND_DWORDS = (int)(sizeof(Cand) / 4);
static_assert(sizeof(Cand) == 48, "Cand is read as 12 dwords");

// A seed of the seed kernel before sorting: k1 = iso | strand:1 | gtx:27 | x:xb
// (sorted by k1, then y; k1 >> xb is the candidate: isoform, strand, subject
// tx). xb = SeedParams::xbits, the bits of the longest transcript length: the
// isoform field has 36 - xb bits (engine limit: max_iso()).
struct LSeed {
    uint64_t k1;
    uint32_t y, len;
};
constexpr int GTX_BITS = 27;
__host__ __device__ __forceinline__ uint64_t seed_key(uint32_t iso, uint32_t strand, uint32_t gtx, uint32_t x, int xb)
{
    return ((uint64_t)iso << (xb + GTX_BITS + 1)) | ((uint64_t)strand << (xb + GTX_BITS)) | ((uint64_t)gtx << xb) |
           (uint64_t)x;
}
__host__ __device__ __forceinline__ uint32_t key_iso(uint64_t k, int xb) { return (uint32_t)(k >> (xb + GTX_BITS + 1)); }
__host__ __device__ __forceinline__ uint32_t key_strand(uint64_t k, int xb) { return (uint32_t)(k >> (xb + GTX_BITS)) & 1u; }
__host__ __device__ __forceinline__ uint32_t key_gtx(uint64_t k, int xb) { return (uint32_t)(k >> xb) & (uint32_t)(MAX_TX - 1); }
__host__ __device__ __forceinline__ uint32_t key_x(uint64_t k, int xb) { return (uint32_t)k & ((1u << xb) - 1u); }
// bits of a transcript position (x < max_len) and the isoforms per gene the
// key then holds (it_iso in the seed kernel's LDS is 16-bit: at most 65535)
__host__ __device__ __forceinline__ int pos_bits(int64_t max_len)
{
    int b = 1;
    while (b < 24 && (1ll << b) <= max_len) b++;
    return b;
}
__host__ __device__ __forceinline__ uint32_t max_iso(int xb)
{
    const int ib = 64 - (xb + GTX_BITS + 1);
    return ib >= 16 ? 65535u : (1u << ib) - 1u;
}

// seed_kernel: per query gene, lookups -> canonical seeds -> candidates.
struct SeedParams {
    int32_t word;                 // W
    int32_t stride;               // W - 16 + 1
    int32_t pre_mode;             // canonical pre-test: 1 = previous word's hits (LDS), 0 = sequence windows
    int32_t sym;                  // spec 5b: subjects are higher-numbered samples only
    int32_t share;                // shared searches: query = lower sample, seeds carry SEED_F / SEED_R
    // Shared searches with DUST. The reverse pass (rev = 1; queries = the
    // higher samples, subjects = the near-mask index) emits the reverse-search
    // seeds the forward pass cannot find (no usable word of the lower sample's
    // transcript inside) as SEED_R seeds in forward-candidate coordinates:
    // rseeds[i] with the forward query's gene in rseed_gene[i]. The forward
    // pass merges them into its candidates: rs_key = those genes sorted,
    // rs_idx = the permutation, rs_n entries.
    int32_t rev;
    int32_t xbits;                // seed-key position bits (pos_bits(max_len)); max_iso(xbits) isoforms per gene
    uint32_t max_iso;
    int32_t tmw;                  // words per query sample of tmask
    const int32_t *trange;        // [n_samples][2]: first and one-past-last subject sample of each query sample
    const uint32_t *tx_pos;       // isoform index of a transcript in its gene
    // genes with more than ISO_LDS isoforms: the word-item prefix of each
    // isoform, at gene_tx_off[g] + g + i (i = 0..niso; stride P.stride)
    const uint32_t *iso_pre_g;
    const uint32_t *iso_list;     // ... those genes of [gene_begin, gene_end) (the ISOG launch)
    uint32_t iso_n;
    LSeed *rseeds;
    uint32_t *rseed_gene;
    uint64_t rseed_cap;
    unsigned long long *rseed_n;
    const LSeed *rs_rec;
    const uint32_t *rs_key, *rs_idx;
    uint32_t rs_n;
    const uint32_t *rs_range;     // [(g - gene_begin) * 2]: gene g's reverse-only seeds [rs_key lower bounds of g, g + 1)
    uint32_t *list2;              // shared searches: slots of the candidates with e1 != SEED_NONE
    unsigned long long *list2_n;
    uint32_t gene_begin, gene_end;   // shard
    GSeed *seeds;
    uint64_t seed_cap;            // per allocation shard
    unsigned long long *seed_count;  // [NSHARD]
    Cand *cands;
    uint64_t cand_cap;            // per allocation shard
    unsigned long long *cand_count;  // [NSHARD]
    uint32_t *gc_off, *gc_cnt;    // [(g - gene_begin) * N + T] candidates of (gene, sample)
    const uint64_t *tmask;        // [n_samples][tmw] subject samples (> query sample) of this shard
    unsigned int *status;         // bit 0 overflow, bit 1 gene limit, bit 3 big list full, bit 4 seed index > 16 bits
    unsigned long long *prof;     // RC_ROW_TIMING builds: block cycles per phase
    // (gene, sample) passes whose seeds overflow LDS: ((gene - gene_begin) << 16) | sample
    uint64_t *big_out;            // the LDS kernel appends here
    unsigned long long *big_n;
    const uint64_t *big_list;     // the global-memory kernel's entries (one workgroup each)
    uint64_t *big_retry;          // entries that overflowed big_cap too
    unsigned long long *big_retry_n;
    uint64_t big_list_cap;
    uint32_t big_cap;             // seeds per workgroup in global scratch (power of two)
    LSeed *big_seeds;
    uint32_t *big_seg;            // big_cap + 1 per workgroup
    uint8_t *big_segT;            // big_cap per workgroup
};

// extend_kernel: one wave per candidate, greedy X-drop, purge, e-value cut.
struct ExtParams {
    int32_t xdrop;
    int32_t sym;                  // spec 5b: also apply the mirrored direction's e-value cut
    int32_t max_len;
    const int32_t *thr;           // [n_samples][max_len + 1] min score_half
    const int32_t *bits10;        // [2 * max_len + 2]
    const Cand *cands;
    const GSeed *seeds;
    const unsigned long long *shard_prefix;   // NSHARD + 1 prefix of candidate counts
    uint64_t n_cand;
    uint64_t cand_cap;
    DHsp *cand_hsp;               // first HSP of each candidate (absolute index)
    uint8_t *cand_nh;             // HSPs kept per candidate
    uint32_t *cand_ovf;           // overflow offset of HSPs 2..nh
    DHsp *ovf;
    uint64_t ovf_cap;
    unsigned long long *ovf_count;
    unsigned int *status;         // bit 0 overflow
    unsigned long long *counters; // [0] greedy steps, [1] extensions, [2] candidates (one atomic per wave),
                                  // [4] full-band recomputations
    // row kernels: staging slot (u64 words per sequence); win: the slot is
    // shorter than the longest transcript, the windowed instantiation runs
    int32_t dsw;
    int32_t win;
    int32_t *cand_box;            // row kernel: status + right/left results of each candidate's first seed
    int32_t chunk;                // row kernel: candidates per work grab (0: static round robin)
    unsigned long long *work;     // row kernel: work counter
    uint32_t *defer;
    unsigned long long *defer_count;
    const uint32_t *list;               // row kernel list mode: candidate slots list[0, *list_n)
    const unsigned long long *list_n;
    uint32_t *defer2;                   // the 64-lane pass's deferrals (-> extend_kernel)
    unsigned long long *defer2_count;
    unsigned long long *work2;
    // shared searches (RC_SHARE): one candidate set serves both directed
    // searches of a pair; the reverse search's HSPs go to the _r arrays
    int32_t share;
    int32_t which;                      // row kernel: 0 seed e0 -> cand_box, 1 seed e1 -> cand_box2
    int32_t dir;                        // extend_kernel: 0 forward search, 1 reverse search
    int32_t *cand_box2;
    DHsp *cand_hsp_r;
    uint8_t *cand_nh_r;
    uint32_t *cand_ovf_r;
    uint32_t *defer_r;                  // first_finish_kernel: the reverse searches extend_kernel redoes
    unsigned long long *defer_r_count;
    const uint32_t *list2;              // candidates with e1 != SEED_NONE (the seed kernel's list)
    const unsigned long long *list2_n;
    unsigned long long *work3;          // work counter of the row kernel's pass over list2
    // shared searches: candidates whose live diagonals outgrew the 32-lane
    // sliding sub-band, for the 64-lane pass after each 32-lane pass
    uint32_t *wide;                     // the list the running pass appends to (null: none)
    unsigned long long *wide_n;
    uint32_t *wide0, *wide1;            // the e0 pass's and the e1 pass's lists
    unsigned long long *wide0_n, *wide1_n, *work_w0, *work_w1;
    // extend_kernel (shared searches): start a search from its first seed's
    // row-kernel result (cand_box / cand_box2) when it has one
    int32_t reuse_first;
    // shared searches: the state of a 32-lane extension that outgrew its
    // window, saved per wide-list entry (the first res_cap entries), so the
    // 64-lane pass continues it instead of starting over (RES_REC ints each)
    int32_t *resume;
    uint32_t res_cap;
    // why searches leave the row kernels: [0] a transcript past the staging
    // slot (row kernel), [1] a directed search whose first seed the row
    // kernels gave up on, [2] one with a seed outside its first HSP's box
    // (first_finish_kernel)
    unsigned long long *why;
};
constexpr int RES_REC = 80;

// Later-seed rounds: a deferred directed search (a seed outside its first
// HSP's box) extends its next seed -- the first in its order outside every box
// so far, the sequential rule of spec 3 -- on the 64-lane row kernel, one seed
// per search per round, instead of on one wave of extend_kernel; a finished
// search is purged, cut and written by later_finish_kernel. Search state:
// [0] LS_STATE (below), [1] the pending work item, [2] MAX_HSP bound,
// then MAX_HSP boxes of LB_N ints.
enum { LS_STATE = 0, LS_PEND = 1, LS_CAPPED = 2, LS_BOX = 4 };
enum { LB_QA, LB_QB, LB_SA, LB_SB, LB_SC, LB_D, LB_G, LB_O, LB_NI, LB_N };
constexpr int LATER_REC = LS_BOX + MAX_HSP * LB_N;
// LS_STATE: >= 0 finished with that many HSPs; LATER_ACTIVE in a round;
// LATER_FULL: extend_kernel runs the search whole (a row kernel gave a seed
// up, or a seed index past the record's 16 bits)
constexpr int LATER_ACTIVE = -1, LATER_FULL = -2;
// device counters per round: work items, searches still active, the 32-lane
// pass's work counter, its wide list, the 64-lane pass's work counter
constexpr int LATER_CNT = 8;
struct LaterParams {
    int32_t *state;                       // [n_cap][LATER_REC]
    uint64_t n_search, n0;                // searches; the first n0 are forward ones (defer0), then defer1
    uint64_t n_cap;                       // searches with a state (the rest run whole)
    const uint32_t *defer0, *defer1;      // first_finish_kernel's defer lists (candidate slots)
    uint32_t *full0, *full1;              // the searches extend_kernel runs whole, per direction
    unsigned long long *full_n;           // [2]
    int32_t round;                        // 0: start from the first seed's box
    Cand *vc;                             // the round's work: candidate records whose e0 is the seed to extend
    uint32_t *list;                       // their indices (the row kernels' list mode)
    const Cand *vc_in;                    // the previous round's work (the buffers alternate)
    const int32_t *box_in;                // the row kernels' results for it (BOX_REC each)
    const uint32_t *act_in;               // searches still active (rounds > 0)
    const unsigned long long *act_in_n;
    uint32_t *act_out;
    unsigned long long *act_out_n;
    unsigned long long *work_n;           // work items of the round
    unsigned long long *counters;         // [0] (unused), [1] searches run whole
};   // phase, kof, d6, best, best record (i, gap, d6, diagonal), right results, R[32], goe[32]

// DHsp.strand carries, besides the strand (bit 0), the direction flags of a
// freshly extended HSP (bit 1: passes the query->subject e-value cut, bit 2:
// passes the mirrored direction's) and its index in the candidate (bits 3-5).
constexpr int HSP_FWD = 2, HSP_REV = 4, HSP_IDX_SHIFT = 3;

// cand_box record: BOX_REC ints per candidate (align.hip FX_*)
constexpr int BOX_REC = 12;


// group kernels: candidates of each (gene, sample) -> contiguous HSP groups.
// Direct groups (gene of the query sample, higher subject sample) come in
// candidate order; mirrored groups (gene of the higher sample, lower sample)
// are counted, scattered and sorted by (isoform, strand, subject tx, index).
struct GroupParams {
    uint32_t gene_begin, gene_end;
    int32_t N;
    const uint32_t *gc_off, *gc_cnt;   // shard-relative gene index
    const uint8_t *cand_nh;
    const DHsp *cand_hsp;
    const uint32_t *cand_ovf;
    const DHsp *ovf;
    uint32_t *cnt;                // [(g - gene_begin) * N + T] direct HSPs per group
    const uint64_t *scan;         // exclusive scan of cnt
    uint32_t *grp_off, *grp_cnt;  // global-gene group table
    DHsp *out;
    uint64_t base;                // first slot of this launch's direct groups in out (tiles append)
    // mirrored groups, over all candidates
    const unsigned long long *shard_prefix;
    uint64_t n_cand, cand_cap;
    const uint32_t *tx_gene, *tx_pos;   // gene of a transcript, its position in the gene
    const TxInfo *tx;
    // mirrored groups of the tile: the genes [mg0, mg0 + mgw) of its subject
    // samples (the reverse searches' queries) x its query samples [ms0,
    // ms0 + msn), counted in that window rather than over every gene and
    // sample (a C5 rank's tile: 3 M groups instead of 820 M)
    uint32_t mg0, mgw;
    int32_t ms0, msn;
    uint32_t *mcnt;               // [(T - ms0) * mgw + gene - mg0]
    const uint64_t *mscan;        // exclusive scan of mcnt
    uint32_t *mcur;               // per candidate (linear index): its first slot in its mirrored group (pass 0 -> pass 1)
    uint64_t mbase;               // first output slot of the mirrored region
    uint64_t *mkey;               // order keys of the mirrored region (parallel to out)
    uint64_t *mbig;               // mirrored groups too large for one thread's sort (mirror_sort_big_kernel)
    unsigned long long *mbig_n;
    uint32_t n_genes;
};

// Parameters of the two reciprocal-best-hit passes.
// an HSP as the RBH kernel's selection loops read it (hkey_kernel)
struct HKey {
    int32_t bits10;
    uint32_t gene;   // the subject transcript's gene
};
struct RbhParams {
    const DHsp *hsp;
    const HKey *hk;                      // parallel to hsp
    const uint32_t *grp_off, *grp_cnt;   // [grp_index(gene, T)], full gene range
    const uint32_t *tx_gene;
    const TxInfo *tx;
    const uint32_t *sample_gene_begin;
    const uint32_t *pair_item_begin;     // n_pairs + 1
    const int32_t *pair_a, *pair_b;
    int32_t n_pairs, N, top_n, keep_all;
    uint32_t n_genes;
    uint64_t item0, n_items;             // this shard's items [item0, item0 + n_items)
    // pass 0 outputs (per item)
    uint32_t *n_rows, *n_fsel, *n_rsel, *n_edges;
    // pass 1 inputs (exclusive scans) and outputs
    const uint64_t *row_off, *fsel_off, *rsel_off, *edge_off;
    DRow *rows;
    DEdge *edges;
    // pass 2 (counts + rows and edges in fixed per-item slots, labels local to
    // the item; rbh_place_kernel moves them once the offsets are scanned)
    DRow *rows_tmp;               // RBH_RMAX per item
    DEdge *edges_tmp;             // RBH_EMAX per item
    unsigned int *ovf;            // set when an item needs more slots (pass 1 then runs)
};
constexpr int RBH_RMAX = 2, RBH_EMAX = 1;

// ------------------------------------------------------------------------
// 2-bit windows
// ------------------------------------------------------------------------

// 32 bases starting at base position p (base i in bits 2i..2i+1). Branchless:
// both words are read (arrays carry padding words), (hi << 1) << (63 - sh)
// is hi << (64 - sh) for sh > 0 and 0 for sh == 0.
template <typename PT>
__device__ __forceinline__ uint64_t win(const uint64_t *__restrict__ a, PT p)
{
    const PT w = p >> 5;
    const unsigned sh = (unsigned)(p & 31) * 2u;
    const uint64_t lo = a[w], hi = a[w + 1];
    return (lo >> sh) | ((hi << 1) << (63u - sh));
}

// Longest common extension of two forward walks (at most maxn bases).
// Ambiguous bases (mask 0b11) never match. PT: 32-bit positions for LDS-staged
// sequences, 64-bit for the global arrays.
template <bool AMB, typename PT>
__device__ __forceinline__ int lcp(const uint64_t *__restrict__ A, const uint64_t *__restrict__ AA, PT pa,
                                   const uint64_t *__restrict__ B, const uint64_t *__restrict__ BA, PT pb,
                                   int maxn)
{
    int n = 0;
    while (n < maxn) {
        uint64_t x = win(A, pa + (PT)n) ^ win(B, pb + (PT)n);
        if (AMB) x |= win(AA, pa + (PT)n) | win(BA, pb + (PT)n);
        if (x == 0) {
            n += 32;
            continue;
        }
        n += __builtin_ctzll(x) >> 1;
        return n < maxn ? n : maxn;
    }
    return maxn > 0 ? maxn : 0;
}

// lcp, 64 bases per round trip (three words of each array in flight
// together): the seed kernel's right extensions of long exact runs
template <bool AMB, typename PT>
__device__ __forceinline__ int lcp64(const uint64_t *__restrict__ A, const uint64_t *__restrict__ AA, PT pa,
                                     const uint64_t *__restrict__ B, const uint64_t *__restrict__ BA, PT pb,
                                     int maxn)
{
    auto w2 = [](uint64_t lo, uint64_t hi, unsigned sh) { return (lo >> sh) | ((hi << 1) << (63u - sh)); };
    int n = 0;
    while (n < maxn) {
        const PT a = pa + (PT)n, b = pb + (PT)n;
        const uint64_t *pA = A + (a >> 5), *pB = B + (b >> 5);
        const unsigned sa = (unsigned)(a & 31) * 2u, sb = (unsigned)(b & 31) * 2u;
        const uint64_t a0 = pA[0], a1 = pA[1], a2 = pA[2], b0 = pB[0], b1 = pB[1], b2 = pB[2];
        uint64_t x0 = w2(a0, a1, sa) ^ w2(b0, b1, sb), x1 = w2(a1, a2, sa) ^ w2(b1, b2, sb);
        if (AMB) {
            const uint64_t *qA = AA + (a >> 5), *qB = BA + (b >> 5);
            const uint64_t m0 = qA[0], m1 = qA[1], m2 = qA[2], n0 = qB[0], n1 = qB[1], n2 = qB[2];
            x0 |= w2(m0, m1, sa) | w2(n0, n1, sb);
            x1 |= w2(m1, m2, sa) | w2(n1, n2, sb);
        }
        const int k = x0 ? (int)(__builtin_ctzll(x0) >> 1) : (x1 ? 32 + (int)(__builtin_ctzll(x1) >> 1) : 64);
        n += k;
        if (k < 64) return n < maxn ? n : maxn;
    }
    return maxn > 0 ? maxn : 0;
}

// 32 bases at a signed base position (arrays carry two zero words in front,
// so p >= -64 stays in bounds)
__device__ __forceinline__ uint64_t win_s(const uint64_t *__restrict__ a, int64_t p)
{
    const int64_t w = p >> 5;
    const unsigned sh = (unsigned)(p & 31) * 2u;
    const uint64_t lo = a[w], hi = a[w + 1];
    return (lo >> sh) | ((hi << 1) << (63u - sh));
}

// 64 bits of a bit array starting at signed bit b (b >= -64: one guard word in front)
__device__ __forceinline__ uint64_t win_bits(const uint64_t *__restrict__ a, int64_t b)
{
    const int64_t w = b >> 6;
    const unsigned sh = (unsigned)(b & 63);
    const uint64_t lo = a[w], hi = a[w + 1];
    return (lo >> sh) | ((hi << 1) << (63u - sh));
}

__device__ __forceinline__ uint64_t rev2(uint64_t x)
{
    x = ((x >> 2) & 0x3333333333333333ull) | ((x & 0x3333333333333333ull) << 2);
    x = ((x >> 4) & 0x0F0F0F0F0F0F0F0Full) | ((x & 0x0F0F0F0F0F0F0F0Full) << 4);
    return __builtin_bswap64(x);
}

}  // namespace rcg

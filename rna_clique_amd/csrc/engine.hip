// Host side of the MI355X RNA-clique engine: the C ABI of include/rcgpu.h.
//
// Owns the device buffers, drives the kernels of kernels.hip on one HIP
// stream, and converts results back to reference semantics (1-based BLAST
// coordinates, pandas index labels, sorted-label matrix order).
#include "../../include/rcgpu.h"
#include "device.h"
#include "graph_pickle.h"

#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <numeric>
#include <string>
#include <thread>
#include <vector>

// od2_tables.cpp: one pair's gene matches table file
int od2_write_table(const rc_row *rows, uint64_t n, const std::string &ssample, const std::string &qsample,
                    const std::string &path);
// graph_pickle.cpp: a table of the pickle whose gene arrays the caller fills
extern "C" int graph_pickle_table(rc_gpickle *g, int32_t ssample, int32_t qsample, uint64_t n, int64_t **sgene,
                                  int64_t **qgene);

namespace rcg {
void launch_pack(const uint8_t *, uint64_t, uint64_t, uint64_t *, uint64_t *, uint64_t *, uint64_t *, hipStream_t);
void launch_kmer_count(const TxInfo *, uint32_t, const uint64_t *, uint64_t *, hipStream_t);
void launch_kmer_fill(bool, const TxInfo *, uint32_t, const uint64_t *, const uint64_t *, const uint64_t *,
                      uint64_t *, hipStream_t);
void launch_bucket_fill(const uint64_t *, uint64_t, int, uint32_t *, hipStream_t);
uint64_t os_status_words(uint64_t n);
uint64_t os_scratch_words(uint64_t n);
bool os_sort_keys(uint64_t *keys, uint64_t *alt, uint64_t n, int bb, uint32_t *scratch, uint64_t *status,
                  uint32_t &epoch, hipStream_t st, const std::function<void()> &after_prep, bool counted,
                  const TxInfo *gen_tx, const uint64_t *gen_koff, const uint64_t *gen_F, uint32_t gen_ntx,
                  uint32_t *gen_tile);
uint64_t os_gen_tile_words(uint64_t n);
void os_fill_hist(const TxInfo *tx, uint32_t n_tx, const uint64_t *F, const uint64_t *koff, uint64_t *ent,
                  uint64_t n, uint32_t *scratch, hipStream_t st);
void launch_tx_masked(const TxInfo *, uint32_t, const uint64_t *, uint8_t *, hipStream_t);
void launch_edge_check(const DEdge *, uint64_t, uint32_t, uint64_t, unsigned int *, hipStream_t);
void launch_edge_key(const DEdge *, uint64_t, const uint32_t *, uint32_t *, uint32_t *, hipStream_t);
void launch_edge_gather(const DEdge *, const uint32_t *, uint64_t, DEdge *, hipStream_t);
void launch_edge_uv(const DEdge *, const uint32_t *, const uint32_t *, uint64_t, uint32_t *, uint32_t *, uint64_t *,
                    hipStream_t);
void launch_tile_tables(const TileSeg *, uint32_t, uint32_t, const uint64_t *, const uint64_t *, TxInfo *, TxInfo *,
                        uint32_t *, TxInfo *, uint64_t *, uint32_t, uint64_t, uint64_t *, IsoRec *, uint64_t,
                        const uint64_t *, PosTx *, uint64_t, hipStream_t);
void launch_near_fill(bool, const TxInfo *, uint32_t, const uint8_t *, const uint64_t *, const uint64_t *,
                      const uint64_t *, uint64_t *, uint64_t, unsigned long long *, hipStream_t);
void launch_seed(bool, const Db &, const Index &, const SeedParams &, hipStream_t);
void launch_seed_big(bool, const Db &, const Index &, const SeedParams &, uint32_t, hipStream_t);
void launch_rs_range(const uint32_t *, uint32_t, uint32_t, uint32_t, uint32_t *, hipStream_t);
void launch_dust(bool, uint64_t, uint64_t, const uint64_t *, const uint64_t *, const uint64_t *, const TxInfo *, uint32_t, int,
                 int, int, uint32_t *, uint64_t *, uint32_t, int, uint64_t *, hipStream_t);
uint32_t dust_scratch_words(uint32_t);
uint64_t dust_event_words(uint32_t);
void launch_extend(bool, const Db &, const ExtParams &, hipStream_t);
void launch_extend_rows(bool, const Db &, const ExtParams &, int, hipStream_t, bool);
void launch_extend_retry(bool, const Db &, const ExtParams &, hipStream_t);
void launch_later_rounds(bool, const Db &, const ExtParams &, const LaterParams &, Cand *const[2], uint32_t *const[2],
                         int32_t *const[2], uint32_t *const[2], unsigned long long *, hipStream_t);
void launch_later_finish(const ExtParams &, const LaterParams &, hipStream_t);
int row_slot_words_max(bool amb);
void launch_group(const GroupParams &, int, hipStream_t);

void launch_rbh(const RbhParams &, int, hipStream_t);
void launch_hkey(const DHsp *h, uint64_t n, const uint32_t *tx_gene, HKey *out, hipStream_t st);
void launch_rbh_place(const RbhParams &, hipStream_t);
void launch_gather_rows(const DHsp *, const DRow *, uint64_t, DHsp *, hipStream_t);
void launch_cc(const DEdge *, uint64_t, uint32_t, const int32_t *, int, int, uint32_t *, uint32_t *, uint32_t *,
               uint32_t *, uint32_t *, uint8_t *, unsigned long long *, hipStream_t);
void launch_pair_sums(const DEdge *, uint64_t, const uint32_t *, const uint8_t *, unsigned long long *,
                      unsigned long long *, unsigned long long *, unsigned long long *, hipStream_t);
void launch_distance(const unsigned long long *, const unsigned long long *, const int32_t *, const int32_t *,
                     int, int, double *, unsigned int *, hipStream_t);
}  // namespace rcg

using namespace rcg;

static thread_local std::string g_err;
static const size_t FRONT_PAD = 2;   // zero words in front of every packed array

static int fail(int code, const std::string &msg)
{
    g_err = msg;
    return code;
}

int rcg_fail(int code, const std::string &msg)
{
    return fail(code, msg);
}

#define HIPCHK(x)                                                                                    \
    do {                                                                                             \
        hipError_t e_ = (x);                                                                         \
        if (e_ != hipSuccess) return fail(RC_E_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
    } while (0)

#define CHK(x)                  \
    do {                        \
        int r_ = (x);           \
        if (r_ != RC_OK) return r_; \
    } while (0)

// Device bytes the engines of this process hold (now and at most), for the
// HBM footprint checks (rc_timing.dev_bytes / dev_peak_bytes)
static std::atomic<long long> g_dev_bytes{0}, g_dev_peak{0};
static void dev_account(long long b)
{
    const long long v = g_dev_bytes.fetch_add(b) + b;
    long long pk = g_dev_peak.load();
    while (v > pk && !g_dev_peak.compare_exchange_weak(pk, v)) {
    }
}

// Device buffer that only grows (no allocation once sized: reruns are alloc-free).
template <class T>
struct DBuf {
    T *p = nullptr;
    size_t cap = 0;
    int ensure(size_t n)
    {
        if (n <= cap && p) return RC_OK;
        release();
        size_t bytes = std::max<size_t>(n, 1) * sizeof(T);
        if (hipMalloc((void **)&p, bytes) != hipSuccess) {
            (void)hipGetLastError();
            p = nullptr;
            return fail(RC_E_NOMEM, "hipMalloc of " + std::to_string(bytes) + " bytes failed");
        }
        cap = std::max<size_t>(n, 1);
        dev_account((long long)(cap * sizeof(T)));
        return RC_OK;
    }
    // a buffer allocated elsewhere (the growth paths that keep contents)
    void adopt(T *np, size_t ncap)
    {
        dev_account((long long)(ncap * sizeof(T)));   // both are held until the old one goes
        T *op = p;
        const size_t oc = cap;
        p = np;
        cap = ncap;
        if (op) {
            (void)hipFree(op);
            dev_account(-(long long)(oc * sizeof(T)));
        }
    }
    ~DBuf() { release(); }
    void release()
    {
        if (p) {
            (void)hipFree(p);
            dev_account(-(long long)(cap * sizeof(T)));
        }
        p = nullptr;
        cap = 0;
    }
};

// every byte is A/C/G/T in either case (a branch-free inner loop the compiler
// vectorises; the scan stops at the first 64 KiB block holding another byte)
static bool all_acgt(const char *s, uint64_t n)
{
    for (uint64_t i0 = 0; i0 < n; i0 += 65536) {
        const uint64_t i1 = std::min<uint64_t>(n, i0 + 65536);
        unsigned bad = 0;
        for (uint64_t i = i0; i < i1; i++) {
            const unsigned char c = (unsigned char)s[i] | 0x20;
            bad |= (unsigned)((c != 'a') & (c != 'c') & (c != 'g') & (c != 't'));
        }
        if (bad) return false;
    }
    return true;
}

// ------------------------------------------------------------------------
// Karlin-Altschul statistics (BLAST restated; same spec as the oracle)
// ------------------------------------------------------------------------
namespace stats {
const double LAMBDA = 1.28, K = 0.46, ALPHA = 1.5, BETA = -2.0;

// BLAST_ComputeLengthAdjustment
int32_t length_adjustment(double m, double n, double N)
{
    const double logK = std::log(K), adl = ALPHA / LAMBDA;
    double ell = 0, ss, ell_min = 0, ell_max, ell_next = 0;
    bool converged = false;
    {
        const double a = N, mb = m * N + n, c = n * m - std::max(m, n) / K;
        if (c < 0) return 0;
        ell_max = 2 * c / (mb + std::sqrt(mb * mb - 4 * a * c));
    }
    for (int i = 1; i <= 20; i++) {
        ell = ell_next;
        ss = (m - ell) * (n - N * ell);
        const double ell_bar = adl * (logK + std::log(ss)) + BETA;
        if (ell_bar >= ell) {
            ell_min = ell;
            if (ell_bar - ell_min <= 1.0) {
                converged = true;
                break;
            }
            if (ell_min == ell_max) break;
        } else {
            ell_max = ell;
        }
        if (ell_min <= ell_bar && ell_bar <= ell_max)
            ell_next = ell_bar;
        else
            ell_next = (i == 1) ? ell_max : (ell_min + ell_max) / 2;
    }
    if (!converged) return (int32_t)ell_min;
    int32_t adj = (int32_t)ell_min;
    ell = std::ceil(ell_min);
    if (ell <= ell_max) {
        ss = (m - ell) * (n - N * ell);
        if (adl * (logK + std::log(ss)) + BETA >= ell) adj = (int32_t)ell;
    }
    return adj;
}

double search_space(int64_t qlen, int64_t dblen, int64_t dbn)
{
    const int32_t ell = length_adjustment((double)qlen, (double)dblen, (double)dbn);
    double mq = (double)(qlen - ell), nd = (double)(dblen - dbn * (int64_t)ell);
    if (mq < 1) mq = 1;
    if (nd < 1) nd = 1;
    return mq * nd;
}

double evalue(double ss, int32_t score_half) { return ss * K * std::exp(-LAMBDA * (score_half / 2.0)); }

int32_t threshold(double ss, double cutoff)
{
    int32_t lo = 0, hi = 1 << 26;
    if (evalue(ss, hi) > cutoff) return hi;
    while (lo < hi) {
        const int32_t mid = lo + (hi - lo) / 2;
        if (evalue(ss, mid) <= cutoff) hi = mid; else lo = mid + 1;
    }
    return lo;
}

// CAlignFormatUtil::GetScoreString formatting of the bit score, in tenths
int32_t bits10(int32_t score_half)
{
    const double bits = (LAMBDA * (score_half / 2.0) - std::log(K)) / std::log(2.0);
    char buf[64];
    if (bits > 99999) {
        std::snprintf(buf, sizeof buf, "%5.3le", bits);
        return (int32_t)std::llround(std::strtod(buf, nullptr) * 10.0);
    }
    if (bits > 99.9) return (int32_t)((long)bits) * 10;
    std::snprintf(buf, sizeof buf, "%4.1lf", bits);
    return (int32_t)std::llround(std::strtod(buf, nullptr) * 10.0);
}
}  // namespace stats

// ------------------------------------------------------------------------
// engine
// ------------------------------------------------------------------------

struct SampleRec {
    std::string label;
    uint64_t base = 0, nbases = 0;   // base: position in the concatenation of all samples (host bookkeeping)
    uint32_t tx_begin = 0, n_tx = 0;
    uint32_t gene_begin = 0, n_genes = 0;
    bool resident = true;            // bases on this GPU (rc_add_sample with a sequence)
    uint64_t abase = 0;              // resident: offset in d_ascii (a multiple of TILE_ALIGN)
};

// Samples start at multiples of TILE_ALIGN bases in d_ascii and in a tile's
// packed arrays: a 2^POS_TX_SHIFT-base block of the position -> transcript
// table never spans two samples, whatever samples a tile holds.
static const uint64_t TILE_ALIGN = 1ull << POS_TX_SHIFT;
static uint64_t align_up(uint64_t x) { return (x + TILE_ALIGN - 1) & ~(TILE_ALIGN - 1); }

struct rc_engine {
    rc_opts o{};
    hipStream_t st = nullptr;
    hipStream_t st2 = nullptr;   // DUST beside the index build
    std::vector<SampleRec> samples;
    uint64_t total_bases = 0;   // input bases added so far (all samples)
    uint64_t ascii_used = 0;    // bytes of d_ascii in use (resident samples, TILE_ALIGN-aligned)
    std::vector<uint64_t> tx_start{0};
    std::vector<int32_t> tx_sample, tx_gene_id, tx_iso;
    bool has_amb = false;

    // derived on upload
    std::vector<uint32_t> tx_gene, gene_tx_off, gene_tx, sample_gene_begin, sample_tx_begin;
    std::vector<int32_t> gene_sample, gene_id;
    std::vector<int64_t> db_len, db_n;
    std::vector<int32_t> pair_a, pair_b, pair_index;
    std::vector<int64_t> shard_first;   // shard r owns pairs [shard_first[r], shard_first[r + 1])
    std::vector<uint32_t> pair_item_begin;
    int32_t max_len = 0;
    int xbits = 24;                     // seed-key position bits (pos_bits(max_len))
    uint64_t n_items = 0;
    int index_bits = 16;
    uint64_t n_index = 0;               // entries of the loaded tile's index
    uint64_t tile_npos = 0;             // 16-mer positions of the loaded tile's indexed transcripts
    std::vector<TxInfo> h_tx;           // every transcript (start 0: the device table holds tile starts)
    std::vector<uint64_t> sample_kmers; // 16-mer positions of each sample's transcripts
    std::vector<TileSeg> h_segs;        // the loaded tile's samples (load_tile)
    std::vector<uint64_t> h_spos, h_send;

    // tiles of this shard (plan_tiles) and the one whose tables are loaded
    struct Tile {
        std::vector<int> samples;                 // ascending
        std::vector<std::pair<int, int>> pairs;   // (a, b), a < b
        // split tiles (a shard cut into several, every a below every b):
        // the b chunk's samples sit at bstart, the same in every tile of that
        // chunk, so consecutive tiles of one b chunk share its 16-mer index
        // and its DUST masks (only the a part is redone)
        int bchunk = -1;
        uint64_t bstart = 0;
    };
    std::vector<Tile> tiles;
    int64_t tiles_for = -1;
    int tile_loaded = -1;
    std::vector<uint64_t> tile_pos;     // first base of each sample in the loaded tile
    uint64_t tile_total = 0;
    bool tile_direct = false;           // the loaded tile is d_ascii's layout (no gathered copy)
    uint32_t tile_ntx = 0;              // the tile's transcripts (DUST, near-mask index)
    uint32_t tile_nitx = 0;             // ... of its subject samples (the 16-mer index)
    bool tile_share = false;            // the search mode the loaded tile's index list was built for
    std::vector<uint32_t> tile_tx_first;   // first transcript (in d_tile_tx) of each sample of the tile
    // DUST masks given by rc_set_dust_masks (computed once per sample across
    // shards): word offset of each sample's mask in d_dust_imp, ~0 = not given
    std::vector<uint64_t> dust_imp_off;
    // after an rc_dust_masks pass over the loaded tile itself: which samples'
    // masks it recomputed (the others were cleared); empty = every tile sample
    std::vector<char> dmask_only;
    // the b chunk (split tiles) whose index and DUST masks the device holds
    // from this run's previous tile (-1: none)
    int idx_bchunk = -1;
    uint64_t idx_bstart = 0;
    uint64_t hsp_used = 0;              // HSPs appended to d_hsp by the tiles of this run

    // external HSPs
    bool external = false;
    std::map<std::pair<int, int>, std::vector<rc_hsp>> ext;

    // state
    bool uploaded = false, aligned = false, finished = false;
    // this shard's sample pairs [pair0, pair1) and their items [item0, item1)
    uint64_t pair0 = 0, pair1 = 0, item0 = 0, item1 = 0;
    uint64_t n_local_edges = 0;
    bool rbh_done = false;
    bool graph_only = false;        // an imported graph + tables, no alignment (rc_import_edges on a fresh engine)
    int32_t sample_count_given = 0; // > 0: the ideal test's sample count (rc_set_sample_count)

    // device buffers
    DBuf<uint8_t> d_ascii, d_tile_ascii;
    DBuf<TxInfo> d_tile_tx, d_tile_itx;
    DBuf<uint32_t> d_tile_gid;          // global id of each tile transcript
    DBuf<TileSeg> d_tile_segs;
    DBuf<uint64_t> d_tile_send, d_tx_rel, d_kpre;   // tile sample ends; per transcript: start in its sample,
                                                    // 16-mer slots of its sample's transcripts before it
    DBuf<uint64_t> d_F, d_RC, d_AF, d_ARC;
    DBuf<TxInfo> d_tx;
    DBuf<IsoRec> d_giso;
    DBuf<uint32_t> d_tx_gene, d_gene_tx_off, d_gene_tx, d_sample_gene_begin, d_sample_tx_begin;
    DBuf<int32_t> d_gene_sample;
    DBuf<uint64_t> d_kpos_off, d_kcnt;
    // shared searches with DUST: masked tile transcripts, the near-mask index
    // of the reverse pass, its reverse-only seeds (sorted by forward gene)
    DBuf<uint8_t> d_tile_masked;
    DBuf<uint64_t> d_ment, d_ment2;
    DBuf<uint32_t> d_mbucket;
    int mindex_bits = 16;
    uint64_t n_mindex = 0, mnear_cap = 0;
    DBuf<LSeed> d_rseeds;
    DBuf<uint32_t> d_rseed_gene, d_rs_key, d_rs_idx, d_rs_range;
    DBuf<unsigned long long> d_rctr;   // [0] near-index entries, [1] reverse-only seeds
    DBuf<uint64_t> d_rtmask;
    DBuf<int32_t> d_trange, d_rtrange;   // [N][2] subject-sample range of each query sample (tmask / rtmask)
    uint64_t rseed_cap = 0, n_rseeds = 0;
    uint32_t res_cap = 0;
    // fraction of the last run's candidates whose first-seed extension
    // outgrew the 32-lane window (selects the saving row kernel, RC_RESUME)
    double ovf_frac = 0.0;
    DBuf<uint64_t> d_ent, d_ent2;   // (k-mer << 32 | position), unsorted / sorted
    // the index sort's scratch (sort.hip): digit histograms + tile counters,
    // the look-back table (zeroed when allocated; tagged by pass epoch)
    DBuf<uint32_t> d_sort_scratch, d_gen_tile;
    DBuf<uint64_t> d_sort_status;
    uint32_t sort_epoch = 0;
    DBuf<uint32_t> d_bucket;
    DBuf<PosTx> d_pos_tx;
    DBuf<uint64_t> d_sample_pos, d_txstart, d_kpos_rel, d_dmask, d_dust_imp;
    DBuf<uint32_t> d_dust_scratch;
    DBuf<uint64_t> d_dust_events;
    DBuf<unsigned long long> d_prof;
    DBuf<uint8_t> d_tmp;
    DBuf<int32_t> d_thr, d_bits10;
    DBuf<DHsp> d_hsp;
    DBuf<HKey> d_hkey;   // RBH: (bit score, subject gene) per d_hsp entry
    DBuf<GSeed> d_seeds;
    DBuf<Cand> d_cands;
    DBuf<DHsp> d_cand_hsp, d_ovf;
    DBuf<uint8_t> d_cand_nh;
    DBuf<int32_t> d_cand_box, d_cand_box2;
    // shared searches (RC_SHARE, default): the reverse search's HSPs per candidate
    DBuf<DHsp> d_cand_hsp_r;
    DBuf<uint8_t> d_cand_nh_r;
    DBuf<uint32_t> d_cand_ovf_r, d_defer_r, d_list2, d_wide0, d_wide1;
    DBuf<int32_t> d_resume;   // saved 32-lane extension states for the 64-lane pass (RES_REC ints each)
    // later-seed rounds (shared searches): search states, the rounds' work
    // (alternating), active lists, counters
    DBuf<int32_t> d_later, d_lbox0, d_lbox1;
    DBuf<Cand> d_lvc0, d_lvc1;
    DBuf<uint32_t> d_llist0, d_llist1, d_lact0, d_lact1, d_lfull0, d_lfull1;
    DBuf<unsigned long long> d_lcnt;
    bool share = false;
    DBuf<DRow> d_rows_tmp;
    DBuf<DEdge> d_edges_tmp;
    DBuf<uint32_t> d_cand_ovf, d_gc_off, d_gc_cnt, d_gcount, d_defer, d_defer2;
    DBuf<uint64_t> d_gscan, d_mscan, d_mkey, d_tmask, d_mbig;
    DBuf<uint32_t> d_mcnt, d_mcur, d_tx_pos, d_iso_pre, d_iso_list, d_iso_list_r;
    DBuf<unsigned long long> d_shard_cnt, d_shard_prefix;
    uint64_t seed_cap = 0, cand_cap = 0, ovf_cap = 0;   // per-shard / total capacities
    // (gene, sample) seed passes too big for LDS, and their global scratch
    DBuf<uint64_t> d_big_out, d_big_list, d_big_retry;
    DBuf<LSeed> d_big_seeds;
    DBuf<uint32_t> d_big_seg;
    DBuf<uint8_t> d_big_segT;
    uint64_t big_list_cap = 1 << 16;
    uint32_t big_cap = 1 << 13;
    DBuf<uint32_t> d_grp_off, d_grp_cnt;
    DBuf<unsigned long long> d_count;
    DBuf<unsigned int> d_status;
    DBuf<uint32_t> d_pair_item_begin;
    DBuf<int32_t> d_pair_a, d_pair_b, d_pair_index;
    DBuf<uint32_t> d_cnt4;   // 4 * (n_items + 1)
    DBuf<uint64_t> d_off4;   // 4 * (n_items + 1)
    DBuf<DRow> d_rows;
    DBuf<DHsp> d_gather;
    DBuf<DEdge> d_edges;
    uint64_t n_rows = 0, n_edges = 0, n_hsps = 0, n_seeds = 0, n_cands = 0;
    DBuf<uint32_t> d_parent, d_present, d_cnodes, d_cedges, d_sample_present;
    DBuf<uint8_t> d_ideal;
    DBuf<unsigned long long> d_stats, d_num, d_den, d_num_all, d_den_all;
    DBuf<int32_t> d_order;
    DBuf<double> d_dist;

    // host results
    std::vector<unsigned long long> h_num, h_den, h_num_all, h_den_all, h_stats;
    std::vector<double> h_ss;   // search space of a query of length L against sample T: [T][L]
    std::vector<double> h_exp;  // exp(-lambda * S / 2) per raw score in half units S (stats::evalue's factor)
    rc_timing tm{};
    hipEvent_t ev[16] = {};
    hipEvent_t evd[3] = {};   // DUST start / end on st2, its start condition on st

    ~rc_engine()
    {
        for (auto &e : ev)
            if (e) (void)hipEventDestroy(e);
        for (hipEvent_t x : evd)
            if (x) (void)hipEventDestroy(x);
        if (st2) (void)hipStreamDestroy(st2);
        if (st) (void)hipStreamDestroy(st);
    }
};

static int set_device(rc_engine *e) { HIPCHK(hipSetDevice(e->o.device)); return RC_OK; }

static double wall_ms()
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// the alignment's blocking waits on the engine's stream (rc_timing.host_wait_ms)
static int wait_st(rc_engine *e)
{
    const double t0 = wall_ms();
    HIPCHK(hipStreamSynchronize(e->st));
    e->tm.host_wait_ms += wall_ms() - t0;
    return RC_OK;
}

// Both directed searches of a pair from one candidate set (query = the lower
// sample), unless spec 5b or RC_SHARE=0 (one after the other)
static bool share_mode(const rc_engine *e)
{
    const char *sv = getenv("RC_SHARE");
    return !e->o.symmetric && !(sv && atoi(sv) == 0);
}

extern "C" {

void rc_default_opts(rc_opts *o)
{
    o->top_matches = 1;
    o->keep_all = 1;
    o->evalue = 1e-99;
    o->word_size = 28;
    o->xdrop_half = 108;
    o->device = 0;
    o->shard_rank = 0;
    o->shard_count = 1;
    o->symmetric = 0;
    o->dust_level = 20;
    o->dust_window = 64;
    o->dust_linker = 1;
}

const char *rc_last_error(void) { return g_err.c_str(); }

void rc_dev_peak_reset(void) { g_dev_peak.store(g_dev_bytes.load()); }

uint64_t rc_edge_record_size(void) { return sizeof(DEdge); }

int rc_create(const rc_opts *opts, rc_engine **out)
{
    if (!opts || !out) return fail(RC_E_ARG, "null argument");
    if (opts->top_matches < 1) return fail(RC_E_ARG, "top_matches must be >= 1");
    if (opts->word_size < W16 || opts->word_size > 64) return fail(RC_E_ARG, "word_size must be in [16, 64]");
    if (opts->xdrop_half < 0) return fail(RC_E_ARG, "xdrop_half must be >= 0");
    if (opts->dust_level < 0 || (opts->dust_level > 0 && (opts->dust_window < 8 || opts->dust_window > 64 ||
                                                          opts->dust_linker < 0)))
        return fail(RC_E_ARG, "bad DUST parameters");
    if (opts->dust_level > 0 && opts->symmetric)
        return fail(RC_E_ARG, "DUST masks each direction's query: it needs symmetric = 0");
    if (opts->shard_count < 1 || opts->shard_rank < 0 || opts->shard_rank >= opts->shard_count)
        return fail(RC_E_ARG, "bad shard");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        (void)hipGetLastError();
        return fail(RC_E_HIP, "no HIP device available");
    }
    if (opts->device < 0 || opts->device >= ndev) return fail(RC_E_ARG, "bad device ordinal");
    rc_engine *e = new rc_engine();
    e->o = *opts;
    if (hipSetDevice(e->o.device) != hipSuccess || hipStreamCreateWithFlags(&e->st, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&e->st2, hipStreamNonBlocking) != hipSuccess) {
        delete e;
        return fail(RC_E_HIP, "stream creation failed");
    }
    for (auto &ev : e->evd)
        if (hipEventCreate(&ev) != hipSuccess) {
            delete e;
            return fail(RC_E_HIP, "event creation failed");
        }
    for (auto &ev : e->ev)
        if (hipEventCreate(&ev) != hipSuccess) {
            delete e;
            return fail(RC_E_HIP, "event creation failed");
        }
    *out = e;
    return RC_OK;
}

int rc_destroy(rc_engine *e)
{
    if (!e) return RC_OK;
    (void)hipSetDevice(e->o.device);
    delete e;  // DBuf destructors free the device buffers
    return RC_OK;
}

int rc_add_sample(rc_engine *e, const char *label, const char *seq, const uint64_t *tx_offsets,
                  const int32_t *gene, const int32_t *iso, uint32_t n_tx, int32_t *sample_id)
{
    if (!e || !label || !tx_offsets || (n_tx && (!gene || !iso))) return fail(RC_E_ARG, "null argument");
    if (e->uploaded) return fail(RC_E_STATE, "samples must be added before rc_run");
    if (e->samples.size() >= MAX_SAMPLES) return fail(RC_E_LIMIT, "at most 65535 samples per engine");
    if (tx_offsets[0] != 0) return fail(RC_E_ARG, "tx_offsets[0] must be 0");
    for (uint32_t t = 0; t < n_tx; t++) {
        if (tx_offsets[t + 1] < tx_offsets[t]) return fail(RC_E_ARG, "tx_offsets must be non-decreasing");
        if (tx_offsets[t + 1] - tx_offsets[t] > (1u << 24) - 64)
            return fail(RC_E_LIMIT, "transcripts longer than 16 Mbp are not supported");
    }
    const uint64_t nb = tx_offsets[n_tx];
    SampleRec s;
    s.label = label;
    s.base = e->total_bases;
    s.nbases = nb;
    s.tx_begin = (uint32_t)e->tx_sample.size();
    s.n_tx = n_tx;
    // seq == NULL with bases: a sample another GPU aligns (sharded runs hold
    // only the samples of their own pairs); its transcripts and genes still
    // count (graph nodes, e-value statistics)
    s.resident = nb == 0 || seq != nullptr;
    // the bases go straight to HBM (the ASCII array the pack kernels read), at
    // a TILE_ALIGN boundary (the gap filled with 'A'); the device array grows
    // geometrically, old contents moved device-side
    if (nb && seq) {
        CHK(set_device(e));
        s.abase = align_up(e->ascii_used);
        const uint64_t need = align_up(s.abase + nb) + 64;
        if (need > e->d_ascii.cap) {
            const size_t cap = std::max<size_t>({(size_t)need, e->d_ascii.cap + e->d_ascii.cap / 4, (size_t)1 << 28});
            uint8_t *np = nullptr;
            if (hipMalloc((void **)&np, cap) != hipSuccess) {
                (void)hipGetLastError();
                return fail(RC_E_NOMEM, "hipMalloc of " + std::to_string(cap) + " bytes failed");
            }
            if (e->ascii_used)
                HIPCHK(hipMemcpyAsync(np, e->d_ascii.p, e->ascii_used, hipMemcpyDeviceToDevice, e->st));
            HIPCHK(hipStreamSynchronize(e->st));
            e->d_ascii.adopt(np, cap);
        }
        HIPCHK(hipMemsetAsync(e->d_ascii.p + e->ascii_used, 'A', need - e->ascii_used, e->st));
        HIPCHK(hipMemcpyAsync(e->d_ascii.p + s.abase, seq, nb, hipMemcpyHostToDevice, e->st));
        if (!e->has_amb) e->has_amb = !all_acgt(seq, nb);
        HIPCHK(hipStreamSynchronize(e->st));   // the caller's buffer is not retained
        e->ascii_used = s.abase + nb;
    }
    e->total_bases += nb;
    const int32_t sid = (int32_t)e->samples.size();
    for (uint32_t t = 0; t < n_tx; t++) {
        e->tx_start.push_back(s.base + tx_offsets[t + 1]);
        e->tx_sample.push_back(sid);
        e->tx_gene_id.push_back(gene[t]);
        e->tx_iso.push_back(iso[t]);
    }
    e->samples.push_back(s);
    if (sample_id) *sample_id = sid;
    return RC_OK;
}

int rc_add_hsps(rc_engine *e, int32_t q, int32_t s, const rc_hsp *h, uint64_t n)
{
    if (!e || (n && !h)) return fail(RC_E_ARG, "null argument");
    if (e->uploaded) return fail(RC_E_STATE, "HSPs must be added before rc_run");
    const int N = (int)e->samples.size();
    if (q < 0 || q >= N || s < 0 || s >= N || q == s) return fail(RC_E_ARG, "bad sample pair");
    for (uint64_t i = 0; i < n; i++)
        if (h[i].q_tx >= e->samples[q].n_tx || h[i].s_tx >= e->samples[s].n_tx)
            return fail(RC_E_ARG, "HSP transcript index out of range");
    e->external = true;
    auto &v = e->ext[{q, s}];
    v.insert(v.end(), h, h + n);
    return RC_OK;
}

}  // extern "C"

// Build gene numbering, tables and upload everything that does not change
// between runs. Inputs are then resident in HBM; rc_run repacks from them.
static void shard_pairs(rc_engine *e);

// Shard plan. The C(N,2) sample pairs (a < b) are the cells
// of the (a, b) triangle; shard_count shards each take one rectangle
// [a0, a1) x [b0, b1) of it, found by recursive bisection that minimises the
// largest shard's modelled time. Both directed searches of a pair run on its
// shard, so the shard's samples -- the ones it holds, indexes and scans --
// are [a0, a1) u [b0, b1):
//   pair work    2 x (L_a + L_b) per pair (seed hits, extension, RBH)
//   queries      9 x L_s per query sample (the seed kernel's per-gene work)
//   subjects    15 x L_s per subject sample (16-mer index + reverse pass)
// (r04: least squares over the eight C3 rank shards with shared DUST masks,
// scripts/shard_time.py, profiles/r04_n: 0.94 ms per query sample, 1.5 per
// subject sample, 0.41 per pair). Pairs are
// numbered shard by shard, subject-major inside a shard; one shard gives the
// plain subject-major order (0,1), (0,2), (1,2), (0,3), ...
namespace plan {
struct Rect {
    int a0, a1, b0, b1;
};
struct Planner {
    int N;
    std::vector<double> SL;   // prefix sums of sample bases
    std::map<std::array<int, 5>, std::pair<double, std::vector<Rect>>> memo;
    double S(int i, int j) const { return j > i ? SL[j] - SL[i] : 0.0; }
    static Rect norm(Rect r)
    {
        r.a1 = std::min(r.a1, r.b1 - 1);
        r.b0 = std::max(r.b0, r.a0 + 1);
        if (r.a1 <= r.a0 || r.b1 <= r.b0) r = Rect{0, 0, 0, 0};
        return r;
    }
    static bool empty(const Rect &r) { return r.a1 <= r.a0 || r.b1 <= r.b0; }
    double leaf(const Rect &r) const
    {
        if (empty(r)) return 0.0;
        double pw = 0.0;
        for (int b = r.b0; b < r.b1; b++) {
            const int ae = std::min(r.a1, b);
            if (ae > r.a0) pw += S(r.a0, ae) + (double)(ae - r.a0) * (SL[b + 1] - SL[b]);
        }
        // a sample that is both a query and a subject of the rank pays both
        return 2.0 * pw + 9.0 * S(r.a0, r.a1) + 15.0 * S(r.b0, r.b1);
    }
    std::pair<double, std::vector<Rect>> best(Rect r, int k)
    {
        r = norm(r);
        const std::array<int, 5> key{r.a0, r.a1, r.b0, r.b1, k};
        auto it = memo.find(key);
        if (it != memo.end()) return it->second;
        std::pair<double, std::vector<Rect>> res{leaf(r), std::vector<Rect>(k, Rect{0, 0, 0, 0})};
        res.second[0] = r;
        if (k > 1 && !empty(r)) {
            const int k1 = k / 2;
            auto consider = [&](Rect x, Rect y) {
                for (int sw = 0; sw < (k1 == k - k1 ? 1 : 2); sw++) {
                    const int kx = sw ? k - k1 : k1;
                    const auto X = best(x, kx);
                    if (X.first >= res.first) continue;
                    const auto Y = best(y, k - kx);
                    const double c = std::max(X.first, Y.first);
                    if (c < res.first) {
                        res.first = c;
                        res.second = X.second;
                        res.second.insert(res.second.end(), Y.second.begin(), Y.second.end());
                    }
                }
            };
            const int nc = N > 128 ? 12 : 32;   // cut candidates per axis
            const int sa = std::max(1, (r.a1 - r.a0) / nc), sb = std::max(1, (r.b1 - r.b0) / nc);
            for (int c = r.a0 + sa; c < r.a1; c += sa) consider({r.a0, c, r.b0, r.b1}, {c, r.a1, r.b0, r.b1});
            for (int c = r.b0 + sb; c < r.b1; c += sb) consider({r.a0, r.a1, r.b0, c}, {r.a0, r.a1, c, r.b1});
        }
        memo.emplace(key, res);
        return res;
    }
};

// pair order (pair_a, pair_b) and shard cuts pair_first[shard_count + 1]
static void plan_pairs(const int64_t *bases, int N, int shards, std::vector<int32_t> &pa, std::vector<int32_t> &pb,
                       std::vector<int64_t> &first)
{
    pa.clear();
    pb.clear();
    first.assign((size_t)shards + 1, 0);
    std::vector<Rect> rects;
    if (shards == 1) {
        rects.push_back(Planner::norm({0, N, 0, N}));
    } else {
        Planner P;
        P.N = N;
        P.SL.assign((size_t)N + 1, 0.0);
        for (int i = 0; i < N; i++) P.SL[i + 1] = P.SL[i] + (double)std::max<int64_t>(bases[i], 1);
        rects = P.best({0, N, 0, N}, shards).second;
    }
    for (int r = 0; r < shards; r++) {
        first[r] = (int64_t)pa.size();
        const Rect q = rects[r];
        for (int b = q.b0; b < q.b1; b++)
            for (int a = q.a0; a < std::min(q.a1, b); a++) {
                pa.push_back(a);
                pb.push_back(b);
            }
    }
    first[shards] = (int64_t)pa.size();
}
}  // namespace plan

static int upload(rc_engine *e)
{
    if (e->uploaded) return RC_OK;
    CHK(set_device(e));
    const int N = (int)e->samples.size();
    if (N < 2) return fail(RC_E_ARG, "need at least two samples");
    if (N > MAX_SAMPLES) return fail(RC_E_LIMIT, "more than 65535 samples per engine");
    if (e->tx_sample.size() >= MAX_TX) return fail(RC_E_LIMIT, "more than 2^27 transcripts per engine");
    const uint32_t n_tx = (uint32_t)e->tx_sample.size();
    // genes: per sample distinct gene ids ascending; a gene's transcripts in input order
    e->tx_gene.assign(n_tx, 0);
    e->gene_tx_off.assign(1, 0);
    e->gene_tx.clear();
    e->gene_sample.clear();
    e->gene_id.clear();
    e->sample_gene_begin.assign(N + 1, 0);
    e->sample_tx_begin.assign(N + 1, 0);
    e->db_len.assign(N, 0);
    e->db_n.assign(N, 0);
    e->max_len = 0;
    for (int si = 0; si < N; si++) {
        SampleRec &s = e->samples[si];
        e->sample_tx_begin[si] = s.tx_begin;
        s.gene_begin = (uint32_t)e->gene_sample.size();
        e->sample_gene_begin[si] = s.gene_begin;
        std::vector<std::pair<int32_t, uint32_t>> byg;
        for (uint32_t t = 0; t < s.n_tx; t++) byg.push_back({e->tx_gene_id[s.tx_begin + t], s.tx_begin + t});
        std::stable_sort(byg.begin(), byg.end(),
                         [](const std::pair<int32_t, uint32_t> &a, const std::pair<int32_t, uint32_t> &b) {
                             return a.first < b.first;
                         });
        for (size_t i = 0; i < byg.size(); i++) {
            if (i == 0 || byg[i].first != byg[i - 1].first) {
                if (i) e->gene_tx_off.push_back((uint32_t)e->gene_tx.size());
                e->gene_sample.push_back(si);
                e->gene_id.push_back(byg[i].first);
            }
            e->tx_gene[byg[i].second] = (uint32_t)(e->gene_sample.size() - 1);
            e->gene_tx.push_back(byg[i].second);
        }
        if (!byg.empty()) e->gene_tx_off.push_back((uint32_t)e->gene_tx.size());
        s.n_genes = (uint32_t)e->gene_sample.size() - s.gene_begin;
        for (uint32_t t = 0; t < s.n_tx; t++) {
            const uint64_t L = e->tx_start[s.tx_begin + t + 1] - e->tx_start[s.tx_begin + t];
            e->db_len[si] += (int64_t)L;
            e->max_len = std::max<int32_t>(e->max_len, (int32_t)L);
        }
        e->db_n[si] = s.n_tx;
    }
    e->sample_tx_begin[N] = n_tx;
    e->sample_gene_begin[N] = (uint32_t)e->gene_sample.size();
    const uint32_t n_genes = (uint32_t)e->gene_sample.size();
    // the seed key's position field holds the longest transcript; its
    // isoform field the rest (max_iso: 65535 unless transcripts reach 2^21)
    e->xbits = pos_bits(e->max_len);
    for (uint32_t g = 0; g < n_genes; g++)
        if (e->gene_tx_off[g + 1] - e->gene_tx_off[g] > max_iso(e->xbits))
            return fail(RC_E_LIMIT, "gene " + std::to_string(e->gene_id[g]) + " has more than " +
                                        std::to_string(max_iso(e->xbits)) + " transcripts");
    // pairs (a < b) in the shard plan's order (plan::plan_pairs): every
    // shard a rectangle [a0, a1) x [b0, b1) of the pair triangle; items =
    // (pair, gene of b). (Outputs are per pair and do not depend on this.)
    {
        std::vector<int64_t> bases(N);
        for (int i = 0; i < N; i++) bases[i] = e->db_len[i];
        plan::plan_pairs(bases.data(), N, e->o.shard_count, e->pair_a, e->pair_b, e->shard_first);
    }
    e->pair_item_begin.assign(1, 0);
    e->pair_index.assign((size_t)N * N, -1);
    uint64_t items = 0;
    for (size_t p = 0; p < e->pair_a.size(); p++) {
        const int a = e->pair_a[p], b = e->pair_b[p];
        e->pair_index[a * N + b] = e->pair_index[b * N + a] = (int32_t)p;
        items += e->samples[b].n_genes;
        if (items > 0xFFFFFFFFull) return fail(RC_E_LIMIT, "too many (pair, gene) items");
        e->pair_item_begin.push_back((uint32_t)items);
    }
    e->n_items = items;
    shard_pairs(e);

    // device copies of what does not change between runs
    auto up = [&](auto &buf, const auto &vec) -> int {
        using T = typename std::remove_reference<decltype(vec)>::type::value_type;
        CHK(buf.ensure(vec.size()));
        if (!vec.empty())
            HIPCHK(hipMemcpyAsync(buf.p, vec.data(), vec.size() * sizeof(T), hipMemcpyHostToDevice, e->st));
        return RC_OK;
    };
    e->h_tx.assign(n_tx, TxInfo{});
    for (uint32_t t = 0; t < n_tx; t++) {
        e->h_tx[t].start = 0;   // a position in the current tile (load_tile)
        e->h_tx[t].len = (uint32_t)(e->tx_start[t + 1] - e->tx_start[t]);
        e->h_tx[t].sample = e->tx_sample[t];
    }
    CHK(up(e->d_tx, e->h_tx));
    {
        // per transcript: its start within its sample and the 16-mer slots of
        // the sample's transcripts before it (the tile tables' inputs)
        std::vector<uint64_t> rel(n_tx), kpre(n_tx);
        e->sample_kmers.assign(N, 0);
        for (int si = 0; si < N; si++) {
            const SampleRec &S = e->samples[si];
            uint64_t k = 0;
            for (uint32_t t = S.tx_begin; t < S.tx_begin + S.n_tx; t++) {
                rel[t] = e->tx_start[t] - S.base;
                kpre[t] = k;
                const int64_t L = (int64_t)e->h_tx[t].len;
                k += (uint64_t)(L >= W16 ? L - W16 + 1 : 0);
            }
            e->sample_kmers[si] = k;
        }
        CHK(up(e->d_tx_rel, rel));
        CHK(up(e->d_kpre, kpre));
        HIPCHK(hipStreamSynchronize(e->st));   // (rel, kpre are about to go)
    }
    {
        std::vector<IsoRec> giso(e->gene_tx.size());
        for (size_t k = 0; k < giso.size(); k++) {
            const TxInfo &x = e->h_tx[e->gene_tx[k]];
            giso[k] = IsoRec{(uint32_t)x.start, x.len, e->gene_tx[k], 0u};
        }
        CHK(up(e->d_giso, giso));
    }
    CHK(up(e->d_tx_gene, e->tx_gene));
    std::vector<uint32_t> tx_pos(n_tx, 0);
    for (uint32_t g = 0; g < n_genes; g++)
        for (uint32_t i = e->gene_tx_off[g]; i < e->gene_tx_off[g + 1]; i++) tx_pos[e->gene_tx[i]] = i - e->gene_tx_off[g];
    CHK(up(e->d_tx_pos, tx_pos));
    {
        // word-item prefix of every gene's isoforms (the seed kernel reads it
        // for genes with more than ISO_LDS isoforms): gene g's entries at
        // gene_tx_off[g] + g + i, i = 0..niso
        const int stride = e->o.word_size - W16 + 1;
        std::vector<uint32_t> ipre((size_t)n_tx + n_genes + 1, 0);
        for (uint32_t g = 0; g < n_genes; g++) {
            uint32_t pre = 0;
            const uint32_t b = e->gene_tx_off[g], n = e->gene_tx_off[g + 1] - b;
            for (uint32_t i = 0; i <= n; i++) {
                ipre[(size_t)b + g + i] = pre;
                if (i < n) {
                    const int64_t L = (int64_t)e->h_tx[e->gene_tx[b + i]].len;
                    pre += L >= W16 ? 2u * (uint32_t)((L - W16) / stride + 1) : 0u;
                }
            }
        }
        CHK(up(e->d_iso_pre, ipre));
    }
    CHK(up(e->d_gene_tx_off, e->gene_tx_off));
    CHK(up(e->d_gene_tx, e->gene_tx));
    CHK(up(e->d_gene_sample, e->gene_sample));
    CHK(up(e->d_sample_gene_begin, e->sample_gene_begin));
    CHK(up(e->d_sample_tx_begin, e->sample_tx_begin));
    CHK(up(e->d_pair_item_begin, e->pair_item_begin));
    CHK(up(e->d_pair_a, e->pair_a));
    CHK(up(e->d_pair_b, e->pair_b));
    CHK(up(e->d_pair_index, e->pair_index));
    // statistics tables
    std::vector<int32_t> thr((size_t)N * (e->max_len + 1));
    e->h_ss.assign((size_t)N * (e->max_len + 1), 0.0);
    for (int T = 0; T < N; T++)
        for (int32_t L = 0; L <= e->max_len; L++) {
            const size_t k = (size_t)T * (e->max_len + 1) + L;
            e->h_ss[k] = stats::search_space(L, e->db_len[T], e->db_n[T]);
            thr[k] = L ? stats::threshold(e->h_ss[k], e->o.evalue) : (1 << 26);
        }
    e->h_exp.resize((size_t)2 * e->max_len + 2);
    for (size_t sc = 0; sc < e->h_exp.size(); sc++) e->h_exp[sc] = std::exp(-stats::LAMBDA * ((int32_t)sc / 2.0));
    std::vector<int32_t> b10((size_t)2 * e->max_len + 2);
    for (size_t sc = 0; sc < b10.size(); sc++) b10[sc] = stats::bits10((int32_t)sc);
    CHK(up(e->d_thr, thr));
    CHK(up(e->d_bits10, b10));
    CHK(e->d_status.ensure(4));
    CHK(e->d_count.ensure(16));
    HIPCHK(hipStreamSynchronize(e->st));
    e->tile_loaded = -1;
    e->uploaded = true;
    return RC_OK;
}

static double ev_ms(rc_engine *e, int a, int b)
{
    float ms = 0;
    if (hipEventElapsedTime(&ms, e->ev[a], e->ev[b]) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return ms;
}

// ------------------------------------------------------------------------
// tiles
// ------------------------------------------------------------------------
//
// A tile is the unit of one alignment pass: a set of samples packed into one
// working copy (positions relative to the tile, < 2^32) and indexed together,
// and the directed searches between them. A shard's pairs form a rectangle
// [a0, a1) x [b0, b1) of the pair triangle; when its samples fit one tile
// (rc_opts-independent cap RC_TILE_BASES, default 2^32 - 2^24 bases) the
// shard is one tile, else the a- and b-ranges are cut into chunks of at most
// half the cap and every (a chunk, b chunk) with pairs is a tile. Each pass
// appends its HSPs to the shard's store; reciprocal best hits then run over
// all the shard's pairs.

static uint64_t tile_cap()
{
    const char *v = getenv("RC_TILE_BASES");   // test knob: force small tiles
    if (v) return std::max<uint64_t>(strtoull(v, nullptr, 10), TILE_ALIGN);
    return (1ull << 32) - (1ull << 24);
}

static void plan_tiles(rc_engine *e)
{
    e->tiles.clear();
    std::vector<std::pair<int, int>> pairs;
    for (uint64_t p = e->pair0; p < e->pair1; p++) pairs.push_back({e->pair_a[p], e->pair_b[p]});
    if (pairs.empty()) return;
    auto bases = [&](int s) { return align_up(e->samples[s].nbases); };
    const uint64_t cap = tile_cap();
    std::vector<int> A, B, U;
    for (auto &pr : pairs) {
        A.push_back(pr.first);
        B.push_back(pr.second);
        U.push_back(pr.first);
        U.push_back(pr.second);
    }
    for (auto *v : {&A, &B, &U}) {
        std::sort(v->begin(), v->end());
        v->erase(std::unique(v->begin(), v->end()), v->end());
    }
    uint64_t ub = 0;
    for (int s : U) ub += bases(s);
    auto chunks = [&](const std::vector<int> &R, uint64_t lim) {
        std::vector<std::vector<int>> out(1);
        uint64_t acc = 0;
        for (int s : R) {
            if (!out.back().empty() && acc + bases(s) > lim) {
                out.push_back({});
                acc = 0;
            }
            out.back().push_back(s);
            acc += bases(s);
        }
        return out;
    };
    const bool multi = ub > cap;
    const auto CA = !multi ? std::vector<std::vector<int>>{U} : chunks(A, cap / 2);
    const auto CB = !multi ? std::vector<std::vector<int>>{U} : chunks(B, cap / 2);
    const bool no_split = getenv("RC_TILE_SPLIT") && atoi(getenv("RC_TILE_SPLIT")) == 0;   // (per plan: tests flip it)
    uint64_t amax = 0;
    for (size_t j = 0; j < CB.size(); j++)
        for (size_t i = 0; i < CA.size(); i++) {
            rc_engine::Tile t;
            std::vector<char> ina(e->samples.size(), 0), inb(e->samples.size(), 0);
            for (int s : CA[i]) ina[s] = 1;
            for (int s : CB[j]) inb[s] = 1;
            int amax_s = -1, bmin_s = INT32_MAX;
            for (auto &pr : pairs)
                if (ina[pr.first] && inb[pr.second]) {
                    t.pairs.push_back(pr);
                    amax_s = std::max(amax_s, pr.first);
                    bmin_s = std::min(bmin_s, pr.second);
                }
            if (t.pairs.empty()) continue;
            for (auto &pr : t.pairs) {
                t.samples.push_back(pr.first);
                t.samples.push_back(pr.second);
            }
            std::sort(t.samples.begin(), t.samples.end());
            t.samples.erase(std::unique(t.samples.begin(), t.samples.end()), t.samples.end());
            if (multi && !no_split && amax_s < bmin_s) {
                // every a below every b: the b part (all of CB[j]: each of its
                // samples pairs with the a's) after a part padded to the
                // largest a part of any split tile
                t.bchunk = (int)j;
                uint64_t ab = 0;
                for (int s : t.samples)
                    if (s <= amax_s) ab += bases(s);
                amax = std::max(amax, ab);
            }
            e->tiles.push_back(t);
        }
    for (auto &t : e->tiles)
        if (t.bchunk >= 0) t.bstart = amax;
}

// Device tables of tile ti: packed working copy (gathered from d_ascii unless
// the tile is d_ascii's layout), transcript starts, sample ranges, the
// position -> transcript blocks and transcript-start bits, and the tile's
// transcripts for the index. Kept while the same tile is loaded.
static int load_tile(rc_engine *e, int ti)
{
    const rc_engine::Tile &T = e->tiles[ti];
    const int N = (int)e->samples.size();
    e->tile_pos.assign(N + 1, 0);
    std::vector<char> in(N, 0);
    for (int s : T.samples) in[s] = 1;
    // layout: tile samples in ascending order, each at a TILE_ALIGN boundary;
    // d_ascii holds exactly that layout when the tile is every resident sample.
    // A split tile's b part starts at T.bstart (after the a part's padding)
    uint64_t pos = 0;
    bool direct = T.bchunk < 0;
    int amax_s = -1;
    if (T.bchunk >= 0)
        for (auto &pr : T.pairs) amax_s = std::max(amax_s, pr.first);
    for (int s = 0; s < N; s++) {
        if (!in[s]) continue;
        if (T.bchunk >= 0 && s > amax_s && pos < T.bstart) pos = T.bstart;
        e->tile_pos[s] = pos;
        direct = direct && e->samples[s].abase == pos;
        pos += align_up(e->samples[s].nbases);
    }
    for (int s = 0; s < N; s++)
        if (e->samples[s].resident && e->samples[s].nbases && !in[s]) direct = false;
    const uint64_t total = pos;
    if (total >= (1ull << 32)) return fail(RC_E_LIMIT, "a tile of more than 2^32 bases");
    e->tile_total = total;
    e->tile_direct = direct;
    // the 16-mer index holds the tile's subject samples only: the b of each
    // pair (shared searches and spec 5b: query = the lower sample), or both
    const bool share = share_mode(e);
    if (e->tile_loaded == ti && e->tile_share == share) return RC_OK;
    std::vector<char> subj(N, 0);
    for (auto &pr : T.pairs) {
        subj[pr.second] = 1;
        if (!share && !e->o.symmetric) subj[pr.first] = 1;
    }
    // Per tile sample one TileSeg; the device builds every per-transcript and
    // per-base table from them (launch_tile_tables): transcript starts in the
    // tile, the tile's transcripts and the index's with their closed-form
    // k-mer slots, the transcript-start bits and the position -> transcript
    // blocks. The host keeps O(samples) bookkeeping only.
    auto &segs = e->h_segs;
    auto &spos = e->h_spos;   // sample ranges, monotone over all N + 1 (a sample outside the tile is empty)
    auto &send = e->h_send;   // one past each tile sample's padded range (0: not in the tile)
    segs.clear();
    spos.assign(N + 1, total);
    send.assign(N, 0);
    {
        uint64_t next = total;
        for (int s = N; s >= 0; s--) {
            if (s < N && in[s]) next = e->tile_pos[s];
            spos[s] = next;
        }
    }
    uint32_t n_ttx = 0, n_itx = 0;
    uint64_t npos = 0;
    e->tile_tx_first.assign(N + 1, 0);
    for (int s = 0; s < N; s++) {
        e->tile_tx_first[s] = n_ttx;
        if (!in[s]) continue;
        const SampleRec &S = e->samples[s];
        send[s] = e->tile_pos[s] + align_up(S.nbases);
        if (!S.n_tx) continue;
        TileSeg g;
        g.pos = e->tile_pos[s];
        g.kbase = npos;
        g.pad_bit = S.nbases < align_up(S.nbases) ? e->tile_pos[s] + S.nbases : ~0ull;
        g.tx0 = S.tx_begin;
        g.ntx = S.n_tx;
        g.ttx0 = n_ttx;
        g.itx0 = subj[s] ? n_itx : ~0u;
        segs.push_back(g);
        n_ttx += S.n_tx;
        if (subj[s]) {
            n_itx += S.n_tx;
            npos += e->sample_kmers[s];
        }
    }
    e->tile_tx_first[N] = n_ttx;
    if (npos > 0xFFFFFFFFull) return fail(RC_E_LIMIT, "more than 2^32 seed positions in a tile");
    const uint64_t nblocks = (total >> POS_TX_SHIFT) + 2, nwb = (total >> 6) + 4;
    CHK(e->d_tile_segs.ensure(std::max<size_t>(segs.size(), 1)));
    CHK(e->d_tile_tx.ensure(std::max<uint32_t>(n_ttx, 1)));
    CHK(e->d_tile_gid.ensure(std::max<uint32_t>(n_ttx, 1)));
    CHK(e->d_tile_itx.ensure(std::max<uint32_t>(n_itx, 1)));
    CHK(e->d_kpos_off.ensure((size_t)n_itx + 1));
    CHK(e->d_pos_tx.ensure(nblocks));
    CHK(e->d_sample_pos.ensure(spos.size()));
    CHK(e->d_tile_send.ensure(send.size()));
    CHK(e->d_txstart.ensure(nwb));
    if (!segs.empty())
        HIPCHK(hipMemcpyAsync(e->d_tile_segs.p, segs.data(), segs.size() * sizeof(TileSeg), hipMemcpyHostToDevice, e->st));
    HIPCHK(hipMemcpyAsync(e->d_sample_pos.p, spos.data(), spos.size() * 8, hipMemcpyHostToDevice, e->st));
    HIPCHK(hipMemcpyAsync(e->d_tile_send.p, send.data(), send.size() * 8, hipMemcpyHostToDevice, e->st));
    HIPCHK(hipMemsetAsync(e->d_txstart.p, 0, nwb * 8, e->st));
    launch_tile_tables(e->d_tile_segs.p, (uint32_t)segs.size(), n_ttx, e->d_tx_rel.p, e->d_kpre.p, e->d_tx.p,
                       e->d_tile_tx.p, e->d_tile_gid.p, e->d_tile_itx.p, e->d_kpos_off.p, n_itx, npos,
                       e->d_txstart.p, e->d_giso.p, e->gene_tx.size(), e->d_tile_send.p, e->d_pos_tx.p, nblocks,
                       e->st);
    HIPCHK(hipGetLastError());
    e->tile_npos = npos;
    e->tile_ntx = n_ttx;
    e->tile_nitx = n_itx;
    e->tile_share = share;
    // the packed working copy's source: d_ascii itself or a gathered copy
    if (!direct) {
        CHK(e->d_tile_ascii.ensure(total + 64));
        HIPCHK(hipMemsetAsync(e->d_tile_ascii.p, 'A', total + 64, e->st));
        for (int s = 0; s < N; s++)
            if (in[s] && e->samples[s].nbases)
                HIPCHK(hipMemcpyAsync(e->d_tile_ascii.p + e->tile_pos[s], e->d_ascii.p + e->samples[s].abase,
                                      e->samples[s].nbases, hipMemcpyDeviceToDevice, e->st));
    }
    // (no wait: the host tables above are engine members, kept until the
    // next load, which comes after this tile's last wait)
    e->tile_loaded = ti;
    return RC_OK;
}

// Sort index entries ent[0, npos) on key bits [bb, 64) into ent2 and build the
// bucket table over the top k-mer bits: about one bucket per entry (times
// 2^extra), at most 2^28 (RC_INDEX_BITS_MAX; 28 measured best at C3 -- a 1 GiB
// table instead of 4 GiB, same seed-kernel time)
// the first pass's key generator (sort.hip KeyGen): keys from the packed
// sequence instead of the fill's entry array
struct GenArgs {
    const TxInfo *tx;
    const uint64_t *koff;
    const uint64_t *F;
    uint32_t n_tx;
};
static int sort_index(rc_engine *e, DBuf<uint64_t> &ent, DBuf<uint64_t> &ent2, uint64_t npos, unsigned bb, int extra,
                      DBuf<uint32_t> &bucket, int &bits_out, const std::function<int()> &after_prep = nullptr,
                      bool counted = false, const GenArgs *gen = nullptr)
{
    static const bool lib = getenv("RC_SORT") && !strcmp(getenv("RC_SORT"), "rocprim");
    bool prepped = false;   // after_prep runs exactly once, also for an empty index
    if (lib) {   // A/B only: rocPRIM's onesweep
        // (rocPRIM sorts up to 2^20 items with a merge sort that did not keep
        // the input order for a partial bit range: there, all 64 bits -- the
        // same result, positions are unique)
        const unsigned lb = bb == 32 && npos <= (1ull << 20) ? 0u : bb;
        prepped = true;
        if (after_prep) CHK(after_prep());
        size_t tmp = 0;
        HIPCHK(rocprim::radix_sort_keys(nullptr, tmp, ent.p, ent2.p, (size_t)npos, lb, 64u, e->st));
        CHK(e->d_tmp.ensure(tmp));
        HIPCHK(rocprim::radix_sort_keys(e->d_tmp.p, tmp, ent.p, ent2.p, (size_t)npos, lb, 64u, e->st));
    } else if (npos) {
        // sort.hip: 8-bit LSD passes ping-ponging between the two buffers;
        // the result must end in ent2
        if (npos > 0xFFFFFFFFull) return fail(RC_E_LIMIT, "more than 2^32 index entries");
        CHK(e->d_sort_scratch.ensure(os_scratch_words(npos)));
        const uint64_t words = os_status_words(npos);
        if (e->d_sort_status.cap < words) {
            CHK(e->d_sort_status.ensure(words));
            HIPCHK(hipMemsetAsync(e->d_sort_status.p, 0, words * sizeof(uint64_t), e->st));
        }
        int prc = RC_OK;
        if (gen) CHK(e->d_gen_tile.ensure(os_gen_tile_words(npos)));
        const bool in_alt = os_sort_keys(ent.p, ent2.p, npos, (int)bb, e->d_sort_scratch.p, e->d_sort_status.p,
                                         e->sort_epoch, e->st, [&]() {
                                             prepped = true;
                                             if (after_prep) prc = after_prep();
                                         }, counted, gen ? gen->tx : nullptr, gen ? gen->koff : nullptr,
                                         gen ? gen->F : nullptr, gen ? gen->n_tx : 0u,
                                         gen ? e->d_gen_tile.p : nullptr);
        CHK(prc);
        HIPCHK(hipGetLastError());
        if (!in_alt) {
            std::swap(ent.p, ent2.p);
            std::swap(ent.cap, ent2.cap);
        }
    }
    if (!prepped && after_prep) CHK(after_prep());
    const char *ibv = getenv("RC_INDEX_BITS_MAX");
    const int bmax = ibv ? std::max(16, std::min(30, atoi(ibv))) : 28;
    int bits = 16;
    while (bits < bmax && (1ull << bits) < (npos << extra)) bits++;
    bits_out = bits;
    CHK(bucket.ensure((1ull << bits) + 1));
    launch_bucket_fill(ent2.p, npos, bits, bucket.p, e->st);
    return RC_OK;
}

// A seed index: every 16-mer position of the transcripts txl[0, n_tx), whose
// slots koff / kpos (closed form when no base is ambiguous) give the order.
static int build_index_of(rc_engine *e, const TxInfo *txl, uint32_t n_tx, uint64_t npos, const uint64_t *kpos,
                          DBuf<uint64_t> &ent, DBuf<uint64_t> &ent2, DBuf<uint32_t> &bucket, int &bits_out,
                          uint64_t &n_out, const std::function<int()> &after_fill = nullptr)
{
    const bool amb = e->has_amb;
    const uint64_t *offs = kpos;
    if (amb) {
        CHK(e->d_kcnt.ensure(n_tx + 1));
        HIPCHK(hipMemsetAsync(e->d_kcnt.p, 0, (n_tx + 1) * sizeof(uint64_t), e->st));
        if (n_tx) launch_kmer_count(txl, n_tx, e->d_AF.p + FRONT_PAD, e->d_kcnt.p, e->st);
        size_t tmp = 0;
        CHK(e->d_kpos_rel.ensure(n_tx + 1));
        HIPCHK(rocprim::exclusive_scan(nullptr, tmp, e->d_kcnt.p, e->d_kpos_rel.p, (uint64_t)0, (size_t)n_tx + 1,
                                       rocprim::plus<uint64_t>(), e->st));
        CHK(e->d_tmp.ensure(tmp));
        HIPCHK(rocprim::exclusive_scan(e->d_tmp.p, tmp, e->d_kcnt.p, e->d_kpos_rel.p, (uint64_t)0,
                                       (size_t)n_tx + 1, rocprim::plus<uint64_t>(), e->st));
        HIPCHK(hipMemcpyAsync(&npos, e->d_kpos_rel.p + n_tx, sizeof(uint64_t), hipMemcpyDeviceToHost, e->st));
        CHK(wait_st(e));
        offs = e->d_kpos_rel.p;
    }
    CHK(ent.ensure(std::max<uint64_t>(npos, 1)));
    CHK(ent2.ensure(std::max<uint64_t>(npos, 1)));
    // without ambiguity codes the fill also counts the sort's segment
    // histograms (sort.hip), so the sort does not read the keys to count them
    static const bool lib = getenv("RC_SORT") && !strcmp(getenv("RC_SORT"), "rocprim");
    const bool counted = !amb && !lib && npos > 0 && npos <= 0xFFFFFFFFull;
    // RC_GEN=1: the sort's first pass computes the keys from the sequence
    // instead of reading the entry array the fill writes (measured slower:
    // index phase 61.1 vs 57.9 ms at C3 -- the per-key transcript search and
    // sequence windows cost more than the 25.6 GB of traffic they save)
    static const bool genv = getenv("RC_GEN") && atoi(getenv("RC_GEN")) == 1;
    const bool gen = counted && genv && n_tx;
    const GenArgs ga{txl, offs, e->d_F.p + FRONT_PAD, n_tx};
    if (counted) {
        CHK(e->d_sort_scratch.ensure(os_scratch_words(npos)));
        os_fill_hist(txl, n_tx, e->d_F.p + FRONT_PAD, offs, gen ? nullptr : ent.p, npos, e->d_sort_scratch.p, e->st);
    } else if (n_tx) {
        launch_kmer_fill(amb, txl, n_tx, e->d_F.p + FRONT_PAD, amb ? e->d_AF.p + FRONT_PAD : nullptr, offs, ent.p,
                         e->st);
    }
    // sort on the k-mer (bits 32..63); the fill order is position order and the
    // radix sort is stable, so positions stay ascending per k-mer. after_fill
    // (DUST on the second stream) starts once the sort's one-block table
    // kernels are queued: beside DUST's waves they crawled (4.2 ms vs 14 us).
    CHK(sort_index(e, ent, ent2, npos, 32u, 0, bucket, bits_out, after_fill, counted, gen ? &ga : nullptr));
    n_out = npos;
    return RC_OK;
}

// The seed index of the loaded tile: every 16-mer position of its subject samples' transcripts.
static int build_index(rc_engine *e, const std::function<int()> &after_fill = nullptr)
{
    return build_index_of(e, e->d_tile_itx.p, e->tile_nitx, e->tile_npos, e->d_kpos_off.p, e->d_ent,
                          e->d_ent2, e->d_bucket, e->index_bits, e->n_index, after_fill);
}

// Shared searches with DUST: the reverse pass's index. A reverse search whose
// SUBJECT a holds a masked base may have seeds the forward pass does not find
// (runs none of whose aligned words of a is usable); every 16-mer of such a
// run has a masked base of a nearby, so the index holds only the positions of
// masked transcripts with a masked base in [pos - 12, pos + 28)
// (near_fill_kernel), sorted on all 64 key bits, with 4 buckets per entry.
static int build_masked_index(rc_engine *e)
{
    const uint32_t n = e->tile_ntx;
    CHK(e->d_tile_masked.ensure(std::max<uint32_t>(n, 1)));
    launch_tx_masked(e->d_tile_tx.p, n, e->d_dmask.p + 1, e->d_tile_masked.p, e->st);
    HIPCHK(hipGetLastError());
    CHK(e->d_rctr.ensure(4));
    if (!e->mnear_cap) e->mnear_cap = e->tile_total / 32 + (1u << 20);
    unsigned long long cnt = 0;
    for (;;) {
        CHK(e->d_ment.ensure(e->mnear_cap));
        CHK(e->d_ment2.ensure(e->mnear_cap));
        HIPCHK(hipMemsetAsync(e->d_rctr.p, 0, sizeof(unsigned long long), e->st));
        launch_near_fill(e->has_amb, e->d_tile_tx.p, n, e->d_tile_masked.p, e->d_F.p + FRONT_PAD,
                         e->has_amb ? e->d_AF.p + FRONT_PAD : nullptr, e->d_dmask.p + 1, e->d_ment.p, e->mnear_cap,
                         e->d_rctr.p, e->st);
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(&cnt, e->d_rctr.p, sizeof cnt, hipMemcpyDeviceToHost, e->st));
        CHK(wait_st(e));
        if (cnt <= e->mnear_cap) break;
        e->mnear_cap = cnt + cnt / 4 + (1u << 20);
    }
    CHK(sort_index(e, e->d_ment, e->d_ment2, cnt, 0u, 2, e->d_mbucket, e->mindex_bits));
    e->n_mindex = cnt;
    e->tm.near_index += (double)cnt;
    return RC_OK;
}

// Genes of [g0, g1) with more than ISO_LDS isoforms (the seed kernel's ISOG
// launch), appended to `list`; returns their count
static uint32_t iso_genes(const rc_engine *e, uint32_t g0, uint32_t g1, std::vector<uint32_t> &list)
{
    uint32_t n = 0;
    for (uint32_t g = g0; g < g1; g++)
        if (e->gene_tx_off[g + 1] - e->gene_tx_off[g] > (uint32_t)ISO_LDS) {
            list.push_back(g);
            n++;
        }
    return n;
}

static Db make_db(rc_engine *e)
{
    Db db;
    db.F = e->d_F.p + FRONT_PAD;
    db.RC = e->d_RC.p + FRONT_PAD;
    db.AF = e->has_amb ? e->d_AF.p + FRONT_PAD : nullptr;
    db.ARC = e->has_amb ? e->d_ARC.p + FRONT_PAD : nullptr;
    db.total = e->tile_total;
    db.tx = e->d_tx.p;
    db.tx_gene = e->d_tx_gene.p;
    db.gene_tx_off = e->d_gene_tx_off.p;
    db.gene_tx = e->d_gene_tx.p;
    db.giso = e->d_giso.p;
    db.gene_sample = e->d_gene_sample.p;
    db.sample_gene_begin = e->d_sample_gene_begin.p;
    db.sample_tx_begin = e->d_sample_tx_begin.p;
    db.sample_pos_begin = e->d_sample_pos.p;
    db.txstart = e->d_txstart.p + 1;
    db.dmask = e->o.dust_level > 0 ? e->d_dmask.p + 1 : nullptr;
    db.n_samples = (int32_t)e->samples.size();
    return db;
}

static void shard_pairs(rc_engine *e)
{
    e->pair0 = (uint64_t)e->shard_first[e->o.shard_rank];
    e->pair1 = (uint64_t)e->shard_first[e->o.shard_rank + 1];
    e->item0 = e->pair_item_begin[e->pair0];
    e->item1 = e->pair_item_begin[e->pair1];
}

// The directed searches of tile ti: per query sample the bit set of its
// subject samples (spec 5b: only a -> b of a pair), and the runs of
// consecutive query samples (one seed launch each: their genes are contiguous).
// Subject-sample bit rows (tmw words per query sample) and the range of
// each row's set bits ([first, one past last), empty N, 0).
static int mask_words(int N) { return (N + 63) / 64; }
static void mask_ranges(const std::vector<uint64_t> &mask, int N, std::vector<int32_t> &range)
{
    const int tw = mask_words(N);
    range.assign((size_t)2 * N, 0);
    for (int q = 0; q < N; q++) {
        int lo = N, hi = 0;
        for (int w = 0; w < tw; w++) {
            const uint64_t m = mask[(size_t)q * tw + w];
            if (!m) continue;
            lo = std::min(lo, 64 * w + __builtin_ctzll(m));
            hi = std::max(hi, 64 * w + 64 - __builtin_clzll(m));
        }
        range[2 * q] = lo;
        range[2 * q + 1] = hi;
    }
}

static void tile_plan(rc_engine *e, int ti, std::vector<uint64_t> &tmask, std::vector<std::pair<int, int>> &runs)
{
    const int N = (int)e->samples.size(), tw = mask_words(N);
    tmask.assign((size_t)tw * N, 0);
    std::vector<char> q(N, 0);
    for (auto &pr : e->tiles[ti].pairs) {
        const int a = pr.first, b = pr.second;
        tmask[(size_t)tw * a + (b >> 6)] |= 1ull << (b & 63);
        q[a] = 1;
        if (!e->o.symmetric && !e->share) {   // the pair's second directed search: query b, subject a
            tmask[(size_t)tw * b + (a >> 6)] |= 1ull << (a & 63);
            q[b] = 1;
        }
    }
    runs.clear();
    for (int s = 0; s < N;) {
        if (!q[s]) {
            s++;
            continue;
        }
        int t = s;
        while (t < N && q[t]) t++;
        runs.push_back({s, t});
        s = t;
    }
}

// The reverse pass of shared searches with DUST: queries = the
// higher sample of each pair of tile ti, subjects = the near-mask index ixm.
// It keeps only the reverse-search runs the forward pass cannot see, as SEED_R
// seeds in forward-candidate coordinates; they are sorted by the forward
// query's gene (rs_key, rs_idx) for the forward pass to merge. n_rs = count.
static int reverse_pass(rc_engine *e, int ti, const Db &db, const Index &ixm, uint32_t &n_rs)
{
    const int N = (int)e->samples.size(), tw = mask_words(N);
    std::vector<uint64_t> rmask((size_t)tw * N, 0);
    std::vector<char> q(N, 0);
    for (auto &pr : e->tiles[ti].pairs) {
        rmask[(size_t)tw * pr.second + (pr.first >> 6)] |= 1ull << (pr.first & 63);
        q[pr.second] = 1;
    }
    std::vector<std::pair<int, int>> runs;
    for (int s0 = 0; s0 < N;) {
        if (!q[s0]) {
            s0++;
            continue;
        }
        int t = s0;
        while (t < N && q[t]) t++;
        runs.push_back({s0, t});
        s0 = t;
    }
    std::vector<int32_t> rrange;
    mask_ranges(rmask, N, rrange);
    CHK(e->d_rtmask.ensure(rmask.size()));
    CHK(e->d_rtrange.ensure(rrange.size()));
    HIPCHK(hipMemcpyAsync(e->d_rtmask.p, rmask.data(), rmask.size() * 8, hipMemcpyHostToDevice, e->st));
    HIPCHK(hipMemcpyAsync(e->d_rtrange.p, rrange.data(), rrange.size() * 4, hipMemcpyHostToDevice, e->st));
    std::vector<uint32_t> ilist, ioff(1, 0);
    for (auto &r : runs) ioff.push_back(ioff.back() + iso_genes(e, e->sample_gene_begin[r.first],
                                                                 e->sample_gene_begin[r.second], ilist));
    CHK(e->d_iso_list_r.ensure(std::max<size_t>(ilist.size(), 1)));
    if (!ilist.empty())
        HIPCHK(hipMemcpyAsync(e->d_iso_list_r.p, ilist.data(), ilist.size() * 4, hipMemcpyHostToDevice, e->st));
    CHK(e->d_rctr.ensure(4));
    CHK(e->d_big_out.ensure(std::max<uint64_t>(e->big_list_cap, 1)));
    if (!e->rseed_cap) e->rseed_cap = 1u << 20;
    unsigned long long cnt = 0;
    for (;;) {
        CHK(e->d_rseeds.ensure(e->rseed_cap));
        CHK(e->d_rseed_gene.ensure(e->rseed_cap));
        HIPCHK(hipMemsetAsync(e->d_rctr.p + 1, 0, 2 * sizeof(unsigned long long), e->st));
        HIPCHK(hipMemsetAsync(e->d_status.p, 0, 4 * sizeof(unsigned int), e->st));
        for (size_t ri = 0; ri < runs.size(); ri++) {
            const auto &r = runs[ri];
            SeedParams S{};
            S.iso_list = e->d_iso_list_r.p + ioff[ri];
            S.iso_n = ioff[ri + 1] - ioff[ri];
            S.word = e->o.word_size;
            S.stride = e->o.word_size - W16 + 1;
            const char *pm = getenv("RC_SEED_PRE");
            S.pre_mode = pm ? atoi(pm) : 1;
            S.rev = 1;
            S.tx_pos = e->d_tx_pos.p;
            S.iso_pre_g = e->d_iso_pre.p;
            S.rseeds = e->d_rseeds.p;
            S.rseed_gene = e->d_rseed_gene.p;
            S.rseed_cap = e->rseed_cap;
            S.rseed_n = e->d_rctr.p + 1;
            S.gene_begin = e->sample_gene_begin[r.first];
            S.gene_end = e->sample_gene_begin[r.second];
            S.tmask = e->d_rtmask.p;
            S.tmw = tw;
            S.trange = e->d_rtrange.p;
            S.xbits = e->xbits;
            S.max_iso = max_iso(e->xbits);
            S.status = e->d_status.p;
            S.big_out = e->d_big_out.p;   // (never used: the pass keeps no seeds of its own)
            S.big_n = e->d_rctr.p + 2;
            S.big_list_cap = 0;
            launch_seed(e->has_amb, db, ixm, S, e->st);
            HIPCHK(hipGetLastError());
        }
        unsigned int status = 0;
        HIPCHK(hipMemcpyAsync(&cnt, e->d_rctr.p + 1, sizeof cnt, hipMemcpyDeviceToHost, e->st));
        HIPCHK(hipMemcpyAsync(&status, e->d_status.p, sizeof status, hipMemcpyDeviceToHost, e->st));
        CHK(wait_st(e));
        if (status & 2u)
            return fail(RC_E_LIMIT, "a query gene has more than " + std::to_string(max_iso(e->xbits)) + " isoforms");
        if (cnt <= e->rseed_cap) break;
        e->rseed_cap = cnt + cnt / 4 + 1024;
    }
    if (cnt > 0xFFFFFFFFull) return fail(RC_E_LIMIT, "more than 2^32 reverse-only seeds in a tile");
    n_rs = (uint32_t)cnt;
    e->n_rseeds += cnt;
    e->tm.reverse_seeds += (double)cnt;
    if (cnt) {
        CHK(e->d_rs_key.ensure(cnt));
        CHK(e->d_rs_idx.ensure(cnt));
        size_t tmp = 0;
        rocprim::counting_iterator<uint32_t> iota(0u);
        HIPCHK(rocprim::radix_sort_pairs(nullptr, tmp, e->d_rseed_gene.p, e->d_rs_key.p, iota, e->d_rs_idx.p,
                                         (size_t)cnt, 0u, 32u, e->st));
        CHK(e->d_tmp.ensure(tmp));
        HIPCHK(rocprim::radix_sort_pairs(e->d_tmp.p, tmp, e->d_rseed_gene.p, e->d_rs_key.p, iota, e->d_rs_idx.p,
                                         (size_t)cnt, 0u, 32u, e->st));
    }
    return RC_OK;
}

static int load_external(rc_engine *e)
{
    const int N = (int)e->samples.size();
    const uint32_t n_genes = (uint32_t)e->gene_sample.size();
    std::vector<std::vector<DHsp>> grp((size_t)n_genes * N);
    for (auto &kv : e->ext) {
        const int q = kv.first.first, s = kv.first.second;
        for (const rc_hsp &h : kv.second) {
            DHsp d;
            d.q_tx = e->samples[q].tx_begin + h.q_tx;
            d.s_tx = e->samples[s].tx_begin + h.s_tx;
            d.qstart = h.qstart; d.qend = h.qend; d.sstart = h.sstart; d.send = h.send;
            d.length = h.length; d.nident = h.nident; d.mismatch = h.mismatch; d.gaps = h.gaps;
            d.gapopen = h.gapopen; d.score_half = h.score_half; d.bits10 = h.bits10; d.strand = h.strand;
            grp[grp_index(e->tx_gene[d.q_tx], s, n_genes)].push_back(d);
        }
    }
    std::vector<DHsp> all;
    std::vector<uint32_t> off(grp.size()), cnt(grp.size());
    for (size_t i = 0; i < grp.size(); i++) {
        off[i] = (uint32_t)all.size();
        cnt[i] = (uint32_t)grp[i].size();
        all.insert(all.end(), grp[i].begin(), grp[i].end());
    }
    CHK(e->d_hsp.ensure(all.size()));
    CHK(e->d_grp_off.ensure(off.size()));
    CHK(e->d_grp_cnt.ensure(cnt.size()));
    if (!all.empty()) HIPCHK(hipMemcpyAsync(e->d_hsp.p, all.data(), all.size() * sizeof(DHsp), hipMemcpyHostToDevice, e->st));
    HIPCHK(hipMemcpyAsync(e->d_grp_off.p, off.data(), off.size() * 4, hipMemcpyHostToDevice, e->st));
    HIPCHK(hipMemcpyAsync(e->d_grp_cnt.p, cnt.data(), cnt.size() * 4, hipMemcpyHostToDevice, e->st));
    HIPCHK(hipStreamSynchronize(e->st));
    e->n_hsps = all.size();
    return RC_OK;
}

// d_hsp grows across tiles with its contents kept
static int grow_hsp(rc_engine *e, uint64_t n)
{
    if (n <= e->d_hsp.cap && e->d_hsp.p) return RC_OK;
    const size_t cap = std::max<size_t>(n, e->d_hsp.cap + e->d_hsp.cap / 2);
    DHsp *np = nullptr;
    if (hipMalloc((void **)&np, cap * sizeof(DHsp)) != hipSuccess) {
        (void)hipGetLastError();
        return fail(RC_E_NOMEM, "hipMalloc of " + std::to_string(cap * sizeof(DHsp)) + " bytes failed");
    }
    if (e->hsp_used) HIPCHK(hipMemcpyAsync(np, e->d_hsp.p, e->hsp_used * sizeof(DHsp), hipMemcpyDeviceToDevice, e->st));
    CHK(wait_st(e));
    e->d_hsp.adopt(np, cap);
    return RC_OK;
}

// One alignment pass over tile ti: pack, DUST, index, seeds (one launch per
// run of query samples), extension, and the (query gene, subject sample) HSP
// groups appended to the shard's store.
// The loaded tile's packed working copy (FRONT_PAD zero words in front, zero
// words behind); ev[0] marks the start of the packing.
static int pack_tile(rc_engine *e)
{
    const uint64_t total = e->tile_total;
    const uint64_t nwords = (total + 31) / 32 + 2;
    CHK(e->d_F.ensure(nwords + 4 + FRONT_PAD));
    CHK(e->d_RC.ensure(nwords + 4 + FRONT_PAD));
    HIPCHK(hipMemsetAsync(e->d_F.p, 0, FRONT_PAD * 8, e->st));
    HIPCHK(hipMemsetAsync(e->d_RC.p, 0, FRONT_PAD * 8, e->st));
    HIPCHK(hipMemsetAsync(e->d_F.p + FRONT_PAD + nwords, 0, 4 * 8, e->st));
    HIPCHK(hipMemsetAsync(e->d_RC.p + FRONT_PAD + nwords, 0, 4 * 8, e->st));
    if (e->has_amb) {
        CHK(e->d_AF.ensure(nwords + 4 + FRONT_PAD));
        CHK(e->d_ARC.ensure(nwords + 4 + FRONT_PAD));
        HIPCHK(hipMemsetAsync(e->d_AF.p, 0, (nwords + 4 + FRONT_PAD) * 8, e->st));
        HIPCHK(hipMemsetAsync(e->d_ARC.p, 0, (nwords + 4 + FRONT_PAD) * 8, e->st));
    }
    HIPCHK(hipEventRecord(e->ev[0], e->st));
    launch_pack(e->tile_direct ? e->d_ascii.p : e->d_tile_ascii.p, total, nwords, e->d_F.p + FRONT_PAD,
                e->d_RC.p + FRONT_PAD, e->has_amb ? e->d_AF.p + FRONT_PAD : nullptr,
                e->has_amb ? e->d_ARC.p + FRONT_PAD : nullptr, e->st);
    HIPCHK(hipGetLastError());
    return RC_OK;
}

// DUST masks of the given tile samples (ascending) into d_dmask, on stream st:
// one launch per run of consecutive samples (the transcripts' ranges only,
// not the padding between a split tile's parts)
static int dust_samples(rc_engine *e, const std::vector<int> &ss, hipStream_t st)
{
    const uint32_t dblocks = 256 * 28;   // at least the resident waves of the chunk kernel (<= 7 per SIMD): their scratch
    CHK(e->d_dust_scratch.ensure(dust_scratch_words(dblocks)));
    CHK(e->d_dust_events.ensure(dust_event_words(dblocks)));
    const char *dwv = getenv("RC_DUST_WAVES");
    const int dwaves = dwv ? atoi(dwv) : 0;   // 0: every resident wave (measured best; 1-3 starve DUST)
    int f = -1, l = -1;
    auto flush = [&]() {
        if (f >= 0) {
            const uint32_t tx0 = e->tile_tx_first[f];
            launch_dust(e->has_amb, e->tile_pos[f], e->tile_pos[l] + align_up(e->samples[l].nbases),
                        e->d_F.p + FRONT_PAD, e->has_amb ? e->d_AF.p + FRONT_PAD : nullptr, e->d_txstart.p + 1,
                        e->d_tile_tx.p + tx0, e->tile_tx_first[l + 1] - tx0, e->o.dust_level, e->o.dust_window,
                        e->o.dust_linker, e->d_dust_scratch.p, e->d_dust_events.p, dblocks, dwaves,
                        e->d_dmask.p + 1, st);
        }
        f = l = -1;
    };
    for (int s : ss) {
        if (f >= 0 && e->tile_pos[s] != e->tile_pos[l] + align_up(e->samples[l].nbases)) flush();
        if (f < 0) f = s;
        l = s;
    }
    flush();
    HIPCHK(hipGetLastError());
    return RC_OK;
}

static int align_tile(rc_engine *e, int ti)
{
    {
        const double t0 = wall_ms();
        CHK(load_tile(e, ti));
        e->tm.load_ms += wall_ms() - t0;
    }
    const int N = (int)e->samples.size();
    const uint64_t total = e->tile_total;
    const uint32_t n_genes = (uint32_t)e->gene_sample.size();
    CHK(pack_tile(e));
    const bool dust = e->o.dust_level > 0;
    // a split tile of the b chunk the previous tile had: its 16-mer index
    // (the b part's) and the b part's DUST masks are on the device already
    const rc_engine::Tile &TT = e->tiles[ti];
    // (only while the index holds the b part alone: with one directed search
    // at a time -- RC_SHARE=0, not spec 5b -- it holds the a part's samples
    // too, and they differ from tile to tile)
    const bool b_only_index = share_mode(e) || e->o.symmetric;
    const bool reuse = b_only_index && TT.bchunk >= 0 && TT.bchunk == e->idx_bchunk && TT.bstart == e->idx_bstart &&
                       e->d_dmask.cap >= (total >> 6) + 4;
    const uint64_t dtot = reuse ? TT.bstart : total;   // masks cleared: the a part only when reusing
    // the samples whose masks DUST computes here, in tile order: a split
    // tile's a part and (unless its masks are kept) its b part, all samples
    // of any other tile -- except those given by rc_set_dust_masks, whose
    // masks are copied in (samples start at 256-base boundaries: whole words)
    std::vector<int> dust_here;
    e->dmask_only.clear();   // every sample of this tile gets its mask
    if (dust) {
        const size_t mw = (total >> 6) + 4;
        CHK(e->d_dmask.ensure(mw));
        HIPCHK(hipMemsetAsync(e->d_dmask.p, 0, (reuse ? 1 + (dtot >> 6) : mw) * 8, e->st));
        for (int s : TT.samples) {
            if (reuse && e->tile_pos[s] >= TT.bstart) continue;
            const uint64_t io = s < (int)e->dust_imp_off.size() ? e->dust_imp_off[s] : ~0ull;
            if (io == ~0ull) {
                dust_here.push_back(s);
            } else if (e->samples[s].nbases) {
                HIPCHK(hipMemcpyAsync(e->d_dmask.p + 1 + (e->tile_pos[s] >> 6), e->d_dust_imp.p + io,
                                      ((e->samples[s].nbases + 63) >> 6) * 8, hipMemcpyDeviceToDevice, e->st));
            }
        }
    }
    HIPCHK(hipEventRecord(e->ev[1], e->st));
    // DUST masks of the tile's transcripts (the query side), bit per base, on
    // the second stream: a compute-bound scan beside the HBM-bound index
    // build, started with the fill (r03, hand-written sort and DUST: index
    // phase 55.7 vs 58.1 ms at C3 when started after the sort's table kernels;
    // RC_DUST_EARLY=0 starts it there).
    auto start_dust = [&]() -> int {
        HIPCHK(hipEventRecord(e->evd[2], e->st));
        HIPCHK(hipStreamWaitEvent(e->st2, e->evd[2], 0));
        HIPCHK(hipEventRecord(e->evd[0], e->st2));
        CHK(dust_samples(e, dust_here, e->st2));
        HIPCHK(hipEventRecord(e->evd[1], e->st2));
        return RC_OK;
    };
    const char *dev = getenv("RC_DUST_EARLY");
    const int dmode = dev ? atoi(dev) : 1;   // 1: beside the fill (default), 0: after the sort's table kernels, 2: before the index
    const bool dust_early = dmode != 0;
    if (dust && dmode == 2) {
        // DUST alone on the engine's stream, then the index build alone
        HIPCHK(hipEventRecord(e->evd[0], e->st));
        CHK(dust_samples(e, dust_here, e->st));
        HIPCHK(hipEventRecord(e->evd[1], e->st));
    } else if (dust && dust_early) {
        CHK(start_dust());
    }
    if (reuse) {
        if (dust && !dust_early) CHK(start_dust());
        e->tm.index_reused += 1.0;
    } else {
        CHK(build_index(e, dust && !dust_early ? std::function<int()>(start_dust) : nullptr));
    }
    e->idx_bchunk = TT.bchunk;
    e->idx_bstart = TT.bstart;
    HIPCHK(hipGetLastError());
    if (dust) HIPCHK(hipStreamWaitEvent(e->st, e->evd[1], 0));
    e->share = share_mode(e);   // (load_tile built the index list for it)
    // shared searches with DUST: reverse-search runs with no usable word of
    // the forward query inside come from a reverse pass over a near-mask index
    const bool revpass = e->share && dust;
    if (revpass) CHK(build_masked_index(e));
    HIPCHK(hipEventRecord(e->ev[2], e->st));

    std::vector<uint64_t> tmask;
    std::vector<std::pair<int, int>> runs;
    tile_plan(e, ti, tmask, runs);
    const size_t R = runs.size(), RT = R;
    const int tw = mask_words(N);
    std::vector<int32_t> trange;
    mask_ranges(tmask, N, trange);
    CHK(e->d_tmask.ensure(tmask.size()));
    CHK(e->d_trange.ensure(trange.size()));
    HIPCHK(hipMemcpyAsync(e->d_tmask.p, tmask.data(), tmask.size() * 8, hipMemcpyHostToDevice, e->st));
    HIPCHK(hipMemcpyAsync(e->d_trange.p, trange.data(), trange.size() * 4, hipMemcpyHostToDevice, e->st));
    // per run: its genes [g0, g1) and its slice of the (gene, sample) arrays
    std::vector<uint32_t> rg0(RT), rg1(RT);
    std::vector<uint32_t> ilist, ioff(1, 0);
    std::vector<size_t> gcb(RT + 1, 0), cnb(R + 1, 0);
    for (size_t r = 0; r < RT; r++) {
        rg0[r] = e->sample_gene_begin[runs[r].first];
        rg1[r] = e->sample_gene_begin[runs[r].second];
        gcb[r + 1] = gcb[r] + (size_t)(rg1[r] - rg0[r]) * N;
        if (r < R) cnb[r + 1] = cnb[r] + (size_t)(rg1[r] - rg0[r]) * N + 1;
        ioff.push_back(ioff.back() + iso_genes(e, rg0[r], rg1[r], ilist));
    }
    CHK(e->d_iso_list.ensure(std::max<size_t>(ilist.size(), 1)));
    if (!ilist.empty())
        HIPCHK(hipMemcpyAsync(e->d_iso_list.p, ilist.data(), ilist.size() * 4, hipMemcpyHostToDevice, e->st));
    CHK(e->d_gc_off.ensure(std::max<size_t>(gcb[RT], 1)));
    CHK(e->d_gc_cnt.ensure(std::max<size_t>(gcb[RT], 1)));
    CHK(e->d_gcount.ensure(std::max<size_t>(cnb[R], 1)));
    CHK(e->d_gscan.ensure(std::max<size_t>(cnb[R], 1)));
    CHK(e->d_shard_cnt.ensure(2 * NSHARD));
    CHK(e->d_shard_prefix.ensure(NSHARD + 1));
    {
        // (query gene, subject sample) searches of the tile
        uint64_t nb = 1;
        for (size_t r = 0; r < RT; r++)
            for (int q = runs[r].first; q < runs[r].second; q++) {
                uint64_t ns = 0;
                for (int w = 0; w < tw; w++) ns += (uint64_t)__builtin_popcountll(tmask[(size_t)tw * q + w]);
                nb += (uint64_t)(e->sample_gene_begin[q + 1] - e->sample_gene_begin[q]) * ns;
            }
        e->seed_cap = std::max<uint64_t>(e->seed_cap, nb * 16 / NSHARD + 4096);
        e->cand_cap = std::max<uint64_t>(e->cand_cap, nb * 2 / NSHARD + 1024);
        // (RC_OVF_CAP0: a smaller first guess, for tests of the overflow retry)
        const char *oc = getenv("RC_OVF_CAP0");
        e->ovf_cap = std::max<uint64_t>(e->ovf_cap, oc ? (uint64_t)std::max(1, atoi(oc)) : nb / 4 + 1024);
    }
    Db db = make_db(e);
    Index ix;
    ix.ent = e->d_ent2.p;
    ix.bucket = e->d_bucket.p;
    ix.pos_tx = e->d_pos_tx.p;
    ix.bits = e->index_bits;
    Index ixm = ix;   // the reverse pass's: masked transcripts only
    ixm.ent = e->d_ment2.p;
    ixm.bucket = e->d_mbucket.p;
    ixm.bits = e->mindex_bits;
    // --- seeds ---
    std::vector<unsigned long long> shard_cnt(2 * NSHARD);
    CHK(e->d_count.ensure(34));
    unsigned long long *big_n = e->d_count.p + 12, *big_retry_n = e->d_count.p + 13;
    uint64_t n_big = 0;
    HIPCHK(hipEventRecord(e->ev[3], e->st));
    uint32_t n_rs = 0;
    if (revpass && e->n_mindex) CHK(reverse_pass(e, ti, db, ixm, n_rs));
    for (int attempt = 0;; attempt++) {
        if (attempt == 6) return fail(RC_E_NOMEM, "seed/candidate buffers kept overflowing");
        if (e->seed_cap * NSHARD > 0xFFFFFFFFull || e->cand_cap * NSHARD > 0xFFFFFFFFull)
            return fail(RC_E_LIMIT, "more than 2^32 seeds or candidates in a tile: use more shards or smaller tiles");
        CHK(e->d_seeds.ensure(e->seed_cap * NSHARD));
        CHK(e->d_cands.ensure(e->cand_cap * NSHARD));
        if (e->share) CHK(e->d_list2.ensure(e->cand_cap * NSHARD));
        HIPCHK(hipMemsetAsync(e->d_count.p + 16, 0, sizeof(unsigned long long), e->st));
        CHK(e->d_big_out.ensure(e->big_list_cap));
        HIPCHK(hipMemsetAsync(e->d_shard_cnt.p, 0, 2 * NSHARD * sizeof(unsigned long long), e->st));
        HIPCHK(hipMemsetAsync(e->d_status.p, 0, 4 * sizeof(unsigned int), e->st));
        if (gcb[RT]) HIPCHK(hipMemsetAsync(e->d_gc_cnt.p, 0, gcb[RT] * 4, e->st));
        CHK(e->d_prof.ensure(10));
        HIPCHK(hipMemsetAsync(e->d_prof.p, 0, 10 * sizeof(unsigned long long), e->st));
        bool again = false;
        n_big = 0;
        for (size_t r = 0; r < RT && !again; r++) {
            HIPCHK(hipMemsetAsync(big_n, 0, 2 * sizeof(unsigned long long), e->st));
            SeedParams S{};
            S.word = e->o.word_size;
            S.stride = e->o.word_size - W16 + 1;
            {
                const char *pm = getenv("RC_SEED_PRE");   // A/B knob; 1 = hit-list pre-test
                S.pre_mode = pm ? atoi(pm) : 1;
            }
            S.sym = e->o.symmetric;
            S.share = e->share ? 1 : 0;
            S.tx_pos = e->d_tx_pos.p;
            S.iso_pre_g = e->d_iso_pre.p;
            S.rs_rec = e->d_rseeds.p;
            S.rs_key = e->d_rs_key.p;
            S.rs_idx = e->d_rs_idx.p;
            S.rs_n = n_rs;
            S.list2 = e->d_list2.p;
            S.list2_n = e->d_count.p + 16;
            S.gene_begin = rg0[r];
            S.gene_end = rg1[r];
            if (n_rs) {
                CHK(e->d_rs_range.ensure((size_t)2 * (rg1[r] - rg0[r]) + 2));
                launch_rs_range(e->d_rs_key.p, n_rs, rg0[r], rg1[r], e->d_rs_range.p, e->st);
                S.rs_range = e->d_rs_range.p;
            }
            S.iso_list = e->d_iso_list.p + ioff[r];
            S.iso_n = ioff[r + 1] - ioff[r];
            S.seeds = e->d_seeds.p;
            S.seed_cap = e->seed_cap;
            S.seed_count = e->d_shard_cnt.p;
            S.cands = e->d_cands.p;
            S.cand_cap = e->cand_cap;
            S.cand_count = e->d_shard_cnt.p + NSHARD;
            S.gc_off = e->d_gc_off.p + gcb[r];
            S.gc_cnt = e->d_gc_cnt.p + gcb[r];
            S.tmask = e->d_tmask.p;
            S.tmw = tw;
            S.trange = e->d_trange.p;
            S.xbits = e->xbits;
            S.max_iso = max_iso(e->xbits);
            S.status = e->d_status.p;
            S.big_out = e->d_big_out.p;
            S.big_n = big_n;
            S.big_retry_n = big_retry_n;
            S.big_list_cap = e->big_list_cap;
            S.prof = e->d_prof.p;
            launch_seed(e->has_amb, db, ix, S, e->st);
            HIPCHK(hipGetLastError());
            unsigned int status = 0;
            unsigned long long nb = 0;   // (big_n: d_count[12], next to the extension's counters [0, 11))
            HIPCHK(hipMemcpyAsync(&status, e->d_status.p, sizeof status, hipMemcpyDeviceToHost, e->st));
            HIPCHK(hipMemcpyAsync(&nb, big_n, sizeof nb, hipMemcpyDeviceToHost, e->st));
            CHK(wait_st(e));
            if (status & 2u)
                return fail(RC_E_LIMIT, "a query gene has more than " + std::to_string(max_iso(e->xbits)) + " isoforms");
            if (status & 16u)
                return fail(RC_E_LIMIT, "a candidate's first seed of a directed search is past seed 65534");
            if (status & 8u) {   // the big-pass list itself overflowed
                e->big_list_cap = std::max<uint64_t>(4 * e->big_list_cap, nb + 1024);
                again = true;
                break;
            }
            again = (status & 1u) != 0;
            // (gene, sample) passes whose seeds overflow LDS: global-memory
            // passes, at most BIG_CHUNK workgroups per launch; entries that
            // overflow big_cap too are rerun with twice the scratch
            const uint64_t BIG_CHUNK = 2048;
            uint64_t *list = e->d_big_out.p;
            n_big += nb;
            while (!again && nb) {
                if ((uint64_t)e->big_cap > (1ull << 22))
                    return fail(RC_E_LIMIT, "a (query gene, subject sample) pass has more than 2^22 seeds");
                const uint64_t chunk = std::min<uint64_t>(nb, BIG_CHUNK);
                CHK(e->d_big_list.ensure(nb));
                CHK(e->d_big_retry.ensure(nb));
                CHK(e->d_big_seeds.ensure(chunk * e->big_cap));
                CHK(e->d_big_seg.ensure(chunk * (e->big_cap + 1)));
                CHK(e->d_big_segT.ensure(chunk * e->big_cap));
                if (list != e->d_big_list.p)
                    HIPCHK(hipMemcpyAsync(e->d_big_list.p, list, nb * 8, hipMemcpyDeviceToDevice, e->st));
                HIPCHK(hipMemsetAsync(big_retry_n, 0, sizeof(unsigned long long), e->st));
                SeedParams B = S;
                B.big_retry = e->d_big_retry.p;
                B.big_list_cap = nb;
                B.big_cap = e->big_cap;
                B.big_seeds = e->d_big_seeds.p;
                B.big_seg = e->d_big_seg.p;
                B.big_segT = e->d_big_segT.p;
                for (uint64_t c0 = 0; c0 < nb; c0 += chunk) {
                    B.big_list = e->d_big_list.p + c0;
                    launch_seed_big(e->has_amb, db, ix, B, (uint32_t)std::min<uint64_t>(chunk, nb - c0), e->st);
                    HIPCHK(hipGetLastError());
                }
                unsigned long long nr = 0;
                HIPCHK(hipMemcpyAsync(&status, e->d_status.p, sizeof status, hipMemcpyDeviceToHost, e->st));
                HIPCHK(hipMemcpyAsync(&nr, big_retry_n, sizeof nr, hipMemcpyDeviceToHost, e->st));
                CHK(wait_st(e));
                if (status & 16u)
                    return fail(RC_E_LIMIT, "a candidate's first seed of a directed search is past seed 65534");
                again = (status & 1u) != 0;
                nb = nr;
                // the retry entries become the next list (buffers swapped, not copied)
                std::swap(e->d_big_list.p, e->d_big_retry.p);
                std::swap(e->d_big_list.cap, e->d_big_retry.cap);
                list = e->d_big_list.p;
                if (nb) e->big_cap *= 2;
            }
        }
        HIPCHK(hipEventRecord(e->ev[9], e->st));
        HIPCHK(hipMemcpyAsync(shard_cnt.data(), e->d_shard_cnt.p, 2 * NSHARD * 8, hipMemcpyDeviceToHost, e->st));
        CHK(wait_st(e));
        if (!again) break;
        uint64_t ms = 0, mc = 0;
        for (int i = 0; i < NSHARD; i++) {
            ms = std::max<uint64_t>(ms, shard_cnt[i]);
            mc = std::max<uint64_t>(mc, shard_cnt[NSHARD + i]);
        }
        e->seed_cap = std::max<uint64_t>(e->seed_cap, ms * 5 / 4 + 4096);
        e->cand_cap = std::max<uint64_t>(e->cand_cap, mc * 5 / 4 + 1024);
    }
    e->tm.big_passes += (double)n_big;
    std::vector<unsigned long long> prefix(NSHARD + 1, 0);
    for (int i = 0; i < NSHARD; i++) prefix[i + 1] = prefix[i] + shard_cnt[NSHARD + i];
    const uint64_t n_cand = prefix[NSHARD];
    for (int i = 0; i < NSHARD; i++) e->n_seeds += shard_cnt[i];
    e->n_cands += n_cand;
    HIPCHK(hipMemcpyAsync(e->d_shard_prefix.p, prefix.data(), (NSHARD + 1) * 8, hipMemcpyHostToDevice, e->st));
    // --- extension ---
    const uint64_t slots = e->cand_cap * NSHARD;
    CHK(e->d_cand_hsp.ensure(slots));
    CHK(e->d_cand_nh.ensure(slots));
    CHK(e->d_cand_ovf.ensure(slots));
    CHK(e->d_cand_box.ensure(slots * BOX_REC));
    if (e->share) {
        CHK(e->d_cand_box2.ensure(slots * BOX_REC));
        CHK(e->d_cand_hsp_r.ensure(slots));
        CHK(e->d_cand_nh_r.ensure(slots));
        CHK(e->d_cand_ovf_r.ensure(slots));
        CHK(e->d_defer_r.ensure(std::max<uint64_t>(n_cand, 1)));
        CHK(e->d_wide0.ensure(std::max<uint64_t>(n_cand, 1)));
        CHK(e->d_wide1.ensure(std::max<uint64_t>(n_cand, 1)));
        {
            // room to continue the first 12 M overflowing extensions of a pass
            // (3.8 GB); later ones start over in the 64-lane pass
            const char *rv = getenv("RC_RESUME");
            e->res_cap = (rv && atoi(rv) == 0) ? 0u : (uint32_t)std::min<uint64_t>(n_cand, 12u << 20);
            if (!(rv && atoi(rv) == 1) && e->ovf_frac <= 0.02) e->res_cap = 0;   // not needed: no buffer
            if (e->res_cap) CHK(e->d_resume.ensure((size_t)e->res_cap * RES_REC));
        }
    }
    CHK(e->d_defer.ensure(std::max<uint64_t>(n_cand, 1)));
    CHK(e->d_defer2.ensure(std::max<uint64_t>(n_cand, 1)));
    // later-seed rounds: their parameters once they ran (a retry finishes
    // the searches again from the states, and extend_kernel takes the lists
    // of the searches they left whole instead of first_finish_kernel's)
    bool later_on = false;
    LaterParams lat{};
    for (int attempt = 0;; attempt++) {
        if (attempt == 4) return fail(RC_E_NOMEM, "HSP overflow buffer kept overflowing");
        CHK(e->d_ovf.ensure(e->ovf_cap));
        if (attempt == 0) {
            HIPCHK(hipMemsetAsync(e->d_count.p, 0, 12 * sizeof(unsigned long long), e->st));
            HIPCHK(hipMemsetAsync(e->d_count.p + 14, 0, 2 * sizeof(unsigned long long), e->st));
            HIPCHK(hipMemsetAsync(e->d_count.p + 17, 0, 2 * sizeof(unsigned long long), e->st));
            HIPCHK(hipMemsetAsync(e->d_count.p + 20, 0, 7 * sizeof(unsigned long long), e->st));
        } else {
            // a retry redoes extend_kernel only: its overflow count restarts,
            // every other counter and list stands
            HIPCHK(hipMemsetAsync(e->d_count.p, 0, sizeof(unsigned long long), e->st));
        }
        HIPCHK(hipMemsetAsync(e->d_status.p, 0, 4 * sizeof(unsigned int), e->st));
        ExtParams X{};
        X.xdrop = e->o.xdrop_half;
        X.sym = e->o.symmetric;
        X.max_len = e->max_len;
        X.thr = e->d_thr.p;
        X.bits10 = e->d_bits10.p;
        X.cands = e->d_cands.p;
        X.seeds = e->d_seeds.p;
        X.shard_prefix = e->d_shard_prefix.p;
        X.n_cand = n_cand;
        X.cand_cap = e->cand_cap;
        X.cand_hsp = e->d_cand_hsp.p;
        X.cand_nh = e->d_cand_nh.p;
        X.cand_ovf = e->d_cand_ovf.p;
        X.ovf = e->d_ovf.p;
        X.ovf_cap = e->ovf_cap;
        X.ovf_count = e->d_count.p;
        X.status = e->d_status.p;
        X.counters = e->d_count.p + 1;
        {
            // row staging slot (u64 words): whole transcripts when the longest
            // fits the slot the 32-lane kernel has at full occupancy, else
            // windows of that slot (the windowed instantiation). RC_WIN_WORDS
            // forces windows of that many words (tests: many refills).
            const int need = ((e->max_len + 31) >> 5) + 4;
            const int smax = row_slot_words_max(e->has_amb);
            const char *wwv = getenv("RC_WIN_WORDS");
            const int forced = wwv ? std::max(4, atoi(wwv)) : 0;
            X.win = forced ? 1 : (need > smax ? 1 : 0);
            X.dsw = forced ? std::min(forced, smax) : std::min(need, smax);
        }
        X.defer = e->d_defer.p;
        X.defer_count = e->d_count.p + 6;
        X.work = e->d_count.p + 7;
        X.defer2 = e->d_defer2.p;
        X.defer2_count = e->d_count.p + 14;
        X.work2 = e->d_count.p + 15;
        X.cand_box = e->d_cand_box.p;
        X.share = e->share ? 1 : 0;
        X.which = 0;
        X.dir = 0;
        X.cand_box2 = e->d_cand_box2.p;
        X.cand_hsp_r = e->d_cand_hsp_r.p;
        X.cand_nh_r = e->d_cand_nh_r.p;
        X.cand_ovf_r = e->d_cand_ovf_r.p;
        X.defer_r = e->d_defer_r.p;
        X.defer_r_count = e->d_count.p + 17;
        X.list2 = e->d_list2.p;
        X.list2_n = e->d_count.p + 16;
        X.work3 = e->d_count.p + 18;
        X.wide0 = e->share ? e->d_wide0.p : nullptr;
        X.wide1 = e->d_wide1.p;
        X.wide0_n = e->d_count.p + 20;
        X.wide1_n = e->d_count.p + 21;
        {
            // save overflowing extensions for the 64-lane pass when the last
            // run had many (C3v: 39 %, C3: 0.002 %): the saving kernel costs
            // the plain one 7 % (RC_RESUME=1 always, 0 never)
            const char *rv = getenv("RC_RESUME");
            const bool on = rv ? atoi(rv) == 1 : e->ovf_frac > 0.02;
            X.resume = e->res_cap && on ? e->d_resume.p : nullptr;
            X.res_cap = e->res_cap;
        }
        X.work_w0 = e->d_count.p + 22;
        X.work_w1 = e->d_count.p + 23;
        X.why = e->d_count.p + 24;   // [24, 27): deferral causes
        {
            const char *cv = getenv("RC_ROW_CHUNK");
            X.chunk = cv ? atoi(cv) : 8;
            const char *rv = getenv("RC_REUSE");   // 0: extend_kernel redoes every search's first seed
            X.reuse_first = rv ? atoi(rv) : 1;
        }
        if (attempt == 0) {
            HIPCHK(hipEventRecord(e->ev[10], e->st));
            // sub-band row width of the extension (16 or 32 diagonals); RC_ROW_WIDTH overrides
            const char *rwv = getenv("RC_ROW_WIDTH");
            const int rw = rwv ? atoi(rwv) : 32;
            launch_extend_rows(e->has_amb, db, X, rw, e->st, false);
            HIPCHK(hipGetLastError());
            // only the searches the row kernels left (defer lists) can have
            // more than one HSP, at most MAX_HSP - 1 more each: the overflow
            // buffer at twice their count (about 1.1 more each at C3v), so a
            // first run rarely redoes extend_kernel
            unsigned long long dn[3] = {0, 0, 0};
            HIPCHK(hipMemcpyAsync(&dn[0], X.defer_count, sizeof dn[0], hipMemcpyDeviceToHost, e->st));
            HIPCHK(hipMemcpyAsync(&dn[1], e->d_count.p + 17, sizeof dn[1], hipMemcpyDeviceToHost, e->st));
            if (X.defer2_count)
                HIPCHK(hipMemcpyAsync(&dn[2], X.defer2_count, sizeof dn[2], hipMemcpyDeviceToHost, e->st));
            CHK(wait_st(e));
            const uint64_t want = std::min<uint64_t>(2 * (dn[0] + dn[1] + dn[2]), (uint64_t)(MAX_HSP - 1) *
                                                     (dn[0] + dn[1] + dn[2])) + 1024;
            if (want > e->ovf_cap && !getenv("RC_OVF_CAP0")) {
                e->ovf_cap = want;
                CHK(e->d_ovf.ensure(e->ovf_cap));
                X.ovf = e->d_ovf.p;
                X.ovf_cap = e->ovf_cap;
            }
            // later-seed rounds: the deferred searches' later seeds on the row
            // kernels (RC_LATER=0: extend_kernel runs them whole); searches
            // past RC_LATER_CAP (default 24 M, 12 GB of state and work) run whole
            const char *lv = getenv("RC_LATER");
            const uint64_t nsrch = dn[0] + dn[1];
            if (e->share && X.reuse_first && !(lv && atoi(lv) == 0) && nsrch) {
                const char *cv = getenv("RC_LATER_CAP");
                const uint64_t cap = cv ? (uint64_t)std::max(atoll(cv), 1ll) : (24ull << 20);
                const uint64_t n = std::min(nsrch, cap);
                CHK(e->d_later.ensure(n * LATER_REC));
                CHK(e->d_lbox0.ensure(n * BOX_REC));
                CHK(e->d_lbox1.ensure(n * BOX_REC));
                CHK(e->d_lvc0.ensure(n));
                CHK(e->d_lvc1.ensure(n));
                CHK(e->d_llist0.ensure(n));
                CHK(e->d_llist1.ensure(n));
                CHK(e->d_lact0.ensure(n));
                CHK(e->d_lact1.ensure(n));
                CHK(e->d_lfull0.ensure(std::max<uint64_t>(dn[0], 1)));
                CHK(e->d_lfull1.ensure(std::max<uint64_t>(dn[1], 1)));
                const size_t nc = (size_t)MAX_HSP * LATER_CNT + 4;
                CHK(e->d_lcnt.ensure(nc));
                HIPCHK(hipMemsetAsync(e->d_lcnt.p, 0, nc * sizeof(unsigned long long), e->st));
                lat = LaterParams{};
                lat.state = e->d_later.p;
                lat.n_search = nsrch;
                lat.n0 = dn[0];
                lat.n_cap = n;
                lat.defer0 = X.defer;
                lat.defer1 = X.defer_r;
                lat.full0 = e->d_lfull0.p;
                lat.full1 = e->d_lfull1.p;
                lat.counters = e->d_lcnt.p + (size_t)MAX_HSP * LATER_CNT;
                lat.full_n = lat.counters + 2;
                Cand *const vc[2] = {e->d_lvc0.p, e->d_lvc1.p};
                uint32_t *const ls[2] = {e->d_llist0.p, e->d_llist1.p};
                int32_t *const bx[2] = {e->d_lbox0.p, e->d_lbox1.p};
                uint32_t *const ac[2] = {e->d_lact0.p, e->d_lact1.p};
                launch_later_rounds(e->has_amb, db, X, lat, vc, ls, bx, ac, e->d_lcnt.p, e->st);
                HIPCHK(hipGetLastError());
                later_on = true;
            }
            if (later_on) {
                launch_later_finish(X, lat, e->st);
                X.defer = lat.full0;
                X.defer_count = lat.full_n;
                X.defer_r = lat.full1;
                X.defer_r_count = lat.full_n + 1;
            }
            launch_extend_retry(e->has_amb, db, X, e->st);
        } else {
            if (later_on) {
                launch_later_finish(X, lat, e->st);
                X.defer = lat.full0;
                X.defer_count = lat.full_n;
                X.defer_r = lat.full1;
                X.defer_r_count = lat.full_n + 1;
            }
            X.counters = nullptr;   // (the first attempt counted this work)
            launch_extend_retry(e->has_amb, db, X, e->st);
            e->tm.ext_retries += 1.0;
        }
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(e->ev[11], e->st));
        unsigned long long ovn = 0, ctr[11] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, nfull = 0;
        HIPCHK(hipMemcpyAsync(&nfull, e->d_count.p + 14, sizeof nfull, hipMemcpyDeviceToHost, e->st));
        unsigned long long nwide[2] = {0, 0};   // shared searches: candidates the 64-lane passes took
        HIPCHK(hipMemcpyAsync(nwide, e->d_count.p + 20, sizeof nwide, hipMemcpyDeviceToHost, e->st));
        unsigned long long why[3] = {0, 0, 0};
        HIPCHK(hipMemcpyAsync(why, e->d_count.p + 24, sizeof why, hipMemcpyDeviceToHost, e->st));
        unsigned long long ndr = 0, nl2 = 0;   // shared searches: reverse searches redone whole, second first seeds
        HIPCHK(hipMemcpyAsync(&ndr, e->d_count.p + 17, sizeof ndr, hipMemcpyDeviceToHost, e->st));
        HIPCHK(hipMemcpyAsync(&nl2, e->d_count.p + 16, sizeof nl2, hipMemcpyDeviceToHost, e->st));
        unsigned int status = 0;
        HIPCHK(hipMemcpyAsync(&ovn, e->d_count.p, sizeof ovn, hipMemcpyDeviceToHost, e->st));
        HIPCHK(hipMemcpyAsync(ctr, e->d_count.p + 1, sizeof ctr, hipMemcpyDeviceToHost, e->st));
        HIPCHK(hipMemcpyAsync(&status, e->d_status.p, sizeof status, hipMemcpyDeviceToHost, e->st));
        CHK(wait_st(e));
        if (ctr[8] || ctr[9]) {   // built with RC_ROW_TIMING: wave cycles in transitions / steps
            unsigned long long tfs[3] = {0, 0, 0};   // fetches, window slides, extension starts (parts of the transitions)
            HIPCHK(hipMemcpy(tfs, e->d_count.p + 28, sizeof tfs, hipMemcpyDeviceToHost));
            HIPCHK(hipMemset(e->d_count.p + 28, 0, sizeof tfs));
            fprintf(stderr, "row kernel wave-cycles: transitions %.4g (fetches %.4g, window slides %.4g, extension "
                            "starts %.4g) steps %.4g\n",
                    (double)ctr[8], (double)tfs[0], (double)tfs[1], (double)tfs[2], (double)ctr[9]);
            // 32-lane rows: steps and candidates within a 16-lane window, its slides (profiles/r06_row16)
            unsigned long long r16[3] = {0, 0, 0};
            HIPCHK(hipMemcpy(&r16[0], e->d_count.p + 27, 8, hipMemcpyDeviceToHost));
            HIPCHK(hipMemcpy(&r16[1], e->d_count.p + 31, 8, hipMemcpyDeviceToHost));
            HIPCHK(hipMemcpy(&r16[2], e->d_count.p + 32, 8, hipMemcpyDeviceToHost));
            HIPCHK(hipMemset(e->d_count.p + 27, 0, 8));
            HIPCHK(hipMemset(e->d_count.p + 31, 0, 16));
            fprintf(stderr, "row steps before a live span over 14 diagonals %.4g of %.4g; candidates never over 14: "
                            "%.4g of %.4g; 16-lane window slides %.4g\n", (double)r16[0], (double)ctr[0],
                    (double)r16[1], (double)ctr[2], (double)r16[2]);
            unsigned long long pr[10];
            HIPCHK(hipMemcpy(pr, e->d_prof.p, sizeof pr, hipMemcpyDeviceToHost));
            fprintf(stderr, "seed kernel block-cycles: prologue %.4g words: usable %.4g lookup %.4g scan %.4g "
                            "hits %.4g (loads %.4g pretest %.4g full test %.4g) sort %.4g write %.4g\n",
                    (double)pr[8], (double)pr[9], (double)pr[0], (double)pr[1], (double)(pr[2] + pr[5] + pr[6] + pr[7]),
                    (double)pr[5], (double)pr[6], (double)pr[7], (double)pr[3], (double)pr[4]);
        }
        if (!(status & 1u)) {
            e->tm.ext_steps += (double)ctr[0];
            e->tm.ext_calls += (double)ctr[1];
            // candidates the one-wave kernel took (the 64-lane pass's list, or the row kernel's)
            const char *r64 = getenv("RC_ROW64");
            e->tm.ext_fullband += (r64 && atoi(r64)) ? (double)nfull : (double)ctr[3];
            e->ovf_frac = n_cand ? (double)ctr[3] / (double)n_cand : 0.0;
            e->tm.ext_deferred += (double)ctr[5] + (double)ndr;
            e->tm.ext_second += e->share ? (double)nl2 : 0.0;
            e->tm.band_bound += (double)ctr[7];
            e->tm.ext_slides += (double)ctr[4];
            e->tm.ext_wide += (double)(nwide[0] + nwide[1]);
            e->tm.maxhsp_bound += (double)ctr[10];
            e->tm.defer_length += (double)why[0];
            e->tm.defer_gaveup += (double)why[1];
            e->tm.defer_outside += (double)why[2];
            if (later_on) {   // later-seed rounds: seeds extended on the row kernels, searches run whole
                std::vector<unsigned long long> lc((size_t)MAX_HSP * LATER_CNT + 4);
                HIPCHK(hipMemcpy(lc.data(), e->d_lcnt.p, lc.size() * sizeof(unsigned long long),
                                 hipMemcpyDeviceToHost));
                for (int r = 0; r < MAX_HSP; r++) e->tm.later_seeds += (double)lc[(size_t)r * LATER_CNT];
                e->tm.later_whole += (double)lc[(size_t)MAX_HSP * LATER_CNT + 1];
            }
            break;
        }
        e->ovf_cap = std::max<uint64_t>(e->ovf_cap, ovn * 5 / 4 + 1024);
    }
    // --- groups: (query gene, subject sample) -> contiguous HSPs, appended ---
    // Direct groups of every run first, in candidate order; mirrored groups
    // (spec 5b: the subject->query direction of the same alignments) follow,
    // each sorted into the order that search emits.
    GroupParams G{};
    G.N = N;
    G.cand_nh = e->d_cand_nh.p;
    G.cand_hsp = e->d_cand_hsp.p;
    G.cand_ovf = e->d_cand_ovf.p;
    G.ovf = e->d_ovf.p;
    G.shard_prefix = e->d_shard_prefix.p;
    G.n_cand = n_cand;
    G.cand_cap = e->cand_cap;
    G.tx_gene = e->d_tx_gene.p;
    G.tx_pos = e->d_tx_pos.p;
    G.tx = e->d_tx.p;
    G.n_genes = n_genes;
    G.grp_off = e->d_grp_off.p;
    G.grp_cnt = e->d_grp_cnt.p;
    auto exscan = [&](const uint32_t *in, uint64_t *out, size_t n) -> int {
        size_t tmp = 0;
        HIPCHK(rocprim::exclusive_scan(nullptr, tmp, in, out, (uint64_t)0, n, rocprim::plus<uint64_t>(), e->st));
        CHK(e->d_tmp.ensure(tmp));
        HIPCHK(rocprim::exclusive_scan(e->d_tmp.p, tmp, in, out, (uint64_t)0, n, rocprim::plus<uint64_t>(), e->st));
        return RC_OK;
    };
    auto run_group = [&](size_t r) {
        GroupParams g = G;
        g.gene_begin = rg0[r];
        g.gene_end = rg1[r];
        g.gc_off = e->d_gc_off.p + gcb[r];
        g.gc_cnt = e->d_gc_cnt.p + gcb[r];
        g.cnt = e->d_gcount.p + cnb[r];
        g.scan = e->d_gscan.p + cnb[r];
        return g;
    };
    std::vector<uint64_t> nd(R, 0);
    for (size_t r = 0; r < R; r++) {
        const size_t nsgrp = cnb[r + 1] - cnb[r] - 1;
        HIPCHK(hipMemsetAsync(e->d_gcount.p + cnb[r] + nsgrp, 0, 4, e->st));
        launch_group(run_group(r), 0, e->st);
        CHK(exscan(e->d_gcount.p + cnb[r], e->d_gscan.p + cnb[r], nsgrp + 1));
        HIPCHK(hipMemcpyAsync(&nd[r], e->d_gscan.p + cnb[r] + nsgrp, 8, hipMemcpyDeviceToHost, e->st));
    }
    uint64_t nm = 0;
    // the other direction's groups: mirror images (spec 5b), or the reverse
    // searches of the shared candidate set (their own HSPs, in their order)
    const bool mirror = e->o.symmetric || e->share;
    if (e->share) {
        G.cand_nh = e->d_cand_nh_r.p;
        G.cand_hsp = e->d_cand_hsp_r.p;
        G.cand_ovf = e->d_cand_ovf_r.p;
    }
    if (mirror) {
        // the window of the tile's mirrored groups: every HSP is between a
        // query transcript of a pair's a (lower sample) and a subject
        // transcript of its b, so its mirrored group is (gene of b, sample a)
        int a_lo = N, a_hi = 0, b_lo = N, b_hi = 0;
        for (const auto &pr : TT.pairs) {
            a_lo = std::min(a_lo, pr.first);
            a_hi = std::max(a_hi, pr.first + 1);
            b_lo = std::min(b_lo, pr.second);
            b_hi = std::max(b_hi, pr.second + 1);
        }
        if (a_hi <= a_lo || b_hi <= b_lo) a_lo = a_hi = b_lo = b_hi = 0;
        G.ms0 = a_lo;
        G.msn = a_hi - a_lo;
        G.mg0 = e->sample_gene_begin[b_lo];
        G.mgw = e->sample_gene_begin[b_hi] - e->sample_gene_begin[b_lo];
        const size_t nwin = (size_t)G.mgw * (size_t)G.msn;
        CHK(e->d_mcnt.ensure(nwin + 1));
        CHK(e->d_mcur.ensure(std::max<uint64_t>(n_cand, 1)));   // per candidate: its slots' start in its group
        CHK(e->d_mscan.ensure(nwin + 1));
        G.mcnt = e->d_mcnt.p;
        G.mcur = e->d_mcur.p;
        HIPCHK(hipMemsetAsync(e->d_mcnt.p, 0, (nwin + 1) * 4, e->st));
        launch_group(G, 2, e->st);   // mirrored groups (spec 5b)
        CHK(exscan(e->d_mcnt.p, e->d_mscan.p, nwin + 1));
        HIPCHK(hipMemcpyAsync(&nm, e->d_mscan.p + nwin, 8, hipMemcpyDeviceToHost, e->st));
    }
    CHK(wait_st(e));
    uint64_t ndt = 0;
    for (uint64_t v : nd) ndt += v;
    const uint64_t nh = e->hsp_used + ndt + nm;
    if (nh > 0xFFFFFFFFull) return fail(RC_E_LIMIT, "more than 2^32 HSPs on one GPU: use more shards");
    CHK(grow_hsp(e, nh));
    uint64_t base = e->hsp_used;
    for (size_t r = 0; r < R; r++) {
        GroupParams g = run_group(r);
        g.cand_nh = e->d_cand_nh.p;
        g.cand_hsp = e->d_cand_hsp.p;
        g.cand_ovf = e->d_cand_ovf.p;
        g.out = e->d_hsp.p;
        g.base = base;
        launch_group(g, 1, e->st);
        base += nd[r];
    }
    if (mirror) {
        CHK(e->d_mkey.ensure(2 * nm + 2));
        CHK(e->d_mbig.ensure(nm / 33 + 2));
        HIPCHK(hipMemsetAsync(e->d_count.p + 19, 0, sizeof(unsigned long long), e->st));
        G.mscan = e->d_mscan.p;
        G.out = e->d_hsp.p;
        G.mbase = base;
        G.mkey = e->d_mkey.p;
        G.mbig = e->d_mbig.p;
        G.mbig_n = e->d_count.p + 19;
        launch_group(G, 3, e->st);
        launch_group(G, 4, e->st);
    }
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(e->ev[4], e->st));
    CHK(wait_st(e));
    e->hsp_used = nh;
    e->tm.pack_ms += ev_ms(e, 0, 1);
    e->tm.index_ms += ev_ms(e, 1, 2);
    if (e->o.dust_level > 0 && !e->external) {
        float dms = 0;
        if (hipEventElapsedTime(&dms, e->evd[0], e->evd[1]) == hipSuccess) e->tm.dust_ms += dms;
    }
    e->tm.align_ms += ev_ms(e, 2, 4);
    e->tm.seed_kernel_ms += ev_ms(e, 3, 9);
    e->tm.align_kernel_ms += ev_ms(e, 10, 11);
    return RC_OK;
}

static int do_align_tiles(rc_engine *e);

static int do_align(rc_engine *e)
{
    CHK(upload(e));
    CHK(set_device(e));
    e->aligned = e->finished = e->rbh_done = false;
    e->tm = rc_timing{};
    const double t0 = wall_ms();
    const int rc = do_align_tiles(e);
    e->tm.align_wall_ms = wall_ms() - t0;
    return rc;
}

static int do_align_tiles(rc_engine *e)
{
    if (e->external) {
        HIPCHK(hipEventRecord(e->ev[0], e->st));
        CHK(load_external(e));
        HIPCHK(hipEventRecord(e->ev[1], e->st));
        HIPCHK(hipEventSynchronize(e->ev[1]));
        e->tm.align_ms = ev_ms(e, 0, 1);
        e->aligned = true;
        return RC_OK;
    }
    const int N = (int)e->samples.size();
    // the samples of this shard's pairs must be on this GPU (a graph-only
    // engine, rc_import_edges on a fresh engine, aligns nothing and needs none)
    for (uint64_t p = e->pair0; p < e->pair1; p++)
        for (int s : {(int)e->pair_a[p], (int)e->pair_b[p]})
            if (!e->samples[s].resident)
                return fail(RC_E_STATE, "sample " + e->samples[s].label +
                                            " is aligned by this shard but was added without its sequence");
    const size_t ngrp = (size_t)e->gene_sample.size() * N;
    CHK(e->d_grp_off.ensure(ngrp));
    CHK(e->d_grp_cnt.ensure(ngrp));
    HIPCHK(hipMemsetAsync(e->d_grp_cnt.p, 0, ngrp * 4, e->st));
    HIPCHK(hipMemsetAsync(e->d_grp_off.p, 0, ngrp * 4, e->st));
    if (e->tiles_for != (int64_t)e->pair0 || e->tiles.empty()) {
        plan_tiles(e);
        e->tiles_for = (int64_t)e->pair0;
        e->tile_loaded = -1;
    }
    e->hsp_used = 0;
    e->n_seeds = e->n_cands = 0;
    e->idx_bchunk = -1;   // every run builds its indexes and masks anew
    // the tile loaded last goes first (its tables stay on the device)
    const int nt = (int)e->tiles.size();
    const int first = (e->tile_loaded >= 0 && e->tile_loaded < nt) ? e->tile_loaded : 0;
    for (int k = 0; k < nt; k++) CHK(align_tile(e, (first + k) % nt));
    e->tm.tiles = (double)nt;
    e->n_hsps = e->hsp_used;
    e->aligned = true;
    return RC_OK;
}

// Top-N + reciprocal best hits for this shard's items -> table rows, edges.
static int do_rbh(rc_engine *e)
{
    if (!e->aligned) return fail(RC_E_STATE, "rc_finish before rc_align");
    CHK(set_device(e));
    const int N = (int)e->samples.size();
    const uint64_t ni = e->item1 - e->item0;
    const size_t np = e->pair_a.size();
    e->finished = false;
    HIPCHK(hipEventRecord(e->ev[5], e->st));
    CHK(e->d_cnt4.ensure(4 * (ni + 1)));
    CHK(e->d_off4.ensure(4 * (ni + 1)));
    HIPCHK(hipMemsetAsync(e->d_cnt4.p, 0, 4 * (ni + 1) * 4, e->st));
    // the RBH selection loops' 8-byte view of the group table (bit score,
    // subject gene): r05, rbh_kernel 6.5 -> see DESIGN §4
    CHK(e->d_hkey.ensure(std::max<uint64_t>(e->n_hsps, 1)));   // (n_hsps: aligned or imported)
    launch_hkey(e->d_hsp.p, e->n_hsps, e->d_tx_gene.p, e->d_hkey.p, e->st);
    RbhParams R{};
    R.hsp = e->d_hsp.p;
    R.hk = e->d_hkey.p;
    R.grp_off = e->d_grp_off.p;
    R.grp_cnt = e->d_grp_cnt.p;
    R.n_genes = (uint32_t)e->gene_sample.size();
    R.tx_gene = e->d_tx_gene.p;
    R.tx = e->d_tx.p;
    R.sample_gene_begin = e->d_sample_gene_begin.p;
    R.pair_item_begin = e->d_pair_item_begin.p;
    R.pair_a = e->d_pair_a.p;
    R.pair_b = e->d_pair_b.p;
    R.n_pairs = (int32_t)np;
    R.N = N;
    R.top_n = e->o.top_matches;
    R.keep_all = e->o.keep_all;
    R.item0 = e->item0;
    R.n_items = ni;
    R.n_rows = e->d_cnt4.p;
    R.n_fsel = e->d_cnt4.p + (ni + 1);
    R.n_rsel = e->d_cnt4.p + 2 * (ni + 1);
    R.n_edges = e->d_cnt4.p + 3 * (ni + 1);
    // one pass over the groups: counts, and rows/edges in per-item slots
    CHK(e->d_rows_tmp.ensure(std::max<uint64_t>(ni, 1) * RBH_RMAX));
    CHK(e->d_edges_tmp.ensure(std::max<uint64_t>(ni, 1) * RBH_EMAX));
    HIPCHK(hipMemsetAsync(e->d_status.p + 1, 0, sizeof(unsigned int), e->st));
    R.rows_tmp = e->d_rows_tmp.p;
    R.edges_tmp = e->d_edges_tmp.p;
    R.ovf = e->d_status.p + 1;
    launch_rbh(R, 2, e->st);
    HIPCHK(hipGetLastError());
    for (int k = 0; k < 4; k++) {
        size_t tmp = 0;
        const uint32_t *in = e->d_cnt4.p + k * (ni + 1);
        uint64_t *out = e->d_off4.p + k * (ni + 1);
        HIPCHK(rocprim::exclusive_scan(nullptr, tmp, in, out, (uint64_t)0, (size_t)ni + 1, rocprim::plus<uint64_t>(),
                                       e->st));
        CHK(e->d_tmp.ensure(tmp));
        HIPCHK(rocprim::exclusive_scan(e->d_tmp.p, tmp, in, out, (uint64_t)0, (size_t)ni + 1,
                                       rocprim::plus<uint64_t>(), e->st));
    }
    uint64_t tot[4] = {0, 0, 0, 0};
    for (int k = 0; k < 4; k++)
        HIPCHK(hipMemcpyAsync(&tot[k], e->d_off4.p + k * (ni + 1) + ni, 8, hipMemcpyDeviceToHost, e->st));
    unsigned int slot_ovf = 0;
    HIPCHK(hipMemcpyAsync(&slot_ovf, e->d_status.p + 1, sizeof slot_ovf, hipMemcpyDeviceToHost, e->st));
    HIPCHK(hipStreamSynchronize(e->st));
    e->n_rows = tot[0];
    e->n_edges = tot[3];
    e->n_local_edges = tot[3];
    CHK(e->d_rows.ensure(e->n_rows));
    CHK(e->d_edges.ensure(e->n_edges));
    R.row_off = e->d_off4.p;
    R.fsel_off = e->d_off4.p + (ni + 1);
    R.rsel_off = e->d_off4.p + 2 * (ni + 1);
    R.edge_off = e->d_off4.p + 3 * (ni + 1);
    R.rows = e->d_rows.p;
    R.edges = e->d_edges.p;
    if (slot_ovf || getenv("RC_RBH_TWO_PASS"))
        launch_rbh(R, 1, e->st);   // an item had more rows or edges than its slots: full second pass
    else
        launch_rbh_place(R, e->st);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(e->ev[6], e->st));
    HIPCHK(hipEventSynchronize(e->ev[6]));
    e->tm.rbh_ms = ev_ms(e, 5, 6);
    e->rbh_done = true;
    return RC_OK;
}

// Gene matches graph over d_edges[0, n_edges): connected components, ideal
// filter, restricted pair sums.
static int do_graph(rc_engine *e)
{
    if (!e->rbh_done) return fail(RC_E_STATE, "graph phase before rc_finish");
    CHK(set_device(e));
    const int N = (int)e->samples.size();
    const uint32_t n_genes = (uint32_t)e->gene_sample.size();
    const size_t np = e->pair_a.size();
    HIPCHK(hipEventRecord(e->ev[6], e->st));
    CHK(e->d_parent.ensure(n_genes));
    CHK(e->d_present.ensure(n_genes));
    CHK(e->d_cnodes.ensure(n_genes));
    CHK(e->d_cedges.ensure(n_genes));
    CHK(e->d_ideal.ensure(n_genes));
    CHK(e->d_sample_present.ensure(N));
    CHK(e->d_stats.ensure(8));
    HIPCHK(hipMemsetAsync(e->d_sample_present.p, 0, N * 4, e->st));
    HIPCHK(hipMemsetAsync(e->d_stats.p, 0, 8 * 8, e->st));
    launch_cc(e->d_edges.p, e->n_edges, n_genes, e->d_gene_sample.p, N, e->sample_count_given, e->d_parent.p,
              e->d_present.p, e->d_cnodes.p,
              e->d_cedges.p, e->d_sample_present.p, e->d_ideal.p, e->d_stats.p, e->st);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(e->ev[7], e->st));
    CHK(e->d_num.ensure(np));
    CHK(e->d_den.ensure(np));
    CHK(e->d_num_all.ensure(np));
    CHK(e->d_den_all.ensure(np));
    HIPCHK(hipMemsetAsync(e->d_num.p, 0, np * 8, e->st));
    HIPCHK(hipMemsetAsync(e->d_den.p, 0, np * 8, e->st));
    HIPCHK(hipMemsetAsync(e->d_num_all.p, 0, np * 8, e->st));
    HIPCHK(hipMemsetAsync(e->d_den_all.p, 0, np * 8, e->st));
    launch_pair_sums(e->d_edges.p, e->n_edges, e->d_parent.p, e->d_ideal.p, e->d_num.p, e->d_den.p,
                     e->d_num_all.p, e->d_den_all.p, e->st);
    HIPCHK(hipGetLastError());
    e->h_num.assign(np, 0);
    e->h_den.assign(np, 0);
    e->h_num_all.assign(np, 0);
    e->h_den_all.assign(np, 0);
    e->h_stats.assign(8, 0);
    if (np) {
        HIPCHK(hipMemcpyAsync(e->h_num.data(), e->d_num.p, np * 8, hipMemcpyDeviceToHost, e->st));
        HIPCHK(hipMemcpyAsync(e->h_den.data(), e->d_den.p, np * 8, hipMemcpyDeviceToHost, e->st));
        HIPCHK(hipMemcpyAsync(e->h_num_all.data(), e->d_num_all.p, np * 8, hipMemcpyDeviceToHost, e->st));
        HIPCHK(hipMemcpyAsync(e->h_den_all.data(), e->d_den_all.p, np * 8, hipMemcpyDeviceToHost, e->st));
    }
    HIPCHK(hipMemcpyAsync(e->h_stats.data(), e->d_stats.p, 8 * 8, hipMemcpyDeviceToHost, e->st));
    HIPCHK(hipEventRecord(e->ev[8], e->st));
    HIPCHK(hipStreamSynchronize(e->st));
    e->tm.graph_ms = ev_ms(e, 6, 7);
    e->tm.reduce_ms = ev_ms(e, 7, 8);
    e->tm.total_ms = e->tm.pack_ms + e->tm.index_ms + e->tm.align_ms + e->tm.rbh_ms + e->tm.graph_ms + e->tm.reduce_ms;
    e->finished = true;
    return RC_OK;
}

static int do_finish(rc_engine *e)
{
    CHK(do_rbh(e));
    if (e->o.shard_count == 1) return do_graph(e);
    return RC_OK;
}

// ------------------------------------------------------------------------
// results
// ------------------------------------------------------------------------

static rc_hsp to_rc_hsp(const rc_engine *e, const DHsp &d, int qs_, int ss_)
{
    rc_hsp h;
    h.q_tx = d.q_tx - e->samples[qs_].tx_begin;
    h.s_tx = d.s_tx - e->samples[ss_].tx_begin;
    h.qstart = d.qstart; h.qend = d.qend; h.sstart = d.sstart; h.send = d.send;
    h.length = d.length; h.nident = d.nident; h.mismatch = d.mismatch; h.gaps = d.gaps;
    h.gapopen = d.gapopen; h.score_half = d.score_half; h.bits10 = d.bits10; h.strand = d.strand & 1;
    const int64_t qlen = (int64_t)(e->tx_start[d.q_tx + 1] - e->tx_start[d.q_tx]);
    const double ss = qlen <= e->max_len ? e->h_ss[(size_t)ss_ * (e->max_len + 1) + (size_t)qlen]
                                         : stats::search_space(qlen, e->db_len[ss_], e->db_n[ss_]);
    // stats::evalue, its exp() taken from the table (the same product, in
    // the same order: bit-identical)
    h.evalue = d.score_half >= 0 && (size_t)d.score_half < e->h_exp.size() ? ss * stats::K * e->h_exp[d.score_half]
                                                                            : stats::evalue(ss, d.score_half);
    return h;
}

static int copy_groups(rc_engine *e, std::vector<uint32_t> &off, std::vector<uint32_t> &cnt)
{
    const size_t n = (size_t)e->gene_sample.size() * e->samples.size();
    off.resize(n);
    cnt.resize(n);
    if (!n) return RC_OK;
    HIPCHK(hipMemcpy(off.data(), e->d_grp_off.p, n * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(cnt.data(), e->d_grp_cnt.p, n * 4, hipMemcpyDeviceToHost));
    return RC_OK;
}

extern "C" {

int rc_upload(rc_engine *e)
{
    if (!e) return fail(RC_E_ARG, "null engine");
    return upload(e);
}

int rc_align(rc_engine *e)
{
    if (!e) return fail(RC_E_ARG, "null engine");
    return do_align(e);
}

int rc_finish(rc_engine *e)
{
    if (!e) return fail(RC_E_ARG, "null engine");
    return do_finish(e);
}

int rc_run(rc_engine *e)
{
    if (!e) return fail(RC_E_ARG, "null engine");
    if (e->o.shard_count != 1) return fail(RC_E_STATE, "sharded engines use rc_align / rc_finish / rc_import_edges");
    CHK(do_align(e));
    return do_finish(e);
}

int rc_set_sample_count(rc_engine *e, int32_t sample_count)
{
    if (!e) return fail(RC_E_ARG, "null engine");
    if (sample_count < 0) return fail(RC_E_ARG, "sample_count must be >= 0");
    e->sample_count_given = sample_count;
    return RC_OK;
}

int rc_hsps(rc_engine *e, int32_t q, int32_t s, rc_hsp *buf, uint64_t cap, uint64_t *n)
{
    if (!e || !n) return fail(RC_E_ARG, "null argument");
    if (!e->aligned) return fail(RC_E_STATE, "no alignment yet");
    const int N = (int)e->samples.size();
    if (q < 0 || q >= N || s < 0 || s >= N) return fail(RC_E_ARG, "bad sample");
    CHK(set_device(e));
    std::vector<uint32_t> off, cnt;
    CHK(copy_groups(e, off, cnt));
    const SampleRec &Q = e->samples[q];
    const uint32_t ng = (uint32_t)e->gene_sample.size();
    uint64_t tot = 0;
    for (uint32_t g = Q.gene_begin; g < Q.gene_begin + Q.n_genes; g++) tot += cnt[grp_index(g, s, ng)];
    *n = tot;
    if (!buf) return RC_OK;
    if (cap < tot) return fail(RC_E_CAPACITY, "buffer too small");
    uint64_t w = 0;
    std::vector<DHsp> tmp;
    for (uint32_t g = Q.gene_begin; g < Q.gene_begin + Q.n_genes; g++) {
        const uint32_t c = cnt[grp_index(g, s, ng)];
        if (!c) continue;
        tmp.resize(c);
        HIPCHK(hipMemcpy(tmp.data(), e->d_hsp.p + off[grp_index(g, s, ng)], c * sizeof(DHsp), hipMemcpyDeviceToHost));
        for (uint32_t i = 0; i < c; i++) buf[w++] = to_rc_hsp(e, tmp[i], q, s);
    }
    return RC_OK;
}

// A pair's rows on the host: its table rows (DRow) and their HSPs, fetched
// from the device (the engine's stream; one caller at a time).
struct PairRaw {
    int32_t s1 = 0, s2 = 0;
    uint64_t n = 0;
    const DRow *rows = nullptr;   // n rows and their HSPs: in the vectors, or in a pinned slab
    const DHsp *hs = nullptr;
    std::vector<DRow> vrows;
    std::vector<DHsp> vhs;
    std::shared_ptr<char> slab;   // (returned to its pool when the last holder lets go)
};

// Pinned host slabs the rows of many pairs come to by DMA (rc_write_outputs):
// at most `cap` of them, allocated as needed, each holding `bytes`; a slab
// goes back to the pool when its pair's last consumer drops it. Pageable
// copies faulted fresh pages for every pair (3.6 GB at C3).
struct SlabPool {
    std::mutex mu;
    std::condition_variable cv;
    std::vector<char *> all, free;
    size_t bytes = 0, cap = 0;
    ~SlabPool()
    {
        for (char *p : all) (void)hipHostFree(p);
    }
    // a slab (blocks while all `cap` are in use); nullptr if pinning fails
    std::shared_ptr<char> get()
    {
        std::unique_lock<std::mutex> lk(mu);
        if (free.empty() && all.size() < cap) {
            char *p = nullptr;
            if (hipHostMalloc((void **)&p, bytes, hipHostMallocDefault) != hipSuccess) {
                (void)hipGetLastError();
                return nullptr;
            }
            all.push_back(p);
            free.push_back(p);
        }
        cv.wait(lk, [&] { return !free.empty(); });
        char *p = free.back();
        free.pop_back();
        return std::shared_ptr<char>(p, [this](char *q) {
            {
                std::lock_guard<std::mutex> g(mu);
                free.push_back(q);
            }
            cv.notify_all();
        });
    }
};

static int pair_row_range(rc_engine *e, int32_t s1, int32_t s2, uint64_t &r0, uint64_t &r1)
{
    if (!e->rbh_done || e->graph_only) return fail(RC_E_STATE, "no gene matches tables on this engine");
    const int N = (int)e->samples.size();
    if (s1 < 0 || s1 >= N || s2 < 0 || s2 >= N || s1 >= s2) return fail(RC_E_ARG, "need s1 < s2 (input order)");
    CHK(set_device(e));
    const uint64_t p = (uint64_t)e->pair_index[s1 * N + s2];
    if (p < e->pair0 || p >= e->pair1) return fail(RC_E_ARG, "pair belongs to another shard");
    const uint64_t ib = e->pair_item_begin[p] - e->item0, ie = e->pair_item_begin[p + 1] - e->item0;
    HIPCHK(hipMemcpy(&r0, e->d_off4.p + ib, 8, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(&r1, e->d_off4.p + ie, 8, hipMemcpyDeviceToHost));
    return RC_OK;
}

// a pair's rows and their HSPs to the host: into `pool`'s pinned slabs when
// given and big enough, else into the PairRaw's own vectors
static int fetch_pair(rc_engine *e, int32_t s1, int32_t s2, PairRaw &out, SlabPool *pool = nullptr,
                      const uint64_t *range = nullptr)
{
    uint64_t r0 = 0, r1 = 0;
    if (range) {
        r0 = range[0];
        r1 = range[1];
    } else {
        CHK(pair_row_range(e, s1, s2, r0, r1));
    }
    const uint64_t nr = r1 - r0;
    out.s1 = s1;
    out.s2 = s2;
    out.n = nr;
    if (!nr) return RC_OK;
    CHK(e->d_gather.ensure(nr));
    launch_gather_rows(e->d_hsp.p, e->d_rows.p + r0, nr, e->d_gather.p, e->st);
    HIPCHK(hipGetLastError());
    DRow *rows = nullptr;
    DHsp *hs = nullptr;
    if (pool && nr * (sizeof(DRow) + sizeof(DHsp)) <= pool->bytes) out.slab = pool->get();
    if (out.slab) {
        hs = reinterpret_cast<DHsp *>(out.slab.get());
        rows = reinterpret_cast<DRow *>(out.slab.get() + nr * sizeof(DHsp));
    } else {
        out.vrows.resize(nr);
        out.vhs.resize(nr);
        rows = out.vrows.data();
        hs = out.vhs.data();
    }
    HIPCHK(hipMemcpyAsync(rows, e->d_rows.p + r0, nr * sizeof(DRow), hipMemcpyDeviceToHost, e->st));
    HIPCHK(hipMemcpyAsync(hs, e->d_gather.p, nr * sizeof(DHsp), hipMemcpyDeviceToHost, e->st));
    HIPCHK(hipStreamSynchronize(e->st));
    out.rows = rows;
    out.hs = hs;
    return RC_OK;
}

// rc_row records of fetched rows (host only: thread-safe, the engine's host
// tables are read only)
static void convert_rows(const rc_engine *e, const PairRaw &raw, rc_row *buf)
{
    const int32_t s1 = raw.s1, s2 = raw.s2;
    const uint64_t nr = raw.n;
    const DRow *rows = raw.rows;
    const DHsp *hs = raw.hs;
    for (uint64_t i = 0; i < nr; i++) {
        const DHsp &d = hs[i];
        rc_row &r = buf[i];
        const bool rev = rows[i].reverse != 0;
        // forward rows: query in s2, subject in s1; reverse rows the other way round
        const int qs_ = rev ? s1 : s2, ss_ = rev ? s2 : s1;
        r.hsp = to_rc_hsp(e, d, qs_, ss_);
        const uint32_t tq = rev ? d.s_tx : d.q_tx;   // transcript of s2 (qgene side)
        const uint32_t ts = rev ? d.q_tx : d.s_tx;   // transcript of s1 (sgene side)
        r.qgene = e->tx_gene_id[tq];
        r.qiso = e->tx_iso[tq];
        r.sgene = e->tx_gene_id[ts];
        r.siso = e->tx_iso[ts];
        r.q_tx = tq - e->samples[s2].tx_begin;
        r.s_tx = ts - e->samples[s1].tx_begin;
        r.reverse = rev ? 1 : 0;
        r.label = rows[i].label;
    }
}

int rc_pair_rows(rc_engine *e, int32_t s1, int32_t s2, rc_row *buf, uint64_t cap, uint64_t *n)
{
    if (!e || !n) return fail(RC_E_ARG, "null argument");
    uint64_t r0 = 0, r1 = 0;
    CHK(pair_row_range(e, s1, s2, r0, r1));
    *n = r1 - r0;
    if (!buf) return RC_OK;
    if (cap < r1 - r0) return fail(RC_E_CAPACITY, "buffer too small");
    if (r1 == r0) return RC_OK;
    PairRaw raw;
    CHK(fetch_pair(e, s1, s2, raw));
    convert_rows(e, raw, buf);
    return RC_OK;
}

int rc_graph_stats(rc_engine *e, rc_stats *s)
{
    if (!e || !s) return fail(RC_E_ARG, "null argument");
    if (!e->finished) return fail(RC_E_STATE, "no results yet");
    s->components = (int64_t)e->h_stats[0];
    s->ideal_components = (int64_t)e->h_stats[1];
    s->ideal_nodes = (int64_t)e->h_stats[2];
    s->nodes = (int64_t)e->h_stats[3];
    s->sample_count = (int32_t)e->h_stats[4];
    s->pad = 0;
    s->edges = (int64_t)e->n_edges;
    s->hsps = (int64_t)e->n_hsps;
    s->seeds = (int64_t)e->n_seeds;
    s->candidates = (int64_t)e->n_cands;
    s->table_rows = (int64_t)e->n_rows;
    return RC_OK;
}

int rc_edges(rc_engine *e, rc_edge *buf, uint64_t cap, uint64_t *n)
{
    if (!e || !n) return fail(RC_E_ARG, "null argument");
    if (!e->finished) return fail(RC_E_STATE, "no results yet");
    *n = e->n_edges;
    if (!buf) return RC_OK;
    if (cap < e->n_edges) return fail(RC_E_CAPACITY, "buffer too small");
    CHK(set_device(e));
    std::vector<DEdge> ed(e->n_edges);
    if (!ed.empty()) HIPCHK(hipMemcpy(ed.data(), e->d_edges.p, ed.size() * sizeof(DEdge), hipMemcpyDeviceToHost));
    for (size_t i = 0; i < ed.size(); i++) {
        buf[i].sample_a = e->gene_sample[ed[i].a];
        buf[i].gene_a = e->gene_id[ed[i].a];
        buf[i].sample_b = e->gene_sample[ed[i].b];
        buf[i].gene_b = e->gene_id[ed[i].b];
    }
    return RC_OK;
}

int rc_ideal_nodes(rc_engine *e, int32_t *sample, int32_t *gene, uint64_t cap, uint64_t *n)
{
    if (!e || !n) return fail(RC_E_ARG, "null argument");
    if (!e->finished) return fail(RC_E_STATE, "no results yet");
    CHK(set_device(e));
    const uint32_t ng = (uint32_t)e->gene_sample.size();
    std::vector<uint32_t> parent(ng), present(ng);
    std::vector<uint8_t> ideal(ng);
    if (ng) {
        HIPCHK(hipMemcpy(parent.data(), e->d_parent.p, ng * 4, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(present.data(), e->d_present.p, ng * 4, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(ideal.data(), e->d_ideal.p, ng, hipMemcpyDeviceToHost));
    }
    uint64_t c = 0;
    for (uint32_t v = 0; v < ng; v++)
        if (present[v] && ideal[parent[v]]) {
            if (sample && gene) {
                if (c >= cap) return fail(RC_E_CAPACITY, "buffer too small");
                sample[c] = e->gene_sample[v];
                gene[c] = e->gene_id[v];
            }
            c++;
        }
    *n = c;
    return RC_OK;
}

int rc_pair_sums(rc_engine *e, int64_t *num, int64_t *den)
{
    if (!e || !num || !den) return fail(RC_E_ARG, "null argument");
    if (!e->finished) return fail(RC_E_STATE, "no results yet");
    const int N = (int)e->samples.size();
    for (int a = 0; a < N; a++)
        for (int b = 0; b < N; b++) {
            if (a == b) {
                num[a * N + b] = den[a * N + b] = 0;
                continue;
            }
            const int p = e->pair_index[a * N + b];
            num[a * N + b] = (int64_t)e->h_num[p];
            den[a * N + b] = (int64_t)e->h_den[p];
        }
    return RC_OK;
}

// Unfiltered sums: every gene matches table row of the pair
// (UnfilteredSimilarity, unfiltered_distance.py:9-16 over similarities_from_dfs,
// similarity_computer.py:21-42).
int rc_pair_sums_unfiltered(rc_engine *e, int64_t *num, int64_t *den)
{
    if (!e || !num || !den) return fail(RC_E_ARG, "null argument");
    if (!e->finished) return fail(RC_E_STATE, "no results yet");
    const int N = (int)e->samples.size();
    for (int a = 0; a < N; a++)
        for (int b = 0; b < N; b++) {
            if (a == b) {
                num[a * N + b] = den[a * N + b] = 0;
                continue;
            }
            const int p = e->pair_index[a * N + b];
            num[a * N + b] = (int64_t)e->h_num_all[p];
            den[a * N + b] = (int64_t)e->h_den_all[p];
        }
    return RC_OK;
}

int rc_distance_subset(rc_engine *e, const int32_t *order, int32_t n, double *out)
{
    if (!e || (n && (!order || !out))) return fail(RC_E_ARG, "null argument");
    if (!e->finished) return fail(RC_E_STATE, "no results yet");
    const int N = (int)e->samples.size();
    if (n < 0 || n > N) return fail(RC_E_ARG, "bad sample count");
    std::vector<int> seen(N, 0);
    for (int i = 0; i < n; i++) {
        if (order[i] < 0 || order[i] >= N || seen[order[i]]) return fail(RC_E_ARG, "order must hold distinct sample ids");
        seen[order[i]] = 1;
    }
    if (!n) return RC_OK;
    CHK(set_device(e));
    CHK(e->d_order.ensure(n));
    CHK(e->d_dist.ensure((size_t)n * n));
    HIPCHK(hipMemcpyAsync(e->d_order.p, order, n * 4, hipMemcpyHostToDevice, e->st));
    HIPCHK(hipMemsetAsync(e->d_status.p, 0, 4 * sizeof(unsigned int), e->st));
    launch_distance(e->d_num.p, e->d_den.p, e->d_pair_index.p, e->d_order.p, N, n, e->d_dist.p, e->d_status.p,
                    e->st);
    HIPCHK(hipGetLastError());
    unsigned int status = 0;
    HIPCHK(hipMemcpyAsync(out, e->d_dist.p, (size_t)n * n * 8, hipMemcpyDeviceToHost, e->st));
    HIPCHK(hipMemcpyAsync(&status, e->d_status.p, 4, hipMemcpyDeviceToHost, e->st));
    HIPCHK(hipStreamSynchronize(e->st));
    if (status & 4u) return fail(RC_E_NO_IDEAL, "No ideal components found. Cannot report distances!");
    return RC_OK;
}

int rc_distance(rc_engine *e, const int32_t *order, double *out)
{
    if (!e) return fail(RC_E_ARG, "null argument");
    return rc_distance_subset(e, order, (int32_t)e->samples.size(), out);
}

int rc_dust_mask(rc_engine *e, int32_t s, uint8_t *buf, uint64_t cap, uint64_t *n)
{
    if (!e || !n) return fail(RC_E_ARG, "null argument");
    if (!e->aligned) return fail(RC_E_STATE, "no alignment yet");
    if (s < 0 || s >= (int)e->samples.size()) return fail(RC_E_ARG, "bad sample");
    const SampleRec &S = e->samples[s];
    *n = S.nbases;
    if (!buf) return RC_OK;
    if (cap < S.nbases) return fail(RC_E_CAPACITY, "buffer too small");
    if (!S.nbases) return RC_OK;
    if (e->o.dust_level <= 0 || e->external) {
        std::memset(buf, 0, S.nbases);
        return RC_OK;
    }
    // the mask of the loaded tile, where the sample sits at tile_pos[s]
    if (e->tile_loaded < 0) return fail(RC_E_STATE, "no tile loaded");
    const auto &ts = e->tiles[e->tile_loaded].samples;
    if (std::find(ts.begin(), ts.end(), s) == ts.end())
        return fail(RC_E_STATE, "the sample is not in the last alignment pass (tile)");
    if (!e->dmask_only.empty() && !e->dmask_only[s])
        return fail(RC_E_STATE, "the last rc_dust_masks pass did not mask this sample");
    CHK(set_device(e));
    const uint64_t b0 = e->tile_pos[s];
    const uint64_t w0 = b0 >> 6, w1 = (b0 + S.nbases + 63) >> 6;
    std::vector<uint64_t> words(w1 - w0);
    HIPCHK(hipMemcpy(words.data(), e->d_dmask.p + 1 + w0, words.size() * 8, hipMemcpyDeviceToHost));
    for (uint64_t i = 0; i < S.nbases; i++) {
        const uint64_t p = b0 + i;
        buf[i] = (uint8_t)((words[(p >> 6) - w0] >> (p & 63)) & 1);
    }
    return RC_OK;
}

// DUST masks computed once per sample across shards: each
// sample's mask is made on one rank that holds it (rc_dust_masks), the masks
// are exchanged, and every rank hands them to its engine (rc_set_dust_masks),
// whose alignment then copies them into its tiles instead of running DUST.
// Layout: the listed samples in order, ceil(bases / 64) words each, bit b of
// word w = base 64 w + b of the sample (1: masked); bits past the last base 0.
static uint64_t mask_words(const rc_engine *e, const int32_t *samples, int32_t n)
{
    uint64_t w = 0;
    for (int32_t i = 0; i < n; i++) w += (e->samples[samples[i]].nbases + 63) >> 6;
    return w;
}

int rc_dust_masks(rc_engine *e, const int32_t *samples, int32_t n, uint64_t *out, uint64_t cap_words,
                  uint64_t *n_words, int on_device)
{
    if (!e || !n_words || n < 0 || (n && !samples)) return fail(RC_E_ARG, "null argument");
    CHK(upload(e));
    const int N = (int)e->samples.size();
    for (int32_t i = 0; i < n; i++) {
        if (samples[i] < 0 || samples[i] >= N) return fail(RC_E_ARG, "bad sample");
        if (!e->samples[samples[i]].resident)
            return fail(RC_E_STATE, "sample " + e->samples[samples[i]].label + " was added without its sequence");
    }
    const uint64_t words = mask_words(e, samples, n);
    *n_words = words;
    if (!out) return RC_OK;
    if (cap_words < words) return fail(RC_E_CAPACITY, "buffer too small");
    CHK(set_device(e));
    // passes of their own: the tile tables of a previous run are replaced. Its
    // results stay valid: HSP groups, RBH rows and edges read only the
    // transcripts' lengths and samples, never a tile's positions or masks
    std::vector<int> ss(samples, samples + n);
    std::sort(ss.begin(), ss.end());
    ss.erase(std::unique(ss.begin(), ss.end()), ss.end());
    std::vector<std::vector<uint64_t>> oof(N);   // word offsets of each listed sample in `out` (any repeats)
    {
        uint64_t o = 0;
        for (int32_t i = 0; i < n; i++) {
            oof[samples[i]].push_back(o);
            o += (e->samples[samples[i]].nbases + 63) >> 6;
        }
    }
    if (e->tiles_for != (int64_t)e->pair0 || e->tiles.empty()) {
        plan_tiles(e);
        e->tiles_for = (int64_t)e->pair0;
        e->tile_loaded = -1;
    }
    // the shard's own alignment tile when it is a single tile holding these
    // samples (its tables stay loaded for rc_align), else tiles of these
    // samples alone, as many as the 2^32-base tile limit takes (a C5 rank
    // masks ~4 Gbp); each packed, its DUST masks copied out
    bool own = e->tiles.size() == 1;
    for (int s : ss)
        own = own && std::binary_search(e->tiles[0].samples.begin(), e->tiles[0].samples.end(), s);
    std::vector<std::vector<int>> chunks;
    if (own) {
        chunks.push_back(ss);
    } else {
        const uint64_t cap = tile_cap();
        uint64_t acc = 0;
        for (int s : ss) {
            const uint64_t b = align_up(e->samples[s].nbases);
            if (chunks.empty() || (acc + b > cap && !chunks.back().empty())) {
                chunks.push_back({});
                acc = 0;
            }
            chunks.back().push_back(s);
            acc += b;
        }
    }
    const bool dust = e->o.dust_level > 0 && !e->external;
    int rc = RC_OK;
    for (size_t c = 0; c < chunks.size() && rc == RC_OK; c++) {
        int ti = 0;
        if (!own) {
            rc_engine::Tile T;
            T.samples = chunks[c];
            e->tiles.push_back(T);
            e->tile_loaded = -1;
            ti = (int)e->tiles.size() - 1;
        }
        rc = load_tile(e, ti);
        if (rc == RC_OK) rc = pack_tile(e);
        if (rc == RC_OK && dust) {
            const size_t mw = (e->tile_total >> 6) + 4;
            rc = e->d_dmask.ensure(mw);
            if (rc == RC_OK && hipMemsetAsync(e->d_dmask.p, 0, mw * 8, e->st) != hipSuccess)
                rc = fail(RC_E_HIP, "hipMemsetAsync");
            if (rc == RC_OK) rc = dust_samples(e, chunks[c], e->st);
        }
        for (size_t k = 0; rc == RC_OK && k < chunks[c].size(); k++) {
            const int s = chunks[c][k];
            const uint64_t nb = e->samples[s].nbases, nw = (nb + 63) >> 6;
            if (!nw) continue;
            for (uint64_t w0 : oof[s]) {
                hipError_t h = hipSuccess;
                if (dust) {
                    h = hipMemcpyAsync(out + w0, e->d_dmask.p + 1 + (e->tile_pos[s] >> 6), nw * 8,
                                       on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, e->st);
                } else if (on_device) {
                    h = hipMemsetAsync(out + w0, 0, nw * 8, e->st);
                } else {
                    std::memset(out + w0, 0, nw * 8);
                }
                if (h != hipSuccess) rc = fail(RC_E_HIP, "mask copy");
            }
        }
        if (rc == RC_OK && hipStreamSynchronize(e->st) != hipSuccess) rc = fail(RC_E_HIP, "hipStreamSynchronize");
        if (!own) {
            e->tiles.pop_back();
            e->tile_loaded = -1;
        }
    }
    if (own) {   // the loaded tile's masks now hold the listed samples only
        e->dmask_only.assign(N, 0);
        for (int s : ss) e->dmask_only[s] = 1;
    }
    // bits past each sample's last base cleared (its last word)
    uint64_t o = 0;
    for (int32_t i = 0; rc == RC_OK && dust && i < n; i++) {
        const uint64_t nb = e->samples[samples[i]].nbases, nw = (nb + 63) >> 6;
        o += nw;
        if (!nw || !(nb & 63)) continue;
        const uint64_t keep = (1ull << (nb & 63)) - 1ull;
        if (on_device) {
            uint64_t w = 0;
            if (hipMemcpy(&w, out + o - 1, 8, hipMemcpyDeviceToHost) != hipSuccess ||
                (w &= keep, hipMemcpy(out + o - 1, &w, 8, hipMemcpyHostToDevice)) != hipSuccess)
                rc = fail(RC_E_HIP, "mask tail");
        } else {
            out[o - 1] &= keep;
        }
    }
    e->idx_bchunk = -1;
    return rc;
}

int rc_set_dust_masks(rc_engine *e, const int32_t *samples, int32_t n, const uint64_t *bits, uint64_t n_words,
                      int on_device)
{
    if (!e || n < 0 || (n && !samples)) return fail(RC_E_ARG, "null argument");
    CHK(upload(e));
    const int N = (int)e->samples.size();
    for (int32_t i = 0; i < n; i++)
        if (samples[i] < 0 || samples[i] >= N) return fail(RC_E_ARG, "bad sample");
    const uint64_t words = mask_words(e, samples, n);
    if (n_words != words) return fail(RC_E_ARG, "mask words do not match the samples' lengths");
    if (words && !bits) return fail(RC_E_ARG, "null argument");
    CHK(set_device(e));
    e->dust_imp_off.assign(N, ~0ull);
    CHK(e->d_dust_imp.ensure(std::max<uint64_t>(words, 1)));
    if (words)
        HIPCHK(hipMemcpy(e->d_dust_imp.p, bits, words * 8, on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice));
    uint64_t o = 0;
    for (int32_t i = 0; i < n; i++) {
        e->dust_imp_off[samples[i]] = o;
        o += (e->samples[samples[i]].nbases + 63) >> 6;
    }
    return RC_OK;
}

int rc_timings(rc_engine *e, rc_timing *t)
{
    if (!e || !t) return fail(RC_E_ARG, "null argument");
    *t = e->tm;
    t->dev_bytes = (double)g_dev_bytes.load();
    t->dev_peak_bytes = (double)g_dev_peak.load();
    return RC_OK;
}

int rc_export_edges(rc_engine *e, void *buf, uint64_t cap, uint64_t *n, int on_device)
{
    if (!e || !n) return fail(RC_E_ARG, "null argument");
    if (!e->rbh_done) return fail(RC_E_STATE, "rc_export_edges before rc_finish");
    CHK(set_device(e));
    const uint64_t tot = e->n_local_edges;
    *n = tot;
    if (!buf) return RC_OK;
    if (cap < tot) return fail(RC_E_CAPACITY, "buffer too small");
    if (e->n_edges != e->n_local_edges || e->graph_only)
        return fail(RC_E_STATE, "edges already replaced by rc_import_edges");
    if (tot)
        HIPCHK(hipMemcpy(buf, e->d_edges.p, tot * sizeof(DEdge), on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost));
    return RC_OK;
}

int rc_import_edges(rc_engine *e, const void *buf, uint64_t n, int on_device)
{
    return rc_import_edge_parts(e, buf, &n, 1, n, on_device);
}

// parts blocks of records, block r at record r * stride of buf with counts[r]
// valid records: the concatenation is imported (an all-gather's padded
// receive buffer goes in as it is, no compacted copy outside the engine)
int rc_import_edge_parts(rc_engine *e, const void *buf, const uint64_t *counts, int32_t parts, uint64_t stride,
                         int on_device)
{
    if (!e || parts < 0 || (parts && !counts)) return fail(RC_E_ARG, "null argument");
    uint64_t n = 0;
    for (int32_t r = 0; r < parts; r++) {
        if (counts[r] > stride) return fail(RC_E_ARG, "a part holds more records than the stride");
        n += counts[r];
    }
    if (n && !buf) return fail(RC_E_ARG, "null argument");
    if (!e->rbh_done) {
        // a fresh engine (samples added, nothing aligned): graph-only mode,
        // the records describe an imported graph and its tables
        if (e->aligned || e->external) return fail(RC_E_STATE, "rc_import_edges before rc_finish");
        CHK(upload(e));
        e->graph_only = e->rbh_done = true;
    }
    CHK(set_device(e));
    const uint32_t ng = (uint32_t)e->gene_sample.size();
    const uint64_t np = e->pair_a.size();
    const DEdge *src = static_cast<const DEdge *>(buf);
    if (!on_device) {
        for (int32_t r = 0; r < parts; r++) {
            const DEdge *ed = src + (uint64_t)r * stride;
            for (uint64_t i = 0; i < counts[r]; i++) {
                const bool node = ed[i].pair == NODE_REC;
                if (ed[i].a >= ng || ed[i].b >= ng || (!node && (ed[i].pair & ~EDGE_SUM_ONLY) >= np) ||
                    (node && ed[i].a != ed[i].b))
                    return fail(RC_E_ARG, "edge record out of range");
            }
        }
    }
    if (on_device) {
        // the same range check on the device, over the caller's blocks before
        // anything of the engine's is replaced: a malformed all-gather must
        // not reach the union-find kernels, and a refused import leaves the
        // engine's own edges in place
        unsigned int bad = 0;
        HIPCHK(hipMemsetAsync(e->d_status.p + 2, 0, sizeof(unsigned int), e->st));
        for (int32_t r = 0; r < parts; r++)
            if (counts[r]) launch_edge_check(src + (uint64_t)r * stride, counts[r], ng, np, e->d_status.p + 2, e->st);
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(&bad, e->d_status.p + 2, sizeof bad, hipMemcpyDeviceToHost, e->st));
        HIPCHK(hipStreamSynchronize(e->st));
        if (bad) return fail(RC_E_ARG, "edge record out of range");
    }
    // the local edges are replaced: their buffer goes before the new one is
    // allocated (a sharded rank's peak holds the gathered records once)
    if (e->d_edges.cap < n) e->d_edges.release();
    CHK(e->d_edges.ensure(n));
    const hipMemcpyKind kind = on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    uint64_t o = 0;
    for (int32_t r = 0; r < parts; r++) {
        if (counts[r])
            HIPCHK(hipMemcpyAsync(e->d_edges.p + o, src + (uint64_t)r * stride, counts[r] * sizeof(DEdge), kind, e->st));
        o += counts[r];
    }
    e->n_edges = n;
    e->n_local_edges = 0;   // the local edges are gone
    HIPCHK(hipStreamSynchronize(e->st));   // (the caller's host buffer is not retained)
    return do_graph(e);
}

// Free the alignment working set of a finished run: tile copies, indexes,
// seeds, candidates, extension and grouping scratch. What the results need
// stays (inputs, HSP store and groups, table rows, edges, graph arrays); the
// next rc_align allocates the rest again.
int rc_trim(rc_engine *e)
{
    if (!e) return fail(RC_E_ARG, "null engine");
    CHK(set_device(e));
    HIPCHK(hipStreamSynchronize(e->st));
    HIPCHK(hipStreamSynchronize(e->st2));
    e->d_tile_ascii.release(); e->d_tile_tx.release(); e->d_tile_itx.release(); e->d_tile_gid.release();
    e->d_tile_segs.release(); e->d_tile_send.release();
    e->d_F.release(); e->d_RC.release(); e->d_AF.release(); e->d_ARC.release();
    e->d_kpos_off.release(); e->d_kcnt.release(); e->d_kpos_rel.release();
    e->d_tile_masked.release(); e->d_ment.release(); e->d_ment2.release(); e->d_mbucket.release();
    e->d_rseeds.release(); e->d_rseed_gene.release(); e->d_rs_key.release(); e->d_rs_idx.release();
    e->d_rs_range.release(); e->d_rctr.release(); e->d_rtmask.release(); e->d_trange.release(); e->d_rtrange.release();
    e->d_ent.release(); e->d_ent2.release(); e->d_sort_scratch.release(); e->d_gen_tile.release();
    e->d_sort_status.release(); e->d_bucket.release(); e->d_pos_tx.release(); e->d_sample_pos.release();
    e->d_txstart.release(); e->d_dmask.release(); e->d_dust_scratch.release(); e->d_dust_events.release();
    e->d_prof.release(); e->d_tmp.release(); e->d_seeds.release(); e->d_cands.release();
    e->d_cand_hsp.release(); e->d_ovf.release(); e->d_cand_nh.release(); e->d_cand_box.release(); e->d_hkey.release();
    e->d_cand_box2.release(); e->d_cand_hsp_r.release(); e->d_cand_nh_r.release(); e->d_cand_ovf_r.release();
    e->d_defer_r.release(); e->d_list2.release(); e->d_wide0.release(); e->d_wide1.release(); e->d_resume.release();
    e->d_later.release(); e->d_lbox0.release(); e->d_lbox1.release(); e->d_lvc0.release(); e->d_lvc1.release();
    e->d_llist0.release(); e->d_llist1.release(); e->d_lact0.release(); e->d_lact1.release(); e->d_lcnt.release();
    e->d_lfull0.release(); e->d_lfull1.release();
    e->d_rows_tmp.release(); e->d_edges_tmp.release(); e->d_cand_ovf.release(); e->d_gc_off.release();
    e->d_gc_cnt.release(); e->d_gcount.release(); e->d_defer.release(); e->d_defer2.release(); e->d_gscan.release();
    e->d_mscan.release(); e->d_mkey.release(); e->d_tmask.release(); e->d_mbig.release(); e->d_mcnt.release();
    e->d_mcur.release(); e->d_big_out.release(); e->d_big_list.release(); e->d_big_retry.release();
    e->d_big_seeds.release(); e->d_big_seg.release(); e->d_big_segT.release(); e->d_cnt4.release();
    e->tile_loaded = -1;   // (rc_dust_mask reads a loaded tile: none now)
    e->idx_bchunk = -1;
    e->mnear_cap = 0;
    e->res_cap = 0;
    return RC_OK;
}

// The sample pairs in the engine's subject-major order ((0,1), (0,2), (1,2),
// (0,3), ...), cut into shard_count contiguous ranges of about equal sequence
// length (L_a + L_b per pair, the byte model of SURVEY.md §8d): pair p goes to
// the shard whose share of the total holds the midpoint of p's cost interval.
// A shard's second samples are then a contiguous sample range, and its seed
// index covers only those samples.
int rc_plan_shards(const int64_t *sample_bases, int32_t n_samples, int32_t shard_count, int64_t *pair_first)
{
    return rc_plan_pairs(sample_bases, n_samples, shard_count, nullptr, nullptr, pair_first);
}

int rc_plan_pairs(const int64_t *sample_bases, int32_t n_samples, int32_t shard_count, int32_t *pair_a,
                  int32_t *pair_b, int64_t *pair_first)
{
    if (!pair_first || shard_count < 1 || n_samples < 0 || (n_samples && !sample_bases))
        return fail(RC_E_ARG, "bad argument");
    if (n_samples > MAX_SAMPLES) return fail(RC_E_LIMIT, "more than 65535 samples");
    std::vector<int32_t> pa, pb;
    std::vector<int64_t> first;
    plan::plan_pairs(sample_bases, n_samples, shard_count, pa, pb, first);
    std::copy(first.begin(), first.end(), pair_first);
    if (pair_a) std::copy(pa.begin(), pa.end(), pair_a);
    if (pair_b) std::copy(pb.begin(), pb.end(), pair_b);
    return RC_OK;
}

int rc_pair_order(rc_engine *e, int32_t *pair_a, int32_t *pair_b)
{
    if (!e || !pair_a || !pair_b) return fail(RC_E_ARG, "null argument");
    CHK(upload(e));
    std::copy(e->pair_a.begin(), e->pair_a.end(), pair_a);
    std::copy(e->pair_b.begin(), e->pair_b.end(), pair_b);
    return RC_OK;
}

int rc_shard_pairs(rc_engine *e, int64_t *first, int64_t *last)
{
    if (!e || !first || !last) return fail(RC_E_ARG, "null argument");
    CHK(upload(e));
    *first = (int64_t)e->pair0;
    *last = (int64_t)e->pair1;
    return RC_OK;
}

// graph.pkl from the engine's graph edges: build_graph over every pair's
// table in combinations order (find_all_pairs.py:224-228 as the one-process
// order; build_graph.py:40-68) needs, per pair, its distinct (s-gene, q-gene)
// edges in the order of their first table rows -- the order of the edge
// records of that pair. The records (all pairs: a single-shard run's own, a
// sharded run's after rc_import_edges) are stably sorted on the device by
// their pair's combinations rank and copied to the host; tbeg[k] is the first
// record of the k-th non-empty pair.
// graph.pkl's tables from the edge records: sorted on the device into every
// pair's table in combinations order (stable: record order inside a pair),
// then handed to the writer as node-slot pairs -- a record's genes are global
// gene indices, sample-major, so sample s's nodes are the slots
// [gene_base[s], gene_base[s + 1]) -- with the tables' row ranges. One
// record per edge (the RBH kernel aggregates an edge's rows into it), so the
// writer skips its edge deduplication.
static int edge_slots(rc_engine *e, GraphSlots &G)
{
    if (!e->finished) return fail(RC_E_STATE, "no results yet");
    CHK(set_device(e));
    const uint64_t n = e->n_edges;
    const int N = (int)e->samples.size();
    if (n > 0xFFFFFFFFull) return fail(RC_E_LIMIT, "more than 2^32 graph edges");
    const size_t ncomb = e->pair_a.size();
    std::vector<uint32_t> comb(ncomb);
    for (size_t p = 0; p < ncomb; p++) {
        const uint64_t a = (uint64_t)e->pair_a[p], b = (uint64_t)e->pair_b[p];
        comb[p] = (uint32_t)(a * (2 * (uint64_t)N - a - 1) / 2 + (b - a - 1));
    }
    G = GraphSlots();
    G.ns = N;
    G.base.assign((size_t)N + 1, 0);
    for (int32_t s : e->gene_sample) G.base[(size_t)s + 1]++;
    for (int s = 0; s < N; s++) G.base[s + 1] += G.base[s];
    G.slot_gene = e->gene_id.data();
    G.unique = true;
    G.rows = n;
    std::vector<uint64_t> first(ncomb, ~0ull);
    if (n) {
        DBuf<uint32_t> dcomb, k0, k1, v0, v1;
        DBuf<uint64_t> dfirst;
        CHK(dcomb.ensure(ncomb));
        CHK(dfirst.ensure(std::max<size_t>(ncomb, 1)));
        CHK(k0.ensure(n));
        CHK(k1.ensure(n));
        CHK(v0.ensure(n));
        CHK(v1.ensure(n));
        HIPCHK(hipMemcpyAsync(dcomb.p, comb.data(), ncomb * 4, hipMemcpyHostToDevice, e->st));
        HIPCHK(hipMemsetAsync(dfirst.p, 0xFF, ncomb * 8, e->st));
        launch_edge_key(e->d_edges.p, n, dcomb.p, k0.p, v0.p, e->st);
        HIPCHK(hipGetLastError());
        size_t tmp = 0;
        HIPCHK(rocprim::radix_sort_pairs(nullptr, tmp, k0.p, k1.p, v0.p, v1.p, (size_t)n, 0u, 32u, e->st));
        CHK(e->d_tmp.ensure(tmp));
        HIPCHK(rocprim::radix_sort_pairs(e->d_tmp.p, tmp, k0.p, k1.p, v0.p, v1.p, (size_t)n, 0u, 32u, e->st));
        uint32_t last = 0;
        HIPCHK(hipMemcpyAsync(&last, k1.p + n - 1, 4, hipMemcpyDeviceToHost, e->st));
        // the (a, b) arrays reuse the sort's input buffers
        launch_edge_uv(e->d_edges.p, v1.p, k1.p, n, k0.p, v0.p, dfirst.p, e->st);
        HIPCHK(hipGetLastError());
        G.U = Raw<uint32_t>(n);
        G.V = Raw<uint32_t>(n);
        HIPCHK(hipMemcpyAsync(G.U.data(), k0.p, n * 4, hipMemcpyDeviceToHost, e->st));
        HIPCHK(hipMemcpyAsync(G.V.data(), v0.p, n * 4, hipMemcpyDeviceToHost, e->st));
        if (ncomb) HIPCHK(hipMemcpyAsync(first.data(), dfirst.p, ncomb * 8, hipMemcpyDeviceToHost, e->st));
        HIPCHK(hipStreamSynchronize(e->st));
        if (last == ~0u)
            return fail(RC_E_STATE, "an imported graph with isolated nodes or rows outside it: no graph.pkl from edges");
    }
    // the tables: combinations with records, in order (a table ends where the
    // next one starts)
    uint64_t end = n;
    std::vector<GraphSlots::Tab> rev;
    for (size_t c = ncomb; c-- > 0;) {
        if (first[c] == ~0ull) continue;
        const uint64_t o = first[c];
        rev.push_back(GraphSlots::Tab{e->gene_sample[G.U[o]], e->gene_sample[G.V[o]], o, end - o});
        end = o;
    }
    G.tabs.assign(rev.rbegin(), rev.rend());
    return RC_OK;
}

static int write_graph_slots(const rc_engine *e, GraphSlots &G, const char *path)
{
    std::vector<const char *> names;
    for (const SampleRec &s : e->samples) names.push_back(s.label.c_str());
    return graph_pickle_write_slots(G, path, (int32_t)names.size(), names.data());
}

extern "C" int rc_write_graph(rc_engine *e, const char *path, int32_t threads)
{
    if (!e || !path) return fail(RC_E_ARG, "null argument");
    const char *otv = getenv("RC_OUT_TIMING");
    const bool otime = otv && atoi(otv);
    const auto t0 = std::chrono::steady_clock::now();
    (void)threads;   // (the writer sizes its own pool)
    GraphSlots G;
    CHK(edge_slots(e, G));
    if (otime)
        fprintf(stderr, "rc_write_graph: edge records sorted and fetched %.3f s\n",
                std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    return write_graph_slots(e, G, path);
}

// The outputs a run writes next to matrix.h5: the od2 gene matches tables of
// the given pairs (paths[i] for pair (s1[i], s2[i]), table_paths may be NULL)
// and graph.pkl (graph_path, may be NULL; build_graph's graph over the pairs
// in the given order -- every pair of a single-shard engine, in combinations
// order). Each pair's rows leave the device once; the calling thread fetches
// them in order, `threads` workers convert and write the tables (od2_tables.
// cpp), one more thread builds and writes the pickle (graph_pickle.cpp) --
// all outside the Python interpreter.
int rc_write_outputs(rc_engine *e, int32_t n_pairs, const int32_t *s1, const int32_t *s2,
                     const char *const *table_paths, const char *graph_path, int32_t threads)
{
    if (!e || n_pairs < 0 || (n_pairs && (!s1 || !s2))) return fail(RC_E_ARG, "null argument");
    if (!table_paths && !graph_path) return RC_OK;
    if (graph_path && e->o.shard_count != 1)
        return fail(RC_E_STATE, "a sharded engine holds only its own pairs' rows: graph.pkl comes from the edges");
    const int nt = std::max(1, std::min(64, (int)threads));
    // RC_OUT_TIMING=1: where the time goes (stderr)
    const char *otv = getenv("RC_OUT_TIMING");
    const bool otime = otv && atoi(otv);
    std::atomic<long long> t_fetch{0}, t_conv{0}, t_write{0}, t_gadd{0}, t_gwrite{0};
    auto now_ns = []() {
        return (long long)std::chrono::duration_cast<std::chrono::nanoseconds>(
                   std::chrono::steady_clock::now().time_since_epoch()).count();
    };
    const long long t_start = now_ns();
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::pair<int, std::shared_ptr<PairRaw>>> tq, gq;
    bool closed = false;
    int in_flight = 0, err = RC_OK;
    std::string err_msg;
    auto set_err = [&](int code) {
        {
            std::lock_guard<std::mutex> lk(mu);
            if (err == RC_OK) {
                err = code;
                err_msg = rc_last_error();
            }
        }
        cv.notify_all();   // the fetch loop may be waiting for room
    };
    // graph.pkl over every pair in combinations order comes from the edge
    // records (sorted on the device first), written on its own thread beside
    // the tables; other pair lists (and imported graphs) take the rows
    GraphSlots gslots;
    bool edge_graph = false;
    if (graph_path) {
        const int N = (int)e->samples.size();
        bool all = (int64_t)n_pairs == (int64_t)N * (N - 1) / 2;
        for (int a = 0, k = 0; all && a < N; a++)
            for (int b = a + 1; all && b < N; b++, k++) all = s1[k] == a && s2[k] == b;
        edge_graph = all && edge_slots(e, gslots) == RC_OK;
    }
    auto worker = [&]() {
        std::vector<rc_row> buf;
        for (;;) {
            std::pair<int, std::shared_ptr<PairRaw>> job;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return !tq.empty() || closed; });
                if (tq.empty()) return;
                job = std::move(tq.front());
                tq.pop_front();
            }
            const PairRaw &raw = *job.second;
            const int32_t js1 = raw.s1, js2 = raw.s2;
            const long long c0 = now_ns();
            buf.resize(raw.n);
            convert_rows(e, raw, buf.data());
            job.second.reset();   // (its slab goes back once the grapher is done too)
            const long long c1 = now_ns();
            const int rc = od2_write_table(buf.data(), buf.size(), e->samples[js1].label, e->samples[js2].label,
                                           table_paths[job.first]);
            t_conv += c1 - c0;
            t_write += now_ns() - c1;
            if (rc != RC_OK) set_err(rc);
            {
                std::lock_guard<std::mutex> lk(mu);
                in_flight--;
            }
            cv.notify_all();
        }
    };
    auto grapher = [&]() {
        rc_gpickle *g = nullptr;
        bool ok = true;
        if (rc_graph_pickle_begin(&g) != RC_OK) {
            // keep draining the queue (in_flight must still go down)
            set_err(RC_E_NOMEM);
            g = nullptr;
            ok = false;
        }
        for (;;) {
            std::pair<int, std::shared_ptr<PairRaw>> job;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return !gq.empty() || closed; });
                if (gq.empty()) break;
                job = std::move(gq.front());
                gq.pop_front();
            }
            const PairRaw &raw = *job.second;
            const long long a0 = now_ns();
            const size_t n = raw.n;
            // the table's gene arrays, written in place (node numbering and
            // edges happen in parallel when the pickle is written)
            int64_t *sg = nullptr, *qg = nullptr;
            if (ok && graph_pickle_table(g, raw.s1, raw.s2, n, &sg, &qg) != RC_OK) {
                set_err(RC_E_LIMIT);
                ok = false;
            }
            if (ok)
                for (size_t i = 0; i < n; i++) {
                    const DHsp &d = raw.hs[i];
                    const bool rev = raw.rows[i].reverse != 0;
                    qg[i] = e->tx_gene_id[rev ? d.s_tx : d.q_tx];   // qgene: the transcript of s2
                    sg[i] = e->tx_gene_id[rev ? d.q_tx : d.s_tx];
                }
            t_gadd += now_ns() - a0;
            {
                std::lock_guard<std::mutex> lk(mu);
                in_flight--;
            }
            cv.notify_all();
        }
        if (ok) {
            const long long w0 = now_ns();
            std::vector<const char *> names;
            for (const SampleRec &s : e->samples) names.push_back(s.label.c_str());
            if (rc_graph_pickle_write(g, graph_path, (int32_t)names.size(), names.data()) != RC_OK) set_err(RC_E_IO);
            t_gwrite += now_ns() - w0;
        }
        rc_graph_pickle_free(g);
    };
    // every pair's row range first: the pinned slabs are sized to the largest
    std::vector<uint64_t> ranges(2 * (size_t)n_pairs);
    uint64_t max_rows = 0;
    for (int i = 0; i < n_pairs && (table_paths || !edge_graph); i++) {
        CHK(pair_row_range(e, s1[i], s2[i], ranges[2 * i], ranges[2 * i + 1]));
        max_rows = std::max<uint64_t>(max_rows, ranges[2 * i + 1] - ranges[2 * i]);
    }
    SlabPool slabs;
    slabs.bytes = std::max<uint64_t>(max_rows, 1) * (sizeof(DRow) + sizeof(DHsp));
    slabs.cap = (size_t)(2 * nt + 8);
    auto edge_grapher = [&]() {
        const long long w0 = now_ns();
        const int rc = write_graph_slots(e, gslots, graph_path);
        if (rc != RC_OK) set_err(rc);
        t_gwrite += now_ns() - w0;
    };
    std::vector<std::thread> pool;
    if (table_paths)
        for (int i = 0; i < nt; i++) pool.emplace_back(worker);
    if (graph_path) pool.emplace_back(edge_graph ? std::function<void()>(edge_grapher) : std::function<void()>(grapher));
    const bool row_graph = graph_path && !edge_graph;
    const int per_job = (table_paths ? 1 : 0) + (row_graph ? 1 : 0);
    const int max_flight = 4 * nt + 4;
    int rc = RC_OK;
    for (int i = 0; i < n_pairs && rc == RC_OK && per_job; i++) {
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return in_flight < max_flight * per_job || err != RC_OK; });
            if (err != RC_OK) break;
        }
        auto raw = std::make_shared<PairRaw>();
        const long long f0 = now_ns();
        rc = fetch_pair(e, s1[i], s2[i], *raw, &slabs, &ranges[2 * (size_t)i]);
        t_fetch += now_ns() - f0;
        if (rc != RC_OK) break;
        {
            std::lock_guard<std::mutex> lk(mu);
            if (table_paths) tq.push_back({i, raw});
            if (row_graph) gq.push_back({i, raw});
            in_flight += per_job;
        }
        cv.notify_all();
    }
    {
        std::lock_guard<std::mutex> lk(mu);
        closed = true;
    }
    cv.notify_all();
    for (std::thread &t : pool) t.join();
    if (otime)
        fprintf(stderr, "rc_write_outputs: %.3f s wall; fetch %.3f s, convert %.3f, table write %.3f (thread-s, %d threads), "
                        "graph add %.3f, graph write %.3f\n", (now_ns() - t_start) * 1e-9, t_fetch * 1e-9, t_conv * 1e-9,
                t_write * 1e-9, nt, t_gadd * 1e-9, t_gwrite * 1e-9);
    if (rc != RC_OK) return rc;
    if (err != RC_OK) return fail(err, err_msg);
    return RC_OK;
}

}  // extern "C"

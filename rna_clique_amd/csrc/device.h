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
constexpr int MAX_ISO = 127;    // transcripts per gene (7-bit field of the seed key)

// Transcript record (16 B, one load).
struct TxInfo {
    uint64_t start;   // global base offset of the transcript
    uint32_t len;
    int32_t sample;
};

// HSP of a directed search (56 B), BLAST tabular coordinates.
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

// Final gene-matches-table row: index of the HSP + flags.
struct DRow {
    uint32_t hsp;          // index into the top-hit array
    int32_t reverse;
    int32_t label;
    uint32_t pad;
};

// Everything the kernels need to see, passed by value.
struct Db {
    const uint64_t *F, *RC;     // 2-bit packed forward / reverse-complement
    const uint64_t *AF, *ARC;   // ambiguity masks (2 bits per base) or null
    uint64_t total;             // bases
    const TxInfo *tx;
    const uint32_t *tx_gene;    // global gene of each transcript
    const uint32_t *gene_tx_off, *gene_tx;   // CSR: transcripts of each gene
    const int32_t *gene_sample;
    const uint32_t *sample_gene_begin;       // n_samples + 1
    const uint32_t *sample_tx_begin;         // n_samples + 1
    int32_t n_samples;
};

struct Index {
    const uint32_t *keys;       // sorted 16-mer keys
    const uint2 *ent;           // (gtx, offset) in key order
    const uint32_t *bucket;     // 2^bits + 1 offsets
    int32_t bits;
};

struct AlignParams {
    int32_t word;               // W
    int32_t stride;             // W - 16 + 1
    int32_t xdrop;              // half units
    int32_t max_len;            // longest transcript
    const int32_t *thr;         // [n_samples][max_len + 1] min score_half
    const int32_t *bits10;      // [2 * max_len + 2]
    uint32_t gene_begin, gene_end;   // shard
    DHsp *out;                  // scratch HSPs
    uint64_t out_cap;
    unsigned long long *out_count;
    uint32_t *grp_off;          // [(g - gene_begin) * n_samples + T] scratch offset
    uint32_t *grp_cnt;          // count
    unsigned int *status;       // bit 0 scratch overflow, bit 1 gene limit
};

// Parameters of the two reciprocal-best-hit passes.
struct RbhParams {
    const DHsp *hsp;
    const uint32_t *grp_off, *grp_cnt;   // [gene * N + T], full gene range
    const uint32_t *tx_gene;
    const TxInfo *tx;
    const uint32_t *sample_gene_begin;
    const uint32_t *pair_item_begin;     // n_pairs + 1
    const int32_t *pair_a, *pair_b;
    int32_t n_pairs, N, top_n, keep_all;
    uint64_t n_items;
    // pass 0 outputs (per item)
    uint32_t *n_rows, *n_fsel, *n_rsel, *n_edges;
    // pass 1 inputs (exclusive scans) and outputs
    const uint64_t *row_off, *fsel_off, *rsel_off, *edge_off;
    DRow *rows;
    DEdge *edges;
};

}  // namespace rcg

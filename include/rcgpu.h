/*
 * rcgpu.h -- C ABI of the MI355X pairwise-distance engine for RNA-clique.
 *
 * One engine = one GPU. It replaces, for a whole set of samples at once:
 *
 *   BlastDBCache(db).makedb(fasta)                      find_all_pairs.py:120-159
 *   TabularBlastnSearch(query=t2, subject=t1, evalue=..,
 *     additional_columns=["gaps","nident","sstrand"])   find_homologs.py:124,209
 *   HomologFinder(...).get_match_table(t1, t2)          find_homologs.py:215-302
 *   find_all_pairs(...) over combinations(inputs, 2)    find_all_pairs.py:161-233
 *   build_graph(tables)                                 build_graph.py:40-68
 *   SampleSimilarity(graph, tables).valid/.restricted   filtered_distance.py:162-247
 *   ComparisonSimilarityComputer.get_dissimilarity_*    similarity_computer.py:216-375
 *
 * Conventions: every function returns 0 on success or a negative RC_E_* code;
 * the message of the last failure on the calling thread is rc_last_error().
 * The engine copies every input (no caller pointer is retained) and writes
 * outputs only into caller buffers sized by a prior call with buf == NULL.
 * Samples are numbered in the order they are added; that order plays the role
 * of the reference's `inputs` order (itertools.combinations(inputs, 2): for a
 * pair (a, b) with a < b, a is t1 = `ssample`, b is t2 = `qsample`).
 * An engine is not thread-safe; calls block until the GPU work is done.
 */
#ifndef RCGPU_H
#define RCGPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RC_OK 0
#define RC_E_ARG (-1)        /* bad argument */
#define RC_E_STATE (-2)      /* call out of order (e.g. rows before rc_run) */
#define RC_E_HIP (-3)        /* HIP runtime error */
#define RC_E_NOMEM (-4)      /* device or host allocation failed */
#define RC_E_NO_IDEAL (-5)   /* a pair has no ideal-component rows:
                                NoIdealComponentsError, filtered_distance.py:242-247 */
#define RC_E_CAPACITY (-6)   /* caller buffer too small */
#define RC_E_LIMIT (-7)      /* input beyond a documented engine limit: */
/*   samples per engine            65535
 *   transcripts per engine        2^27
 *   transcript length             16 Mbp
 *   transcripts (isoforms) / gene 65535 while the longest transcript is under
 *                                 1 Mbp; 2^(36 - b) - 1 for a longest length of
 *                                 b bits (4095 at 16 Mbp)
 *   bases per alignment tile      2^32 (a shard is cut into tiles below that)
 *   seeds per (query gene, subject sample) pass 2^22 */
#define RC_E_IO (-8)         /* file could not be written */

typedef struct rc_engine rc_engine;

/* Run options. Defaults (rc_default_opts) follow config.py:77-81. */
typedef struct rc_opts {
    int32_t top_matches;   /* N of highest_bitscores (config.py:77), >= 1 */
    int32_t keep_all;      /* keep ties (config.py:81); 0 = keep "first" */
    double evalue;         /* BLAST e-value cutoff (config.py:79) */
    int32_t word_size;     /* seed length W, 16..64 (megablast default 28) */
    int32_t xdrop_half;    /* greedy X-drop in half-score units (108 = 100 bits) */
    int32_t device;        /* HIP device ordinal */
    int32_t shard_rank;    /* rc_align() processes query genes of this shard */
    int32_t shard_count;   /* number of shards (1 = everything) */
    int32_t symmetric;     /* 0 (default): both directed searches of a pair run
                              independently, as BLAST runs them (find_homologs.py:
                              235-246); 1: spec 5b -- each pair extended once, the
                              higher sample's search reported as mirror images */
    int32_t dust_level;    /* symmetric DUST on the query words (blastn default
                              -dust 20 64 1); 0 = off */
    int32_t dust_window;
    int32_t dust_linker;
} rc_opts;

/* One HSP of a directed search, BLAST tabular semantics (1-based, inclusive;
 * qstart < qend; sstart > send on the minus strand). q_tx / s_tx are transcript
 * indices within their samples (input order). */
typedef struct rc_hsp {
    uint32_t q_tx, s_tx;
    int32_t qstart, qend, sstart, send;
    int32_t length, nident, mismatch, gaps, gapopen;
    int32_t score_half;    /* raw score x 2 (match 2, mismatch -4, gap -5) */
    int32_t bits10;        /* bit score as BLAST prints it, in tenths */
    int32_t strand;        /* 0 plus, 1 minus (sstrand) */
    double evalue;
} rc_hsp;

/* One row of a gene matches table (docs/formats.md:231-252) of pair (s1, s2):
 * qgene/qiso belong to s2 (`qsample`), sgene/siso to s1 (`ssample`). For
 * reverse rows the coordinates are those of the t1-query search, exactly as the
 * reference's column rename leaves them (find_homologs.py:248-255). */
typedef struct rc_row {
    int32_t qgene, qiso, sgene, siso;
    uint32_t q_tx, s_tx;   /* transcript indices (qgene's sample / sgene's) */
    int32_t reverse;
    int32_t label;         /* pandas index label the reference would keep */
    rc_hsp hsp;            /* q_tx/s_tx in hsp are those of the search row */
} rc_row;

typedef struct rc_stats {
    int64_t nodes;            /* vertices of the gene matches graph */
    int64_t edges;            /* distinct undirected edges */
    int64_t components;
    int64_t ideal_components;
    int64_t ideal_nodes;
    int32_t sample_count;     /* distinct samples among vertices (filtered_distance.py:171-182) */
    int32_t pad;
    int64_t hsps;             /* HSPs of all directed searches after the e-value cut */
    int64_t table_rows;       /* rows of all gene matches tables */
    int64_t seeds;            /* seeds (maximal exact runs >= W) of this engine's shard */
    int64_t candidates;       /* (query tx, strand, subject tx) with >= 1 seed */
} rc_stats;

typedef struct rc_edge {
    int32_t sample_a, gene_a, sample_b, gene_b;   /* sample_a < sample_b */
} rc_edge;

typedef struct rc_timing {
    double pack_ms, index_ms, align_ms, topn_ms, rbh_ms, graph_ms, reduce_ms, total_ms;
    double seed_kernel_ms;    /* device time of the seed kernel (lookups, seeds) */
    double align_kernel_ms;   /* device time of the extension kernel */
    double ext_steps;         /* greedy X-drop steps executed (wave-level) */
    double ext_calls;         /* greedy extensions (left + right per HSP attempt) */
    double ext_fullband;      /* candidates whose frontier left the row kernel's sub-band (extended whole
                                 by the one-wave full-band kernel; RC_ROW64=1: by 64-lane rows first) */
    double ext_deferred;      /* candidates the one-wave kernel took (sub-band exits, seeds outside the
                                 first HSP box, transcripts past the row staging slot) */
    double big_passes;        /* (query gene, subject sample) seed passes run from global memory */
    double tiles;             /* alignment passes (tiles) of this shard's samples */
    double dust_ms;           /* device time of DUST (on its own stream, beside the index build) */
    double band_bound;        /* extensions whose frontier reached the 64-diagonal band edge (spec 3) */
    double maxhsp_bound;      /* candidates with a seed outside their MAX_HSP (8) HSP boxes (spec 3) */
    double ext_second;        /* shared searches: candidates whose reverse search starts at another seed
                                 (a second first-seed extension) */
    double near_index;        /* shared searches with DUST: entries of the reverse pass's near-mask index */
    double reverse_seeds;     /* shared searches with DUST: reverse-search seeds only the reverse pass finds */
    double ext_slides;        /* row-kernel window slides (the sliding 32-diagonal sub-band) */
    double ext_wide;          /* first-seed extensions whose live diagonals outgrew the sliding sub-band,
                                 redone on 64-lane rows (the spec's whole band) */
    double dev_bytes;         /* device memory the engines of this process hold now (bytes) */
    double dev_peak_bytes;    /* ... and the most they held at once */
    double defer_length;      /* candidates with a transcript past the row kernels' staging slot */
    double defer_gaveup;      /* directed searches the one-wave kernel took because the row kernels gave
                                 up on their first seed (transcript length) */
    double defer_outside;     /* directed searches the one-wave kernel took because a seed lies outside
                                 their first HSP's box (more than one HSP) */
    double index_reused;      /* alignment tiles that reused the previous tile's 16-mer index and subject
                                 DUST masks (split tiles of one subject chunk) */
    double ext_retries;       /* extend_kernel reruns after the HSP overflow buffer overflowed (the buffer
                                 grows to fit; the row kernels' results are kept) */
    double load_ms;           /* host wall time loading alignment tiles (tile tables, working copy) */
    double align_wall_ms;     /* host wall time of rc_align (every tile, kernels and host work) */
    double host_wait_ms;      /* host wall time blocked on the engine's stream inside rc_align */
    double later_seeds;       /* later seeds of deferred searches extended on the row kernels (the
                                 later-seed rounds, one seed per search per round) */
    double later_whole;       /* deferred searches extend_kernel ran whole (a row kernel gave a seed up,
                                 or past the rounds' capacity, RC_LATER_CAP) */
} rc_timing;

void rc_default_opts(rc_opts *opts);

int rc_create(const rc_opts *opts, rc_engine **eng);
int rc_destroy(rc_engine *eng);
const char *rc_last_error(void);
/* Reset the process's device-memory peak (rc_timing.dev_peak_bytes) to what
 * its engines hold now, so that the next engine's own peak can be read. */
void rc_dev_peak_reset(void);

/* Add one sample: `seq` holds all transcripts concatenated (ASCII; A/C/G/T
 * any case, anything else is an ambiguous base), tx_offsets[n_tx + 1] their
 * boundaries; gene / iso the parsed TranscriptID fields (transcripts.py:60-126).
 * `label` is the sample string used in tables and matrix order.
 * seq == NULL (with tx_offsets, gene, iso as usual): a sample this engine does
 * not align -- in a sharded run, one no pair of this shard touches. Its
 * transcripts and genes still count (graph nodes, the e-value search space of
 * searches against it); its bases are not copied to the device. rc_align
 * fails with RC_E_STATE if a pair of this shard has such a sample. */
int rc_add_sample(rc_engine *eng, const char *label, const char *seq,
                  const uint64_t *tx_offsets, const int32_t *gene,
                  const int32_t *iso, uint32_t n_tx, int32_t *sample_id);

/* External-alignment mode: supply the HSPs of directed search
 * (query sample q, subject sample s) yourself -- e.g. real blastn output in
 * BLAST output order -- instead of running the GPU aligner. Either every
 * ordered pair gets rc_add_hsps (missing ones are empty) or none does. */
int rc_add_hsps(rc_engine *eng, int32_t q, int32_t s, const rc_hsp *hsps, uint64_t n);

/* Copy inputs to the device (done implicitly by rc_run); after this the inputs
 * are resident in HBM and rc_run repeats the whole path from them. */
int rc_upload(rc_engine *eng);

/* Phases. rc_run = rc_align + rc_finish (single shard).
 *
 * Sharded use (shard_count > 1, one engine per GPU, every engine given the
 * same samples in the same order -- with their sequences only where this
 * shard needs them, seq == NULL for the others; see rc_add_sample): the C(N,2)
 * sample pairs are cut by rc_plan_pairs into one rectangle [a0, a1) x [b0, b1)
 * of the pair triangle per shard, so a shard's resident samples are
 * [a0, a1) u [b0, b1) (rna_clique_amd.distributed.needed_samples); rc_align
 * runs seed-and-extend for this shard's pairs only (in alignment tiles of
 * < 2^32 bases when its samples do not fit one pass), and rc_finish the top-N and
 * reciprocal-best-hit step for them, producing this shard's gene matches
 * tables and graph edges. The gene matches graph and the ideal-clique filter
 * are global, so the edges are then exchanged (one all-gather) and every shard
 * passes the concatenation to rc_import_edges, which runs connected
 * components, the ideal filter and the pair sums over all edges. Tables
 * (rc_pair_rows) stay on the shard that owns the pair. */
int rc_run(rc_engine *eng);
int rc_align(rc_engine *eng);
int rc_finish(rc_engine *eng);

/* Edge records are opaque and fixed-size (rc_edge_record_size() bytes).
 * export: this shard's edges into a caller buffer (host or device pointer,
 * `on_device` says which; buf == NULL queries the count); import: all shards'
 * edges, concatenated in any order, then the graph phase. */
uint64_t rc_edge_record_size(void);
int rc_export_edges(rc_engine *eng, void *buf, uint64_t cap, uint64_t *n, int on_device);
int rc_import_edges(rc_engine *eng, const void *buf, uint64_t n, int on_device);
/* The same import from `parts` blocks: block r starts at record r * stride of
 * buf and holds counts[r] records (an all-gather's padded receive buffer, taken
 * as it is). Device records are range-checked on the device (RC_E_ARG). */
int rc_import_edge_parts(rc_engine *eng, const void *buf, const uint64_t *counts, int32_t parts, uint64_t stride,
                         int on_device);
/* Free the alignment working set of a finished run (tile copies, 16-mer
 * indexes, seeds, candidates, extension scratch) before the edge exchange;
 * rows, HSPs, edges and inputs stay, and the next rc_align allocates the rest
 * again. rc_dust_mask needs a new rc_align afterwards. */
int rc_trim(rc_engine *eng);
/* Graph-only mode (SampleSimilarity(graph, comparison_dfs), filtered_distance.py:
 * 162-169, and its from_filenames resume path :291-317): on a fresh engine
 * whose samples carry one zero-length transcript per gene (seq may be NULL),
 * rc_import_edges takes host records built by the caller -- rc_edge_record
 * below -- and runs components, the ideal filter, the sums and distances on
 * the GPU. Gene numbering: per sample in ascending gene id, sample-major. */
typedef struct rc_edge_record {
    uint32_t a, b;         /* global gene indices (a == b for an isolated node) */
    uint32_t pair;         /* pair index (rc_pair_order), | RC_EDGE_SUM_ONLY for table
                              rows whose edge is not in the graph, or RC_NODE_ONLY */
    int32_t nident;        /* sum of nident over the edge's table rows */
    int32_t den;           /* sum of length - gaps over them */
} rc_edge_record;
#define RC_EDGE_SUM_ONLY 0x80000000u
#define RC_NODE_ONLY 0x7FFFFFFFu
/* sample_count of the ideal-component test (0: distinct samples among the
 * graph's nodes, filtered_distance.py:171-182) */
int rc_set_sample_count(rc_engine *eng, int32_t sample_count);
/* This shard's sample-pair range [first, last) in the engine's pair order
 * (rc_pair_order). */
int rc_shard_pairs(rc_engine *eng, int64_t *first, int64_t *last);
/* The engine's pair numbering: pair p is (pair_a[p], pair_b[p]), a < b;
 * C(N,2) entries each. */
int rc_pair_order(rc_engine *eng, int32_t *pair_a, int32_t *pair_b);
/* The split itself (no device needed). Each shard takes one rectangle of the
 * (query a, subject b) pair triangle; pairs are numbered shard by shard,
 * subject-major inside a shard (one shard: (0,1), (0,2), (1,2), (0,3), ...).
 * pair_first[shard_count + 1]: shard r owns pairs [pair_first[r],
 * pair_first[r + 1]); pair_a/pair_b (C(N,2) entries, may be NULL) the order.
 * sample_bases = total bases of each sample's transcripts. */
int rc_plan_pairs(const int64_t *sample_bases, int32_t n_samples, int32_t shard_count, int32_t *pair_a,
                  int32_t *pair_b, int64_t *pair_first);
int rc_plan_shards(const int64_t *sample_bases, int32_t n_samples, int32_t shard_count, int64_t *pair_first);

/* Results (after rc_run / rc_finish). */
int rc_hsps(rc_engine *eng, int32_t q, int32_t s, rc_hsp *buf, uint64_t cap, uint64_t *n);
int rc_pair_rows(rc_engine *eng, int32_t s1, int32_t s2, rc_row *buf, uint64_t cap, uint64_t *n);
int rc_graph_stats(rc_engine *eng, rc_stats *stats);
int rc_edges(rc_engine *eng, rc_edge *buf, uint64_t cap, uint64_t *n);
int rc_ideal_nodes(rc_engine *eng, int32_t *sample, int32_t *gene, uint64_t cap, uint64_t *n);
/* num/den: n_samples x n_samples row-major (sample ids), 0 on the diagonal.
 * rc_pair_sums: rows restricted to ideal components (SampleSimilarity,
 * filtered_distance.py:234-247); rc_pair_sums_unfiltered: every row of the
 * pair's gene matches table (UnfilteredSimilarity, unfiltered_distance.py:9-16,
 * similarity_computer.py:21-42). */
int rc_pair_sums(rc_engine *eng, int64_t *num, int64_t *den);
int rc_pair_sums_unfiltered(rc_engine *eng, int64_t *num, int64_t *den);
/* order[n]: sample ids in output order; out: n x n row-major distances.
 * Returns RC_E_NO_IDEAL when some pair has no ideal rows. */
int rc_distance(rc_engine *eng, const int32_t *order, double *out);
/* The same for n distinct samples: order[n], out n x n (the matrix of the
 * samples a SampleSimilarity built from tables knows, filtered_distance.py:
 * 162-169 / similarity_computer.py:216-226: samples = the tables' keys). */
int rc_distance_subset(rc_engine *eng, const int32_t *order, int32_t n, double *out);
int rc_timings(rc_engine *eng, rc_timing *t);
/* The DUST mask of sample `s` after rc_run / rc_align: one byte per base of
 * its concatenated transcripts (1 = masked query base, spec 1b of the oracle);
 * all zero when DUST is off. buf == NULL queries the size. */
int rc_dust_mask(rc_engine *eng, int32_t s, uint8_t *buf, uint64_t cap, uint64_t *n);
/* DUST masks shared across shards (each sample masked once, on one rank that
 * holds it; the rest of the query-side DUST of TabularBlastnSearch's blastn
 * -dust default, find_homologs.py:124, is then a copy). Layout: the listed
 * samples in order, ceil(bases / 64) uint64 words each; bit b of word w =
 * base 64 w + b of the sample's concatenated transcripts (1 = masked); bits
 * past its last base 0.
 * rc_dust_masks: the masks of resident samples, computed in a pass of their
 * own; out == NULL queries n_words. `on_device`: out is a device pointer.
 * Results of an earlier rc_align / rc_finish stay valid (they do not depend
 * on the loaded tile's tables); rc_dust_mask then reads this pass's tile and
 * fails with RC_E_STATE when the pass used a tile of its own, or -- a pass
 * over the loaded tile itself -- for a sample the pass did not list (its mask
 * was cleared; the next rc_align / rc_run masks every sample again).
 * rc_set_dust_masks: masks for these samples (replacing any given before;
 * n = 0 clears them): rc_align copies them into its tiles instead of running
 * DUST on those samples. They must come from engines with the same DUST
 * options. */
int rc_dust_masks(rc_engine *eng, const int32_t *samples, int32_t n, uint64_t *out, uint64_t cap_words,
                  uint64_t *n_words, int on_device);
int rc_set_dust_masks(rc_engine *eng, const int32_t *samples, int32_t n, const uint64_t *bits, uint64_t n_words,
                      int on_device);

/* ---- outputs next to matrix.h5 (od2 tables, graph.pkl) -------------------
 * rc_write_outputs: the gene matches table files of pairs (s1[i], s2[i]) at
 * table_paths[i] (pandas table format, key "gene_matches": write_table,
 * gene_matches_tables.py:42-56; NULL = none) and graph.pkl at graph_path
 * (build_graph over the pairs in the given order + pickle.dump, build_graph.py:
 * 40-68, filtering_step.py:158-159; NULL = none; single-shard engines), each
 * pair's rows fetched once, the files written by `threads` host threads.
 * rc_table_write_rows: one table file from rc_row records (host only). */
int rc_write_outputs(rc_engine *eng, int32_t n_pairs, const int32_t *s1, const int32_t *s2,
                     const char *const *table_paths, const char *graph_path, int32_t threads);
int rc_table_write_rows(const rc_row *rows, uint64_t n, const char *ssample, const char *qsample, const char *path);
/* graph.pkl from the engine's graph edges (every pair, in combinations
 * order: build_graph.py:40-68 over the tables of find_all_pairs' pairs; node
 * and neighbour order included) -- a single-shard engine after rc_run, a
 * sharded one after rc_import_edges. The records are sorted on the device;
 * `threads` host threads build the pickle. RC_E_STATE for an imported graph
 * with isolated nodes or rows outside the graph. */
int rc_write_graph(rc_engine *eng, const char *path, int32_t threads);

/* ---- FASTA input (host only; fasta.cpp) ----------------------------------
 * Replaces the Bio.SeqIO passes of TopGeneSelector (select_top_genes.py:108-127)
 * and the Bio.SeqIO.write of select_top_and_save (select_top_genes_all.py:12-46).
 * A title is the header line without '>' and trailing whitespace; a sequence is
 * the record's lines right-stripped and joined, ' ' and '\r' removed. `keep`
 * (one byte per record, NULL = all) selects records for select/write. */
typedef struct rc_fasta rc_fasta;
int rc_fasta_open(const char *path, rc_fasta **out);
int rc_fasta_close(rc_fasta *f);
int rc_fasta_info(const rc_fasta *f, uint64_t *n_records, uint64_t *n_bases, uint64_t *title_bytes);
/* titles concatenated into buf (title_bytes), offsets[n_records + 1];
 * seq_lens[n_records] (may be NULL) */
int rc_fasta_titles(const rc_fasta *f, char *buf, uint64_t *offsets, uint64_t *seq_lens);
/* (coverage, gene, isoform) of every record under the default rnaSPAdes id
 * pattern (transcripts.py:8 of the reference, matched as re.search does);
 * records it cannot decide (non-ASCII title, no match, > 18 digits) count in
 * n_undecided -- the caller then parses the ids with the regex itself */
int rc_fasta_parse_rnaspades(const rc_fasta *f, double *cov, int64_t *gene, int64_t *iso, uint64_t *n_undecided);
/* selected sequences concatenated into seq; tx_offsets[n_selected + 1] */
int rc_fasta_select(const rc_fasta *f, const uint8_t *keep, uint8_t *seq, uint64_t *tx_offsets);
/* selected records as Bio.SeqIO.write(..., "fasta") writes them (width 60) */
int rc_fasta_write(const rc_fasta *f, const uint8_t *keep, const char *path, int32_t width);

/* ---- graph.pkl (host only; graph_pickle.cpp) -------------------------------
 * Replaces build_graph + pickle.dump (build_graph.py:40-68, filtering_step.py:
 * 158-159): the tables are added in order (per table: sample indices of
 * ssample and qsample, the sgene and qgene columns), then the pickle of the
 * networkx Graph build_graph would make from them is written to `path`
 * (protocol 4; nodes are (names[sample], gene) tuples; node, neighbour and
 * edge order as build_graph inserts them). */
typedef struct rc_gpickle rc_gpickle;
int rc_graph_pickle_begin(rc_gpickle **out);
int rc_graph_pickle_add(rc_gpickle *g, int32_t ssample, int32_t qsample, const int64_t *sgene, const int64_t *qgene,
                        uint64_t n);
int rc_graph_pickle_write(rc_gpickle *g, const char *path, int32_t n_names, const char *const *names);
void rc_graph_pickle_free(rc_gpickle *g);

#ifdef __cplusplus
}
#endif
#endif /* RCGPU_H */

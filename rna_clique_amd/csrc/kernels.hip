// HIP kernels of the MI355X RNA-clique engine (gfx950, wave64).
//
// Pipeline (one rc_run):
//   pack_fwd / pack_rc      ASCII -> 2-bit packed forward + reverse complement
//   kmer_fill + radix sort  16-mer seed index over every sample at once
//   bucket_fill             direct-address bucket table over the sorted keys
//   align_kernel            per query gene: stride lookups, canonical seeds,
//                           wave-parallel greedy X-drop, HSPs per subject sample
//   rbh_kernel (2 passes)   top-N, reciprocal best hits, gene matches rows, edges
//   cc_* kernels            union-find components, ideal-clique test
//   pair_sums / distance    restricted sums and the N x N matrix
//
// The exact semantics are those of oracle/align_oracle.c (alignment) and
// oracle/post_oracle.py (post-alignment, pinned to the reference).
#include "device.h"

#include <algorithm>
#include <climits>

namespace rcg {

// ------------------------------------------------------------------------
// pack
// ------------------------------------------------------------------------

// One thread per 64-bit word (32 bases): 32 input bytes as two 16-B loads,
// coded four bytes at a time in registers. The 2-bit code of A/C/G/T (either
// case) is ((c >> 1) ^ (c >> 2)) & 3 (A 0, C 1, G 2, T 3); any other byte is
// ambiguous (mask 3, code 0).
__global__ void pack_fwd_kernel(const uint8_t *__restrict__ ascii, uint64_t total, uint64_t nwords,
                                uint64_t *__restrict__ F, uint64_t *__restrict__ AF)
{
    for (uint64_t w = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; w < nwords;
         w += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t p0 = w * 32;
        uint32_t d[8];
        if (p0 + 32 <= total) {
            const uint4 *v = reinterpret_cast<const uint4 *>(ascii + p0);
            const uint4 x0 = v[0], x1 = v[1];
            d[0] = x0.x; d[1] = x0.y; d[2] = x0.z; d[3] = x0.w;
            d[4] = x1.x; d[5] = x1.y; d[6] = x1.z; d[7] = x1.w;
        } else {
#pragma unroll
            for (int j = 0; j < 8; j++) {
                uint32_t x = 0;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const uint64_t p = p0 + 4 * j + k;
                    x |= (uint32_t)(p < total ? ascii[p] : (uint8_t)'A') << (8 * k);
                }
                d[j] = x;
            }
        }
        uint64_t word = 0, amb = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint32_t t = (d[j] >> 1) ^ (d[j] >> 2);
#pragma unroll
            for (int k = 0; k < 4; k++) word |= (uint64_t)((t >> (8 * k)) & 3u) << (8 * j + 2 * k);
        }
        if (AF) {
#pragma unroll
            for (int j = 0; j < 8; j++)
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const uint32_t l = ((d[j] >> (8 * k)) & 0xFFu) | 0x20u;
                    const bool ok = l == 'a' || l == 'c' || l == 'g' || l == 't';
                    amb |= (uint64_t)(ok ? 0u : 3u) << (8 * j + 2 * k);
                }
            word &= ~amb;   // ambiguous bases code as 0
        }
        if (p0 + 32 > total) {
            const uint64_t keep = (1ull << (2 * (total - p0))) - 1ull;   // total - p0 < 32
            word &= keep;
            amb &= keep;
        }
        F[w] = word;
        if (AF) AF[w] = amb;
    }
}

// RC word w = reverse complement of the forward window ending at total - 32w.
__global__ void pack_rc_kernel(const uint64_t *__restrict__ F, const uint64_t *__restrict__ AF,
                               uint64_t total, uint64_t nwords, uint64_t *__restrict__ RC,
                               uint64_t *__restrict__ ARC)
{
    for (uint64_t w = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; w < nwords;
         w += (uint64_t)gridDim.x * blockDim.x) {
        const int64_t lo = (int64_t)total - 32 * (int64_t)(w + 1);
        uint64_t x, ax = 0;
        if (lo >= 0) {
            x = win(F, (uint64_t)lo);
            if (AF) ax = win(AF, (uint64_t)lo);
        } else if (lo > -32) {
            x = win(F, 0) << (2 * (unsigned)(-lo));
            if (AF) ax = win(AF, 0) << (2 * (unsigned)(-lo));
        } else {
            x = 0;
        }
        RC[w] = ~rev2(x);
        if (ARC) ARC[w] = rev2(ax);
    }
}

// ------------------------------------------------------------------------
// seed index
// ------------------------------------------------------------------------

// Valid 16-mer windows per transcript (only used when ambiguous bases exist).
__global__ void kmer_count_kernel(const TxInfo *__restrict__ tx, uint32_t n_tx,
                                  const uint64_t *__restrict__ AF, uint64_t *__restrict__ cnt)
{
    const uint32_t t = blockIdx.x;
    if (t >= n_tx) return;
    const TxInfo ti = tx[t];
    __shared__ unsigned long long s;
    if (threadIdx.x == 0) s = 0;
    __syncthreads();
    unsigned long long c = 0;
    for (int64_t o = threadIdx.x; o + W16 <= (int64_t)ti.len; o += blockDim.x)
        if ((win(AF, ti.start + o) & 0xFFFFFFFFull) == 0) c++;
    atomicAdd(&s, c);
    __syncthreads();
    if (threadIdx.x == 0) cnt[t] = s;
}

// One wave per transcript, grid-stride over the transcripts (a block per
// transcript spent more time in dispatch than in its stores, and slowed DUST
// beside it); windows in (gtx, offset) order so that a stable radix sort on
// the key keeps each key's entries sorted by (gtx, offset). AMB: windows with
// an ambiguous base are left out (compacted within the wave).
template <bool AMB>
__global__ __launch_bounds__(256) void kmer_fill_kernel(const TxInfo *__restrict__ tx, uint32_t n_tx,
                                                        const uint64_t *__restrict__ F,
                                                        const uint64_t *__restrict__ AF,
                                                        const uint64_t *__restrict__ out_off,
                                                        uint64_t *__restrict__ ent)
{
    const int lane = threadIdx.x & 63;
    const uint32_t nwave = gridDim.x * 4u;
    for (uint32_t t = blockIdx.x * 4u + (threadIdx.x >> 6); t < n_tx; t += nwave) {
        const TxInfo ti = tx[t];
        const int64_t nwin = (int64_t)ti.len - W16 + 1;
        uint64_t base = out_off[t];
        for (int64_t o0 = 0; o0 < nwin; o0 += 64) {
            const int64_t o = o0 + lane;
            bool ok = o < nwin;
            const uint64_t p = ti.start + (uint64_t)o;
            const uint32_t key = ok ? (uint32_t)win(F, p) : 0u;
            if (!AMB) {
                if (ok) ent[base + (uint64_t)o] = ((uint64_t)key << 32) | p;
            } else {
                if (ok) ok = (win(AF, p) & 0xFFFFFFFFull) == 0;
                const uint64_t m = __ballot(ok);
                if (ok) ent[base + (uint64_t)__popcll(m & ((1ull << lane) - 1ull))] = ((uint64_t)key << 32) | p;
                base += (uint64_t)__popcll(m);
            }
        }
    }
}

// bucket[b] = first sorted index whose key >> (32 - bits) >= b, b in [0, 2^bits].
// bucket[x] = first entry whose top `bits` k-mer bits are >= x (x = 0 .. 2^bits).
// Each thread owns BF_PER consecutive entries: one wide load of its own
// entries (plus the one before) with every load in flight at once, then the
// bucket slots from the previous entry's bucket (exclusive) to each entry's.
constexpr int BF_PER = 4;
constexpr uint32_t FILL_BLOCKS = 256 * 8;   // grid of the wave-per-transcript fill kernels
__global__ __launch_bounds__(256) void bucket_fill_kernel(const uint64_t *__restrict__ ent, uint64_t n, int bits,
                                                          uint32_t *__restrict__ bucket)
{
    const unsigned sh = 64u - (unsigned)bits;
    const uint64_t nb = 1ull << bits;
    const uint64_t i0 = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) * BF_PER;
    if (i0 > n) return;
    uint64_t e[BF_PER + 1];
    e[0] = i0 > 0 ? ent[i0 - 1] : 0ull;
    if (i0 + BF_PER <= n) {
        const ulonglong2 *v = reinterpret_cast<const ulonglong2 *>(ent + i0);
#pragma unroll
        for (int j = 0; j < BF_PER / 2; j++) {
            const ulonglong2 w = v[j];
            e[1 + 2 * j] = w.x;
            e[2 + 2 * j] = w.y;
        }
    } else {
#pragma unroll
        for (int j = 0; j < BF_PER; j++) e[1 + j] = i0 + j < n ? ent[i0 + j] : 0ull;
    }
#pragma unroll
    for (int j = 0; j < BF_PER; j++) {
        const uint64_t i = i0 + j;
        if (i > n) break;
        const uint64_t lo = i > 0 ? (e[j] >> sh) + 1 : 0;
        const uint64_t hi = i < n ? (e[j + 1] >> sh) : nb;
        for (uint64_t x = lo; x <= hi; x++) bucket[x] = (uint32_t)i;
    }
}

// ------------------------------------------------------------------------
// reciprocal best hits -> gene matches rows and edges (find_homologs.py:215-302)
// ------------------------------------------------------------------------



// the RBH kernel's view of the group table: each HSP's bit score and its
// subject transcript's gene (8 bytes instead of the 56-byte record and a
// transcript -> gene gather in every selection loop)
__global__ void hkey_kernel(const DHsp *__restrict__ h, uint64_t n, const uint32_t *__restrict__ tx_gene,
                            HKey *__restrict__ out)
{
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        HKey k;
        k.bits10 = h[i].bits10;
        k.gene = tx_gene[h[i].s_tx];
        out[i] = k;
    }
}
void launch_hkey(const DHsp *h, uint64_t n, const uint32_t *tx_gene, HKey *out, hipStream_t st)
{
    if (!n) return;
    const uint64_t g = std::min<uint64_t>((n + 255) / 256, 65536);
    hipLaunchKernelGGL(hkey_kernel, dim3((unsigned)g), dim3(256), 0, st, h, n, tx_gene, out);
}

// threshold of highest_bitscores(n, keep="all") over one group's bitscores
__device__ __forceinline__ int group_thr(const HKey *h, uint32_t off, uint32_t cnt, int n)
{
    if (cnt == 0) return INT_MAX;
    if ((int)cnt <= n) {
        int m = INT_MAX;
        for (uint32_t i = 0; i < cnt; i++) m = min(m, h[off + i].bits10);
        return m;
    }
    // n-th largest value counting duplicates
    int prev = INT_MAX, taken = 0;
    while (true) {
        int v = INT_MIN, c = 0;
        for (uint32_t i = 0; i < cnt; i++) {
            const int b = h[off + i].bits10;
            if (b < prev && b > v) v = b, c = 0;
            if (b == v) c++;
        }
        taken += c;
        if (taken >= n) return v;
        prev = v;
    }
}

// rank of element i among a group in (bits desc, index asc) order, restricted by pred
template <typename Pred>
__device__ __forceinline__ uint32_t desc_rank(const HKey *h, uint32_t off, uint32_t cnt, uint32_t i, Pred pred)
{
    const int bi = h[off + i].bits10;
    uint32_t r = 0;
    for (uint32_t j = 0; j < cnt; j++)
        if (j != i && pred(j)) {
            const int bj = h[off + j].bits10;
            if (bj > bi || (bj == bi && j < i)) r++;
        }
    return r;
}

// pass 0: per-item counts; pass 1: rows and edges at the scanned offsets;
// pass 2: counts plus rows and edges in per-item slots with item-local labels
// (rbh_place_kernel finishes them) -- one pass over the groups instead of two.
__global__ void rbh_kernel(RbhParams P, int pass)
{
    const bool tmp = pass == 2;
    // items [item0, item0 + n_items) of this shard; per-item arrays are local.
    // The pair of an item: one binary search per block (its first item), then
    // a short walk (a block's 256 items span one or two pairs)
    __shared__ int sh_pair;
    for (uint64_t lb = blockIdx.x * (uint64_t)blockDim.x; lb < P.n_items; lb += (uint64_t)gridDim.x * blockDim.x) {
        __syncthreads();
        if (threadIdx.x == 0) {
            const uint64_t item0 = P.item0 + lb;
            int lo = 0, hi = P.n_pairs;
            while (hi - lo > 1) {
                const int mid = (lo + hi) >> 1;
                if (P.pair_item_begin[mid] <= item0) lo = mid; else hi = mid;
            }
            sh_pair = lo;
        }
        __syncthreads();
        const uint64_t li = lb + threadIdx.x;
        if (li >= P.n_items) continue;
        const uint64_t item = P.item0 + li;
        int pr = sh_pair;
        while (pr + 1 < P.n_pairs && P.pair_item_begin[pr + 1] <= item) pr++;
        const int A = P.pair_a[pr], B = P.pair_b[pr];
        const uint32_t b = P.sample_gene_begin[B] + (uint32_t)(item - P.pair_item_begin[pr]);
        const int N = P.N;
        const size_t fgi = grp_index(b, A, P.n_genes);
        const uint32_t foff = P.grp_off[fgi], fcnt = P.grp_cnt[fgi];
        // the groups' bit scores and subject genes, 8 bytes an HSP (hkey_kernel;
        // the 56-byte records are read for the rows that make edges only)
        const HKey *H = P.hk;
        const DHsp *HF = P.hsp;
        const int fthr = group_thr(H, foff, fcnt, P.top_n);
        // per F_top row: R-existence of its pair
        uint32_t fsel = 0, rsel = 0, nrows = 0, nedges = 0;
        int M = INT_MIN;
        // pass over F_top rows: compute M and counts
        for (uint32_t i = 0; i < fcnt; i++) {
            const HKey &f = H[foff + i];
            if (f.bits10 < fthr) continue;
            const uint32_t a = f.gene;
            const size_t rgi = grp_index(a, B, P.n_genes);
            const uint32_t roff = P.grp_off[rgi], rcnt = P.grp_cnt[rgi];
            const int rthr = group_thr(H, roff, rcnt, P.top_n);
            bool inP = false;
            for (uint32_t j = 0; j < rcnt; j++) {
                const HKey &r = H[roff + j];
                if (r.bits10 >= rthr && r.gene == b) {
                    inP = true;
                    break;
                }
            }
            if (!inP) continue;
            fsel++;
            M = max(M, f.bits10);
            // first F_top row of this pair?
            bool first = true;
            for (uint32_t i2 = 0; i2 < i; i2++) {
                const HKey &f2 = H[foff + i2];
                if (f2.bits10 >= fthr && f2.gene == a) {
                    first = false;
                    break;
                }
            }
            if (!first) continue;
            for (uint32_t j = 0; j < rcnt; j++) {
                const HKey &r = H[roff + j];
                if (r.bits10 >= rthr && r.gene == b) {
                    rsel++;
                    M = max(M, r.bits10);
                }
            }
        }
        // final rows: rows of C at M; pairs in ascending a; F rows then R rows
        // (keep "first": only the first such row)
        uint32_t prev_a = 0;
        bool have_prev = false, done = false;
        const bool fin = pass == 1;
        uint64_t row_w = fin ? P.row_off[li] : 0, edge_w = fin ? P.edge_off[li] : 0;
        const uint64_t fsel_base = fin ? P.fsel_off[li] - P.fsel_off[P.pair_item_begin[pr] - P.item0] : 0;
        const uint64_t fsel_pair_total =
            fin ? P.fsel_off[P.pair_item_begin[pr + 1] - P.item0] - P.fsel_off[P.pair_item_begin[pr] - P.item0] : 0;
        const uint64_t rsel_base = fin ? P.rsel_off[li] - P.rsel_off[P.pair_item_begin[pr] - P.item0] : 0;
        auto put_row = [&](const DRow &row) {
            if (!tmp) P.rows[row_w] = row;
            else if (row_w < (uint64_t)RBH_RMAX) P.rows_tmp[li * RBH_RMAX + row_w] = row;
            else atomicOr(P.ovf, 1u);
            row_w++;
        };
        while (fsel && !done) {
            // next smallest a among selected F rows
            bool found = false;
            uint32_t a = 0;
            for (uint32_t i = 0; i < fcnt; i++) {
                const HKey &f = H[foff + i];
                if (f.bits10 < fthr) continue;
                const uint32_t ai = f.gene;
                if (have_prev && ai <= prev_a) continue;
                if (!found || ai < a) a = ai, found = true;
            }
            if (!found) break;
            prev_a = a;
            have_prev = true;
            const size_t rgi = grp_index(a, B, P.n_genes);
            const uint32_t roff = P.grp_off[rgi], rcnt = P.grp_cnt[rgi];
            const int rthr = group_thr(H, roff, rcnt, P.top_n);
            auto r_sel = [&](uint32_t j) {
                const HKey &r = H[roff + j];
                return r.bits10 >= rthr && r.gene == b;
            };
            bool inP = false;
            for (uint32_t j = 0; j < rcnt; j++)
                if (r_sel(j)) {
                    inP = true;
                    break;
                }
            if (!inP) continue;
            int en = 0, ed = 0, erows = 0;
            // F rows of this pair at M
            for (uint32_t i = 0; i < fcnt && !done; i++) {
                const HKey &f = H[foff + i];
                if (f.bits10 < fthr || f.gene != a || f.bits10 != M) continue;
                if (pass) {
                    // label: rank among F_sel rows of b in F_top order + earlier genes
                    const uint32_t rk = desc_rank(H, foff, fcnt, i, [&](uint32_t j) {
                        const HKey &f2 = H[foff + j];
                        if (f2.bits10 < fthr) return false;
                        const uint32_t a2 = f2.gene;
                        const size_t g2 = grp_index(a2, B, P.n_genes);
                        const uint32_t o2 = P.grp_off[g2], c2 = P.grp_cnt[g2];
                        const int t2 = group_thr(H, o2, c2, P.top_n);
                        for (uint32_t k2 = 0; k2 < c2; k2++)
                            if (H[o2 + k2].bits10 >= t2 && H[o2 + k2].gene == b) return true;
                        return false;
                    });
                    DRow row;
                    row.hsp = foff + i;
                    row.reverse = 0;
                    row.label = (int32_t)(fsel_base + rk);
                    row.pad = 0;
                    put_row(row);
                }
                en += HF[foff + i].nident;
                ed += HF[foff + i].length - HF[foff + i].gaps;
                erows++;
                if (!P.keep_all) done = true;
            }
            // R rows of this pair at M. R_sel order: pairs by the first
            // appearance of their F rows in F_top order (bits desc, index
            // asc), then R_top order; `before` = the R_sel rows of the pairs
            // whose first F_top row precedes this pair's (the same for every
            // R row of the pair: computed once, by direct (bits, index)
            // comparisons -- O(fcnt^2) per pair, not a rank per comparison)
            auto precedes = [&](uint32_t x, uint32_t y) {
                const int bx = H[foff + x].bits10, by = H[foff + y].bits10;
                return bx > by || (bx == by && x < y);
            };
            uint64_t before = 0;
            bool have_before = false;
            for (uint32_t j = 0; j < rcnt && !done; j++) {
                if (!r_sel(j) || H[roff + j].bits10 != M) continue;
                const HKey &r = H[roff + j];
                if (pass) {
                    if (!have_before) {
                        have_before = true;
                        uint32_t afirst = 0xFFFFFFFFu;   // this pair's first F_top row
                        for (uint32_t i = 0; i < fcnt; i++)
                            if (H[foff + i].bits10 >= fthr && H[foff + i].gene == a &&
                                (afirst == 0xFFFFFFFFu || precedes(i, afirst)))
                                afirst = i;
                        for (uint32_t i = 0; i < fcnt; i++) {
                            const HKey &f = H[foff + i];
                            if (f.bits10 < fthr) continue;
                            const uint32_t a2 = f.gene;
                            if (a2 == a || precedes(afirst, i)) continue;
                            // is f the first F_top row of pair a2?
                            bool firstrow = true;
                            for (uint32_t i2 = 0; i2 < fcnt && firstrow; i2++)
                                if (i2 != i && H[foff + i2].bits10 >= fthr && H[foff + i2].gene == a2 &&
                                    precedes(i2, i))
                                    firstrow = false;
                            if (!firstrow) continue;
                            const size_t g2 = grp_index(a2, B, P.n_genes);
                            const uint32_t o2 = P.grp_off[g2], c2 = P.grp_cnt[g2];
                            const int t2 = group_thr(H, o2, c2, P.top_n);
                            for (uint32_t k2 = 0; k2 < c2; k2++)
                                if (H[o2 + k2].bits10 >= t2 && H[o2 + k2].gene == b) before++;
                        }
                    }
                    const uint32_t rk = desc_rank(H, roff, rcnt, j, r_sel);
                    DRow row;
                    row.hsp = roff + j;
                    row.reverse = 1;
                    row.label = (int32_t)(fsel_pair_total + rsel_base + before + rk);
                    row.pad = 0;
                    put_row(row);
                }
                en += HF[roff + j].nident;
                ed += HF[roff + j].length - HF[roff + j].gaps;
                erows++;
                if (!P.keep_all) done = true;
            }
            if (erows) {
                nrows += erows;
                if (pass) {
                    DEdge e;
                    e.a = a;
                    e.b = b;
                    e.pair = (uint32_t)pr;
                    e.nident = en;
                    e.den = ed;
                    if (!tmp) P.edges[edge_w] = e;
                    else if (edge_w < (uint64_t)RBH_EMAX) P.edges_tmp[li * RBH_EMAX + edge_w] = e;
                    else atomicOr(P.ovf, 1u);
                    edge_w++;
                }
                nedges++;
            }
        }
        if (pass != 1) {
            P.n_rows[li] = nrows;
            P.n_fsel[li] = fsel;
            P.n_rsel[li] = rsel;
            P.n_edges[li] = nedges;
        }
    }
}

// ------------------------------------------------------------------------
// graph: union-find components and the ideal-clique test
// ------------------------------------------------------------------------

__device__ __forceinline__ uint32_t uf_find(uint32_t *parent, uint32_t x)
{
    uint32_t curr = parent[x];
    if (curr != x) {
        uint32_t next, prev = x;
        while (curr > (next = parent[curr])) {
            parent[prev] = next;
            prev = curr;
            curr = next;
        }
    }
    return curr;
}

__global__ void cc_init_kernel(uint32_t *parent, uint32_t *present, uint32_t *cnodes, uint32_t *cedges,
                               uint32_t n)
{
    for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < n; v += gridDim.x * blockDim.x) {
        parent[v] = v;
        present[v] = 0;
        cnodes[v] = 0;
        cedges[v] = 0;
    }
}

__global__ void cc_hook_kernel(const DEdge *edges, uint64_t n_edges, uint32_t *parent, uint32_t *present)
{
    for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < n_edges;
         e += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t u = edges[e].a, v = edges[e].b;
        if (edges[e].pair & EDGE_SUM_ONLY) continue;   // a table row whose edge is not in the graph
        present[u] = 1;
        present[v] = 1;
        uint32_t ru = uf_find(parent, u), rv = uf_find(parent, v);
        bool repeat;
        do {
            repeat = false;
            if (ru != rv) {
                uint32_t ret;
                if (ru < rv) {
                    if ((ret = atomicCAS(&parent[rv], rv, ru)) != rv) {
                        rv = ret;
                        repeat = true;
                    }
                } else {
                    if ((ret = atomicCAS(&parent[ru], ru, rv)) != ru) {
                        ru = ret;
                        repeat = true;
                    }
                }
            }
        } while (repeat);
    }
}

__global__ void cc_compress_kernel(uint32_t *parent, uint32_t n)
{
    for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < n; v += gridDim.x * blockDim.x) {
        uint32_t p = parent[v];
        while (p != parent[p]) p = parent[p];
        parent[v] = p;
    }
}

__global__ void cc_count_kernel(const DEdge *edges, uint64_t n_edges, const uint32_t *parent,
                                const uint32_t *present, const int32_t *gene_sample, uint32_t n,
                                uint32_t *cnodes, uint32_t *cedges, uint32_t *sample_present)
{
    const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const uint64_t nt = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t e = tid; e < n_edges; e += nt) {
        const DEdge ed = edges[e];
        if (ed.a != ed.b && !(ed.pair & EDGE_SUM_ONLY)) atomicAdd(&cedges[parent[ed.a]], 1u);   // graph edges only
    }
    for (uint64_t v = tid; v < n; v += nt)
        if (present[v]) {
            atomicAdd(&cnodes[parent[v]], 1u);
            sample_present[gene_sample[v]] = 1;
        }
}

// sum of a per-thread value over the block, one atomic per block
__device__ __forceinline__ void block_atomic_add(unsigned long long *dst, unsigned long long v)
{
    __shared__ unsigned long long part[16];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    __syncthreads();
    if (lane == 0) part[wid] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long s = 0;
        for (int i = 0; i < (int)(blockDim.x >> 6); i++) s += part[i];
        if (s) atomicAdd(dst, s);
    }
}

// stats[0] components, [1] ideal components, [2] ideal nodes, [3] nodes, [4] sample_count
__global__ void cc_ideal_kernel(const uint32_t *parent, const uint32_t *present, const uint32_t *cnodes,
                                const uint32_t *cedges, uint32_t n, const uint32_t *sample_present, int N,
                                int S_given, uint8_t *ideal, unsigned long long *stats)
{
    __shared__ int S;
    if (threadIdx.x == 0) {
        int s = 0;
        for (int i = 0; i < N; i++) s += sample_present[i] ? 1 : 0;
        if (S_given > 0) s = S_given;   // SampleSimilarity(..., sample_count=S)
        S = s;
        if (blockIdx.x == 0) stats[4] = (unsigned long long)s;
    }
    __syncthreads();
    unsigned long long comps = 0, ic = 0, inodes = 0, nodes = 0;
    for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < n; v += gridDim.x * blockDim.x) {
        uint8_t id = 0;
        if (present[v]) nodes++;
        if (parent[v] == v && present[v]) {
            comps++;
            const uint64_t nv = cnodes[v], ne = cedges[v];
            if ((int64_t)nv == S && 2 * ne == nv * (nv - 1)) {
                id = 1;
                ic++;
                inodes += nv;
            }
        }
        ideal[v] = id;
    }
    block_atomic_add(&stats[0], comps);
    block_atomic_add(&stats[1], ic);
    block_atomic_add(&stats[2], inodes);
    block_atomic_add(&stats[3], nodes);
}

// restricted sums per pair (filtered_distance.py:66-124 + similarity_computer.py:37-41)
__global__ void pair_sums_kernel(const DEdge *edges, uint64_t n_edges, const uint32_t *parent,
                                 const uint8_t *ideal, unsigned long long *num, unsigned long long *den,
                                 unsigned long long *num_all, unsigned long long *den_all)
{
    // Restricted sums (edges inside ideal components: SampleSimilarity,
    // filtered_distance.py:234-247) and unfiltered sums (every edge:
    // UnfilteredSimilarity, unfiltered_distance.py:9-16). Edges are stored
    // pair-major, so a wave usually sees one pair: reduce in registers and
    // issue one atomic per sum per wave; mixed waves fall back to lanes.
    const uint64_t nt = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t start = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const uint64_t iters = (n_edges + nt - 1) / nt;
    for (uint64_t it = 0; it < iters; it++) {
        const uint64_t e = start + it * nt;
        uint32_t pair = 0xFFFFFFFFu;
        unsigned long long a = 0, b = 0, ua = 0, ub = 0;
        if (e < n_edges && edges[e].pair != NODE_REC) {
            const DEdge ed = edges[e];
            pair = ed.pair & ~EDGE_SUM_ONLY;
            ua = (unsigned long long)ed.nident;
            ub = (unsigned long long)ed.den;
            // both endpoints in ideal components (restrict_multi,
            // filtered_distance.py:66-124); a graph edge's are in one
            if (ideal[parent[ed.a]] && ideal[parent[ed.b]]) {
                a = ua;
                b = ub;
            }
        }
        const uint32_t p0 = __shfl(pair, 0);
        if (__ballot(pair != p0 && pair != 0xFFFFFFFFu) == 0) {
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) {
                a += __shfl_xor(a, off);
                b += __shfl_xor(b, off);
                ua += __shfl_xor(ua, off);
                ub += __shfl_xor(ub, off);
            }
            if ((threadIdx.x & 63) == 0 && p0 != 0xFFFFFFFFu) {
                if (a || b) {
                    atomicAdd(&num[p0], a);
                    atomicAdd(&den[p0], b);
                }
                if (ua || ub) {
                    atomicAdd(&num_all[p0], ua);
                    atomicAdd(&den_all[p0], ub);
                }
            }
        } else if (pair != 0xFFFFFFFFu) {
            if (a || b) {
                atomicAdd(&num[pair], a);
                atomicAdd(&den[pair], b);
            }
            if (ua || ub) {
                atomicAdd(&num_all[pair], ua);
                atomicAdd(&den_all[pair], ub);
            }
        }
    }
}

// d = float(1 - Fraction(num, den)) = correctly rounded (den - num) / den
__global__ void distance_kernel(const unsigned long long *num, const unsigned long long *den,
                                const int32_t *pair_index, const int32_t *order, int N, int M, double *out,
                                unsigned int *status)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= M * M) return;
    const int i = t / M, j = t % M;
    const int a = order[i], b = order[j];
    if (a == b) {
        out[t] = 0.0;
        return;
    }
    const int p = pair_index[a * N + b];
    const unsigned long long dn = den[p], nm = num[p];
    if (dn == 0) {
        out[t] = __builtin_nan("");
        atomicOr(status, 4u);
        return;
    }
    out[t] = (double)(long long)(dn - nm) / (double)(long long)dn;
}

// ------------------------------------------------------------------------
// launchers (host side)
// ------------------------------------------------------------------------

static inline unsigned grid_for(uint64_t n, unsigned block, unsigned cap = 65536)
{
    uint64_t g = (n + block - 1) / block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (unsigned)g;
}

// rows -> their HSP records, for copying one pair's table to the host
__global__ void gather_rows_kernel(const DHsp *hsp, const DRow *rows, uint64_t n, DHsp *out)
{
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        out[i] = hsp[rows[i].hsp];
}

void launch_pack(const uint8_t *ascii, uint64_t total, uint64_t nwords, uint64_t *F, uint64_t *RC,
                 uint64_t *AF, uint64_t *ARC, hipStream_t st)
{
    hipLaunchKernelGGL(pack_fwd_kernel, dim3(grid_for(nwords, 256)), dim3(256), 0, st, ascii, total, nwords,
                       F, AF);
    hipLaunchKernelGGL(pack_rc_kernel, dim3(grid_for(nwords, 256)), dim3(256), 0, st, F, AF, total, nwords,
                       RC, ARC);
}

void launch_kmer_count(const TxInfo *tx, uint32_t n_tx, const uint64_t *AF, uint64_t *cnt, hipStream_t st)
{
    hipLaunchKernelGGL(kmer_count_kernel, dim3(n_tx), dim3(256), 0, st, tx, n_tx, AF, cnt);
}

void launch_kmer_fill(bool amb, const TxInfo *tx, uint32_t n_tx, const uint64_t *F, const uint64_t *AF,
                      const uint64_t *out_off, uint64_t *ent, hipStream_t st)
{
    if (!n_tx) return;
    const dim3 g(std::min<uint32_t>((n_tx + 3) / 4, FILL_BLOCKS));
    if (amb)
        hipLaunchKernelGGL(kmer_fill_kernel<true>, g, dim3(256), 0, st, tx, n_tx, F, AF, out_off, ent);
    else
        hipLaunchKernelGGL(kmer_fill_kernel<false>, g, dim3(256), 0, st, tx, n_tx, F, AF, out_off, ent);
}

void launch_bucket_fill(const uint64_t *ent, uint64_t n, int bits, uint32_t *bucket, hipStream_t st)
{
    const uint64_t threads = n / BF_PER + 1;   // entries 0 .. n (entry n closes the table)
    hipLaunchKernelGGL(bucket_fill_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st, ent, n, bits, bucket);
}

// ------------------------------------------------------------------------
// tile tables (load_tile): built on the device from one TileSeg per tile
// sample, so a tile load moves O(samples) bytes over PCIe instead of
// per-transcript and per-base tables
// ------------------------------------------------------------------------

// last segment whose ttx0 <= i (segments ascend by ttx0, none empty)
__device__ inline uint32_t seg_of(const TileSeg *segs, uint32_t nseg, uint32_t i)
{
    uint32_t lo = 0, hi = nseg;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (segs[mid].ttx0 <= i) lo = mid; else hi = mid;
    }
    return lo;
}

// One thread per tile transcript: its start in the tile into the global
// transcript table, the tile list (and its global id), the index list with
// its k-mer slot (subject samples), and its start bit (bit start + 64 of
// txb: the seed kernel reads it one word in). Threads < nseg also set the
// bit at the end of their sample's bases when padding follows.
__global__ void tile_tx_kernel(const TileSeg *__restrict__ segs, uint32_t nseg, uint32_t n_ttx,
                               const uint64_t *__restrict__ tx_rel, const uint64_t *__restrict__ kpre,
                               TxInfo *__restrict__ tx, TxInfo *__restrict__ ttx, uint32_t *__restrict__ gid,
                               TxInfo *__restrict__ itx, uint64_t *__restrict__ koff, uint32_t n_itx, uint64_t npos,
                               unsigned long long *__restrict__ txb)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nseg && segs[i].pad_bit != ~0ull) {
        const uint64_t q = segs[i].pad_bit + 64;
        atomicOr(&txb[q >> 6], 1ull << (q & 63));
    }
    if (i == 0) koff[n_itx] = npos;
    if (i >= n_ttx) return;
    const TileSeg S = segs[seg_of(segs, nseg, i)];
    const uint32_t k = i - S.ttx0, t = S.tx0 + k;
    TxInfo x = tx[t];
    x.start = S.pos + tx_rel[t];
    tx[t] = x;
    ttx[i] = x;
    gid[i] = t;
    if (S.itx0 != ~0u) {
        itx[S.itx0 + k] = x;
        koff[S.itx0 + k] = S.kbase + kpre[t];
    }
    const uint64_t q = x.start + 64;
    atomicOr(&txb[q >> 6], 1ull << (q & 63));
}

// The isoform records of every gene follow their transcripts' tile starts.
__global__ void tile_giso_kernel(const TxInfo *__restrict__ tx, IsoRec *__restrict__ giso, uint64_t n)
{
    for (uint64_t k = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; k < n; k += (uint64_t)gridDim.x * blockDim.x)
        giso[k].start = (uint32_t)tx[giso[k].gtx].start;
}

// Position -> transcript blocks: block b (bases [b << POS_TX_SHIFT, ...)) of
// a sample's padded range holds the sample's last transcript starting at or
// before the block's first base; blocks outside every sample are zero.
__global__ void tile_pos_tx_kernel(const TxInfo *__restrict__ ttx, const uint32_t *__restrict__ gid, uint32_t n_ttx,
                                   const uint64_t *__restrict__ send, PosTx *__restrict__ pos_tx, uint64_t nblocks)
{
    for (uint64_t b = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; b < nblocks;
         b += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t p = b << POS_TX_SHIFT;
        uint32_t lo = 0, hi = n_ttx;   // first transcript starting after p
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (ttx[mid].start <= p) lo = mid + 1; else hi = mid;
        }
        PosTx r{0, 0, 0, 0};
        if (lo) {
            const TxInfo x = ttx[lo - 1];
            if (p < send[x.sample]) r = PosTx{gid[lo - 1], (uint32_t)x.start, x.len, x.sample};
        }
        pos_tx[b] = r;
    }
}

void launch_tile_tables(const TileSeg *segs, uint32_t nseg, uint32_t n_ttx, const uint64_t *tx_rel,
                        const uint64_t *kpre, TxInfo *tx, TxInfo *ttx, uint32_t *gid, TxInfo *itx, uint64_t *koff,
                        uint32_t n_itx, uint64_t npos, uint64_t *txb, IsoRec *giso, uint64_t n_giso,
                        const uint64_t *send, PosTx *pos_tx, uint64_t nblocks, hipStream_t st)
{
    const uint32_t n = std::max<uint32_t>(std::max(n_ttx, nseg), 1u);
    hipLaunchKernelGGL(tile_tx_kernel, dim3((n + 255) / 256), dim3(256), 0, st, segs, nseg, n_ttx, tx_rel, kpre, tx,
                       ttx, gid, itx, koff, n_itx, npos, (unsigned long long *)txb);
    if (n_giso)
        hipLaunchKernelGGL(tile_giso_kernel, dim3(grid_for(n_giso, 256)), dim3(256), 0, st, tx, giso, n_giso);
    if (nblocks)
        hipLaunchKernelGGL(tile_pos_tx_kernel, dim3(grid_for(nblocks, 256)), dim3(256), 0, st, ttx, gid, n_ttx, send,
                           pos_tx, nblocks);
}

// 1 iff transcript i of the list holds a DUST-masked base (one thread each)
__global__ void tx_masked_kernel(const TxInfo *txl, uint32_t n, const uint64_t *dmask, uint8_t *out)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const TxInfo t = txl[i];
    uint64_t any = 0;
    for (uint32_t u = 0; u < t.len && !any; u += 64) {
        const uint32_t k = t.len - u < 64 ? t.len - u : 64;
        const uint64_t w = win_bits(dmask, (int64_t)(t.start + u));
        any = k == 64 ? w : (w & ((1ull << k) - 1ull));
    }
    out[i] = any ? 1 : 0;
}

void launch_tx_masked(const TxInfo *txl, uint32_t n, const uint64_t *dmask, uint8_t *out, hipStream_t st)
{
    if (n) hipLaunchKernelGGL(tx_masked_kernel, dim3((n + 255) / 256), dim3(256), 0, st, txl, n, dmask, out);
}

// The reverse pass's index (shared searches with DUST): the 16-mer positions
// of masked transcripts with a DUST-masked base in [pos - 12, pos + 28). A
// run between a and b none of whose aligned words of a is usable has a masked
// base of a there for every 16-mer pos it holds: the 28 bases of the run
// nearest to [pos, pos + 16) lie in that range and hold a whole word of a's
// grid (13 consecutive starts hold one), and that word is masked. So the hits
// of such runs are all here. One wave per
// transcript, one atomic per 64 positions: the order is arbitrary and the
// sort orders all 64 key bits. Entries past `cap` are counted, not written.
template <bool AMB>
__global__ __launch_bounds__(256) void near_fill_kernel(const TxInfo *__restrict__ tx, uint32_t n_tx,
                                                        const uint8_t *__restrict__ masked,
                                                        const uint64_t *__restrict__ F,
                                                        const uint64_t *__restrict__ AF,
                                                        const uint64_t *__restrict__ dmask, uint64_t *__restrict__ ent,
                                                        uint64_t cap, unsigned long long *count)
{
    const int lane = threadIdx.x & 63;
    const uint32_t nwave = gridDim.x * 4u, t0 = blockIdx.x * 4u + (threadIdx.x >> 6);
    // the positions of this wave's transcripts: counted, one atomic for all
    // of them, then written (one counter for every wave: an atomic per 64
    // positions serialised on it)
    auto near = [&](const TxInfo &ti, int64_t o, uint64_t &p) -> bool {
        p = ti.start + (uint64_t)o;
        bool ok = o <= (int64_t)ti.len - W16 && (win_bits(dmask, (int64_t)p - 12) & ((1ull << 40) - 1ull)) != 0;
        if (AMB && ok) ok = (win(AF, p) & 0xFFFFFFFFull) == 0;
        return ok;
    };
    uint64_t n = 0, p = 0;
    for (uint32_t t = t0; t < n_tx; t += nwave) {
        if (!masked[t]) continue;
        const TxInfo ti = tx[t];
        for (int64_t o0 = 0; o0 + W16 <= (int64_t)ti.len; o0 += 64) n += (uint64_t)__popcll(__ballot(near(ti, o0 + lane, p)));
    }
    if (!n) return;
    unsigned long long b = 0;
    if (lane == 0) b = atomicAdd(count, (unsigned long long)n);
    b = (unsigned long long)__shfl((long long)b, 0);
    for (uint32_t t = t0; t < n_tx; t += nwave) {
        if (!masked[t]) continue;
        const TxInfo ti = tx[t];
        for (int64_t o0 = 0; o0 + W16 <= (int64_t)ti.len; o0 += 64) {
            const bool ok = near(ti, o0 + lane, p);
            const uint64_t m = __ballot(ok);
            const uint64_t i = b + (uint64_t)__popcll(m & ((1ull << lane) - 1ull));
            if (ok && i < cap) ent[i] = ((uint64_t)(uint32_t)win(F, p) << 32) | p;
            b += (uint64_t)__popcll(m);
        }
    }
}

void launch_near_fill(bool amb, const TxInfo *tx, uint32_t n_tx, const uint8_t *masked, const uint64_t *F,
                      const uint64_t *AF, const uint64_t *dmask, uint64_t *ent, uint64_t cap,
                      unsigned long long *count, hipStream_t st)
{
    if (!n_tx) return;
    const dim3 g(std::min<uint32_t>((n_tx + 3) / 4, FILL_BLOCKS));
    if (amb)
        hipLaunchKernelGGL(near_fill_kernel<true>, g, dim3(256), 0, st, tx, n_tx, masked, F, AF, dmask, ent, cap, count);
    else
        hipLaunchKernelGGL(near_fill_kernel<false>, g, dim3(256), 0, st, tx, n_tx, masked, F, AF, dmask, ent, cap, count);
}

// After pass 2 and the scans: each item's rows and edges from its slots to
// their offsets, labels made pair-global (F rows: + the item's F_sel base; R
// rows: + the pair's F_sel total + the item's R_sel base).
__global__ void rbh_place_kernel(RbhParams P)
{
    __shared__ int sh_pair;
    for (uint64_t lb = blockIdx.x * (uint64_t)blockDim.x; lb < P.n_items; lb += (uint64_t)gridDim.x * blockDim.x) {
        __syncthreads();
        if (threadIdx.x == 0) {
            const uint64_t item0 = P.item0 + lb;
            int lo = 0, hi = P.n_pairs;
            while (hi - lo > 1) {
                const int mid = (lo + hi) >> 1;
                if (P.pair_item_begin[mid] <= item0) lo = mid; else hi = mid;
            }
            sh_pair = lo;
        }
        __syncthreads();
        const uint64_t li = lb + threadIdx.x;
        if (li >= P.n_items) continue;
        const uint64_t item = P.item0 + li;
        int pr = sh_pair;
        while (pr + 1 < P.n_pairs && P.pair_item_begin[pr + 1] <= item) pr++;
        const uint64_t pb = P.pair_item_begin[pr] - P.item0, pe = P.pair_item_begin[pr + 1] - P.item0;
        const uint32_t nr = P.n_rows[li], ne = P.n_edges[li];
        if (nr) {
            const int32_t fb = (int32_t)(P.fsel_off[li] - P.fsel_off[pb]);
            const int32_t rb = (int32_t)(P.fsel_off[pe] - P.fsel_off[pb] + P.rsel_off[li] - P.rsel_off[pb]);
            const uint64_t o = P.row_off[li];
            for (uint32_t k = 0; k < nr && k < (uint32_t)RBH_RMAX; k++) {
                DRow r = P.rows_tmp[li * RBH_RMAX + k];
                r.label += r.reverse ? rb : fb;
                P.rows[o + k] = r;
            }
        }
        const uint64_t eo = P.edge_off[li];
        for (uint32_t k = 0; k < ne && k < (uint32_t)RBH_EMAX; k++) P.edges[eo + k] = P.edges_tmp[li * RBH_EMAX + k];
    }
}

void launch_rbh_place(const RbhParams &P, hipStream_t st)
{
    if (P.n_items == 0) return;
    hipLaunchKernelGGL(rbh_place_kernel, dim3(grid_for(P.n_items, 256)), dim3(256), 0, st, P);
}

void launch_rbh(const RbhParams &P, int pass, hipStream_t st)
{
    if (P.n_items == 0) return;
    hipLaunchKernelGGL(rbh_kernel, dim3(grid_for(P.n_items, 256)), dim3(256), 0, st, P, pass);
}

void launch_cc(const DEdge *edges, uint64_t n_edges, uint32_t n_nodes, const int32_t *gene_sample, int N,
               int S_given, uint32_t *parent, uint32_t *present, uint32_t *cnodes, uint32_t *cedges,
               uint32_t *sample_present, uint8_t *ideal, unsigned long long *stats, hipStream_t st)
{
    const unsigned gn = grid_for(n_nodes, 256), ge = grid_for(n_edges, 256);
    hipLaunchKernelGGL(cc_init_kernel, dim3(gn), dim3(256), 0, st, parent, present, cnodes, cedges, n_nodes);
    if (n_edges) hipLaunchKernelGGL(cc_hook_kernel, dim3(ge), dim3(256), 0, st, edges, n_edges, parent, present);
    hipLaunchKernelGGL(cc_compress_kernel, dim3(gn), dim3(256), 0, st, parent, n_nodes);
    hipLaunchKernelGGL(cc_count_kernel, dim3(grid_for(n_edges > n_nodes ? n_edges : n_nodes, 256)), dim3(256), 0,
                       st, edges, n_edges, parent, present, gene_sample, n_nodes, cnodes, cedges, sample_present);
    hipLaunchKernelGGL(cc_ideal_kernel, dim3(gn), dim3(256), 0, st, parent, present, cnodes, cedges, n_nodes,
                       sample_present, N, S_given, ideal, stats);
}

void launch_pair_sums(const DEdge *edges, uint64_t n_edges, const uint32_t *parent, const uint8_t *ideal,
                      unsigned long long *num, unsigned long long *den, unsigned long long *num_all,
                      unsigned long long *den_all, hipStream_t st)
{
    if (!n_edges) return;
    hipLaunchKernelGGL(pair_sums_kernel, dim3(grid_for(n_edges, 256)), dim3(256), 0, st, edges, n_edges, parent,
                       ideal, num, den, num_all, den_all);
}

void launch_distance(const unsigned long long *num, const unsigned long long *den, const int32_t *pair_index,
                     const int32_t *order, int N, int M, double *out, unsigned int *status, hipStream_t st)
{
    const int n = M * M;
    if (!n) return;
    hipLaunchKernelGGL(distance_kernel, dim3((n + 255) / 256), dim3(256), 0, st, num, den, pair_index, order, N,
                       M, out, status);
}

// Imported edge records in range (rc_import_edges from the device): node ids
// below n_genes, a pair index (with the sums-only flag) below n_pairs, or a
// node-only record a == b. Any other record sets *bad.
__global__ void edge_check_kernel(const DEdge *edges, uint64_t n, uint32_t ng, uint64_t np, unsigned int *bad)
{
    bool b = false;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const DEdge d = edges[i];
        const bool node = d.pair == NODE_REC;
        b |= d.a >= ng || d.b >= ng || (!node && (uint64_t)(d.pair & ~EDGE_SUM_ONLY) >= np) || (node && d.a != d.b);
    }
    if (__any(b) && (threadIdx.x & 63) == 0) atomicOr(bad, 1u);
}

void launch_edge_check(const DEdge *edges, uint64_t n, uint32_t ng, uint64_t np, unsigned int *bad, hipStream_t st)
{
    if (!n) return;
    hipLaunchKernelGGL(edge_check_kernel, dim3(grid_for(n, 256, 8192)), dim3(256), 0, st, edges, n, ng, np, bad);
}

// graph.pkl from the edge records: each record's sort key (its pair's rank
// in combinations order; flagged records -- sums-only rows, isolated nodes of
// an imported graph -- are marked by ~0u) and its index
__global__ void edge_key_kernel(const DEdge *edges, uint64_t n, const uint32_t *comb_of_pair, uint32_t *key,
                                uint32_t *idx)
{
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t p = edges[i].pair;
        key[i] = (p & EDGE_SUM_ONLY) || p == NODE_REC ? ~0u : comb_of_pair[p];
        idx[i] = (uint32_t)i;
    }
}
__global__ void edge_gather_kernel(const DEdge *edges, const uint32_t *idx, uint64_t n, DEdge *out)
{
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        out[i] = edges[idx[i]];
}

// the sorted records as the graph.pkl writer takes them: node pairs (a, b)
// in two arrays, and the first record of each combination (table) -- keys
// sorted, so a key's first record is where it differs from its predecessor
__global__ void edge_uv_kernel(const DEdge *edges, const uint32_t *idx, const uint32_t *key, uint64_t n, uint32_t *u,
                               uint32_t *v, uint64_t *first)
{
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const DEdge d = edges[idx[i]];
        u[i] = d.a;
        v[i] = d.b;
        const uint32_t k = key[i];
        if (k != ~0u && (i == 0 || key[i - 1] != k)) first[k] = i;
    }
}

void launch_edge_uv(const DEdge *edges, const uint32_t *idx, const uint32_t *key, uint64_t n, uint32_t *u, uint32_t *v,
                    uint64_t *first, hipStream_t st)
{
    if (n) hipLaunchKernelGGL(edge_uv_kernel, dim3(grid_for(n, 256)), dim3(256), 0, st, edges, idx, key, n, u, v, first);
}

void launch_edge_key(const DEdge *edges, uint64_t n, const uint32_t *comb_of_pair, uint32_t *key, uint32_t *idx,
                     hipStream_t st)
{
    if (n) hipLaunchKernelGGL(edge_key_kernel, dim3(grid_for(n, 256)), dim3(256), 0, st, edges, n, comb_of_pair, key, idx);
}
void launch_edge_gather(const DEdge *edges, const uint32_t *idx, uint64_t n, DEdge *out, hipStream_t st)
{
    if (n) hipLaunchKernelGGL(edge_gather_kernel, dim3(grid_for(n, 256)), dim3(256), 0, st, edges, idx, n, out);
}

void launch_gather_rows(const DHsp *hsp, const DRow *rows, uint64_t n, DHsp *out, hipStream_t st)
{
    if (!n) return;
    hipLaunchKernelGGL(gather_rows_kernel, dim3(grid_for(n, 256)), dim3(256), 0, st, hsp, rows, n, out);
}

}  // namespace rcg

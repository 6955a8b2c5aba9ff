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

#include <climits>

namespace rcg {

// ------------------------------------------------------------------------
// 2-bit windows
// ------------------------------------------------------------------------

// 32 bases starting at base position p (base i in bits 2i..2i+1).
__device__ __forceinline__ uint64_t win(const uint64_t *__restrict__ a, uint64_t p)
{
    const uint64_t w = p >> 5;
    const unsigned sh = (unsigned)(p & 31) * 2u;
    const uint64_t lo = a[w];
    if (sh == 0) return lo;
    return (lo >> sh) | (a[w + 1] << (64u - sh));
}

// Longest common extension of two forward walks (at most maxn bases).
// Ambiguous bases (mask 0b11) never match.
template <bool AMB>
__device__ __forceinline__ int lcp(const uint64_t *__restrict__ A, const uint64_t *__restrict__ AA,
                                   uint64_t pa, const uint64_t *__restrict__ B,
                                   const uint64_t *__restrict__ BA, uint64_t pb, int maxn)
{
    int n = 0;
    while (n < maxn) {
        uint64_t x = win(A, pa + n) ^ win(B, pb + n);
        if (AMB) x |= win(AA, pa + n) | win(BA, pb + n);
        if (x == 0) {
            n += 32;
            continue;
        }
        n += __builtin_ctzll(x) >> 1;
        return n < maxn ? n : maxn;
    }
    return maxn > 0 ? maxn : 0;
}

__device__ __forceinline__ uint64_t rev2(uint64_t x)
{
    x = ((x >> 2) & 0x3333333333333333ull) | ((x & 0x3333333333333333ull) << 2);
    x = ((x >> 4) & 0x0F0F0F0F0F0F0F0Full) | ((x & 0x0F0F0F0F0F0F0F0Full) << 4);
    return __builtin_bswap64(x);
}

// ------------------------------------------------------------------------
// pack
// ------------------------------------------------------------------------

__device__ __forceinline__ void code_of(uint8_t c, uint64_t &code, uint64_t &amb)
{
    const uint8_t l = c | 0x20;
    code = (l == 'c') ? 1 : (l == 'g') ? 2 : (l == 't') ? 3 : 0;
    amb = (l == 'a' || l == 'c' || l == 'g' || l == 't') ? 0 : 3;
}

// One thread per 64-bit word (32 bases): 32 input bytes as two 16-B loads.
__global__ void pack_fwd_kernel(const uint8_t *__restrict__ ascii, uint64_t total, uint64_t nwords,
                                uint64_t *__restrict__ F, uint64_t *__restrict__ AF)
{
    for (uint64_t w = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; w < nwords;
         w += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t p0 = w * 32;
        uint8_t b[32];
        if (p0 + 32 <= total) {
            const uint4 *v = reinterpret_cast<const uint4 *>(ascii + p0);
            uint4 x0 = v[0], x1 = v[1];
            *reinterpret_cast<uint4 *>(b) = x0;
            *reinterpret_cast<uint4 *>(b + 16) = x1;
        } else {
#pragma unroll
            for (int i = 0; i < 32; i++) b[i] = (p0 + i < total) ? ascii[p0 + i] : 'A';
        }
        uint64_t word = 0, amb = 0;
#pragma unroll
        for (int i = 0; i < 32; i++) {
            uint64_t c, a;
            code_of(b[i], c, a);
            if (p0 + i >= total) c = 0, a = 0;
            word |= c << (2 * i);
            amb |= a << (2 * i);
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

// One block per transcript; windows in (gtx, offset) order so that a stable
// radix sort on the key keeps each key's entries sorted by (gtx, offset).
template <bool AMB>
__global__ __launch_bounds__(256) void kmer_fill_kernel(const TxInfo *__restrict__ tx, uint32_t n_tx,
                                                        const uint64_t *__restrict__ F,
                                                        const uint64_t *__restrict__ AF,
                                                        const uint64_t *__restrict__ out_off,
                                                        uint32_t *__restrict__ keys,
                                                        uint64_t *__restrict__ vals)
{
    const uint32_t t = blockIdx.x;
    if (t >= n_tx) return;
    const TxInfo ti = tx[t];
    const int64_t nwin = (int64_t)ti.len - W16 + 1;
    if (nwin <= 0) return;
    uint64_t base = out_off[t];
    __shared__ uint32_t wcnt[4];
    for (int64_t o0 = 0; o0 < nwin; o0 += blockDim.x) {
        const int64_t o = o0 + threadIdx.x;
        bool ok = o < nwin;
        uint32_t key = 0;
        if (ok) {
            key = (uint32_t)win(F, ti.start + o);
            if (AMB) ok = (win(AF, ti.start + o) & 0xFFFFFFFFull) == 0;
        }
        if (!AMB) {
            if (ok) {
                keys[base + o] = key;
                vals[base + o] = (uint64_t)t | ((uint64_t)o << 32);
            }
        } else {
            const uint64_t m = __ballot(ok);
            const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
            const uint32_t before = __popcll(m & ((1ull << lane) - 1ull));
            if (lane == 0) wcnt[wid] = __popcll(m);
            __syncthreads();
            uint32_t woff = 0, tot = 0;
            for (int i = 0; i < (int)(blockDim.x >> 6); i++) {
                if (i < wid) woff += wcnt[i];
                tot += wcnt[i];
            }
            if (ok) {
                keys[base + woff + before] = key;
                vals[base + woff + before] = (uint64_t)t | ((uint64_t)o << 32);
            }
            base += tot;
            __syncthreads();
        }
    }
}

// bucket[b] = first sorted index whose key >> (32 - bits) >= b, b in [0, 2^bits].
__global__ void bucket_fill_kernel(const uint32_t *__restrict__ keys, uint64_t n, int bits,
                                   uint32_t *__restrict__ bucket)
{
    const unsigned sh = 32u - (unsigned)bits;
    const uint64_t nb = 1ull << bits;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i <= n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t b = (i < n) ? (uint64_t)(keys[i] >> sh) : nb + 1;
        const uint64_t pb = (i > 0) ? (uint64_t)(keys[i - 1] >> sh) : 0;
        const uint64_t lo = (i > 0) ? pb + 1 : 0;
        const uint64_t hi = (i < n) ? b : nb;
        for (uint64_t x = lo; x <= hi && x <= nb; x++) bucket[x] = (uint32_t)i;
    }
}

// ------------------------------------------------------------------------
// alignment
// ------------------------------------------------------------------------

constexpr int ABLOCK = 256;
constexpr int NWAVE = ABLOCK / 64;
constexpr int SEED_CAP = 2048;
constexpr int HSP_CAP = 128;
constexpr int MAX_SAMPLES = 256;

struct LSeed {
    uint64_t k1;    // iso:7 | strand:1 | gtx:32 | x:24
    uint32_t y, len;
};

struct ExtRes {
    int score, i, j, d, g, o;
};

__device__ __forceinline__ int wave_max(int v)
{
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = max(v, __shfl_xor(v, off));
    return v;
}

// Greedy X-drop extension (oracle/align_oracle.c greedy_ext), one diagonal per
// lane. Returns wave-uniform values.
template <bool AMB>
__device__ ExtRes ext_wave(const uint64_t *A, const uint64_t *AA, uint64_t pa, int alen,
                           const uint64_t *B, const uint64_t *BA, uint64_t pb, int blen, int X,
                           int lane)
{
    const int k = lane + BAND_LO;
    int R = -1, G = 0, O = 0, E = 0;
    int r0 = 0;
    if (lane == -BAND_LO) {
        r0 = lcp<AMB>(A, AA, pa, B, BA, pb, min(alen, blen));
        R = r0;
    }
    r0 = __shfl(r0, -BAND_LO);
    ExtRes best = {2 * r0, r0, r0, 0, 0, 0};
    for (int d = 1; d <= DMAX; ++d) {
        const int goe = G | (O << 13) | (E << 26);
        int Rl = __shfl_up(R, 1), Rr = __shfl_down(R, 1);
        int gl = __shfl_up(goe, 1), gr = __shfl_down(goe, 1);
        if (lane == 0) Rl = -1;
        if (lane == 63) Rr = -1;
        int ni = -1, ng = 0, no = 0, ne = 0;
        if (R >= 0 && R < alen && R - k < blen) {
            ni = R + 1; ng = G; no = O; ne = 0;
        }
        if (Rl >= 0 && Rl < alen) {
            const int c = Rl + 1;
            if (c > ni) {
                ni = c;
                ng = (gl & 8191) + 1;
                no = ((gl >> 13) & 8191) + (((gl >> 26) & 3) == 1 ? 0 : 1);
                ne = 1;
            }
        }
        if (Rr >= 0 && Rr - (k + 1) < blen) {
            const int c = Rr;
            if (c > ni) {
                ni = c;
                ng = (gr & 8191) + 1;
                no = ((gr >> 13) & 8191) + (((gr >> 26) & 3) == 2 ? 0 : 1);
                ne = 2;
            }
        }
        int score = INT_MIN;
        if (ni >= 0 && ni - k >= 0) {
            const int ja = ni - k;
            const int m = min(alen - ni, blen - ja);
            const int s = lcp<AMB>(A, AA, pa + (uint64_t)ni, B, BA, pb + (uint64_t)ja, m);
            if (s > 0) {
                ni += s;
                ne = 0;
            }
            score = 2 * ni - k - 6 * d;
            if (score < best.score - X) ni = -1;
        } else {
            ni = -1;
        }
        R = ni; G = ng; O = no; E = ne;
        const bool live = ni >= 0;
        const uint64_t lm = __ballot(live);
        if (lm == 0) break;
        const int mx = wave_max(live ? score : INT_MIN);
        if (mx > best.score) {
            const uint64_t tm = __ballot(live && score == mx);
            const int bl = __ffsll((unsigned long long)tm) - 1;
            best.score = mx;
            best.i = __shfl(R, bl);
            best.j = best.i - (bl + BAND_LO);
            best.d = d;
            best.g = __shfl(G, bl);
            best.o = __shfl(O, bl);
        }
    }
    return best;
}

// Oriented query helpers. strand 0: q; strand 1: revcomp(q).
struct QGeo {
    uint64_t qs;   // forward start
    int Lq;
};

// array/position of the forward walk of oriented position u
__device__ __forceinline__ uint64_t qfwd_pos(const QGeo &q, int strand, uint64_t total, int u)
{
    return strand ? (total - q.qs - (uint64_t)q.Lq + (uint64_t)u) : (q.qs + (uint64_t)u);
}
// array/position of the walk leftwards from oriented position x (x-1, x-2, ...)
__device__ __forceinline__ uint64_t qrev_pos(const QGeo &q, int strand, uint64_t total, int x)
{
    return strand ? (q.qs + (uint64_t)q.Lq - (uint64_t)x) : (total - q.qs - (uint64_t)x);
}

template <bool AMB>
__global__ __launch_bounds__(ABLOCK) void align_kernel(Db db, Index ix, AlignParams P)
{
    const uint32_t g = P.gene_begin + blockIdx.x;
    if (g >= P.gene_end) return;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;

    __shared__ LSeed seeds[SEED_CAP];
    __shared__ uint16_t seg_begin[SEED_CAP + 1];
    __shared__ uint32_t it_lo[ABLOCK], it_pre[ABLOCK + 1], it_info[ABLOCK];
    __shared__ uint64_t iso_start[MAX_ISO];
    __shared__ uint32_t iso_len[MAX_ISO], iso_gtx[MAX_ISO], iso_pre[MAX_ISO + 1];
    __shared__ DHsp hbuf[HSP_CAP];
    __shared__ uint32_t hkey[HSP_CAP];
    __shared__ uint16_t hord[HSP_CAP];
    __shared__ uint32_t tcnt[MAX_SAMPLES], tpre[MAX_SAMPLES + 1];
    __shared__ uint32_t sh_nseed, sh_nhsp, sh_flags, sh_nseg;
    __shared__ unsigned long long sh_base;

    const int Q = db.gene_sample[g];
    const uint32_t t0 = db.gene_tx_off[g];
    const uint32_t niso = db.gene_tx_off[g + 1] - t0;
    const int N = db.n_samples;
    const uint64_t total = db.total;
    const int stride = P.stride;
    if (niso > (uint32_t)MAX_ISO || N > MAX_SAMPLES) {
        if (tid == 0) atomicOr(P.status, 2u);
        return;
    }
    for (uint32_t i = tid; i < niso; i += ABLOCK) {
        const uint32_t gtx = db.gene_tx[t0 + i];
        const TxInfo ti = db.tx[gtx];
        iso_gtx[i] = gtx;
        iso_start[i] = ti.start;
        iso_len[i] = ti.len;
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t pre = 0;
        for (uint32_t i = 0; i < niso; i++) {
            iso_pre[i] = pre;
            const int L = (int)iso_len[i];
            pre += (L >= W16) ? 2u * (uint32_t)((L - W16) / stride + 1) : 0u;
        }
        iso_pre[niso] = pre;
    }
    __syncthreads();
    const uint32_t n_items = iso_pre[niso];
    const uint32_t gl = g - P.gene_begin;

    int T0 = 0, T1 = N;
    while (T0 < N) {
        if (tid == 0) {
            sh_nseed = 0;
            sh_nhsp = 0;
            sh_flags = 0;
        }
        __syncthreads();
        // ---------------- seeds ----------------
        for (uint32_t ib = 0; ib < n_items; ib += ABLOCK) {
            const uint32_t it = ib + tid;
            uint32_t lo = 0, cnt = 0, info = 0;
            if (it < n_items) {
                uint32_t ii = 0;
                while (ii + 1 < niso && iso_pre[ii + 1] <= it) ii++;
                const uint32_t rem = it - iso_pre[ii];
                const uint32_t ns = (iso_pre[ii + 1] - iso_pre[ii]) >> 1;
                const int strand = rem >= ns ? 1 : 0;
                const int p = (int)(rem - (strand ? ns : 0)) * stride;
                info = ii | ((uint32_t)strand << 7) | ((uint32_t)p << 8);
                QGeo qg = {iso_start[ii], (int)iso_len[ii]};
                const uint64_t qp = qfwd_pos(qg, strand, total, p);
                const uint64_t *QA = strand ? db.RC : db.F;
                bool ok = true;
                if (AMB) {
                    const uint64_t *QM = strand ? db.ARC : db.AF;
                    ok = (win(QM, qp) & 0xFFFFFFFFull) == 0;
                }
                if (ok) {
                    const uint32_t key = (uint32_t)win(QA, qp);
                    const uint32_t b = key >> (32 - ix.bits);
                    uint32_t a0 = ix.bucket[b], a1 = ix.bucket[b + 1];
                    while (a0 < a1 && ix.keys[a0] < key) a0++;
                    uint32_t a2 = a0;
                    while (a2 < a1 && ix.keys[a2] == key) a2++;
                    lo = a0;
                    cnt = a2 - a0;
                }
            }
            it_lo[tid] = lo;
            it_info[tid] = info;
            it_pre[tid] = cnt;
            __syncthreads();
            if (tid == 0) {
                uint32_t s = 0;
                for (int i = 0; i < ABLOCK; i++) {
                    const uint32_t c = it_pre[i];
                    it_pre[i] = s;
                    s += c;
                }
                it_pre[ABLOCK] = s;
            }
            __syncthreads();
            const uint32_t nh = it_pre[ABLOCK];
            for (uint32_t h = tid; h < nh; h += ABLOCK) {
                int lo2 = 0, hi2 = ABLOCK;   // last k with it_pre[k] <= h
                while (hi2 - lo2 > 1) {
                    const int mid = (lo2 + hi2) >> 1;
                    if (it_pre[mid] <= h) lo2 = mid; else hi2 = mid;
                }
                const int k = lo2;
                const uint2 e = ix.ent[it_lo[k] + (h - it_pre[k])];
                const TxInfo st = db.tx[e.x];
                if (st.sample == Q || st.sample < T0 || st.sample >= T1) continue;
                const uint32_t inf = it_info[k];
                const uint32_t ii = inf & 127;
                const int strand = (inf >> 7) & 1;
                const int p = (int)(inf >> 8);
                const int off = (int)e.y;
                QGeo qg = {iso_start[ii], (int)iso_len[ii]};
                const int maxl = min(min(p, off), stride);
                const uint64_t *QL = strand ? db.F : db.RC;
                const uint64_t *QLM = strand ? db.AF : db.ARC;
                const int l = lcp<AMB>(QL, QLM, qrev_pos(qg, strand, total, p), db.RC, db.ARC,
                                       total - st.start - (uint64_t)off, maxl);
                if (l >= stride) continue;
                const uint64_t *QR = strand ? db.RC : db.F;
                const uint64_t *QRM = strand ? db.ARC : db.AF;
                const int maxr = min(qg.Lq - p - W16, (int)st.len - off - W16);
                const int r = lcp<AMB>(QR, QRM, qfwd_pos(qg, strand, total, p + W16), db.F, db.AF,
                                       st.start + (uint64_t)off + W16, maxr);
                const int len = l + W16 + r;
                if (len < P.word) continue;
                const uint32_t slot = atomicAdd(&sh_nseed, 1u);
                if (slot < (uint32_t)SEED_CAP) {
                    LSeed sd;
                    sd.k1 = ((uint64_t)ii << 57) | ((uint64_t)strand << 56) | ((uint64_t)e.x << 24) |
                            (uint64_t)(uint32_t)(p - l);
                    sd.y = (uint32_t)(off - l);
                    sd.len = (uint32_t)len;
                    seeds[slot] = sd;
                } else {
                    atomicOr(&sh_flags, 1u);
                }
            }
            __syncthreads();
        }
        if (sh_flags & 1u) {
            if (T1 - T0 == 1) {
                if (tid == 0) atomicOr(P.status, 2u);
                return;
            }
            T1 = T0 + (T1 - T0) / 2;
            __syncthreads();
            continue;
        }
        const uint32_t nseed = sh_nseed;
        // ---------------- sort seeds by (k1, y) ----------------
        uint32_t np2 = 1;
        while (np2 < nseed) np2 <<= 1;
        for (uint32_t i = nseed + tid; i < np2; i += ABLOCK) {
            seeds[i].k1 = ~0ull;
            seeds[i].y = 0xFFFFFFFFu;
        }
        __syncthreads();
        for (uint32_t kk = 2; kk <= np2; kk <<= 1) {
            for (uint32_t j = kk >> 1; j > 0; j >>= 1) {
                for (uint32_t i = tid; i < np2; i += ABLOCK) {
                    const uint32_t ixj = i ^ j;
                    if (ixj > i) {
                        LSeed a = seeds[i], b = seeds[ixj];
                        const bool gt = (a.k1 > b.k1) || (a.k1 == b.k1 && a.y > b.y);
                        const bool up = (i & kk) == 0;
                        if (gt == up) {
                            seeds[i] = b;
                            seeds[ixj] = a;
                        }
                    }
                }
                __syncthreads();
            }
        }
        // ---------------- candidates (segments) ----------------
        if (tid == 0) {
            uint32_t ns = 0;
            for (uint32_t i = 0; i < nseed; i++)
                if (i == 0 || (seeds[i].k1 >> 24) != (seeds[i - 1].k1 >> 24)) seg_begin[ns++] = (uint16_t)i;
            seg_begin[ns] = (uint16_t)nseed;
            sh_nseg = ns;
        }
        __syncthreads();
        const uint32_t nseg = sh_nseg;
        for (uint32_t sg = wid; sg < nseg; sg += NWAVE) {
            const uint32_t sb = seg_begin[sg], se = seg_begin[sg + 1];
            const uint64_t k1 = seeds[sb].k1;
            const uint32_t ii = (uint32_t)(k1 >> 57);
            const int strand = (int)((k1 >> 56) & 1);
            const uint32_t stx = (uint32_t)(k1 >> 24);
            const TxInfo st = db.tx[stx];
            QGeo qg = {iso_start[ii], (int)iso_len[ii]};
            const int Lq = qg.Lq, Lt = (int)st.len;
            const uint64_t *QR = strand ? db.RC : db.F;
            const uint64_t *QRM = strand ? db.ARC : db.AF;
            const uint64_t *QL = strand ? db.F : db.RC;
            const uint64_t *QLM = strand ? db.AF : db.ARC;
            int bqa = 0, bqb = 0, bsa = 0, bsb = 0, bsc = 0, bd = 0, bg = 0, bo = 0, bni = 0;
            int nh = 0;
            for (uint32_t si = sb; si < se && nh < MAX_HSP; si++) {
                const int x = (int)(uint32_t)(seeds[si].k1 & 0xFFFFFFull);
                const int y = (int)seeds[si].y, len = (int)seeds[si].len;
                const bool inside = lane < nh && bqa <= x && x + len <= bqb && bsa <= y && y + len <= bsb;
                if (__ballot(inside)) continue;
                const ExtRes r = ext_wave<AMB>(QR, QRM, qfwd_pos(qg, strand, total, x + len), Lq - (x + len),
                                               db.F, db.AF, st.start + (uint64_t)(y + len), Lt - (y + len),
                                               P.xdrop, lane);
                const ExtRes l = ext_wave<AMB>(QL, QLM, qrev_pos(qg, strand, total, x), x, db.RC, db.ARC,
                                               total - st.start - (uint64_t)y, y, P.xdrop, lane);
                if (lane == nh) {
                    bqa = x - l.i; bqb = x + len + r.i; bsa = y - l.j; bsb = y + len + r.j;
                    bsc = l.score + 2 * len + r.score;
                    bd = l.d + r.d; bg = l.g + r.g; bo = l.o + r.o;
                    bni = len + (l.i + l.j - 2 * l.d + l.g) / 2 + (r.i + r.j - 2 * r.d + r.g) / 2;
                }
                nh++;
            }
            // purge HSPs with common endpoints: by (score desc, index asc)
            int rank = 0;
            for (int j = 0; j < nh; j++) {
                const int sj = __shfl(bsc, j);
                if (lane < nh && (sj > bsc || (sj == bsc && j < lane))) rank++;
            }
            bool kept = false;
            for (int rr = 0; rr < nh; rr++) {
                const uint64_t m = __ballot(lane < nh && rank == rr);
                const int i = __ffsll((unsigned long long)m) - 1;
                const int qa = __shfl(bqa, i), sa = __shfl(bsa, i), qb = __shfl(bqb, i), sb2 = __shfl(bsb, i);
                const bool conflict = kept && lane < nh &&
                                      ((bqa == qa && bsa == sa) || (bqb == qb && bsb == sb2));
                if (!__ballot(conflict) && lane == i) kept = true;
            }
            const int thr = P.thr[(size_t)st.sample * (size_t)(P.max_len + 1) + (size_t)Lq];
            const bool out = kept && bsc >= thr;
            const uint64_t om = __ballot(out);
            uint32_t wbase = 0;
            if (lane == 0 && om) wbase = atomicAdd(&sh_nhsp, (uint32_t)__popcll(om));
            wbase = __shfl(wbase, 0);
            if (out) {
                const uint32_t slot = wbase + (uint32_t)__popcll(om & ((1ull << lane) - 1ull));
                if (slot < (uint32_t)HSP_CAP) {
                    DHsp h;
                    h.q_tx = iso_gtx[ii];
                    h.s_tx = stx;
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
                    h.strand = strand;
                    hbuf[slot] = h;
                    hkey[slot] = (sg << 3) | (uint32_t)lane;
                } else {
                    atomicOr(&sh_flags, 2u);
                }
            }
        }
        __syncthreads();
        if (sh_flags & 2u) {
            if (T1 - T0 == 1) {
                if (tid == 0) atomicOr(P.status, 2u);
                return;
            }
            T1 = T0 + (T1 - T0) / 2;
            __syncthreads();
            continue;
        }
        // ---------------- order HSPs and group them by subject sample ----------------
        const uint32_t nhsp = sh_nhsp;
        for (uint32_t i = tid; i < nhsp; i += ABLOCK) {
            uint32_t r = 0;
            const uint32_t ki = hkey[i];
            for (uint32_t j = 0; j < nhsp; j++) r += hkey[j] < ki;
            hord[r] = (uint16_t)i;   // keys are unique
        }
        for (int T = tid; T < N; T += ABLOCK) tcnt[T] = 0;
        __syncthreads();
        for (uint32_t i = tid; i < nhsp; i += ABLOCK) {
            const int T = db.tx[hbuf[i].s_tx].sample;
            atomicAdd(&tcnt[T], 1u);
        }
        __syncthreads();
        if (tid == 0) {
            uint32_t s = 0;
            for (int T = 0; T < N; T++) {
                tpre[T] = s;
                s += tcnt[T];
            }
            tpre[N] = s;
            sh_base = nhsp ? atomicAdd(P.out_count, (unsigned long long)nhsp) : 0ull;
            if (sh_base + nhsp > P.out_cap) atomicOr(P.status, 1u);
        }
        __syncthreads();
        const unsigned long long base = sh_base;
        const bool room = base + nhsp <= P.out_cap;
        for (uint32_t r = tid; r < nhsp; r += ABLOCK) {
            const uint32_t i = hord[r];
            const int T = db.tx[hbuf[i].s_tx].sample;
            uint32_t rk = 0;   // rank among earlier (ordered) HSPs of the same sample
            for (uint32_t r2 = 0; r2 < r; r2++) rk += db.tx[hbuf[hord[r2]].s_tx].sample == T;
            if (room) P.out[base + tpre[T] + rk] = hbuf[i];
        }
        for (int T = T0 + tid; T < T1; T += ABLOCK) {
            const size_t gi = (size_t)gl * (size_t)N + (size_t)T;
            P.grp_off[gi] = (uint32_t)(base + tpre[T]);
            P.grp_cnt[gi] = tcnt[T];
        }
        T0 = T1;
        T1 = N;
        __syncthreads();
    }
}

// ------------------------------------------------------------------------
// reciprocal best hits -> gene matches rows and edges (find_homologs.py:215-302)
// ------------------------------------------------------------------------



// threshold of highest_bitscores(n, keep="all") over one group's bitscores
__device__ __forceinline__ int group_thr(const DHsp *h, uint32_t off, uint32_t cnt, int n)
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
__device__ __forceinline__ uint32_t desc_rank(const DHsp *h, uint32_t off, uint32_t cnt, uint32_t i, Pred pred)
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

__global__ void rbh_kernel(RbhParams P, int pass)
{
    for (uint64_t item = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; item < P.n_items;
         item += (uint64_t)gridDim.x * blockDim.x) {
        int lo = 0, hi = P.n_pairs;
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (P.pair_item_begin[mid] <= item) lo = mid; else hi = mid;
        }
        const int pr = lo;
        const int A = P.pair_a[pr], B = P.pair_b[pr];
        const uint32_t b = P.sample_gene_begin[B] + (uint32_t)(item - P.pair_item_begin[pr]);
        const int N = P.N;
        const size_t fgi = (size_t)b * N + A;
        const uint32_t foff = P.grp_off[fgi], fcnt = P.grp_cnt[fgi];
        const DHsp *H = P.hsp;
        const int fthr = group_thr(H, foff, fcnt, P.top_n);
        // per F_top row: R-existence of its pair
        uint32_t fsel = 0, rsel = 0, nrows = 0, nedges = 0;
        int M = INT_MIN;
        // pass over F_top rows: compute M and counts
        for (uint32_t i = 0; i < fcnt; i++) {
            const DHsp &f = H[foff + i];
            if (f.bits10 < fthr) continue;
            const uint32_t a = P.tx_gene[f.s_tx];
            const size_t rgi = (size_t)a * N + B;
            const uint32_t roff = P.grp_off[rgi], rcnt = P.grp_cnt[rgi];
            const int rthr = group_thr(H, roff, rcnt, P.top_n);
            bool inP = false;
            for (uint32_t j = 0; j < rcnt; j++) {
                const DHsp &r = H[roff + j];
                if (r.bits10 >= rthr && P.tx_gene[r.s_tx] == b) {
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
                const DHsp &f2 = H[foff + i2];
                if (f2.bits10 >= fthr && P.tx_gene[f2.s_tx] == a) {
                    first = false;
                    break;
                }
            }
            if (!first) continue;
            for (uint32_t j = 0; j < rcnt; j++) {
                const DHsp &r = H[roff + j];
                if (r.bits10 >= rthr && P.tx_gene[r.s_tx] == b) {
                    rsel++;
                    M = max(M, r.bits10);
                }
            }
        }
        // final rows: rows of C at M; pairs in ascending a; F rows then R rows
        // (keep "first": only the first such row)
        uint32_t prev_a = 0;
        bool have_prev = false, done = false;
        uint64_t row_w = pass ? P.row_off[item] : 0, edge_w = pass ? P.edge_off[item] : 0;
        const uint64_t fsel_base = pass ? P.fsel_off[item] - P.fsel_off[P.pair_item_begin[pr]] : 0;
        const uint64_t fsel_pair_total =
            pass ? P.fsel_off[P.pair_item_begin[pr + 1]] - P.fsel_off[P.pair_item_begin[pr]] : 0;
        const uint64_t rsel_base = pass ? P.rsel_off[item] - P.rsel_off[P.pair_item_begin[pr]] : 0;
        while (fsel && !done) {
            // next smallest a among selected F rows
            bool found = false;
            uint32_t a = 0;
            for (uint32_t i = 0; i < fcnt; i++) {
                const DHsp &f = H[foff + i];
                if (f.bits10 < fthr) continue;
                const uint32_t ai = P.tx_gene[f.s_tx];
                if (have_prev && ai <= prev_a) continue;
                if (!found || ai < a) a = ai, found = true;
            }
            if (!found) break;
            prev_a = a;
            have_prev = true;
            const size_t rgi = (size_t)a * N + B;
            const uint32_t roff = P.grp_off[rgi], rcnt = P.grp_cnt[rgi];
            const int rthr = group_thr(H, roff, rcnt, P.top_n);
            auto r_sel = [&](uint32_t j) {
                const DHsp &r = H[roff + j];
                return r.bits10 >= rthr && P.tx_gene[r.s_tx] == b;
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
                const DHsp &f = H[foff + i];
                if (f.bits10 < fthr || P.tx_gene[f.s_tx] != a || f.bits10 != M) continue;
                if (pass) {
                    // label: rank among F_sel rows of b in F_top order + earlier genes
                    const uint32_t rk = desc_rank(H, foff, fcnt, i, [&](uint32_t j) {
                        const DHsp &f2 = H[foff + j];
                        if (f2.bits10 < fthr) return false;
                        const uint32_t a2 = P.tx_gene[f2.s_tx];
                        const size_t g2 = (size_t)a2 * N + B;
                        const uint32_t o2 = P.grp_off[g2], c2 = P.grp_cnt[g2];
                        const int t2 = group_thr(H, o2, c2, P.top_n);
                        for (uint32_t k2 = 0; k2 < c2; k2++)
                            if (H[o2 + k2].bits10 >= t2 && P.tx_gene[H[o2 + k2].s_tx] == b) return true;
                        return false;
                    });
                    DRow row;
                    row.hsp = foff + i;
                    row.reverse = 0;
                    row.label = (int32_t)(fsel_base + rk);
                    row.pad = 0;
                    P.rows[row_w++] = row;
                }
                en += f.nident;
                ed += f.length - f.gaps;
                erows++;
                if (!P.keep_all) done = true;
            }
            // R rows of this pair at M
            for (uint32_t j = 0; j < rcnt && !done; j++) {
                if (!r_sel(j) || H[roff + j].bits10 != M) continue;
                const DHsp &r = H[roff + j];
                if (pass) {
                    // R_sel order: pairs by first appearance in F_top order, then R_top order
                    uint64_t before = 0;
                    // F_top rank of this pair's first F row
                    uint32_t myfirst = 0xFFFFFFFFu;
                    for (uint32_t i = 0; i < fcnt; i++) {
                        const DHsp &f = H[foff + i];
                        if (f.bits10 >= fthr && P.tx_gene[f.s_tx] == a) {
                            const uint32_t rk = desc_rank(H, foff, fcnt, i, [&](uint32_t jj) {
                                return H[foff + jj].bits10 >= fthr;
                            });
                            myfirst = min(myfirst, rk);
                        }
                    }
                    // R rows of pairs whose first F_top row precedes ours
                    for (uint32_t i = 0; i < fcnt; i++) {
                        const DHsp &f = H[foff + i];
                        if (f.bits10 < fthr) continue;
                        const uint32_t a2 = P.tx_gene[f.s_tx];
                        if (a2 == a) continue;
                        // is f the first F_top row of pair a2?
                        const uint32_t rk = desc_rank(H, foff, fcnt, i, [&](uint32_t jj) {
                            return H[foff + jj].bits10 >= fthr;
                        });
                        bool firstrow = true;
                        for (uint32_t i2 = 0; i2 < fcnt; i2++) {
                            if (i2 == i) continue;
                            const DHsp &f2 = H[foff + i2];
                            if (f2.bits10 < fthr || P.tx_gene[f2.s_tx] != a2) continue;
                            const uint32_t rk2 = desc_rank(H, foff, fcnt, i2, [&](uint32_t jj) {
                                return H[foff + jj].bits10 >= fthr;
                            });
                            if (rk2 < rk) firstrow = false;
                        }
                        if (!firstrow || rk > myfirst) continue;
                        const size_t g2 = (size_t)a2 * N + B;
                        const uint32_t o2 = P.grp_off[g2], c2 = P.grp_cnt[g2];
                        const int t2 = group_thr(H, o2, c2, P.top_n);
                        for (uint32_t k2 = 0; k2 < c2; k2++)
                            if (H[o2 + k2].bits10 >= t2 && P.tx_gene[H[o2 + k2].s_tx] == b) before++;
                    }
                    const uint32_t rk = desc_rank(H, roff, rcnt, j, r_sel);
                    DRow row;
                    row.hsp = roff + j;
                    row.reverse = 1;
                    row.label = (int32_t)(fsel_pair_total + rsel_base + before + rk);
                    row.pad = 0;
                    P.rows[row_w++] = row;
                }
                en += r.nident;
                ed += r.length - r.gaps;
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
                    P.edges[edge_w++] = e;
                }
                nedges++;
            }
        }
        if (!pass) {
            P.n_rows[item] = nrows;
            P.n_fsel[item] = fsel;
            P.n_rsel[item] = rsel;
            P.n_edges[item] = nedges;
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
    for (uint64_t e = tid; e < n_edges; e += nt) atomicAdd(&cedges[parent[edges[e].a]], 1u);
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
                                uint8_t *ideal, unsigned long long *stats)
{
    __shared__ int S;
    if (threadIdx.x == 0) {
        int s = 0;
        for (int i = 0; i < N; i++) s += sample_present[i] ? 1 : 0;
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
                                 const uint8_t *ideal, unsigned long long *num, unsigned long long *den)
{
    // Edges are stored pair-major, so a wave usually sees one pair: reduce in
    // registers and issue one atomic per wave; mixed waves fall back to lanes.
    const uint64_t nt = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t start = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const uint64_t iters = (n_edges + nt - 1) / nt;
    for (uint64_t it = 0; it < iters; it++) {
        const uint64_t e = start + it * nt;
        uint32_t pair = 0xFFFFFFFFu;
        unsigned long long a = 0, b = 0;
        if (e < n_edges) {
            const DEdge ed = edges[e];
            pair = ed.pair;
            if (ideal[parent[ed.a]]) {
                a = (unsigned long long)ed.nident;
                b = (unsigned long long)ed.den;
            }
        }
        const uint32_t p0 = __shfl(pair, 0);
        if (__ballot(pair != p0 && pair != 0xFFFFFFFFu) == 0) {
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) {
                a += __shfl_xor(a, off);
                b += __shfl_xor(b, off);
            }
            if ((threadIdx.x & 63) == 0 && p0 != 0xFFFFFFFFu && (a || b)) {
                atomicAdd(&num[p0], a);
                atomicAdd(&den[p0], b);
            }
        } else if (pair != 0xFFFFFFFFu && (a || b)) {
            atomicAdd(&num[pair], a);
            atomicAdd(&den[pair], b);
        }
    }
}

// d = float(1 - Fraction(num, den)) = correctly rounded (den - num) / den
__global__ void distance_kernel(const unsigned long long *num, const unsigned long long *den,
                                const int32_t *pair_index, const int32_t *order, int N, double *out,
                                unsigned int *status)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= N * N) return;
    const int i = t / N, j = t % N;
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
                      const uint64_t *out_off, uint32_t *keys, uint64_t *vals, hipStream_t st)
{
    if (amb)
        hipLaunchKernelGGL(kmer_fill_kernel<true>, dim3(n_tx), dim3(256), 0, st, tx, n_tx, F, AF, out_off,
                           keys, vals);
    else
        hipLaunchKernelGGL(kmer_fill_kernel<false>, dim3(n_tx), dim3(256), 0, st, tx, n_tx, F, AF, out_off,
                           keys, vals);
}

void launch_bucket_fill(const uint32_t *keys, uint64_t n, int bits, uint32_t *bucket, hipStream_t st)
{
    hipLaunchKernelGGL(bucket_fill_kernel, dim3(grid_for(n + 1, 256)), dim3(256), 0, st, keys, n, bits,
                       bucket);
}

void launch_align(bool amb, const Db &db, const Index &ix, const AlignParams &P, hipStream_t st)
{
    const uint32_t n = P.gene_end - P.gene_begin;
    if (n == 0) return;
    if (amb)
        hipLaunchKernelGGL(align_kernel<true>, dim3(n), dim3(ABLOCK), 0, st, db, ix, P);
    else
        hipLaunchKernelGGL(align_kernel<false>, dim3(n), dim3(ABLOCK), 0, st, db, ix, P);
}

void launch_rbh(const RbhParams &P, int pass, hipStream_t st)
{
    if (P.n_items == 0) return;
    hipLaunchKernelGGL(rbh_kernel, dim3(grid_for(P.n_items, 256)), dim3(256), 0, st, P, pass);
}

void launch_cc(const DEdge *edges, uint64_t n_edges, uint32_t n_nodes, const int32_t *gene_sample, int N,
               uint32_t *parent, uint32_t *present, uint32_t *cnodes, uint32_t *cedges,
               uint32_t *sample_present, uint8_t *ideal, unsigned long long *stats, hipStream_t st)
{
    const unsigned gn = grid_for(n_nodes, 256), ge = grid_for(n_edges, 256);
    hipLaunchKernelGGL(cc_init_kernel, dim3(gn), dim3(256), 0, st, parent, present, cnodes, cedges, n_nodes);
    if (n_edges) hipLaunchKernelGGL(cc_hook_kernel, dim3(ge), dim3(256), 0, st, edges, n_edges, parent, present);
    hipLaunchKernelGGL(cc_compress_kernel, dim3(gn), dim3(256), 0, st, parent, n_nodes);
    hipLaunchKernelGGL(cc_count_kernel, dim3(grid_for(n_edges > n_nodes ? n_edges : n_nodes, 256)), dim3(256), 0,
                       st, edges, n_edges, parent, present, gene_sample, n_nodes, cnodes, cedges, sample_present);
    hipLaunchKernelGGL(cc_ideal_kernel, dim3(gn), dim3(256), 0, st, parent, present, cnodes, cedges, n_nodes,
                       sample_present, N, ideal, stats);
}

void launch_pair_sums(const DEdge *edges, uint64_t n_edges, const uint32_t *parent, const uint8_t *ideal,
                      unsigned long long *num, unsigned long long *den, hipStream_t st)
{
    if (!n_edges) return;
    hipLaunchKernelGGL(pair_sums_kernel, dim3(grid_for(n_edges, 256)), dim3(256), 0, st, edges, n_edges, parent,
                       ideal, num, den);
}

void launch_distance(const unsigned long long *num, const unsigned long long *den, const int32_t *pair_index,
                     const int32_t *order, int N, double *out, unsigned int *status, hipStream_t st)
{
    const int n = N * N;
    if (!n) return;
    hipLaunchKernelGGL(distance_kernel, dim3((n + 255) / 256), dim3(256), 0, st, num, den, pair_index, order, N,
                       out, status);
}

}  // namespace rcg

// The seed index's radix sort, hand-written for gfx950 (replaces rocPRIM's
// onesweep in the index build).
//
// Keys are the index entries (k-mer << 32 | position), sorted stably on the
// key bits [bb, 64) -- the k-mer (bb = 32) for the main index, all 64 bits for
// the reverse pass's near-mask index -- by least-significant-digit passes of 8
// bits. One launch per pass (onesweep: decoupled look-back), with the array
// cut into OS_SEG segments that are independent look-back chains:
//
//   * segments: pass 0's input in OS_SEG equal ranges; pass p's input (pass
//     p-1's output) in the ranges of pass p-1's digit groups (256 / OS_SEG
//     consecutive digits each). A digit's output range is then the segments'
//     shares one after another, so the pass stays stable, and the counts that
//     place them -- how many keys of segment s have digit d -- are counted for
//     every pass before the first (seg_hist_kernel: one read of the keys).
//   * tiles of OS_TILE keys within a segment, taken from a counter in
//     round-robin order over the segments (tile j of every segment, then tile
//     j + 1): a tile's look-back predecessor was taken OS_SEG tiles earlier,
//     so the look-back finds a published prefix after few steps (one chain over
//     the whole array left every tile walking back over the tiles in flight).
//   * each wave ranks its keys stably by digit: item j of lane l is key
//     j * 64 + l of the wave's slice, matched against the wave's other lanes
//     by 8 ballots (one per digit bit) and counted in the wave's own LDS
//     histogram, so equal digits keep their input order;
//   * the tile's per-digit counts are published to the look-back table as
//     {tag, count} granules (agent-scope 64-bit stores; the tag carries the
//     pass's epoch, so the table needs no clearing between passes) and each
//     digit's exclusive prefix over the segment's earlier tiles is summed back
//     to a tile whose inclusive prefix is published;
//   * the keys go to LDS in digit order and leave in runs per digit, each run
//     to consecutive global slots.
#include "device.h"

#include <algorithm>
#include <functional>
#include <utility>

namespace rcg {

namespace {
#ifndef OS_BLOCK_M
#define OS_BLOCK_M 512
#endif
#ifndef OS_ITEMS_M
#define OS_ITEMS_M 16
#endif
#ifndef OS_MINB
#define OS_MINB 2                              // workgroups per CU
#endif
constexpr int OS_BLOCK = OS_BLOCK_M;           // 8 waves
constexpr int OS_WAVES = OS_BLOCK / 64;
constexpr int OS_ITEMS = OS_ITEMS_M;           // keys per thread
constexpr int OS_TILE = OS_BLOCK * OS_ITEMS;   // 8192 keys, 64 KB of LDS
constexpr int RADIX = 256;
constexpr int HIST_BLOCK = 256;
constexpr int HIST_MAXP = 8;
#ifndef OS_SEG_M
#define OS_SEG_M 8
#endif
constexpr int OS_SEG = OS_SEG_M;               // look-back chains per pass (power of 2)
static_assert(OS_SEG >= 1 && OS_SEG <= 16 && (OS_SEG & (OS_SEG - 1)) == 0,
              "seg_hist_kernel holds 8 passes x OS_SEG x 256 counters in LDS (<= 128 KB)");
constexpr int OS_GSH = 8 - (OS_SEG >= 64 ? 6 : OS_SEG >= 32 ? 5 : OS_SEG >= 16 ? 4 : OS_SEG >= 8 ? 3 : OS_SEG >= 4 ? 2
                                                                                         : OS_SEG >= 2 ? 1 : 0);
// scratch (u32 words): per pass the segment histograms H[S][256], segment
// bases SB[S][256], digit bases [256], segment offsets [S + 1], tile bases
// [S + 1]; tile counters; then the claim order of the current pass
constexpr uint64_t OS_PASS_WORDS = 2 * OS_SEG * RADIX + RADIX + 2 * 64 + 2;
constexpr uint64_t OS_FIXED_WORDS = HIST_MAXP * OS_PASS_WORDS + HIST_MAXP;
}   // namespace

typedef __attribute__((address_space(1))) unsigned long long gu64;

struct PassTab {
    uint32_t *H, *SB, *base, *segoff, *tbase;
};
__host__ __device__ inline PassTab pass_tab(uint32_t *scratch, int p)
{
    uint32_t *q = scratch + (uint64_t)p * OS_PASS_WORDS;
    return {q, q + OS_SEG * RADIX, q + 2 * OS_SEG * RADIX, q + 2 * OS_SEG * RADIX + RADIX,
            q + 2 * OS_SEG * RADIX + RADIX + 64};
}

// Segment histograms of every pass, one read of the keys: pass 0 counts digit
// 0 per input segment (index / segsize), pass p >= 1 counts digit p per digit
// group of digit p - 1. Per-block LDS tables (np * S * 256 u32, dynamic),
// added to H at the end.
__global__ __launch_bounds__(HIST_BLOCK) void seg_hist_kernel(const uint64_t *__restrict__ keys, uint64_t n, int bb,
                                                              int np, uint64_t segsize, uint32_t *scratch)
{
    extern __shared__ uint32_t h[];
    const int tab = OS_SEG * RADIX;
    for (int i = threadIdx.x; i < np * tab; i += HIST_BLOCK) h[i] = 0;
    __syncthreads();
    // 8 keys per thread in flight at a time (coalesced: key q of a thread is
    // HIST_BLOCK apart), then their counts
    constexpr int HQ = 8;
    const uint64_t stride = (uint64_t)gridDim.x * HIST_BLOCK * HQ;
    for (uint64_t i0 = (uint64_t)blockIdx.x * HIST_BLOCK * HQ + threadIdx.x; i0 < n; i0 += stride) {
        uint64_t kk[HQ];
#pragma unroll
        for (int q = 0; q < HQ; q++) {
            const uint64_t i = i0 + (uint64_t)q * HIST_BLOCK;
            kk[q] = i < n ? keys[i] : 0ull;
        }
#pragma unroll
        for (int q = 0; q < HQ; q++) {
            const uint64_t i = i0 + (uint64_t)q * HIST_BLOCK;
            if (i >= n) break;
            uint32_t prev = (uint32_t)(i / segsize);
            for (int p = 0; p < np; p++) {
                const uint32_t d = (uint32_t)(kk[q] >> (bb + 8 * p)) & 255u;
                atomicAdd(&h[p * tab + (p ? (prev >> OS_GSH) : prev) * RADIX + d], 1u);
                prev = d;
            }
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < np * tab; i += HIST_BLOCK)
        if (h[i]) atomicAdd(&pass_tab(scratch, i / tab).H[i % tab], h[i]);
}

// Every pass's tables from the histograms (one block, thread d = digit):
// digit bases, segment bases SB[s][d] = base[d] + sum_{s' < s} H[s'][d],
// segment offsets (pass 0: equal ranges; pass p: pass p-1's digit groups),
// tile bases (segment-major tile numbering).
__global__ __launch_bounds__(RADIX) void seg_scan_kernel(uint32_t *scratch, int np, uint64_t n, uint64_t segsize)
{
    __shared__ uint32_t s[RADIX];
    const int d = threadIdx.x;
    for (int p = 0; p < np; p++) {
        const PassTab T = pass_tab(scratch, p);
        uint32_t tot = 0;
        for (int g = 0; g < OS_SEG; g++) tot += T.H[g * RADIX + d];
        s[d] = tot;
        __syncthreads();
        for (int o = 1; o < RADIX; o <<= 1) {
            const uint32_t v = d >= o ? s[d - o] : 0u;
            __syncthreads();
            s[d] += v;
            __syncthreads();
        }
        const uint32_t base = s[d] - tot;
        T.base[d] = base;
        uint32_t acc = base;
        for (int g = 0; g < OS_SEG; g++) {
            T.SB[g * RADIX + d] = acc;
            acc += T.H[g * RADIX + d];
        }
        __syncthreads();
        if (d == 0) {
            const PassTab Q = pass_tab(scratch, p > 0 ? p - 1 : 0);
            uint32_t tb = 0;
            for (int g = 0; g <= OS_SEG; g++) {
                uint64_t off;
                if (g == OS_SEG) off = n;
                else if (p == 0) off = std::min<uint64_t>((uint64_t)g * segsize, n);
                else off = Q.base[g << OS_GSH];
                T.segoff[g] = (uint32_t)off;
            }
            for (int g = 0; g < OS_SEG; g++) {
                T.tbase[g] = tb;
                tb += (T.segoff[g + 1] - T.segoff[g] + OS_TILE - 1) / OS_TILE;
            }
            T.tbase[OS_SEG] = tb;
        }
        __syncthreads();
    }
}

// The claim order of pass p's tiles: tile j of every segment (in segment
// order) before tile j + 1 of any. order[position] = segment-major tile id.
__global__ void tile_order_kernel(const uint32_t *scratch, int p, uint32_t *order, uint32_t tmax)
{
    const PassTab T = pass_tab(const_cast<uint32_t *>(scratch), p);
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= tmax || g >= T.tbase[OS_SEG]) return;
    int sg = 0;
    while (sg + 1 < OS_SEG && T.tbase[sg + 1] <= g) sg++;
    const uint32_t j = g - T.tbase[sg];
    uint32_t pos = 0;
    for (int q = 0; q < OS_SEG; q++) {
        const uint32_t nt = T.tbase[q + 1] - T.tbase[q];
        pos += std::min(nt, j) + (q < sg && nt > j ? 1u : 0u);
    }
    order[pos] = g;
}

// The index fill (kernels.hip kmer_fill_kernel, no ambiguity codes: entry
// koff[t] + o is window o of transcript t) with the sort's segment
// histograms counted on the way, so the sort does not read the keys to count
// them. Wave per transcript, grid-stride; per-block LDS tables.
__global__ __launch_bounds__(1024) void kmer_fill_hist_kernel(const TxInfo *__restrict__ tx, uint32_t n_tx,
                                                             const uint64_t *__restrict__ F,
                                                             const uint64_t *__restrict__ out_off,
                                                             uint64_t *__restrict__ ent, int np, uint64_t segsize,
                                                             uint32_t *scratch)
{
    extern __shared__ uint32_t h[];
    const int tab = OS_SEG * RADIX;
    for (int i = threadIdx.x; i < np * tab; i += blockDim.x) h[i] = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const uint32_t wpb = blockDim.x >> 6, nwave = gridDim.x * wpb;
    for (uint32_t t = blockIdx.x * wpb + (threadIdx.x >> 6); t < n_tx; t += nwave) {
        const TxInfo ti = tx[t];
        const int64_t nwin = (int64_t)ti.len - W16 + 1;
        const uint64_t base = out_off[t];
        for (int64_t o0 = 0; o0 < nwin; o0 += 64) {
            // the segment of the 64 entries: one division per wave (a segment
            // holds at least 64 entries once n >= 64 OS_SEG)
            const uint64_t i0 = base + (uint64_t)o0;
            const uint32_t s0 = (uint32_t)(i0 / segsize);
            const uint64_t nb = (uint64_t)(s0 + 1) * segsize;
            const int64_t o = o0 + lane;
            if (o >= nwin) continue;
            const uint64_t p = ti.start + (uint64_t)o;
            const uint32_t key = (uint32_t)win(F, p);
            const uint64_t i = base + (uint64_t)o;
            if (ent) ent[i] = ((uint64_t)key << 32) | p;   // null: the first pass generates the keys itself
            uint32_t prev = segsize >= 64 ? s0 + (i >= nb ? 1u : 0u) : (uint32_t)(i / segsize);
            for (int q = 0; q < np; q++) {
                const uint32_t d = (key >> (8 * q)) & 255u;
                atomicAdd(&h[q * tab + (q ? (prev >> OS_GSH) : prev) * RADIX + d], 1u);
                prev = d;
            }
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < np * tab; i += blockDim.x)
        if (h[i]) atomicAdd(&pass_tab(scratch, i / tab).H[i % tab], h[i]);
}

__device__ __forceinline__ uint32_t lanes_below(uint64_t m)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Pass 0 without the entry array: key i of the fill order is window
// i - koff[t] of tile transcript t (koff[t] <= i < koff[t + 1]), so the first
// pass computes it from the packed sequence instead of reading 8 bytes the
// fill would have written (transcripts without ambiguity codes).
struct KeyGen {
    const TxInfo *tx;
    const uint64_t *koff;   // n_tx + 1 entries
    const uint64_t *F;
    uint32_t n_tx;
    uint32_t *tile_tx;      // per pass-0 tile: its first transcript
};

// the transcript of entry i: last t with koff[t] <= i (binary search)
__device__ __forceinline__ uint32_t gen_tx_of(const uint64_t *koff, uint32_t n_tx, uint64_t i)
{
    uint32_t lo = 0, hi = n_tx;   // koff[lo] <= i < koff[hi]
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (koff[mid] <= i) lo = mid; else hi = mid;
    }
    return lo;
}

// the first transcript of every pass-0 tile (one thread per tile)
__global__ void gen_tile_tx_kernel(const uint32_t *scratch, KeyGen G, uint32_t tmax)
{
    const PassTab T = pass_tab(const_cast<uint32_t *>(scratch), 0);
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= tmax || g >= T.tbase[OS_SEG]) return;
    int sg = 0;
    while (sg + 1 < OS_SEG && T.tbase[sg + 1] <= g) sg++;
    const uint64_t t0 = (uint64_t)T.segoff[sg] + (uint64_t)(g - T.tbase[sg]) * OS_TILE;
    G.tile_tx[g] = gen_tx_of(G.koff, G.n_tx, t0);
}

#ifdef OS_STATS
__device__ unsigned long long os_stats[4];   // look-back loads, not-ready polls, tiles
#endif

// One tile: load; the tile's digit counts (LDS atomics) published at once;
// waves 0-3 then walk the look-back (one digit per thread) while waves 4-7
// rank their keys, and rank theirs after it; the keys go to LDS in digit
// order and out in runs.
template <bool GEN>
__global__ __launch_bounds__(OS_BLOCK, OS_MINB * OS_WAVES / 4) void onesweep_kernel(const uint64_t *__restrict__ in,
                                                                     uint64_t *__restrict__ out, int shift,
                                                                     const uint32_t *scratch, int p,
                                                                     const uint32_t *__restrict__ order,
                                                                     gu64 *status, uint32_t epoch, uint32_t *tile_ctr,
                                                                     uint64_t n_all, KeyGen G)
{
    static_assert(OS_BLOCK >= RADIX && OS_TILE <= 65536 && OS_ITEMS % 2 == 0, "one look-back thread per digit; 16-bit ranks");
    __shared__ uint64_t s_keys[OS_TILE];
    __shared__ uint32_t s_hist[OS_WAVES * RADIX];
    __shared__ uint32_t s_cnt[RADIX];
    __shared__ uint32_t s_start[RADIX];
    __shared__ uint64_t s_goff[RADIX];
    __shared__ uint32_t s_wsum[RADIX / 64];
    __shared__ uint32_t s_tile;
    constexpr int GTX = 64;   // GEN: the tile's transcripts staged (first entry, start); more: searched in HBM
    __shared__ uint64_t s_gk[GEN ? GTX + 1 : 1], s_gs[GEN ? GTX : 1];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const PassTab T = pass_tab(const_cast<uint32_t *>(scratch), p);
    if (tid == 0) {
        const uint32_t c = atomicAdd(tile_ctr, 1u);
        s_tile = c < T.tbase[OS_SEG] ? order[c] : 0xFFFFFFFFu;
    }
    for (int i = tid; i < OS_WAVES * RADIX; i += OS_BLOCK) s_hist[i] = 0;
    if (tid < RADIX) s_cnt[tid] = 0;
    __syncthreads();
    const uint32_t tile = s_tile;   // segment-major tile id (look-back index)
    if (tile == 0xFFFFFFFFu) return;
    int sg = 0;
    while (sg + 1 < OS_SEG && T.tbase[sg + 1] <= tile) sg++;
    const uint32_t tj = tile - T.tbase[sg];   // the tile's index within its segment
    const uint64_t t0 = (uint64_t)T.segoff[sg] + (uint64_t)tj * OS_TILE;
    const uint64_t n = std::min<uint64_t>(t0 + OS_TILE, T.segoff[sg + 1]);   // keys [t0, n)
    const uint64_t wbase = t0 + (uint64_t)w * (64 * OS_ITEMS) + (uint64_t)lane;
    uint64_t k[OS_ITEMS];
    if constexpr (GEN) {
        // the tile's transcripts from its first: their first entries and starts
        const uint32_t tf = G.tile_tx[tile];
        for (int q = tid; q <= GTX; q += OS_BLOCK) {
            const uint32_t t = tf + (uint32_t)q;
            s_gk[q] = t <= G.n_tx ? G.koff[t] : ~0ull;
            if (q < GTX) s_gs[q] = t < G.n_tx ? G.tx[t].start : 0ull;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < OS_ITEMS; j++) {
            const uint64_t i = wbase + (uint64_t)j * 64;
            uint64_t key = 0;
            if (i < n) {
                uint64_t st, k0;
                if (s_gk[GTX] > i) {   // among the staged transcripts: last q with first entry <= i
                    int lo = 0, hi = GTX;
                    while (hi - lo > 1) {
                        const int mid = (lo + hi) >> 1;
                        if (s_gk[mid] <= i) lo = mid; else hi = mid;
                    }
                    st = s_gs[lo];
                    k0 = s_gk[lo];
                } else {
                    const uint32_t t = gen_tx_of(G.koff, G.n_tx, i);
                    st = G.tx[t].start;
                    k0 = G.koff[t];
                }
                const uint64_t pos = st + (i - k0);
                key = ((uint64_t)(uint32_t)win(G.F, pos) << 32) | pos;
            }
            k[j] = key;
        }
    } else {
#pragma unroll
        for (int j = 0; j < OS_ITEMS; j++) {
            const uint64_t i = wbase + (uint64_t)j * 64;
            k[j] = i < n ? in[i] : 0ull;
        }
    }
    // the tile's digit counts
#pragma unroll
    for (int j = 0; j < OS_ITEMS; j++)
        if (wbase + (uint64_t)j * 64 < n) atomicAdd(&s_cnt[(uint32_t)(k[j] >> shift) & 255u], 1u);
    __syncthreads();
    const uint64_t gt_mask = lane == 63 ? 0ull : ~0ull << (lane + 1);
    uint32_t *hw = s_hist + w * RADIX;
    uint32_t r[OS_ITEMS / 2];   // two 16-bit ranks per register (a rank < OS_TILE)
    // stable rank of each key among the wave's keys of its digit
    auto rank = [&]() {
#pragma unroll
        for (int j = 0; j < OS_ITEMS; j++) {
            const bool valid = wbase + (uint64_t)j * 64 < n;
            const uint32_t d = (uint32_t)(k[j] >> shift) & 255u;
            uint64_t peers = __ballot(valid);
#pragma unroll
            for (int b = 0; b < 8; b++) {
                const bool bit = (d >> b) & 1u;
                const uint64_t m = __ballot(bit);
                peers &= bit ? m : ~m;
            }
            const uint32_t old = hw[d];
            const uint32_t rk = old + lanes_below(peers);
            if (j & 1) r[j >> 1] |= rk << 16;
            else r[j >> 1] = rk;
            if (valid && (peers & gt_mask) == 0) hw[d] = old + (uint32_t)__popcll(peers);
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
        }
    };
    if (tid < RADIX) {
        // publish this tile's count, then the exclusive prefix of the segment's
        // earlier tiles (decoupled look-back) and the inclusive one
        const uint32_t tot = s_cnt[tid];
        const uint64_t AGG = (uint64_t)(2u * epoch) << 32, INC = (uint64_t)(2u * epoch + 1u) << 32;
        gu64 *mine = status + (uint64_t)tile * RADIX + tid;
        uint32_t excl = 0;
#ifdef OS_STATS
        unsigned long long nl = 0, nw = 0;
#endif
        if (tj == 0) {
            __hip_atomic_store(mine, INC | tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            __hip_atomic_store(mine, AGG | tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            int64_t t = (int64_t)tile - 1;
            for (;;) {
                const uint64_t v = __hip_atomic_load(status + (uint64_t)t * RADIX + tid, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
                const uint32_t tag = (uint32_t)(v >> 32);
#ifdef OS_STATS
                nl++;
#endif
                if (tag == 2u * epoch + 1u) {
                    excl += (uint32_t)v;
                    break;
                }
                if (tag == 2u * epoch) {
                    excl += (uint32_t)v;
                    t--;
                } else {
#ifdef OS_STATS
                    nw++;
#endif
                    __builtin_amdgcn_s_sleep(1);
                }
            }
            __hip_atomic_store(mine, INC | (uint64_t)(excl + tot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
#ifdef OS_STATS
        atomicAdd(&os_stats[0], nl);
        atomicAdd(&os_stats[1], nw);
        if (tid == 0) atomicAdd(&os_stats[2], 1ull);
#endif
        // block exclusive scan of the counts over the 256 digits
        uint32_t x = tot;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) s_wsum[w] = x;
        s_start[tid] = x - tot;
        s_goff[tid] = (uint64_t)T.SB[sg * RADIX + tid] + excl;
    }
    rank();
    __syncthreads();
    if (tid < RADIX) {
        uint32_t add = 0;
        for (int v = 0; v < w; v++) add += s_wsum[v];
        const uint32_t st = s_start[tid] + add;
        s_start[tid] = st;
        s_goff[tid] -= st;
        // wave offsets: exclusive over the waves
        uint32_t acc = 0;
#pragma unroll
        for (int v = 0; v < OS_WAVES; v++) {
            const uint32_t c = s_hist[v * RADIX + tid];
            s_hist[v * RADIX + tid] = acc;
            acc += c;
        }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < OS_ITEMS; j++) {
        if (wbase + (uint64_t)j * 64 < n) {
            const uint32_t d = (uint32_t)(k[j] >> shift) & 255u;
            s_keys[s_start[d] + hw[d] + ((r[j >> 1] >> (16 * (j & 1))) & 0xFFFFu)] = k[j];
        }
    }
    __syncthreads();
    const uint32_t cnt = (uint32_t)(n - t0);
#pragma unroll 4
    for (uint32_t s = tid; s < cnt; s += OS_BLOCK) {
        const uint64_t key = s_keys[s];
        const uint64_t gi = s_goff[(uint32_t)(key >> shift) & 255u] + s;
        if (gi < n_all) out[gi] = key;   // always, unless the counts were inconsistent
    }
}

// Sort keys[0, n) stably on bits [bb, 64) by ping-pong passes between keys
// and alt; returns true when the result is in alt (odd pass count), false
// when it is back in keys. Scratch (caller-owned, device): os_scratch_words(n)
// u32, status os_status_words(n) u64 (zeroed once when allocated), epoch a
// counter the caller keeps across calls. n < 2^32.
uint64_t os_status_words(uint64_t n) { return ((n + OS_TILE - 1) / OS_TILE + OS_SEG) * (uint64_t)RADIX; }
uint64_t os_scratch_words(uint64_t n) { return OS_FIXED_WORDS + (n + OS_TILE - 1) / OS_TILE + OS_SEG; }

// after_prep (optional) runs once the tables and the first pass's claim order
// are queued, before the first pass: work for another stream that should not
// starve those one-block kernels (the engine starts DUST there).
// The index fill and the segment histograms of a 32-bit-key sort (bb = 32)
// in one kernel (transcripts without ambiguity codes; koff: first entry of
// each transcript); os_sort_keys(..., counted = true) then skips its count.
// ent == nullptr: counts only (the sort's first pass then generates the keys: os_sort_keys with gen).
void os_fill_hist(const TxInfo *tx, uint32_t n_tx, const uint64_t *F, const uint64_t *koff, uint64_t *ent,
                  uint64_t n, uint32_t *scratch, hipStream_t st)
{
    (void)hipMemsetAsync(scratch, 0, OS_FIXED_WORDS * sizeof(uint32_t), st);
    if (!n_tx || !n) return;
    const int np = 4;
    const uint64_t segsize = (n + OS_SEG - 1) / OS_SEG;
    // 16-wave blocks, two per CU (r05: 4.84-4.97 ms at C3 against 5.71 for
    // 2048 four-wave blocks, whose 32 KB tables made a second, partial round
    // of blocks and twice the closing atomics)
    const dim3 g(std::min<uint32_t>((n_tx + 15) / 16, 512));
    hipLaunchKernelGGL(kmer_fill_hist_kernel, g, dim3(1024), (size_t)np * OS_SEG * RADIX * sizeof(uint32_t), st, tx,
                       n_tx, F, koff, ent, np, segsize, scratch);
}

// gen (bb = 32, counted): the first pass computes the keys from the packed
// sequence F of the transcripts tx[0, n_tx) with first entries koff[0, n_tx]
// (keys need not hold them); gen_tile: scratch of os_gen_tile_words(n) u32.
uint64_t os_gen_tile_words(uint64_t n) { return (n + OS_TILE - 1) / OS_TILE + OS_SEG; }

bool os_sort_keys(uint64_t *keys, uint64_t *alt, uint64_t n, int bb, uint32_t *scratch, uint64_t *status,
                  uint32_t &epoch, hipStream_t st, const std::function<void()> &after_prep, bool counted,
                  const TxInfo *gen_tx, const uint64_t *gen_koff, const uint64_t *gen_F, uint32_t gen_ntx,
                  uint32_t *gen_tile)
{
    const int np = (64 - bb + 7) / 8;
    if (n == 0) return false;
    uint32_t *ctr = scratch + HIST_MAXP * OS_PASS_WORDS, *order = ctr + HIST_MAXP;
    const uint64_t segsize = (n + OS_SEG - 1) / OS_SEG;
    if (!counted) {
        (void)hipMemsetAsync(scratch, 0, OS_FIXED_WORDS * sizeof(uint32_t), st);
        const uint64_t hb = std::min<uint64_t>((n + HIST_BLOCK * 8 - 1) / (HIST_BLOCK * 8), 1024);
        hipLaunchKernelGGL(seg_hist_kernel, dim3((unsigned)hb), dim3(HIST_BLOCK),
                           (size_t)np * OS_SEG * RADIX * sizeof(uint32_t), st, keys, n, bb, np, segsize, scratch);
    }
    hipLaunchKernelGGL(seg_scan_kernel, dim3(1), dim3(RADIX), 0, st, scratch, np, n, segsize);
    const uint32_t tmax = (uint32_t)((n + OS_TILE - 1) / OS_TILE + OS_SEG);
    const unsigned grid = tmax;   // tiles beyond a pass's count exit at once
    uint64_t *src = keys, *dst = alt;
    const bool gen = counted && gen_koff && bb == 32;
    KeyGen G{gen_tx, gen_koff, gen_F, gen_ntx, gen_tile};
    for (int p = 0; p < np; p++) {
        hipLaunchKernelGGL(tile_order_kernel, dim3((tmax + 255) / 256), dim3(256), 0, st, scratch, p, order, tmax);
        if (p == 0 && gen)
            hipLaunchKernelGGL(gen_tile_tx_kernel, dim3((tmax + 255) / 256), dim3(256), 0, st, scratch, G, tmax);
        if (p == 0 && after_prep) after_prep();
        ++epoch;
        if (p == 0 && gen)
            hipLaunchKernelGGL(onesweep_kernel<true>, dim3(grid), dim3(OS_BLOCK), 0, st, src, dst, bb + 8 * p, scratch,
                               p, order, (gu64 *)status, epoch, ctr + p, n, G);
        else
            hipLaunchKernelGGL(onesweep_kernel<false>, dim3(grid), dim3(OS_BLOCK), 0, st, src, dst, bb + 8 * p,
                               scratch, p, order, (gu64 *)status, epoch, ctr + p, n, G);
        std::swap(src, dst);
    }
    return src == alt;
}

}  // namespace rcg

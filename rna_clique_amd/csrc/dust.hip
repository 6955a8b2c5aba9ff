// Symmetric DUST on the query transcripts (blastn's default query filter,
// -dust 20 64 1, used as a soft mask: it removes query words from seeding;
// extension runs through masked bases). Semantics: spec 1b of
// oracle/align_oracle.c (dust_run / dust_tx), bit for bit.
//
// Chunk-parallel. Whether an interval starting at s is perfect depends only
// on the bases from s on (its score, and the perfect intervals inside it,
// which start at or after s), and an interval is final once its start has
// left the window (W bases later). So the masked intervals starting in a
// chunk [c0, c1) of an ACGT run come out of the window scan started fresh at
// c0 and run to c1 + W - 1 (or the run's end): one lane per CHUNK bases, about
// (CHUNK + W) / CHUNK of the sequential work.
//
// The window lives in registers as two bit planes of the last 64 bases (low
// and high bit of each 2-bit base, bit a = the base a positions back), so
// "where in the window does triplet v occur" is a few 64-bit logic ops and a
// window count is a popcount: no per-triplet tables, no LDS, nothing between
// the lanes. Two phases per chunk, in one kernel:
//  A. the window scan (every lane at the same chunk offset each step, the
//     packed words reloading in lockstep): the window score rw and the start
//     Lst of the L-suffix (no triplet more than 2 level / 10 times; a new
//     occurrence past the bound moves Lst past the need-th previous one, a
//     bit position). Where some suffix longer than the L-suffix may pass the
//     level (rw * 10 > L * level: 0.7 % of the bases of random sequence),
//     the step only appends an event (position, rw, L) to the lane's list.
//  B. the lane's events in order: the suffixes past the L-suffix, shortest
//     first, against the perfect intervals found so far (per start, in global
//     scratch), from bit planes rebuilt out of the packed sequence. Deferring
//     this rare pass keeps the scan free of the long divergent loop that one
//     lane in three wave steps would otherwise impose on the whole wave.
#include "device.h"

#include <algorithm>

namespace rcg {

constexpr int DW = 64;          // lanes per block (one wave)
constexpr int DCHUNK = 256;     // bases per lane
constexpr int DWIN_MAX = 64;    // longest DUST window the kernel supports
constexpr int DEVCAP = 32;  // events a lane holds before it runs them (phase B) in the middle of its scan

#ifdef RC_DUST_PROF
__device__ unsigned long long g_dust_prof[4];   // cycles of phase A, phase B; events; B iterations (microbenchmarks)
#endif

__device__ __forceinline__ void dust_mark(uint64_t *mask, uint64_t a, uint64_t b)
{
    while (a < b) {   // bits [a, b): word by word
        const uint64_t w = a >> 6;
        const unsigned sh = (unsigned)(a & 63);
        const uint64_t n = min((uint64_t)(64 - sh), b - a);
        const uint64_t bits = (n == 64 ? ~0ull : ((1ull << n) - 1ull)) << sh;
        atomicOr(reinterpret_cast<unsigned long long *>(mask + w), (unsigned long long)bits);
        a += n;
    }
}

// bit i: base i of the planes (P0 low bits, P1 high bits) is c
__device__ __forceinline__ uint64_t base_eq(uint64_t P0, uint64_t P1, int c)
{
    return (P0 ^ ((c & 1) ? 0ull : ~0ull)) & (P1 ^ ((c & 2) ? 0ull : ~0ull));
}
// bits [lo, hi] (0 <= lo, hi <= 63; empty when hi < lo)
__device__ __forceinline__ uint64_t bit_range(int lo, int hi)
{
    if (hi < lo) return 0ull;
    const uint64_t up = hi >= 63 ? ~0ull : ((1ull << (hi + 1)) - 1ull);
    return up & ~((1ull << lo) - 1ull);
}
// the even bits of x packed into the low 32 (a 2-bit base word -> one bit plane)
__device__ __forceinline__ uint64_t even_bits(uint64_t x)
{
    x &= 0x5555555555555555ull;
    x = (x | (x >> 1)) & 0x3333333333333333ull;
    x = (x | (x >> 2)) & 0x0F0F0F0F0F0F0F0Full;
    x = (x | (x >> 4)) & 0x00FF00FF00FF00FFull;
    x = (x | (x >> 8)) & 0x0000FFFF0000FFFFull;
    return (x | (x >> 16)) & 0x00000000FFFFFFFFull;
}

#ifndef RC_DUST_MINW
#define RC_DUST_MINW 7   // waves per SIMD the registers must allow: 7 measured best (21.4 ms at 5 waves, 20.1 at 7, 21.1 at 8)
#endif
template <bool AMB>
__global__ __launch_bounds__(DW, RC_DUST_MINW) void dust_kernel(uint64_t total, uint64_t nwords, const uint64_t *__restrict__ F,
                                                  const uint64_t *__restrict__ AF,
                                                  const uint64_t *__restrict__ txstart, int T, int W,
                                                  uint64_t *__restrict__ evs, uint32_t *__restrict__ scratch,
                                                  uint64_t *__restrict__ mask)
{
    const int lane = threadIdx.x;
    const int need = (2 * T) / 10;   // occurrences before a new one that break the L-suffix bound
    uint32_t *slot = scratch + ((size_t)blockIdx.x * DW + lane) * DWIN_MAX;   // [run offset of the start & 63]
    uint64_t *ev = evs + (size_t)blockIdx.x * DEVCAP * 3 * DW + lane;         // [event][field][lane]
    const uint64_t nchunk = (total + DCHUNK - 1) / DCHUNK;
    auto word = [&](uint64_t w) -> uint64_t { return w < nwords ? F[w] : 0ull; };
    auto aword = [&](uint64_t w) -> uint64_t { return AMB && w < nwords ? AF[w] : 0ull; };
    for (uint64_t ch = (uint64_t)blockIdx.x * DW + lane; ch < nchunk; ch += (uint64_t)gridDim.x * DW) {
        const uint64_t c0 = ch * DCHUNK, c1 = min(c0 + DCHUNK, total);
        const uint64_t lim = min(c1 + (uint64_t)W, total);   // the scan's reach
        // ---------------- B: the lane's events, in order (state kept across runs of B) ----------------
#ifdef RC_DUST_PROF
        unsigned long long its = 0, tb = 0;
#endif
        uint64_t set = 0, prs = ~0ull;   // slots holding a perfect interval; their run's start
        int pw = 0;                      // window start (run offset) of the previous event
        auto finalize = [&](uint64_t keep_from) {   // the perfect intervals starting before keep_from (run offset) are final
            uint64_t m = set;
            while (m) {
                const int k = __builtin_ctzll(m);
                m &= m - 1;
                const uint64_t a = (uint64_t)pw + (uint64_t)((k - pw) & 63);
                if (a >= keep_from) continue;
                const uint32_t s = slot[k];
                if (prs + a < c1) dust_mark(mask, prs + a, prs + a + ((s >> 20) & 0x1FFu));
                set &= ~(1ull << k);
            }
        };
        int nev = 0;
        auto run_events = [&]() {
#ifdef RC_DUST_PROF
        const unsigned long long tq = __builtin_readcyclecounter();
#endif
        // an event: (j, rw, L, rel) and the bit planes of its window
        uint64_t nx = nev ? ev[0] : 0ull, nq0 = nev ? ev[DW] : 0ull, nq1 = nev ? ev[2 * DW] : 0ull;
        for (int e = 0; e < nev; e++) {
            const uint64_t x = nx, Q0 = nq0, Q1 = nq1;
            if (e + 1 < nev) {   // the next event's loads in flight meanwhile
                nx = ev[(size_t)(3 * e + 3) * DW];
                nq0 = ev[(size_t)(3 * e + 4) * DW];
                nq1 = ev[(size_t)(3 * e + 5) * DW];
            }
            const int rel = (int)(x & 0x1FF), Lq = (int)((x >> 9) & 63), rwe = (int)((x >> 15) & 0x7FF);
            const int32_t j = (int32_t)(x >> 26), pt = j - 2, wstart = max(j + 1 - W, 0), Lst = pt + 1 - Lq;
            const uint64_t r0 = c0 + (uint64_t)rel - (uint64_t)j;   // the run's start
            if (r0 != prs) {
                finalize(~0ull);
                prs = r0;
            } else {
                finalize((uint64_t)wstart);
            }
            pw = wstart;
            // Q0/Q1: bit a = the base a positions before j. The triplet starting
            // at st ends pt - st back; those starting later in (st, pt] end
            // 0 .. pt - st - 1 back.
            auto later = [&](int32_t st) -> int {
                const int a = pt - st;   // the triplet's last base is a back, its first a + 2
                const uint64_t t0 = Q0 >> a, t1 = Q1 >> a;
                const int bl = (int)((t0 & 1) | ((t1 & 1) << 1)), bm = (int)(((t0 >> 1) & 1) | (t1 & 2)),
                          bf = (int)(((t0 >> 2) & 1) | ((t1 >> 1) & 2));
                // bit e: the triplet ending e back equals it (masks from the codes:
                // a select among precomputed masks would be an indexed array, i.e. scratch)
                const uint64_t eq = (base_eq(Q0, Q1, bf) >> 2) & (base_eq(Q0, Q1, bm) >> 1) & base_eq(Q0, Q1, bl);
                return a ? __builtin_popcountll(eq & bit_range(0, a - 1)) : 0;
            };
            int r = 0;
            for (int32_t st = Lst; st <= pt; st++) r += later(st);   // the L-suffix's score
            int mr = 0, ml = 0;
            {   // best ratio of the perfect intervals inside the L-suffix
                uint64_t m = set;
                while (m) {
                    const int k = __builtin_ctzll(m);
                    m &= m - 1;
                    if (wstart + ((k - wstart) & 63) < Lst) continue;
                    const uint32_t s = slot[k];
                    const int sr = (int)(s & 0xFFF), sl = (int)((s >> 12) & 0xFF);
                    if (mr == 0 || sr * ml > mr * sl) { mr = sr; ml = sl; }
                }
            }
            for (int32_t st = Lst - 1; st >= wstart; st--) {
                const int l = pt - st;
                if (T * l >= 10 * rwe) break;   // no longer suffix can pass the level
#ifdef RC_DUST_PROF
                its++;
#endif
                r += later(st);
                const int k = st & 63;
                const bool has = (set >> k) & 1ull;
                const uint32_t s = has ? slot[k] : 0u;
                const int sr = (int)(s & 0xFFF), sl = (int)((s >> 12) & 0xFF);
                if (has && (mr == 0 || sr * ml > mr * sl)) { mr = sr; ml = sl; }
                if (r * 10 > T * l && (mr == 0 || r * ml >= mr * l)) {
                    const int end = j + 1 - st;   // end - start
                    int nr = r, nl = l;
                    if (has && !(r * sl > sr * l)) { nr = sr; nl = sl; }
                    const int ne = has ? max(end, (int)((s >> 20) & 0x1FF)) : end;
                    slot[k] = ((uint32_t)ne << 20) | ((uint32_t)nl << 12) | (uint32_t)nr;
                    set |= 1ull << k;
                    mr = r;
                    ml = l;
                }
            }
#ifdef RC_DUST_PROF
            its += (unsigned long long)Lq;
#endif
        }
        nev = 0;
#ifdef RC_DUST_PROF
        tb += __builtin_readcyclecounter() - tq;
#endif
        };
        // ---------------- A: the window scan over [c0, lim) ----------------
#ifdef RC_DUST_PROF
        const unsigned long long tp0 = __builtin_readcyclecounter();
#endif
        // The scan goes a packed word (32 bases) at a time: the words of the
        // next block are loaded at the top of a block and only rotated in at
        // its end, so their latency hides behind 32 steps (a load rotated per
        // step would make every step wait for it).
        const uint64_t w0 = c0 >> 5;   // c0 is a multiple of 64
        const uint64_t t0i = c0 >> 6, tmax = (total >> 6) + 1;
        uint64_t wpp = 0, wp = 0, wc = word(w0), ac = aword(w0), tc = txstart[t0i];
        const int o = 66 - W;   // the trailing cursor's first base in the 96-base window (wpp, wp, wc)
        uint64_t P0 = 0, P1 = 0;   // bit planes of the last 64 bases, bit a = a bases back
        bool in_run = false, done = false;
        int nb = 0, tri = 0, tri2 = 0, rw = 0, Lst = 0;
        for (uint64_t k = 0; !done && c0 + 32 * k < lim; k++) {
            const uint64_t wn = word(w0 + k + 1), an = aword(w0 + k + 1);
            const uint64_t ti = t0i + ((k + 1) >> 1);
            const uint64_t tn = ti <= tmax ? txstart[ti] : 0ull;
            // the trailing bases of this block (32 k + i - W + 2) and its transcript-start bits
            const uint64_t tw = o < 32 ? (wpp >> (2 * o)) | (wp << (64 - 2 * o))
                                       : (o == 32 ? wp : (wp >> (2 * (o - 32))) | (wc << (64 - 2 * (o - 32))));
            const uint32_t txb = (uint32_t)(tc >> (32 * (k & 1)));
            for (int i = 0; i < 32; i++) {
                const uint64_t rel = 32 * k + (uint64_t)i;
                const uint64_t u = c0 + rel;
                if (u >= lim) {
                    done = true;
                    break;
                }
                const bool amb = AMB && ((ac >> (2 * i)) & 3u);
                const int b = (int)((wc >> (2 * i)) & 3u);
                // the trailing cursor: the triplet that leaves the window starts at u - W
                if ((int64_t)rel - W + 2 >= 0) tri2 = ((tri2 << 2) | (int)((tw >> (2 * i)) & 3u)) & 63;
                if (in_run && (amb || ((txb >> i) & 1u))) in_run = false;   // ambiguous base or next transcript
                if (amb) {
                    if (u >= c1) {
                        done = true;
                        break;
                    }
                    continue;
                }
                if (!in_run) {
                    if (u >= c1) {   // runs starting past the chunk are the next lane's
                        done = true;
                        break;
                    }
                    in_run = true;
                    nb = rw = Lst = 0;
                }
                nb++;
                tri = ((tri << 2) | b) & 63;
                P0 = (P0 << 1) | (uint64_t)(b & 1);
                P1 = (P1 << 1) | (uint64_t)(b >> 1);
                if (nb < 3) continue;
                const int32_t j = nb - 1;        // run offset of u
                const int32_t pt = j - 2;        // start of the new triplet
                const int32_t wstart = max(j + 1 - W, 0);
                // the window without the new triplet, after the leaving one (start
                // j - W) is gone: the triplets ending 1 .. W - 3 bases back that
                // start in the run. Bit e of trip(v): the triplet ending e back is v.
                const uint64_t wm = bit_range(1, min(W - 3, j - 2));
                auto trip = [&](int v) -> uint64_t {
                    return (base_eq(P0, P1, v >> 4) >> 2) & (base_eq(P0, P1, (v >> 2) & 3) >> 1) & base_eq(P0, P1, v & 3);
                };
                if (j >= W) rw -= __builtin_popcountll(trip(tri2) & wm);   // its partners in the window
                const uint64_t e3 = trip(tri) & wm;
                const int cw = __builtin_popcountll(e3);
                rw += cw;
                Lst = max(Lst, wstart);
                if (cw >= need) {   // the need-th previous occurrence (need-th lowest bit) is in the window
                    uint64_t m = e3;
                    for (int q = 1; q < need; q++) m &= m - 1;
                    const int p = need ? pt - (int)__builtin_ctzll(m) : pt;
                    if (p >= Lst) Lst = p + 1;
                }
                if (rw * 10 <= (pt - Lst + 1) * T) continue;
                // rare: B tries the longer suffixes; event = j | rw | L | rel
#ifndef RC_DUST_NO_B
                ev[(size_t)(3 * nev) * DW] = ((uint64_t)j << 26) | ((uint64_t)rw << 15) | ((uint64_t)(pt - Lst + 1) << 9) | rel;
                ev[(size_t)(3 * nev + 1) * DW] = P0;
                ev[(size_t)(3 * nev + 2) * DW] = P1;
                if (++nev == DEVCAP) run_events();
#else
                nev++;
#endif
            }
            wpp = wp;
            wp = wc;
            wc = wn;
            ac = an;
            if (k & 1) tc = tn;
        }
#ifdef RC_DUST_PROF
        const unsigned long long tp1 = __builtin_readcyclecounter();
#endif
#ifndef RC_DUST_NO_B
        run_events();
#endif
        finalize(~0ull);   // the last run's intervals (its end, or the scan's reach)
#ifdef RC_DUST_PROF
        const unsigned long long tp2 = __builtin_readcyclecounter();
        if (lane == 0) {
            atomicAdd(&g_dust_prof[0], tp1 - tp0);   // the scan (with any runs of B in it)
            atomicAdd(&g_dust_prof[1], tp2 - tp1);   // the last run of B
        }
        atomicAdd(&g_dust_prof[3], its);
        atomicAdd(&g_dust_prof[2], (unsigned long long)nev);
#endif
    }
}

// gaps shorter than `linker` between masked runs of one transcript (spec 1b;
// a no-op for linker <= 1): one thread per transcript over its mask words
__global__ void dust_linker_kernel(const TxInfo *__restrict__ tx, uint32_t n_tx, int linker, uint64_t *mask)
{
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < n_tx; t += gridDim.x * blockDim.x) {
        const TxInfo ti = tx[t];
        int64_t last = -1;   // end of the last masked run (transcript offset)
        for (int64_t u = 0; u < (int64_t)ti.len;) {
            const uint64_t g = ti.start + (uint64_t)u;
            const uint64_t w = win_bits(mask, (int64_t)g);
            const int room = (int)min<int64_t>(64, (int64_t)ti.len - u);
            const uint64_t vm = room == 64 ? ~0ull : ((1ull << room) - 1ull);
            const uint64_t set = w & vm;
            if (!set) {
                u += room;
                continue;
            }
            const int a = __builtin_ctzll(set);
            const uint64_t clear_above = ~(set >> a) & (vm >> a);
            const int len = clear_above ? __builtin_ctzll(clear_above) : room - a;
            const int64_t s = u + a;
            if (last >= 0 && s > last && s - last < linker) dust_mark(mask, ti.start + (uint64_t)last, ti.start + (uint64_t)s);
            last = s + len;
            u = s + len;
        }
    }
}

void launch_dust(bool amb, uint64_t total, const uint64_t *F, const uint64_t *AF, const uint64_t *txstart,
                 const TxInfo *tx, uint32_t n_tx, int level, int window, int linker, uint32_t *scratch,
                 uint64_t *events, uint32_t scratch_blocks, int max_waves, uint64_t *mask, hipStream_t st)
{
    if (total == 0) return;
    const uint64_t nchunk = (total + DCHUNK - 1) / DCHUNK;
    // every block resident at once (the chunks then split evenly: a second
    // round of blocks would double the kernel's time for a few waves)
    int dev = 0, ncu = 0, per_cu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &per_cu, amb ? (const void *)dust_kernel<true> : (const void *)dust_kernel<false>, DW, 0);
    // max_waves > 0: at most that many waves per SIMD (room for kernels on other streams)
    if (max_waves > 0) per_cu = std::min(per_cu, 4 * max_waves);
    const uint64_t resident = (uint64_t)std::max(ncu, 1) * (uint64_t)std::max(per_cu, 1);
    const uint64_t g = std::min<uint64_t>(std::min<uint64_t>((nchunk + DW - 1) / DW, scratch_blocks), resident);
    const uint64_t nwords = (total + 31) / 32 + 2;   // readable packed words (the arrays carry padding)
    if (amb)
        hipLaunchKernelGGL(dust_kernel<true>, dim3((unsigned)g), dim3(DW), 0, st, total, nwords, F, AF, txstart, level,
                           window, events, scratch, mask);
    else
        hipLaunchKernelGGL(dust_kernel<false>, dim3((unsigned)g), dim3(DW), 0, st, total, nwords, F, AF, txstart,
                           level, window, events, scratch, mask);
    if (linker > 1 && n_tx)
        hipLaunchKernelGGL(dust_linker_kernel, dim3((n_tx + 255) / 256 < 65536 ? (n_tx + 255) / 256 : 65536), dim3(256),
                           0, st, tx, n_tx, linker, mask);
}

uint32_t dust_scratch_words(uint32_t blocks) { return blocks * DW * DWIN_MAX; }
uint64_t dust_event_words(uint32_t blocks) { return (uint64_t)blocks * DW * DEVCAP * 3; }

}  // namespace rcg

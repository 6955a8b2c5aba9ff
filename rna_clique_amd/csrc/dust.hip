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
//  B. the events, owner lane by owner lane, each by the whole wave (one lane
//     per suffix, prefix sums and a max-scan over the lanes in DPP) against
//     the perfect intervals found so far (per start: the owner's slots, in
//     global scratch between rounds of B, in the lanes while they run).
//     Deferring this rare pass keeps the scan free of the long divergent
//     loop one lane in three wave steps would otherwise impose on the wave.
#include "device.h"

#include <algorithm>

namespace rcg {

constexpr int DW = 64;          // lanes per block (one wave)
#ifndef RC_DUST_CHUNK
#define RC_DUST_CHUNK 1024
#endif
constexpr int DCHUNK = RC_DUST_CHUNK;   // bases per lane (a multiple of 64)
static_assert(DCHUNK % 64 == 0 && DCHUNK + 64 < 4096, "an event's chunk offset has 12 bits");
constexpr int DWIN_MAX = 64;    // longest DUST window the kernel supports
constexpr int DEVCAP = 64;  // events a lane holds (phase B runs between scan blocks when one nears this)


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
#define RC_DUST_MINW 5   // waves per SIMD the registers must allow (r03: 22.7 ms at 5, 24.7 at 6, 25.5 at 7 on 1.6 Gbp random)
#endif

// wave-uniform 64-bit lane read
__device__ __forceinline__ uint64_t rl64(uint64_t v, int l)
{
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l) << 32) |
           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
}

// the number of triplets ending 0 .. a - 1 bases before j that equal the one
// ending a back, from the window's bit planes (bit e: the base e back)
__device__ __forceinline__ int dust_later(uint64_t Q0, uint64_t Q1, int a)
{
    const uint64_t t0 = Q0 >> a, t1 = Q1 >> a;
    const int bl = (int)((t0 & 1) | ((t1 & 1) << 1)), bm = (int)(((t0 >> 1) & 1) | (t1 & 2)),
              bf = (int)(((t0 >> 2) & 1) | ((t1 >> 1) & 2));
    const uint64_t eq = (base_eq(Q0, Q1, bf) >> 2) & (base_eq(Q0, Q1, bm) >> 1) & base_eq(Q0, Q1, bl);
    return a ? __builtin_popcountll(eq & bit_range(0, a - 1)) : 0;
}

// DPP scans over the wave (lane order): row_shr 1, 2, 4, 8 inside the rows of
// 16, then row_bcast 15 and 31 across them
__device__ __forceinline__ int dpp_add_scan(int v)
{
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);   // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);   // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);   // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);   // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);   // row_bcast:15
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);   // row_bcast:31
    return v;
}
// a ratio n / d packed as n | d << 16; RID = 0 / 1 (below every perfect one)
constexpr uint32_t RID = 1u << 16;
// a, unless b's ratio is larger (ties keep a)
__device__ __forceinline__ uint32_t rmax(uint32_t a, uint32_t b)
{
    return (b & 0xFFFFu) * (a >> 16) > (a & 0xFFFFu) * (b >> 16) ? b : a;
}
__device__ __forceinline__ uint32_t dpp_max_scan(uint32_t v)
{
    const int RI = (int)RID;
    v = rmax(v, (uint32_t)__builtin_amdgcn_update_dpp(RI, (int)v, 0x111, 0xF, 0xF, false));
    v = rmax(v, (uint32_t)__builtin_amdgcn_update_dpp(RI, (int)v, 0x112, 0xF, 0xF, false));
    v = rmax(v, (uint32_t)__builtin_amdgcn_update_dpp(RI, (int)v, 0x114, 0xF, 0xF, false));
    v = rmax(v, (uint32_t)__builtin_amdgcn_update_dpp(RI, (int)v, 0x118, 0xF, 0xF, false));
    v = rmax(v, (uint32_t)__builtin_amdgcn_update_dpp(RI, (int)v, 0x142, 0xA, 0xF, false));
    v = rmax(v, (uint32_t)__builtin_amdgcn_update_dpp(RI, (int)v, 0x143, 0xC, 0xF, false));
    return v;
}
// the value of the lane below (lane 0: RID): an inclusive scan made exclusive
__device__ __forceinline__ uint32_t dpp_shr1(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_update_dpp((int)RID, (int)v, 0x138, 0xF, 0xF, false);   // wave_shr:1
}

template <bool AMB>
__global__ __launch_bounds__(DW, RC_DUST_MINW) void dust_kernel(uint64_t begin, uint64_t total, uint64_t nwords,
                                                  const uint64_t *__restrict__ F,
                                                  const uint64_t *__restrict__ AF,
                                                  const uint64_t *__restrict__ txstart, int T, int W,
                                                  uint64_t *__restrict__ evs, uint32_t *__restrict__ scratch,
                                                  uint64_t *__restrict__ mask)
{
    const int lane = threadIdx.x;
    const int need = (2 * T) / 10;   // occurrences before a new one that break the L-suffix bound
    uint32_t *const slot0 = scratch + (size_t)blockIdx.x * DW * DWIN_MAX;   // [lane][run offset of a start & 63]
    uint32_t *const slot = slot0 + lane * DWIN_MAX;
    // the lane's triplet counts over the window (64 bytes, lane stride 68:
    // spread over the LDS banks): the window score moves by the counts of the
    // entering and the leaving triplet, so the bit-plane match of a triplet
    // is only needed where the L-suffix bound may move
    __shared__ uint32_t cnt_lds[DW * 17];
    uint8_t *const C = reinterpret_cast<uint8_t *>(cnt_lds + 17 * lane);
    uint64_t *ev = evs + (size_t)blockIdx.x * DEVCAP * 3 * DW + lane;         // [event][field][lane]
    const uint64_t nchunk = (total - begin + DCHUNK - 1) / DCHUNK;   // chunks of [begin, total)
    auto word = [&](uint64_t w) -> uint64_t { return w < nwords ? F[w] : 0ull; };
    auto aword = [&](uint64_t w) -> uint64_t { return AMB && w < nwords ? AF[w] : 0ull; };
    // wave-uniform chunk rounds (the whole wave meets in phase B); a lane past
    // the last chunk scans nothing
    for (uint64_t chb = (uint64_t)blockIdx.x * DW; chb < nchunk; chb += (uint64_t)gridDim.x * DW) {
        const uint64_t ch = chb + (uint64_t)lane;
        const bool have = ch < nchunk;
        const uint64_t c0 = have ? begin + ch * DCHUNK : total, c1 = have ? min(c0 + DCHUNK, total) : total;
        const uint64_t lim = have ? min(c1 + (uint64_t)W, total) : total;   // the scan's reach
        // ---------------- B: the events, in order per lane (state kept across runs of B) ----------------
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
        // Every lane's events, owner by owner (wave-uniform call): the whole
        // wave works on one event at a time, lane a on the suffix ending at j
        // that starts a triplets back (st = pt - a). Its score is a prefix
        // sum over the lanes of "the later copies of the triplet at st"; the
        // best ratio it is compared with -- the perfect intervals inside the
        // L-suffix, then every shorter suffix's slot and every shorter suffix
        // that passes the level (a passing one that does not beat the running
        // best leaves it unchanged) -- is an exclusive max-scan over the same
        // lanes: align_oracle.c dust_run's loop over the longer suffixes,
        // without its walk. The owner's slots sit in the lanes (lane k: slot
        // k) while its events run, one load and one store per owner.
        int nev = 0;
        const uint64_t *const evb = evs + (size_t)blockIdx.x * DEVCAP * 3 * DW;
        auto run_events = [&]() {
            for (uint64_t hm = __ballot(nev > 0); hm; hm &= hm - 1) {
                const int o = __builtin_ctzll(hm);
                const int n = __builtin_amdgcn_readlane(nev, o);
                uint64_t xv = 0, q0v = 0, q1v = 0;   // lane e: the owner's event e
                if (lane < n) {
                    xv = evb[(size_t)(3 * lane) * DW + o];
                    q0v = evb[(size_t)(3 * lane + 1) * DW + o];
                    q1v = evb[(size_t)(3 * lane + 2) * DW + o];
                }
                const uint64_t oc0 = rl64(c0, o), oc1 = rl64(c1, o);
                uint64_t oset = rl64(set, o), oprs = rl64(prs, o);
                int opw = __builtin_amdgcn_readlane(pw, o);
                uint32_t *const os = slot0 + o * DWIN_MAX;
                uint32_t sv = ((oset >> lane) & 1ull) ? os[lane] : 0u;
                for (int e = 0; e < n; e++) {
                    const uint64_t x = rl64(xv, e), Q0 = rl64(q0v, e), Q1 = rl64(q1v, e);
                    const int rel = (int)(x & 0xFFF), Lq = (int)((x >> 12) & 63), rwe = (int)((x >> 18) & 0x7FF);
                    const int32_t j = (int32_t)(x >> 29), pt = j - 2, wstart = max(j + 1 - W, 0);
                    const uint64_t r0 = oc0 + (uint64_t)rel - (uint64_t)j;   // the run's start
                    // finalize: the owner's intervals that start before the
                    // window (all of them on a new run)
                    bool mine = (oset >> lane) & 1ull;
                    if (mine) {
                        const uint64_t a = (uint64_t)opw + (uint64_t)((lane - opw) & 63);
                        if (r0 != oprs || a < (uint64_t)wstart) {
                            if (oprs + a < oc1) dust_mark(mask, oprs + a, oprs + a + ((sv >> 20) & 0x1FFu));
                            mine = false;
                        }
                    }
                    oset = __ballot(mine);
                    oprs = r0;
                    opw = wstart;
                    // lane a: the suffix starting at st = pt - a (l = a)
                    const int span = pt - wstart;   // the window's last lane
                    const bool valid = lane <= span;
                    const int r = dpp_add_scan(valid ? dust_later(Q0, Q1, lane) : 0);
                    const int ki = (pt - lane) & 63;
                    const uint32_t si = (uint32_t)__shfl((int)sv, ki);
                    const bool has = valid && ((oset >> ki) & 1ull);
                    const bool act = valid && lane >= Lq && T * lane < 10 * rwe;   // the loop's prefix (its break)
                    const bool pass = act && r * 10 > T * lane;
                    if (!__ballot(pass)) continue;   // no longer suffix reaches the level: nothing is perfect
                    uint32_t c = has ? (si & 0xFFFu) | (((si >> 12) & 0xFFu) << 16) : RID;
                    if (pass) c = rmax(c, (uint32_t)r | ((uint32_t)lane << 16));
                    if (lane >= Lq && !act) c = RID;
                    const uint32_t ex = rmax(dpp_shr1(dpp_max_scan(c)), has ? (si & 0xFFFu) | (((si >> 12) & 0xFFu) << 16) : RID);
                    const int en = (int)(ex & 0xFFFF), ed = (int)(ex >> 16);
                    const bool perfect = pass && r * ed >= en * lane;
                    uint32_t nv = 0;
                    if (perfect) {
                        const int sr = (int)(si & 0xFFF), sl = (int)((si >> 12) & 0xFF);
                        const int end = j + 1 - (pt - lane);
                        int nr = r, nl = lane;
                        if (has && !(r * sl > sr * lane)) { nr = sr; nl = sl; }
                        const int ne = has ? max(end, (int)((si >> 20) & 0x1FF)) : end;
                        nv = ((uint32_t)ne << 20) | ((uint32_t)nl << 12) | (uint32_t)nr;
                    }
                    // back to the slot lanes: slot k came from lane (pt - k) & 63
                    const uint64_t pb = __ballot(perfect);
                    if (pb) {
                        const int src = (pt - lane) & 63;
                        const uint32_t t = (uint32_t)__shfl((int)nv, src);
                        if ((pb >> src) & 1ull) sv = t;
                        const uint64_t rv = __builtin_bitreverse64(pb);
                        const int sh = (pt + 1) & 63;
                        oset |= sh ? (rv << sh) | (rv >> (64 - sh)) : rv;
                    }
                }
                if ((oset >> lane) & 1ull) os[lane] = sv;
                if (lane == o) {
                    set = oset;
                    prs = oprs;
                    pw = opw;
                }
            }
            nev = 0;
        };
        // ---------------- A: the window scan over [c0, lim) ----------------
        // The scan goes a packed word (32 bases) at a time: the words of the
        // next block are loaded at the top of a block and only rotated in at
        // its end, so their latency hides behind 32 steps (a load rotated per
        // step would make every step wait for it). Blocks are wave-uniform
        // rounds, so phase B can run between them when a lane's events near
        // the buffer's capacity.
        const uint64_t w0 = c0 >> 5;   // c0 is a multiple of 64
        const uint64_t t0i = c0 >> 6, tmax = (total >> 6) + 1;
        uint64_t wpp = 0, wp = 0, wc = have ? word(w0) : 0ull, ac = have ? aword(w0) : 0ull,
                 tc = have ? txstart[t0i] : 0ull;
        const int o = 66 - W;   // the trailing cursor's first base in the 96-base window (wpp, wp, wc)
        uint64_t P0 = 0, P1 = 0;   // bit planes of the last 64 bases, bit a = a bases back
        bool in_run = false, done = !have;
        int nb = 0, tri = 0, tri2 = 0, rw = 0, Lst = 0;
        // chunk-relative limits (32-bit: a chunk scan is < 2^12 bases)
        const uint32_t limr = (uint32_t)(lim - c0), c1r = (uint32_t)(c1 - c0);
        for (uint32_t k = 0;; k++) {
            if (!done && 32 * k >= limr) done = true;
            if (!__ballot(!done)) break;
            if (!done) {
                const uint64_t wn = word(w0 + k + 1), an = aword(w0 + k + 1);
                const uint64_t ti = t0i + ((k + 1) >> 1);
                const uint64_t tn = ti <= tmax ? txstart[ti] : 0ull;
                // the trailing bases of this block (32 k + i - W + 2) and its transcript-start bits
                const uint64_t tw = o < 32 ? (wpp >> (2 * o)) | (wp << (64 - 2 * o))
                                           : (o == 32 ? wp : (wp >> (2 * (o - 32))) | (wc << (64 - 2 * (o - 32))));
                const uint32_t txb = (uint32_t)(tc >> (32 * (k & 1)));
                const uint32_t nval = min(32u, limr - 32 * k);   // the block's bases before the scan's reach
                for (uint32_t i = 0; i < nval; i++) {
                    const uint32_t rel = 32 * k + i;
                    const bool amb = AMB && ((ac >> (2 * i)) & 3u);
                    const int b = (int)((wc >> (2 * i)) & 3u);
                    // the trailing cursor: the triplet that leaves the window
                    // starts at u - W (its first steps shift in bases from before
                    // the chunk; they are out of it before a triplet leaves)
                    tri2 = ((tri2 << 2) | (int)((tw >> (2 * i)) & 3u)) & 63;
                    if (AMB && amb) {
                        in_run = false;
                        if (rel >= c1r) {
                            done = true;
                            break;
                        }
                        continue;
                    }
                    if (!in_run || ((txb >> i) & 1u)) {   // a run starts: the chunk's first base or a transcript's
                        if (rel >= c1r) {   // runs starting past the chunk are the next lane's
                            done = true;
                            break;
                        }
                        in_run = true;
                        nb = rw = Lst = 0;
                        for (int q = 0; q < 16; q++) cnt_lds[17 * lane + q] = 0u;
                    }
                    nb++;
                    tri = ((tri << 2) | b) & 63;
                    P0 = (P0 << 1) | (uint64_t)(b & 1);
                    P1 = (P1 << 1) | (uint64_t)(b >> 1);
                    if (nb < 3) continue;
                    const int32_t j = nb - 1;        // run offset of u
                    const int32_t pt = j - 2;        // start of the new triplet
                    const int32_t wstart = max(j + 1 - W, 0);
                    // the leaving triplet (start j - W, once j >= W; before
                    // that a spare counter byte takes the update): its
                    // partners are its other copies
                    const bool leave = j >= W;
                    const int ls = leave ? tri2 : 64;
                    const int c2 = (int)C[ls] - 1;
                    C[ls] = (uint8_t)c2;
                    rw -= leave ? c2 : 0;
                    const int cw = (int)C[tri];   // the new triplet's copies in the window
                    C[tri] = (uint8_t)(cw + 1);
                    rw += cw;
                    Lst = max(Lst, wstart);
                    if (cw >= need) {   // the need-th previous occurrence (need-th lowest bit) is in the window
                        // the window without the new triplet: the triplets ending
                        // 1 .. W - 3 bases back that start in the run; bit e: the
                        // triplet ending e back is the new one
                        const uint64_t wm = bit_range(1, min(W - 3, j - 2));
                        uint64_t m = (base_eq(P0, P1, tri >> 4) >> 2) & (base_eq(P0, P1, (tri >> 2) & 3) >> 1) &
                                     base_eq(P0, P1, tri & 3) & wm;
                        for (int q = 1; q < need; q++) m &= m - 1;
                        const int p = need ? pt - (int)__builtin_ctzll(m) : pt;
                        if (p >= Lst) Lst = p + 1;
                    }
                    // (24-bit multiplies: full rate; rw < 2^11, L < 64)
                    if (__mul24(rw, 10) <= __mul24(pt - Lst + 1, T)) continue;
                    // rare: B tries the longer suffixes; event = j | rw | L | rel
                    ev[(size_t)(3 * nev) * DW] = ((uint64_t)j << 29) | ((uint64_t)rw << 18) | ((uint64_t)(pt - Lst + 1) << 12) | rel;
                    ev[(size_t)(3 * nev + 1) * DW] = P0;
                    ev[(size_t)(3 * nev + 2) * DW] = P1;
                    nev++;
                }
                if (nval < 32) done = true;   // the scan's reach
                wpp = wp;
                wp = wc;
                wc = wn;
                ac = an;
                if (k & 1) tc = tn;
            }
            // a block adds at most 32 events per lane
            if (__ballot(nev > DEVCAP - 32)) run_events();
        }
        run_events();
        finalize(~0ull);   // the last run's intervals (its end, or the scan's reach)
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

// the masks of the transcripts in [begin, total) (begin: a multiple of DCHUNK
// where a transcript starts; the packed arrays are read from position 0)
void launch_dust(bool amb, uint64_t begin, uint64_t total, const uint64_t *F, const uint64_t *AF, const uint64_t *txstart,
                 const TxInfo *tx, uint32_t n_tx, int level, int window, int linker, uint32_t *scratch,
                 uint64_t *events, uint32_t scratch_blocks, int max_waves, uint64_t *mask, hipStream_t st)
{
    if (total <= begin) return;
    const uint64_t nchunk = (total - begin + DCHUNK - 1) / DCHUNK;
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
        hipLaunchKernelGGL(dust_kernel<true>, dim3((unsigned)g), dim3(DW), 0, st, begin, total, nwords, F, AF, txstart, level,
                           window, events, scratch, mask);
    else
        hipLaunchKernelGGL(dust_kernel<false>, dim3((unsigned)g), dim3(DW), 0, st, begin, total, nwords, F, AF,
                           txstart, level, window, events, scratch, mask);
    if (linker > 1 && n_tx)
        hipLaunchKernelGGL(dust_linker_kernel, dim3((n_tx + 255) / 256 < 65536 ? (n_tx + 255) / 256 : 65536), dim3(256),
                           0, st, tx, n_tx, linker, mask);
}

uint32_t dust_scratch_words(uint32_t blocks) { return blocks * DW * DWIN_MAX; }
uint64_t dust_event_words(uint32_t blocks) { return (uint64_t)blocks * DW * DEVCAP * 3; }

}  // namespace rcg

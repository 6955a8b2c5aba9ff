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
// (CHUNK + W) / CHUNK of the sequential work, and every lane busy.
//
// Per lane state in LDS, laid out [entry][lane] (every lane its own bank):
// triplet window counts with each triplet's last start, and a ring of
// previous-occurrence links. The L-suffix of the published algorithm (no
// triplet more than 2 level / 10 times) then moves by following at most 4
// links instead of a walk, and its counts -- needed only on the rare steps
// where some suffix may pass the level -- are recounted there. Perfect
// intervals by start (mod 64) live in global scratch (rare; a 64-bit register
// mask says which slots hold one). Every lane of a wave is at the same chunk
// offset each step, so the register windows of packed bases reload in
// lockstep with the next word already in flight.
#include "device.h"

#include <algorithm>

namespace rcg {

constexpr int DW = 64;          // lanes per block (one wave)
constexpr int DCHUNK = 256;     // bases per lane
constexpr int DWIN_MAX = 64;    // longest DUST window the kernel supports

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

constexpr uint32_t DNONE = 511;   // "no earlier occurrence" in the occurrence links

template <bool AMB>
__global__ __launch_bounds__(DW) void dust_kernel(uint64_t total, uint64_t nwords, const uint64_t *__restrict__ F,
                                                  const uint64_t *__restrict__ AF,
                                                  const uint64_t *__restrict__ txstart, int T, int W,
                                                  uint32_t *__restrict__ scratch, uint64_t *__restrict__ mask)
{
    // every lane owns one column of each array (no barriers: one wave)
    //   cnt[t]:  window count (bits 0-6) | run offset of t's last start (7-15) |
    //            count of the rare suffix pass (16-22), valid when its tag (23-30)
    //            is the pass's
    //   prv[p & 63]: run offset of the previous start of the triplet starting at p
    //   qtr[p & 63]: the triplet starting at p (the window's, for the rare pass)
    __shared__ uint32_t cnt[64][DW];
    __shared__ uint16_t prv[64][DW];
    __shared__ uint8_t qtr[64][DW];
    const int lane = threadIdx.x;
    constexpr uint32_t CWM = 0x7Fu, SCM = 0x7FFFu << 16;
    uint32_t tag = 0;   // the rare pass's counts: tag, then count
    auto scount = [&](uint32_t ce) -> int { return (ce >> 23) == tag ? (int)((ce >> 16) & 0x7Fu) : 0; };
    auto sbump = [&](uint32_t ce) -> uint32_t {
        return (ce & ~SCM) | (tag << 23) | ((uint32_t)(scount(ce) + 1) << 16);
    };
    uint32_t *slot = scratch + ((size_t)blockIdx.x * DW + lane) * DWIN_MAX;   // [absolute start & 63]
    const uint64_t nchunk = (total + DCHUNK - 1) / DCHUNK;
    auto word = [&](uint64_t w) -> uint64_t { return w < nwords ? F[w] : 0ull; };
    auto aword = [&](uint64_t w) -> uint64_t { return AMB && w < nwords ? AF[w] : 0ull; };
    for (uint64_t ch = (uint64_t)blockIdx.x * DW + lane; ch < nchunk; ch += (uint64_t)gridDim.x * DW) {
        const uint64_t c0 = ch * DCHUNK, c1 = min(c0 + DCHUNK, total);
        const uint64_t lim = min(c1 + (uint64_t)W, total);   // the scan's reach
        // the window scan over [c0, lim): every lane of the wave at the same
        // chunk offset rel each step, so the 32-base register windows (lead
        // and the trailing cursor W - 2 behind) reload in lockstep, the next
        // word already in flight
        const uint64_t w0 = c0 >> 5;   // c0 is a multiple of 64
        uint64_t curw = word(w0), nxtw = word(w0 + 1), cura = aword(w0), nxta = aword(w0 + 1);
        uint64_t curt = txstart[c0 >> 6], nxtt = txstart[(c0 >> 6) + 1];
        uint64_t curw2 = curw, nxtw2 = nxtw;
        bool in_run = false;
        uint64_t rs = 0, set = 0;
        int nb = 0, tri = 0, tri2 = 0, rw = 0, Lst = 0;
        auto finalize = [&](uint64_t a, uint32_t s) {   // interval at absolute start a
            if (a < c1) dust_mark(mask, a, a + ((s >> 20) & 0x1FFu));
        };
        auto end_run = [&]() {   // every perfect interval left is final
            const uint64_t b0 = rs + (uint64_t)max(nb - W, 0);
            while (set) {
                const int k = __builtin_ctzll(set);
                set &= set - 1;
                finalize(b0 + (uint64_t)((k - (int)(b0 & 63)) & 63), slot[k]);
            }
            in_run = false;
        };
        for (uint64_t rel = 0; c0 + rel < lim; rel++) {
            const uint64_t u = c0 + rel;
            if (rel && (rel & 31) == 0) {
                curw = nxtw;
                nxtw = word(w0 + (rel >> 5) + 1);
                if (AMB) {
                    cura = nxta;
                    nxta = aword(w0 + (rel >> 5) + 1);
                }
            }
            if (rel && (rel & 63) == 0) {
                curt = nxtt;
                nxtt = (c0 >> 6) + (rel >> 6) + 1 <= (total >> 6) + 1 ? txstart[(c0 >> 6) + (rel >> 6) + 1] : 0ull;
            }
            const unsigned sh = 2u * (unsigned)(rel & 31);
            const bool amb = AMB && ((cura >> sh) & 3u);
            const int b = (int)((curw >> sh) & 3u);
            // the trailing cursor: the triplet that leaves the window starts at u - W
            const int64_t rel2 = (int64_t)rel - W + 2;
            if (rel2 >= 0) {
                if (rel2 && (rel2 & 31) == 0) {
                    curw2 = nxtw2;
                    nxtw2 = word(w0 + (uint64_t)(rel2 >> 5) + 1);
                }
                tri2 = ((tri2 << 2) | (int)((curw2 >> (2u * (unsigned)(rel2 & 31))) & 3u)) & 63;
            }
            if (in_run && (amb || ((curt >> (rel & 63)) & 1ull))) end_run();   // ambiguous base or next transcript
            if (amb) {
                if (u >= c1) break;
                continue;
            }
            if (!in_run) {
                if (u >= c1) break;   // runs starting past the chunk are the next lane's
                in_run = true;
                rs = u;
                nb = rw = Lst = 0;
                set = 0;
                for (int k = 0; k < 64; k++) cnt[k][lane] = DNONE << 7;
                tag = 0;
            }
            nb++;
            tri = ((tri << 2) | b) & 63;
            if (nb < 3) continue;
            const int32_t j = nb - 1;        // run offset of u
            const int32_t pt = j - 2;        // start of the new triplet
            const int32_t wstart = max(j + 1 - W, 0);
            if (wstart > 0) {   // the start wstart - 1 left the window: final
                const uint64_t a = rs + (uint64_t)(wstart - 1);
                const int k = (int)(a & 63);
                if ((set >> k) & 1ull) {
                    finalize(a, slot[k]);
                    set &= ~(1ull << k);
                }
            }
            if (j >= W) {   // the window was full: its oldest triplet (start j - W) leaves
                const uint32_t co = cnt[tri2][lane] - 1u;
                cnt[tri2][lane] = co;
                rw -= (int)(co & CWM);
            }
            const int t3 = tri;
            const uint32_t c = cnt[t3][lane];
            const int cw = (int)(c & CWM);
            rw += cw;
            prv[pt & 63][lane] = (uint16_t)((c >> 7) & 0x1FFu);
            qtr[pt & 63][lane] = (uint8_t)t3;
            cnt[t3][lane] = (c & SCM) | ((uint32_t)pt << 7) | (uint32_t)(cw + 1);
            // L-suffix: the longest suffix of the window in which no triplet
            // occurs more than 2 level / 10 times (4 at level 20)
            Lst = max(Lst, wstart);
            if ((cw + 1) * 10 > 2 * T) {
                int need = (2 * T) / 10, p = pt;   // occurrences before pt that would exceed the bound
                bool over = true;
                for (int k = 0; k < need; k++) {
                    p = (int)prv[p & 63][lane];
                    if (p == (int)DNONE || p < Lst) {
                        over = false;
                        break;
                    }
                }
                if (over) Lst = p + 1;
            }
            const int Lq = pt - Lst + 1;
            if (rw * 10 <= Lq * T) continue;
            // rare: the suffixes longer than Lq that could score above the
            // level (10 r > level (n - 1) and r <= rw), shortest first, against
            // the best ratio of the perfect intervals inside them
            auto tri_at = [&](int32_t st) -> int { return qtr[st & 63][lane]; };
            if (++tag == 256) {   // tags wrapped: clear every count of the pass
                for (int k = 0; k < 64; k++) cnt[k][lane] &= ~SCM;
                tag = 1;
            }
            int r = 0;
            for (int32_t st = Lst; st <= pt; st++) {   // the L-suffix's counts
                const int tt = tri_at(st);
                const uint32_t ce = cnt[tt][lane];
                r += scount(ce);
                cnt[tt][lane] = sbump(ce);
            }
            int mr = 0, ml = 0;
            for (int32_t st = Lst; st <= j; st++) {
                const int k = (int)((rs + (uint64_t)st) & 63);
                if (!((set >> k) & 1ull)) continue;
                const uint32_t s = slot[k];
                const int sr = (int)(s & 0xFFF), sl = (int)((s >> 12) & 0xFF);
                if (mr == 0 || sr * ml > mr * sl) { mr = sr; ml = sl; }
            }
            for (int32_t st = Lst - 1; st >= wstart; st--) {
                const int l = pt - st;
                if (T * l >= 10 * rw) break;   // no longer suffix can pass the level
                const int tt = tri_at(st);
                const uint32_t ce = cnt[tt][lane];
                r += scount(ce);
                cnt[tt][lane] = sbump(ce);
                const int k = (int)((rs + (uint64_t)st) & 63);
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
        }
        if (in_run) end_run();   // the run reaches lim
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
                 uint32_t scratch_blocks, uint64_t *mask, hipStream_t st)
{
    if (total == 0) return;
    const uint64_t nchunk = (total + DCHUNK - 1) / DCHUNK;
    const uint64_t g = std::min<uint64_t>((nchunk + DW - 1) / DW, scratch_blocks);
    const uint64_t nwords = (total + 31) / 32 + 2;   // readable packed words (the arrays carry padding)
    if (amb)
        hipLaunchKernelGGL(dust_kernel<true>, dim3((unsigned)g), dim3(DW), 0, st, total, nwords, F, AF, txstart, level,
                           window, scratch, mask);
    else
        hipLaunchKernelGGL(dust_kernel<false>, dim3((unsigned)g), dim3(DW), 0, st, total, nwords, F, AF, txstart,
                           level, window, scratch, mask);
    if (linker > 1 && n_tx)
        hipLaunchKernelGGL(dust_linker_kernel, dim3((n_tx + 255) / 256 < 65536 ? (n_tx + 255) / 256 : 65536), dim3(256),
                           0, st, tx, n_tx, linker, mask);
}

uint32_t dust_scratch_words(uint32_t blocks) { return blocks * DW * DWIN_MAX; }

}  // namespace rcg

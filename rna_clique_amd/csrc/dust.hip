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
// Per lane state: triplet counts in LDS laid out [triplet][lane] as dwords
// (every lane its own bank): window (bits 0-9), L-suffix (10-19), scratch
// (20-29). Perfect intervals by start (mod 64) in global scratch -- they are
// rare, and a 64-bit register mask says which slots hold one. A lane stages
// its chunk's packed bases and transcript-start bits in LDS first; the scan
// then advances every lane of the wave to the same chunk offset each step, so
// the register windows reload in lockstep (no divergent memory waits).
#include "device.h"

#include <algorithm>

namespace rcg {

#ifndef DUST_VARIANT
#define DUST_VARIANT 0   // microbenchmark knob (scripts/micro): 1 no find-perfect, 2 no counts, 3 staging only
#endif
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

constexpr int SBW = (DCHUNK + DWIN_MAX) / 32 + 2;   // packed words of a chunk's bases (+ tail)
constexpr int STW = (DCHUNK + DWIN_MAX) / 64 + 2;   // transcript-start words of a chunk

template <bool AMB>
__global__ __launch_bounds__(DW) void dust_kernel(uint64_t total, uint64_t nwords, const uint64_t *__restrict__ F,
                                                  const uint64_t *__restrict__ AF,
                                                  const uint64_t *__restrict__ txstart, int T, int W,
                                                  uint32_t *__restrict__ scratch, uint64_t *__restrict__ mask)
{
    // every lane owns one column of each array (no barriers: one wave)
    __shared__ uint32_t cnt[64][DW];
    __shared__ uint64_t sb[SBW][DW];
    __shared__ uint64_t sa[AMB ? SBW : 1][DW];
    __shared__ uint64_t stx[STW][DW];
    const int lane = threadIdx.x;
    const uint32_t CW = 0x3FFu, CV = 0x3FFu << 10, CS = 0x3FFu << 20;
    uint32_t *slot = scratch + ((size_t)blockIdx.x * DW + lane) * DWIN_MAX;   // [absolute start & 63]
    const uint64_t nchunk = (total + DCHUNK - 1) / DCHUNK;
    auto code_at = [&](uint64_t rel) -> int {   // base at chunk offset rel (inside a run: never ambiguous)
        return (int)((sb[rel >> 5][lane] >> (2u * (unsigned)(rel & 31))) & 3u);
    };
    for (uint64_t ch = (uint64_t)blockIdx.x * DW + lane; ch < nchunk; ch += (uint64_t)gridDim.x * DW) {
        const uint64_t c0 = ch * DCHUNK, c1 = min(c0 + DCHUNK, total);
        const uint64_t lim = min(c1 + (uint64_t)W, total);   // the scan's reach
        // stage the chunk: packed bases (c0 is a multiple of 64) and transcript-start bits
        for (int i = 0; i < SBW; i++) {
            const uint64_t w = (c0 >> 5) + (uint64_t)i;
            sb[i][lane] = w < nwords ? F[w] : 0ull;
            if (AMB) sa[i][lane] = w < nwords ? AF[w] : 0ull;
        }
        for (int i = 0; i < STW; i++) {
            const uint64_t w = (c0 >> 6) + (uint64_t)i;
            stx[i][lane] = w <= (total >> 6) + 1 ? txstart[w] : 0ull;
        }
        // the window scan over [c0, lim): positions advance in lockstep across
        // the wave (every lane at chunk offset rel), runs start and end per lane
        if (DUST_VARIANT == 3) continue;
        bool in_run = false;
        uint64_t rs = 0, set = 0, curw = 0, cura = 0, curt = 0, curw2 = 0;
        int nb = 0, tri = 0, tri2 = 0, qn = 0, rw = 0, rv = 0, Lq = 0;
        auto finalize = [&](uint64_t a, uint32_t s) {   // interval at absolute start a
            if (a < c1) dust_mark(mask, a, a + ((s >> 20) & 0x1FFu));
        };
        auto end_run = [&]() {   // every perfect interval left is final
            const uint64_t base = rs + (uint64_t)max(nb - W, 0);
            while (set) {
                const int k = __builtin_ctzll(set);
                set &= set - 1;
                finalize(base + (uint64_t)((k - (int)(base & 63)) & 63), slot[k]);
            }
            in_run = false;
        };
        for (uint64_t rel = 0; c0 + rel < lim; rel++) {
            const uint64_t u = c0 + rel;
            if ((rel & 31) == 0) {
                curw = sb[rel >> 5][lane];
                if (AMB) cura = sa[rel >> 5][lane];
            }
            if ((rel & 63) == 0) curt = stx[rel >> 6][lane];
            const unsigned sh = 2u * (unsigned)(rel & 31);
            const bool amb = AMB && ((cura >> sh) & 3u);
            const int b = (int)((curw >> sh) & 3u);
            // the trailing cursor (bases W - 2 behind) feeds the triplet that drops out
            const int64_t rel2 = (int64_t)rel - W + 2;
            if (rel2 >= 0) {
                if ((rel2 & 31) == 0) curw2 = sb[rel2 >> 5][lane];
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
                nb = qn = rw = rv = Lq = 0;
                set = 0;
                for (int k = 0; k < 64; k++) cnt[k][lane] = 0;
            }
            nb++;
            tri = ((tri << 2) | b) & 63;
            if (nb < 3) continue;
            const int32_t j = nb - 1;   // run offset of u
            const int32_t wstart = max(j + 1 - W, 0);
            if (wstart > 0) {   // the start wstart - 1 left the window: final
                const uint64_t a = rs + (uint64_t)(wstart - 1);
                const int k = (int)(a & 63);
                if ((set >> k) & 1ull) {
                    finalize(a, slot[k]);
                    set &= ~(1ull << k);
                }
            }
            const int t3 = tri;
            if (DUST_VARIANT == 2) {
                rw += t3 + tri2;
                continue;
            }
            if (qn == W - 2) {   // drop the oldest triplet (it starts at u - W)
                const int o = tri2;
                qn--;
                uint32_t co = cnt[o][lane] - 1u;
                rw -= (int)(co & CW);
                if (Lq > qn) {
                    Lq--;
                    co -= 1u << 10;
                    rv -= (int)((co & CV) >> 10);
                }
                cnt[o][lane] = co;
            }
            qn++;
            Lq++;
            uint32_t ct = cnt[t3][lane];
            rw += (int)(ct & CW);
            rv += (int)((ct & CV) >> 10);
            ct += 1u + (1u << 10);
            cnt[t3][lane] = ct;
            // window triplet q (0 = oldest) starts at run offset wstart + q
            auto tri_at = [&](int32_t st) {
                const uint64_t r0 = rs + (uint64_t)st - c0;
                return code_at(r0) * 16 + code_at(r0 + 1) * 4 + code_at(r0 + 2);
            };
            if ((int)((ct & CV) >> 10) * 10 > 2 * T) {   // shrink the suffix past the previous copy
                int o;
                do {
                    o = tri_at(wstart + qn - Lq);
                    uint32_t co = cnt[o][lane] - (1u << 10);
                    rv -= (int)((co & CV) >> 10);
                    cnt[o][lane] = co;
                    Lq--;
                } while (o != t3);
            }
            if (rw * 10 <= Lq * T || DUST_VARIANT == 1) continue;
            // suffixes longer than Lq, shortest first, against the best ratio of
            // the perfect intervals inside them
            int r = rv, mr = 0, ml = 0;
            for (int32_t st = wstart + qn - Lq; st <= j; st++) {
                const int k = (int)((rs + (uint64_t)st) & 63);
                if (!((set >> k) & 1ull)) continue;
                const uint32_t s = slot[k];
                const int sr = (int)(s & 0xFFF), sl = (int)((s >> 12) & 0xFF);
                if (mr == 0 || sr * ml > mr * sl) { mr = sr; ml = sl; }
            }
            for (int q = qn - Lq - 1; q >= 0; q--) {
                const int tt = tri_at(wstart + q);
                const uint32_t ce = cnt[tt][lane];
                r += (int)((ce & CV) >> 10) + (int)((ce & CS) >> 20);
                cnt[tt][lane] = ce + (1u << 20);
                const int l = qn - q - 1;
                const int32_t st = wstart + q;
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
            for (int q = qn - Lq - 1; q >= 0; q--) cnt[tri_at(wstart + q)][lane] &= ~CS;   // scratch counts to 0
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

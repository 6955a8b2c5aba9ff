// Microbenchmark of the DUST kernel on random packed sequence (build with
// -DDUST_VARIANT=... to time variants). Not part of the product.
#include "../../rna_clique_amd/csrc/device.h"
#include <cstdio>
#include <cstdlib>
#include <vector>
namespace rcg {
void launch_dust(bool, uint64_t, uint64_t, const uint64_t *, const uint64_t *, const uint64_t *, const TxInfo *, uint32_t, int,
                 int, int, uint32_t *, uint64_t *, uint32_t, int, uint64_t *, hipStream_t);
uint32_t dust_scratch_words(uint32_t);
uint64_t dust_event_words(uint32_t);
}
using namespace rcg;
int main(int argc, char **argv)
{
    const uint64_t total = argc > 1 ? strtoull(argv[1], 0, 10) : 1600000000ull;
    const uint64_t nw = (total + 31) / 32 + 4;
    std::vector<uint64_t> h(nw);
    uint64_t x = 88172645463325252ull;
    for (auto &v : h) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; v = x; }
    std::vector<uint64_t> tb((total >> 6) + 4, 0);
    for (uint64_t p = 0; p < total; p += 1000) { const uint64_t q = p + 64; tb[q >> 6] |= 1ull << (q & 63); }
    // argv[3]: fraction of the 1000-base transcripts ending in a 30-base poly-A tail (as C3v)
    const double pa = argc > 3 ? atof(argv[3]) : 0.0;
    uint64_t y = 12345;
    for (uint64_t p = 64; p + 1000 <= total; p += 1000) {
        y ^= y << 13; y ^= y >> 7; y ^= y << 17;
        if ((double)(y % 1000000) / 1e6 >= pa) continue;
        for (uint64_t u = p + 1000 - 30; u < p + 1000; u++) h[u >> 5] &= ~(3ull << (2 * (u & 31)));
    }
    uint64_t *F, *TB, *M, *E; uint32_t *S;
    hipMalloc(&F, nw * 8); hipMalloc(&TB, tb.size() * 8); hipMalloc(&M, tb.size() * 8);
    const uint32_t blocks = argc > 2 ? (uint32_t)atoi(argv[2]) : 256 * 10;
    hipMalloc(&S, (size_t)dust_scratch_words(blocks) * 4);
    hipMalloc(&E, (size_t)dust_event_words(blocks) * 8);
    hipMemcpy(F, h.data(), nw * 8, hipMemcpyHostToDevice);
    hipMemcpy(TB, tb.data(), tb.size() * 8, hipMemcpyHostToDevice);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    for (int it = 0; it < 3; it++) {
        hipMemset(M, 0, tb.size() * 8);
        hipEventRecord(a, 0);
        launch_dust(false, 0, total, F, nullptr, TB + 1, nullptr, 0, 20, 64, 1, S, E, blocks, 0, M + 1, 0);
        hipEventRecord(b, 0);
        hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        printf("dust %.3f ms (%s)\n", ms, hipGetErrorString(hipGetLastError()));
    }
    std::vector<uint64_t> m(tb.size());
    hipMemcpy(m.data(), M, m.size() * 8, hipMemcpyDeviceToHost);
    uint64_t c = 0; for (auto v : m) c += __builtin_popcountll(v);
    printf("masked %llu of %llu\n", (unsigned long long)c, (unsigned long long)total);
    return 0;
}

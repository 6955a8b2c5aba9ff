// Check + time the hand-written onesweep (rna_clique_amd/csrc/sort.hip)
// against rocPRIM's radix_sort_keys on the index's key shapes. Not part of
// the product. Cases: C3-size conserved k-mers (bits 32..63), a skewed set
// (a third of the keys share one k-mer, as poly-A windows do), small and
// ragged sizes, and the near-mask index's full 64-bit sort.
// Usage: onesweep_micro [n]   (default 1.6e9)
#include <cstdio>
#include "../../rna_clique_amd/csrc/sort.hip"

#include <rocprim/device/device_radix_sort.hpp>

using namespace rcg;

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                             \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
            exit(1);                                                                      \
        }                                                                                 \
    } while (0)

__global__ void gen(uint64_t *ent, uint64_t n, int kind)
{
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t x = (i % (n / 32 + 1)) * 0x9E3779B97F4A7C15ull;
        x ^= x >> 29;
        uint32_t key = (uint32_t)(x * 0xBF58476D1CE4E5B9ull >> 32);
        if (kind == 1 && (i % 3) == 0) key = 0;
        uint64_t lo = (uint32_t)i;
        if (kind == 2) lo = (uint32_t)(x >> 7);   // full 64-bit keys with repeats
        ent[i] = ((uint64_t)key << 32) | lo;
    }
}

__global__ void cmp(const uint64_t *a, const uint64_t *b, uint64_t n, unsigned long long *bad)
{
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        if (a[i] != b[i]) atomicAdd(bad, 1ull);
}

__global__ void copyk(const uint64_t *__restrict__ a, uint64_t *__restrict__ b, uint64_t n)
{
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        b[i] = a[i];
}

int main(int argc, char **argv)
{
    const uint64_t N = argc > 1 ? strtoull(argv[1], 0, 10) : 1600000000ull;
    hipStream_t st;
    CK(hipStreamCreate(&st));
    uint64_t *src, *a, *b, *ref;
    CK(hipMalloc(&src, N * 8));
    CK(hipMalloc(&a, N * 8));
    CK(hipMalloc(&b, N * 8));
    CK(hipMalloc(&ref, N * 8));
    uint32_t *scratch;
    CK(hipMalloc(&scratch, os_scratch_words(N) * 4));
    uint64_t *status;
    CK(hipMalloc(&status, os_status_words(N) * 8));
    CK(hipMemset(status, 0, os_status_words(N) * 8));
    unsigned long long *bad;
    CK(hipMalloc(&bad, 8));
    void *tmp = nullptr;
    size_t tb = 0;
    for (unsigned bbq : {0u, 32u}) {
        size_t q = 0;
        CK(rocprim::radix_sort_keys(nullptr, q, src, ref, (size_t)N, bbq, 64u, st));
        tb = std::max(tb, q);
    }
    CK(hipMalloc(&tmp, tb + 1));
    uint32_t epoch = 0;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    struct Case { uint64_t n; int kind, bb; };
    std::vector<Case> cases = {{N, 0, 32}, {N, 1, 32}, {1, 0, 32}, {1000, 0, 32}, {8191, 0, 32}, {8193, 0, 32},
                               {(1u << 20) + 3, 1, 32}, {N / 80, 2, 0}, {12345, 2, 0}};
    int fails = 0;
    if (getenv("OS_COPY")) {
        hipLaunchKernelGGL(copyk, dim3(256 * 16), dim3(256), 0, st, src, a, N);
        float ms;
        CK(hipEventRecord(e0, st));
        hipLaunchKernelGGL(copyk, dim3(256 * 16), dim3(256), 0, st, src, a, N);
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("copy of %llu keys: %.3f ms = %.0f GB/s (read + write)\n", (unsigned long long)N, ms, 16.0 * N / ms / 1e6);
    }
    if (getenv("OS_ONLY_BIG")) cases.resize(2);
    for (const Case &c : cases) {
        hipLaunchKernelGGL(gen, dim3(8192), dim3(256), 0, st, src, c.n, c.kind);
        // the reference sorts all 64 bits below 2^20 keys (its merge sort is
        // not stable on a partial bit range; positions are unique there)
        const unsigned rbb = c.n <= (1u << 20) ? 0u : (unsigned)c.bb;
        size_t t = 0;
        CK(rocprim::radix_sort_keys(nullptr, t, src, ref, (size_t)c.n, rbb, 64u, st));
        const size_t tc = t;
        CK(rocprim::radix_sort_keys(tmp, t, src, ref, (size_t)c.n, rbb, 64u, st));
        float best = 1e30f, best_r = 1e30f;
        bool in_alt = false;
        for (int rep = 0; rep < 3; rep++) {
            CK(hipMemcpyAsync(a, src, c.n * 8, hipMemcpyDeviceToDevice, st));
            CK(hipGetLastError());
            CK(hipEventRecord(e0, st));
            in_alt = os_sort_keys(a, b, c.n, c.bb, scratch, status, epoch, st, nullptr, false, nullptr, nullptr, nullptr, 0, nullptr);
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = std::min(best, ms);
            CK(hipEventRecord(e0, st));
            t = tc;
            CK(rocprim::radix_sort_keys(tmp, t, src, ref, (size_t)c.n, rbb, 64u, st));
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&ms, e0, e1));
            best_r = std::min(best_r, ms);
        }
        CK(hipMemsetAsync(bad, 0, 8, st));
        hipLaunchKernelGGL(cmp, dim3(8192), dim3(256), 0, st, in_alt ? b : a, ref, c.n, bad);
        unsigned long long nb = 0;
        CK(hipMemcpy(&nb, bad, 8, hipMemcpyDeviceToHost));
#ifdef OS_STATS
        {
            unsigned long long hs[4] = {0, 0, 0, 0}, z[4] = {0, 0, 0, 0};
            CK(hipMemcpyFromSymbol(hs, HIP_SYMBOL(os_stats), sizeof hs));
            CK(hipMemcpyToSymbol(HIP_SYMBOL(os_stats), z, sizeof z));
            printf("  stats: tiles %llu  look-back loads per digit-tile %.2f  not-ready polls %.2f\n", hs[2],
                   hs[0] / (256.0 * hs[2] + 1e-9), hs[1] / (256.0 * hs[2] + 1e-9));
        }
#endif
        printf("n=%llu kind=%d bb=%d  onesweep %.3f ms  rocprim %.3f ms  mismatches %llu\n", (unsigned long long)c.n,
               c.kind, c.bb, best, best_r, nb);
        fails += nb != 0;
    }
    CK(hipGetLastError());
    printf(fails ? "FAIL\n" : "OK\n");
    return fails ? 1 : 0;
}

// Microbenchmark of the seed-index sort variants at C3 size (1.6 G entries).
// Not part of the product. (a) today's: u64 (k-mer << 32 | position) keys,
// bits 32..63, rocPRIM default onesweep (8-bit digits); (b) u32 k-mer keys +
// u32 position values (SoA), default config; (c) the same pairs with 11-bit
// onesweep digits (3 passes). Prints ms per sort and checks (b), (c) against (a).
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

__global__ void gen(uint64_t *ent, uint32_t *k, uint32_t *v, uint64_t n)
{
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        // k-mers shared by 32 "samples" (as orthologs share them), positions ascending
        uint64_t x = (i % (n / 32)) * 0x9E3779B97F4A7C15ull;
        x ^= x >> 29;
        const uint32_t key = (uint32_t)(x * 0xBF58476D1CE4E5B9ull >> 32);
        ent[i] = ((uint64_t)key << 32) | (uint32_t)i;
        k[i] = key;
        v[i] = (uint32_t)i;
    }
}

__global__ void check(const uint64_t *ent, const uint32_t *k, const uint32_t *v, uint64_t n, unsigned long long *bad)
{
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        if (ent[i] != (((uint64_t)k[i] << 32) | v[i])) atomicAdd(bad, 1ull);
}

template <class F>
static float timed(F f, hipStream_t st)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    f();   // warm-up (allocations are outside)
    CK(hipEventRecord(a, st));
    f();
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms;
}

int main(int argc, char **argv)
{
    const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 1600000000ull;
    hipStream_t st;
    CK(hipStreamCreate(&st));
    uint64_t *e0, *e1;
    uint32_t *k0, *k1, *v0, *v1;
    CK(hipMalloc(&e0, n * 8));
    CK(hipMalloc(&e1, n * 8));
    CK(hipMalloc(&k0, n * 4));
    CK(hipMalloc(&k1, n * 4));
    CK(hipMalloc(&v0, n * 4));
    CK(hipMalloc(&v1, n * 4));
    hipLaunchKernelGGL(gen, dim3(8192), dim3(256), 0, st, e0, k0, v0, n);
    void *tmp = nullptr;
    size_t tb = 0, t1 = 0, t2 = 0;
    CK(rocprim::radix_sort_keys(nullptr, tb, e0, e1, (size_t)n, 32u, 64u, st));
    CK(rocprim::radix_sort_pairs(nullptr, t1, k0, k1, v0, v1, (size_t)n, 0u, 32u, st));
    using C11 = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                           rocprim::radix_sort_onesweep_config<rocprim::kernel_config<256, 12>,
                                                                               rocprim::kernel_config<256, 12>, 11,
                                                                               rocprim::block_radix_rank_algorithm::match>>;
    CK(rocprim::radix_sort_pairs<C11>(nullptr, t2, k0, k1, v0, v1, (size_t)n, 0u, 32u, st));
    const size_t tt = std::max(tb, std::max(t1, t2));
    CK(hipMalloc(&tmp, tt));
    const float ma = timed([&] { CK(rocprim::radix_sort_keys(tmp, tb, e0, e1, (size_t)n, 32u, 64u, st)); }, st);
    const float mb = timed([&] { CK(rocprim::radix_sort_pairs(tmp, t1, k0, k1, v0, v1, (size_t)n, 0u, 32u, st)); }, st);
    unsigned long long *bad;
    CK(hipMalloc(&bad, 8));
    CK(hipMemsetAsync(bad, 0, 8, st));
    hipLaunchKernelGGL(check, dim3(8192), dim3(256), 0, st, e1, k1, v1, n, bad);
    unsigned long long hb = 0;
    CK(hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost));
    const float mc = timed([&] { CK(rocprim::radix_sort_pairs<C11>(tmp, t2, k0, k1, v0, v1, (size_t)n, 0u, 32u, st)); }, st);
    CK(hipMemsetAsync(bad, 0, 8, st));
    hipLaunchKernelGGL(check, dim3(8192), dim3(256), 0, st, e1, k1, v1, n, bad);
    unsigned long long hc = 0;
    CK(hipMemcpy(&hc, bad, 8, hipMemcpyDeviceToHost));
    printf("n %llu: u64 keys (8-bit) %.2f ms | u32 pairs default %.2f ms (mismatch %llu) | u32 pairs 11-bit %.2f ms "
           "(mismatch %llu)\n",
           (unsigned long long)n, ma, mb, hb, mc, hc);
    return 0;
}

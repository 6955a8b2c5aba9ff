// Random-line read rate of the chip (the seed kernel's access shape: every
// lane its own random 8-B word, most lines missing L2). Not part of the product.
//
//   rand_micro [GB] [iters]
// For each (blocks per CU, loads in flight per lane, dependent chain yes/no)
// prints the rate in G lines/s. Independent: each lane issues K loads of a
// hashed address, sums them, repeats. Chained: the next address depends on
// the value loaded (pointer chase), K chains per lane.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

__device__ __forceinline__ uint64_t mix(uint64_t x)
{
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

template <int K, bool CHAIN>
__global__ __launch_bounds__(256) void rand_kernel(const uint64_t *__restrict__ buf, uint64_t nw, int iters,
                                                   uint64_t *out)
{
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t st[K];
#pragma unroll
    for (int k = 0; k < K; k++) st[k] = mix(t * K + k + 1);
    uint64_t acc = 0;
    for (int i = 0; i < iters; i++) {
        uint64_t v[K];
#pragma unroll
        for (int k = 0; k < K; k++) v[k] = buf[st[k] % nw];
#pragma unroll
        for (int k = 0; k < K; k++) {
            acc += v[k];
            st[k] = CHAIN ? mix(v[k] ^ st[k]) : mix(st[k] + 0x9e3779b97f4a7c15ull);
        }
    }
    if (acc == 0x12345) out[0] = acc;
}

template <int K, bool CHAIN>
static void run(const uint64_t *buf, uint64_t nw, int bpc, int iters, uint64_t *out, int cus)
{
    const int blocks = bpc * cus;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    rand_kernel<K, CHAIN><<<blocks, 256>>>(buf, nw, 2, out);
    hipEventRecord(a, 0);
    rand_kernel<K, CHAIN><<<blocks, 256>>>(buf, nw, iters, out);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double lines = (double)blocks * 256 * K * iters;
    printf("blocks/CU %2d  K %d  %-5s  %8.3f ms  %6.2f G lines/s  (%.0f ns per load round)\n", bpc, K,
           CHAIN ? "chain" : "indep", ms, lines / ms / 1e6, ms * 1e6 / iters);
}

int main(int argc, char **argv)
{
    const double gb = argc > 1 ? atof(argv[1]) : 16.0;
    const int iters = argc > 2 ? atoi(argv[2]) : 64;
    const uint64_t nw = (uint64_t)(gb * 1e9 / 8);
    uint64_t *buf, *out;
    if (hipMalloc(&buf, nw * 8) != hipSuccess) return 1;
    hipMalloc(&out, 8);
    hipMemset(buf, 0x5a, nw * 8);
    int cus = 256;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    printf("buffer %.1f GB, %d CUs\n", gb, cus);
    for (int bpc : {1, 2, 4, 8}) {
        run<1, false>(buf, nw, bpc, iters, out, cus);
        run<4, false>(buf, nw, bpc, iters, out, cus);
        run<1, true>(buf, nw, bpc, iters, out, cus);
        run<4, true>(buf, nw, bpc, iters, out, cus);
    }
    printf("%s\n", hipGetErrorString(hipGetLastError()));
    return 0;
}

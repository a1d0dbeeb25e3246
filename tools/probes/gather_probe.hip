// tools/probes/gather_probe.hip -- random-gather ceiling of the block sort's
// key loads (dev probe): every workgroup gathers from the table of "its" XCD
// (workgroup i runs on XCD i mod 8 under round-robin dealing), 16-B (or 8-B)
// loads at uniformly random 16-B-aligned offsets of a T-byte table, K loads in
// flight per thread (independent), grid = CUs x W workgroups of 256 threads.
// Prints G loads/s per configuration.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { if ((x) != hipSuccess) { fprintf(stderr, "%s failed\n", #x); exit(1); } } while (0)

template <int K, int W16>
__global__ void __launch_bounds__(256) k_gather(const uint4* __restrict__ tab, uint32_t words_per_tab, uint32_t iters,
                                                 uint32_t* __restrict__ out)
{
    const uint32_t x = blockIdx.x & 7u;
    const uint4* t = tab + (uint64_t)x * words_per_tab;
    uint32_t s = blockIdx.x * 2654435761u + threadIdx.x * 40503u + 12345u;
    uint32_t acc = 0;
    for (uint32_t it = 0; it < iters; ++it) {
        uint32_t idx[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            s ^= s << 13; s ^= s >> 17; s ^= s << 5;
            idx[k] = s % words_per_tab;
        }
        if constexpr (W16) {
            uint4 v[K];
#pragma unroll
            for (int k = 0; k < K; ++k) v[k] = t[idx[k]];
#pragma unroll
            for (int k = 0; k < K; ++k) acc += v[k].x ^ v[k].w;
        } else {
            uint2 v[K];
            const uint2* t2 = reinterpret_cast<const uint2*>(t);
#pragma unroll
            for (int k = 0; k < K; ++k) v[k] = t2[2 * idx[k]];
#pragma unroll
            for (int k = 0; k < K; ++k) acc += v[k].x ^ v[k].y;
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <int K, int W16>
void run(const uint4* tab, uint32_t tab_bytes, int wpc, int ncu, uint32_t* out)
{
    const uint32_t words = tab_bytes / 16;
    const uint32_t iters = 256;
    const dim3 g(ncu * wpc);
    hipLaunchKernelGGL((k_gather<K, W16>), g, dim3(256), 0, 0, tab, words, 16, out);
    CK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a, 0));
    hipLaunchKernelGGL((k_gather<K, W16>), g, dim3(256), 0, 0, tab, words, iters, out);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    const double loads = (double)g.x * 256 * iters * K;
    printf("table %7u KB  %2d-B loads  K=%d  WG/CU=%d : %7.1f G loads/s  (%.3f ms)\n", tab_bytes >> 10, W16 ? 16 : 8, K,
           wpc, loads / (ms * 1e-3) / 1e9, ms);
}

int main()
{
    int ncu = 256;
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    ncu = p.multiProcessorCount;
    uint4* tab;
    const size_t maxb = 8ull * (64u << 20);
    CK(hipMalloc(&tab, maxb));
    CK(hipMemset(tab, 1, maxb));
    uint32_t* out;
    CK(hipMalloc(&out, 64));
    for (uint32_t tb : {450u << 10, 2u << 20, 16u << 20}) {
        run<4, 1>(tab, tb, 4, ncu, out);
        run<8, 1>(tab, tb, 4, ncu, out);
        run<8, 1>(tab, tb, 8, ncu, out);
        run<16, 1>(tab, tb, 4, ncu, out);
        run<8, 0>(tab, tb, 4, ncu, out);
    }
    return 0;
}

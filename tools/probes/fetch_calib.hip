// tools/probes/fetch_calib.hip -- calibration of rocprofv3's FETCH_SIZE /
// WRITE_SIZE for the block sort's access widths (dev tool, not product).
//
// MI355X_MICROARCH.md calibrates FETCH_SIZE only for 16-B/lane streaming
// reads (it reports half their bytes) and WRITE_SIZE only for 16-B/lane
// streaming stores.  The block sort mostly does 8- and 16-B random gathers
// and 4-B scattered stores.  Each kernel here touches a KNOWN set of 128-B
// lines exactly once, in a 4 GiB buffer (far past the 256 MiB Infinity
// Cache), so the counter per access can be read against it:
//   stream16   16 B/lane coalesced read of 1 GiB          (guide: FETCH = bytes / 2)
//   gather8    one 8-B read per lane, each in its own line (offset 0)
//   gather16   one 16-B read per lane, each in its own line
//   gpair8     lanes 2i, 2i+1 read offsets 0 and 64 of one line: if the L2
//              fetches whole 128-B lines the second half hits
//   scatter4   one 4-B store per lane, each in its own line
//   scatter16  one 16-B store per lane, each in its own line
//   stream4w   4 B/lane coalesced stores (whole lines written)
// Line of access i: (i * 2654435761) mod 2^25 -- a bijection on 32 Mi lines.
//   hipcc --offload-arch=gfx950 -O3 -o fetch_calib fetch_calib.hip
//   rocprofv3 --kernel-trace --pmc FETCH_SIZE -- ./fetch_calib   (then WRITE_SIZE)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr uint64_t kLines = 1ull << 25;          // 32 Mi lines x 128 B = 4 GiB
constexpr uint32_t kN = 8u << 20;                 // 8 Mi accesses per gather/scatter kernel

__device__ __forceinline__ uint64_t line_of(uint64_t i) { return (i * 2654435761ull) & (kLines - 1); }

__global__ void stream16(const uint4* __restrict__ p, uint64_t n16, uint32_t* __restrict__ sink)
{
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += gridDim.x * 256ull) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void gather8(const uint8_t* __restrict__ b, uint32_t* __restrict__ sink)
{
    const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
    if (i >= kN) return;
    const uint64_t v = *reinterpret_cast<const uint64_t*>(b + line_of(i) * 128);
    if (v == 0x1234567812345678ull) sink[0] = 1;
}

__global__ void gather16(const uint8_t* __restrict__ b, uint32_t* __restrict__ sink)
{
    const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
    if (i >= kN) return;
    const uint4 v = *reinterpret_cast<const uint4*>(b + line_of(i) * 128);
    if ((v.x ^ v.y ^ v.z ^ v.w) == 0x12345678u) sink[0] = 1;
}

__global__ void gpair8(const uint8_t* __restrict__ b, uint32_t* __restrict__ sink)
{
    const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
    if (i >= kN) return;
    const uint64_t v = *reinterpret_cast<const uint64_t*>(b + line_of(i >> 1) * 128 + (i & 1) * 64);
    if (v == 0x1234567812345678ull) sink[0] = 1;
}

__global__ void scatter4(uint8_t* __restrict__ b)
{
    const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
    if (i >= kN) return;
    *reinterpret_cast<uint32_t*>(b + line_of(i) * 128) = (uint32_t)i;
}

__global__ void scatter16(uint8_t* __restrict__ b)
{
    const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
    if (i >= kN) return;
    *reinterpret_cast<uint4*>(b + line_of(i) * 128) = make_uint4((uint32_t)i, 1, 2, 3);
}

__global__ void stream4w(uint32_t* __restrict__ p, uint64_t n4)
{
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n4; i += gridDim.x * 256ull) p[i] = (uint32_t)i;
}

int main()
{
    uint8_t* big = nullptr;
    uint8_t* other = nullptr;
    uint32_t* sink = nullptr;
    const uint64_t bytes = kLines * 128;
    CK(hipMalloc(&big, bytes));
    CK(hipMalloc(&other, 1ull << 30));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(big, 1, bytes));
    CK(hipMemset(other, 2, 1ull << 30));
    const dim3 g(kN / 256);
    // flush the Infinity Cache between kernels: a 1 GiB streamed write
    auto flush = [&]() { hipLaunchKernelGGL(stream4w, dim3(4096), dim3(256), 0, 0, (uint32_t*)other, (1ull << 30) / 4); };
    for (int rep = 0; rep < 2; ++rep) {
        flush();
        hipLaunchKernelGGL(stream16, dim3(8192), dim3(256), 0, 0, (const uint4*)big, (1ull << 30) / 16, sink);
        flush();
        hipLaunchKernelGGL(gather8, g, dim3(256), 0, 0, big, sink);
        flush();
        hipLaunchKernelGGL(gather16, g, dim3(256), 0, 0, big, sink);
        flush();
        hipLaunchKernelGGL(gpair8, g, dim3(256), 0, 0, big, sink);
        flush();
        hipLaunchKernelGGL(scatter4, g, dim3(256), 0, 0, big);
        flush();
        hipLaunchKernelGGL(scatter16, g, dim3(256), 0, 0, big);
    }
    CK(hipDeviceSynchronize());
    printf("accesses per gather/scatter kernel: %u; stream16 bytes %llu; stream4w bytes %llu\n", kN,
           (unsigned long long)(1ull << 30), (unsigned long long)(1ull << 30));
    CK(hipFree(big));
    CK(hipFree(other));
    CK(hipFree(sink));
    return 0;
}

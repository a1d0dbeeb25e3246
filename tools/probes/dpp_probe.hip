// Probe: DPP row_shr / row_bcast wave scans on gfx950 against a plain
// reference (dev tool; prints "dpp ok" or the first mismatch).
//   hipcc -O3 --offload-arch=gfx950 tools/probes/dpp_probe.hip -o starch_amd/_build/dpp_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__device__ __forceinline__ uint32_t dpp_scan_add(uint32_t v)
{
    v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, true);   // row_shr:1
    v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, true);   // row_shr:2
    v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, true);   // row_shr:4
    v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, true);   // row_shr:8
    v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return v;
}

__device__ __forceinline__ uint32_t dpp_scan_max(uint32_t v)
{
    uint32_t t;
    t = __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, true); v = t > v ? t : v;
    t = __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, true); v = t > v ? t : v;
    t = __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, true); v = t > v ? t : v;
    t = __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, true); v = t > v ? t : v;
    t = __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false); v = t > v ? t : v;
    t = __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false); v = t > v ? t : v;
    return v;
}

__global__ void k(uint32_t* o, const uint32_t* in)
{
    const uint32_t x = in[threadIdx.x];
    o[threadIdx.x] = dpp_scan_add(x);
    o[64 + threadIdx.x] = dpp_scan_max(x);
    o[128 + threadIdx.x] = __builtin_amdgcn_readlane(dpp_scan_add(x), 63);
}

int main()
{
    uint32_t h[64], r[192];
    uint32_t* d_in;
    uint32_t* d_o;
    (void)hipMalloc(&d_in, sizeof(h));
    (void)hipMalloc(&d_o, sizeof(r));
    for (int t = 0; t < 50; ++t) {
        for (int i = 0; i < 64; ++i) h[i] = (uint32_t)((i * 2654435761u + t * 97u) >> (t % 20));
        (void)hipMemcpy(d_in, h, sizeof(h), hipMemcpyHostToDevice);
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d_o, d_in);
        (void)hipMemcpy(r, d_o, sizeof(r), hipMemcpyDeviceToHost);
        uint32_t s = 0, m = 0;
        for (int i = 0; i < 64; ++i) {
            s += h[i];
            m = h[i] > m ? h[i] : m;
            if (r[i] != s || r[64 + i] != m) {
                printf("mismatch t=%d lane %d: add %u/%u max %u/%u\n", t, i, r[i], s, r[64 + i], m);
                return 1;
            }
        }
        for (int i = 0; i < 64; ++i)
            if (r[128 + i] != s) { printf("readlane mismatch\n"); return 1; }
    }
    printf("dpp ok\n");
    return 0;
}

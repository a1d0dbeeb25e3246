// Probe: which XCD does workgroup L run on?  (placement check for the per-XCD
// queues; prints a histogram of (L mod 8, XCC_ID) pairs)
//   hipcc -O3 --offload-arch=gfx950 tools/probes/xcc_probe.hip -o starch_amd/_build/xcc_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(unsigned* o)
{
    if (threadIdx.x == 0) o[blockIdx.x] = __builtin_amdgcn_s_getreg(20 | (0 << 6) | (3 << 11));
}
int main()
{
    const int n = 4096;
    unsigned* d;
    hipMalloc(&d, n * 4);
    hipLaunchKernelGGL(k, dim3(n), dim3(256), 0, 0, d);
    unsigned h[4096];
    hipMemcpy(h, d, n * 4, hipMemcpyDeviceToHost);
    int cnt[8][16] = {};
    for (int i = 0; i < n; ++i) cnt[i % 8][h[i] & 15]++;
    for (int r = 0; r < 8; ++r) {
        printf("L%%8=%d:", r);
        for (int x = 0; x < 16; ++x) if (cnt[r][x]) printf(" xcc%d=%d", x, cnt[r][x]);
        printf("\n");
    }
    return 0;
}

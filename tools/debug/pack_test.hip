// debug: the packed sort_w lane mapping on the GPU vs a host model
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>
#include <random>
#include "../../starch_amd/csrc/common.hpp"
__device__ __forceinline__ uint64_t shfl64(uint64_t v, uint32_t src)
{
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, (int)src, 64);
    const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), (int)src, 64);
    return ((uint64_t)hi << 32) | lo;
}
__global__ void k(const uint32_t* sizes, uint32_t cnt, uint32_t* out)   // out[pass*64+lane] = gi<<16 | j
{
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t myitem = lane < cnt ? ((uint64_t)lane << 32 | sizes[lane]) : 0ull;
    const uint32_t msz = lane < cnt ? (uint32_t)myitem : 0u;
    uint32_t pass = 0;
    for (uint32_t done = 0; done < cnt; ++pass) {
        const uint32_t sz = (lane >= done && lane < cnt) ? msz : 0u;
        const uint32_t incl = wave_incl_scan_add(sz);
        const bool take = lane >= done && lane < cnt && incl <= 64u;
        const uint32_t ng = (uint32_t)__popcll(__ballot(take));
        const uint32_t off = incl - sz;
        const uint32_t total = (uint32_t)__shfl((int)incl, (int)(done + ng - 1), 64);
        const uint64_t smask = wave_reduce_or64(take ? (1ull << off) : 0ull);
        const bool valid = lane < total;
        const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
        const uint32_t gi = valid ? done + (uint32_t)__popcll(smask & upto) - 1u : done;
        const uint64_t item = shfl64(myitem, gi);
        const uint32_t goff = (uint32_t)__shfl((int)off, (int)gi, 64);   // every lane: gi may be past `total`
        const uint32_t gstart = valid ? goff : 0u;
        const uint32_t j = valid ? lane - gstart : 0u;
        out[pass * 64 + lane] = valid ? (((uint32_t)(item >> 32)) << 16 | j) : 0xFFFFFFFFu;
        done += ng;
    }
}
int main()
{
    std::mt19937 rng(1);
    int bad = 0;
    uint32_t *ds, *dout;
    hipMalloc(&ds, 64 * 4); hipMalloc(&dout, 64 * 64 * 4);
    for (int t = 0; t < 200; ++t) {
        uint32_t cnt = 1 + rng() % 64;
        std::vector<uint32_t> sz(64, 0);
        for (uint32_t i = 0; i < cnt; ++i) sz[i] = (rng() % 5 == 0) ? 2 + rng() % 63 : 2 + rng() % 3;
        hipMemcpy(ds, sz.data(), 256, hipMemcpyHostToDevice);
        hipMemset(dout, 0xFF, 64 * 64 * 4);
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, ds, cnt, dout);
        std::vector<uint32_t> o(64 * 64);
        hipMemcpy(o.data(), dout, o.size() * 4, hipMemcpyDeviceToHost);
        // host model
        uint32_t done = 0, pass = 0;
        while (done < cnt) {
            uint32_t tot = 0, g = done;
            std::vector<uint32_t> exp(64, 0xFFFFFFFFu);
            while (g < cnt && tot + sz[g] <= 64) { for (uint32_t q = 0; q < sz[g]; ++q) exp[tot + q] = g << 16 | q; tot += sz[g]; ++g; }
            for (int l = 0; l < 64; ++l) if (o[pass * 64 + l] != exp[l]) { if (bad < 10) printf("t %d pass %u lane %d got %08x exp %08x\n", t, pass, l, o[pass*64+l], exp[l]); ++bad; }
            done = g; ++pass;
        }
    }
    printf("bad %d\n", bad);
    return bad != 0;
}

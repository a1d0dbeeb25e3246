// starch_amd/csrc/gen_bed_dev.hip -- the per-position synthetic input (cfg5,
// starch_gen_bed kind 2) generated straight into HBM.  Like gen_bed.cpp this
// is the benchmark's INPUT, not part of the compression path: the 73.6 GB
// cfg5 input takes about a minute on the host and then a PCIe copy; here one
// chromosome (at most 6 GB) is written by the GPU in milliseconds, so the
// full-size cfg5 parity test can cover all 24 chromosomes.
//
// Line p of chromosome c is "<name>\t<p>\t<p+1>\n" (gen_bed.cpp kind 2).  Its
// offset is closed-form: (p - first) * (name + 3) plus the decimal digits of
// first..p-1 and of first+1..p (digit sums over whole decades).
#include <stdint.h>
#include <string.h>

#include "../../include/starch_amd.h"
#include "common.hpp"

namespace {

struct Name { char s[8]; uint32_t len; };
const char* kNames[24] = {"chr1",  "chr10", "chr11", "chr12", "chr13", "chr14", "chr15", "chr16",
                          "chr17", "chr18", "chr19", "chr2",  "chr20", "chr21", "chr22", "chr3",
                          "chr4",  "chr5",  "chr6",  "chr7",  "chr8",  "chr9",  "chrX",  "chrY"};
const uint64_t kLen[24] = {248956422, 133797422, 135086622, 133275309, 114364328, 107043718, 101991189, 90338345,
                           83257441,  80373285,  58617616,  242193529, 64444167,  46709983,  50818468,  198295559,
                           190214555, 181538259, 170805979, 159345973, 145138636, 138394717, 156040895, 57227415};

// sum of the decimal digit counts of 0 .. x-1 (0 has one digit)
__host__ __device__ inline uint64_t digit_sum(uint64_t x)
{
    if (x == 0) return 0;
    uint64_t s = 1;                     // the number 0
    uint64_t lo = 1;
    for (uint32_t k = 1; k <= 19 && lo < x; ++k) {
        const uint64_t hi = lo * 10;    // numbers with k digits: [lo, hi)
        const uint64_t e = x < hi ? x : hi;
        s += (e - lo) * k;
        if (hi / 10 != lo) break;       // overflow guard
        lo = hi;
    }
    return s;
}

__device__ inline uint32_t ndig(uint64_t v)
{
    uint32_t d = 1;
    while (v >= 10) { v /= 10; ++d; }
    return d;
}

__device__ inline void put_dec(uint8_t* o, uint64_t v, uint32_t d)
{
    for (uint32_t i = d; i > 0; --i) { o[i - 1] = (uint8_t)('0' + v % 10); v /= 10; }
}

__global__ void k_gen_perpos(Name nm, uint64_t first, uint64_t count, uint8_t* __restrict__ out)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const uint64_t p = first + i;
    const uint64_t off = i * (nm.len + 3) + (digit_sum(p) - digit_sum(first)) + (digit_sum(p + 1) - digit_sum(first + 1));
    uint8_t* o = out + off;
    for (uint32_t k = 0; k < nm.len; ++k) o[k] = (uint8_t)nm.s[k];
    uint32_t k = nm.len;
    o[k++] = '\t';
    const uint32_t d0 = ndig(p), d1 = ndig(p + 1);
    put_dec(o + k, p, d0);
    k += d0;
    o[k++] = '\t';
    put_dec(o + k, p + 1, d1);
    k += d1;
    o[k] = '\n';
}

}  // namespace

extern "C" int starch_gen_perpos_device(int chrom, uint64_t first, uint64_t count, void* d_dst, uint64_t cap,
                                        uint64_t* len, void* stream)
{
    if (chrom < 0 || chrom >= 24 || !len) return STARCH_ERR_ARG;
    if (first > kLen[chrom] || count > kLen[chrom] - first) return STARCH_ERR_ARG;
    Name nm{};
    nm.len = (uint32_t)strlen(kNames[chrom]);
    memcpy(nm.s, kNames[chrom], nm.len);
    const uint64_t bytes = count * (nm.len + 3) + (digit_sum(first + count) - digit_sum(first)) +
                           (digit_sum(first + count + 1) - digit_sum(first + 1));
    *len = bytes;
    if (!d_dst) return STARCH_OK;
    if (cap < bytes) return STARCH_ERR_MEM;
    if (!count) return STARCH_OK;
    hipStream_t st = static_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(k_gen_perpos, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, st, nm, first, count,
                       static_cast<uint8_t*>(d_dst));
    if (hipGetLastError() != hipSuccess) return STARCH_ERR_DEVICE;
    return STARCH_OK;
}

// starch_amd/csrc/gen_bed.cpp -- deterministic synthetic hg38 BED generator
// (bench + tests).  Host code: it produces the INPUT
// of the benchmark, it is not part of the compression path.
//
// Line i of chromosome c depends only on (seed, c, i) through splitmix64, so
// any subset of chromosomes (a rank's shard) is generated independently and
// identically on the GPU box and in this container.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

#include "../../include/starch_amd.h"

namespace {

struct Chrom { const char* name; uint64_t len; };
const Chrom kHg38[24] = {
    {"chr1", 248956422}, {"chr10", 133797422}, {"chr11", 135086622}, {"chr12", 133275309},
    {"chr13", 114364328}, {"chr14", 107043718}, {"chr15", 101991189}, {"chr16", 90338345},
    {"chr17", 83257441}, {"chr18", 80373285}, {"chr19", 58617616}, {"chr2", 242193529},
    {"chr20", 64444167}, {"chr21", 46709983}, {"chr22", 50818468}, {"chr3", 198295559},
    {"chr4", 190214555}, {"chr5", 181538259}, {"chr6", 170805979}, {"chr7", 159345973},
    {"chr8", 145138636}, {"chr9", 138394717}, {"chrX", 156040895}, {"chrY", 57227415},
};
const uint64_t kGenome = 3088269832ull;

inline uint64_t mix(uint64_t x)
{
    x += 0x9e3779b97f4a7c15ull;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}
inline uint64_t rnd(uint64_t seed, uint64_t c, uint64_t i, uint64_t k)
{
    return mix(seed ^ mix((c << 58) ^ (k << 52) ^ i));
}

inline size_t put_u(char* o, uint64_t v)
{
    char t[24];
    int n = 0;
    do { t[n++] = (char)('0' + v % 10); v /= 10; } while (v);
    for (int k = 0; k < n; ++k) o[k] = t[n - 1 - k];
    return (size_t)n;
}
inline size_t put_fix5(char* o, uint64_t micro)   // micro / 1e5 with 5 decimals
{
    size_t k = put_u(o, micro / 100000);
    o[k++] = '.';
    uint64_t f = micro % 100000;
    for (int d = 4; d >= 0; --d) { o[k + d] = (char)('0' + f % 10); f /= 10; }
    return k + 5;
}

uint64_t lines_of(int kind, int c, uint64_t total)
{
    if (kind == 2) return kHg38[c].len;
    // cumulative rounding: the 24 per-chromosome counts sum to exactly `total`
    uint64_t before = 0;
    for (int k = 0; k < c; ++k) before += kHg38[k].len;
    const uint64_t upto = before + kHg38[c].len;
    const long double t = (long double)total / (long double)kGenome;
    return (uint64_t)((long double)upto * t + 0.5L) - (uint64_t)((long double)before * t + 0.5L);
}

// writes chromosome c's lines (dst may be NULL: size only)
uint64_t gen_chrom(int kind, uint64_t seed, uint64_t total, int c, char* dst)
{
    const uint64_t n = lines_of(kind, c, total);
    const char* name = kHg38[c].name;
    const size_t nl = strlen(name);
    char buf[256];
    uint64_t bytes = 0;
    uint64_t pos = 0;
    const uint64_t L = kHg38[c].len;
    const uint64_t span = kind == 1 ? 2000 : 1000;
    const uint64_t mean = n ? (L - span) / n : 1;
    const uint64_t incmax = mean ? 2 * mean - 1 : 1;   // inc in [1, 2*mean-1], mean spacing = mean
    for (uint64_t i = 0; i < n; ++i) {
        size_t k = 0;
        memcpy(buf, name, nl);
        k = nl;
        buf[k++] = '\t';
        uint64_t s, e;
        if (kind == 2) {
            s = i;
            e = i + 1;
        } else {
            pos += 1 + rnd(seed, c, i, 0) % incmax;
            s = pos;
            e = s + (kind == 0 ? 20 + rnd(seed, c, i, 1) % 980 : 150 + rnd(seed, c, i, 1) % 1850);
        }
        k += put_u(buf + k, s);
        buf[k++] = '\t';
        k += put_u(buf + k, e);
        if (kind == 1) {   // ENCODE narrowPeak BED6+4
            memcpy(buf + k, "\tpeak", 5); k += 5;
            k += put_u(buf + k, i);
            buf[k++] = '\t';
            k += put_u(buf + k, rnd(seed, c, i, 2) % 1001);
            memcpy(buf + k, "\t.\t", 3); k += 3;
            k += put_fix5(buf + k, rnd(seed, c, i, 3) % 10000000ull);
            buf[k++] = '\t';
            k += put_fix5(buf + k, rnd(seed, c, i, 4) % 5000000ull);
            buf[k++] = '\t';
            k += put_fix5(buf + k, rnd(seed, c, i, 5) % 2000000ull);
            buf[k++] = '\t';
            k += put_u(buf + k, rnd(seed, c, i, 6) % (e - s));
        }
        buf[k++] = '\n';
        if (dst) memcpy(dst + bytes, buf, k);
        bytes += k;
    }
    return bytes;
}

}  // namespace

extern "C" int starch_gen_bed(int kind, uint64_t seed, uint64_t total_lines, const int32_t* chroms, int nchroms,
                              void* dst, uint64_t cap, uint64_t* len)
{
    if (kind < 0 || kind > 2 || nchroms < 0 || !len) return STARCH_ERR_ARG;
    for (int k = 0; k < nchroms; ++k) if (chroms[k] < 0 || chroms[k] >= 24) return STARCH_ERR_ARG;
    std::vector<uint64_t> sz(nchroms, 0);
    unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    auto run = [&](bool write, const std::vector<uint64_t>* offs) {
        std::vector<std::thread> th;
        std::vector<int> next(1, 0);
        for (unsigned t = 0; t < hw; ++t) {
            th.emplace_back([&, t]() {
                for (int k = (int)t; k < nchroms; k += (int)hw) {
                    char* d = write ? static_cast<char*>(dst) + (*offs)[k] : nullptr;
                    sz[k] = gen_chrom(kind, seed, total_lines, chroms[k], d);
                }
            });
        }
        for (auto& x : th) x.join();
    };
    run(false, nullptr);
    std::vector<uint64_t> offs(nchroms + 1, 0);
    for (int k = 0; k < nchroms; ++k) offs[k + 1] = offs[k] + sz[k];
    *len = offs[nchroms];
    if (!dst) return STARCH_OK;
    if (cap < offs[nchroms]) return STARCH_ERR_MEM;
    run(true, &offs);
    return STARCH_OK;
}

// per-chromosome byte counts of starch_gen_bed's output (sizes[k] for chroms[k])
extern "C" int starch_gen_bed_sizes(int kind, uint64_t seed, uint64_t total_lines, const int32_t* chroms, int nchroms,
                                    uint64_t* sizes)
{
    if (kind < 0 || kind > 2 || nchroms < 0 || (nchroms && !sizes)) return STARCH_ERR_ARG;
    for (int k = 0; k < nchroms; ++k) if (chroms[k] < 0 || chroms[k] >= 24) return STARCH_ERR_ARG;
    unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<std::thread> th;
    for (unsigned t = 0; t < hw; ++t)
        th.emplace_back([&, t]() {
            for (int k = (int)t; k < nchroms; k += (int)hw) sizes[k] = gen_chrom(kind, seed, total_lines, chroms[k], nullptr);
        });
    for (auto& x : th) x.join();
    return STARCH_OK;
}

// starch_amd/csrc/common.hpp -- shared device/host helpers for the MI355X
// (gfx950, CDNA4) Starch pipeline.  wave64 throughout; all arithmetic integer.
#pragma once
#include <hip/hip_runtime.h>

#include <stdlib.h>
#include <string.h>

#include <memory>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string>
#include <stdexcept>

#define ST_WAVE 64

struct StarchError : std::runtime_error {
    int code;
    StarchError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define HIP_CHECK(expr)                                                                 \
    do {                                                                                \
        hipError_t _e = (expr);                                                         \
        if (_e != hipSuccess)                                                           \
            throw StarchError(-10, std::string("HIP error ") + hipGetErrorString(_e) + \
                                       " at " __FILE__ ":" + std::to_string(__LINE__)); \
    } while (0)

static inline uint64_t ceil_div(uint64_t a, uint64_t b) { return (a + b - 1) / b; }

// ---------------------------------------------------------------------------
// Device workspace: grow-only buffers owned by the context.
// ---------------------------------------------------------------------------
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    void* get(size_t bytes) {
        if (bytes == 0) bytes = 16;
        if (bytes > cap) {
            if (p) HIP_CHECK(hipFree(p));
            p = nullptr;
            size_t want = bytes + bytes / 8 + 256;
            HIP_CHECK(hipMalloc(&p, want));
            cap = want;
        }
        return p;
    }
    template <class T> T* as(size_t count) { return static_cast<T*>(get(count * sizeof(T))); }
    void release() { if (p) (void)hipFree(p); p = nullptr; cap = 0; }
    ~DevBuf() { release(); }
};

// Grow-only pinned host buffer (hipHostMalloc): small device <-> host
// transfers without pageable staging.  The caller orders reuse against the
// copies that read or fill it (stream syncs).
struct PinnedBuf {
    void* p = nullptr;
    size_t cap = 0;
    void* get(size_t bytes) {
        if (bytes == 0) bytes = 16;
        if (bytes > cap) {
            if (p) HIP_CHECK(hipHostFree(p));
            p = nullptr;
            size_t want = bytes + bytes / 2 + 4096;
            HIP_CHECK(hipHostMalloc(&p, want, hipHostMallocDefault));
            cap = want;
        }
        return p;
    }
    template <class T> T* as(size_t count) { return static_cast<T*>(get(count * sizeof(T))); }
    ~PinnedBuf() { if (p) (void)hipHostFree(p); }
};

// Host memory the runtime can DMA from directly for the duration of one call
// (an mmap'ed file, a caller's buffer): registering a page-cached 2.4 GB
// mapping took ~28 ms and its copies then ran at the pinned rate
// (tools/probes/h2d_file_probe.cpp), against ~0.2 s per GB to pin fresh memory
// or ~0.1 s per GB to copy through a staging buffer.  Page-rounded; read-only
// unless `writable`.  If the runtime refuses (already pinned or registered,
// ...) nothing happens and the copies go as before.  STARCH_REGISTER=0: off.
struct HostRegistration {
    void* base = nullptr;
    HostRegistration(const void* p, uint64_t n, uint64_t min_bytes, bool writable = false)
    {
        if (!p || n < min_bytes) return;
        static const bool off = [] { const char* e = getenv("STARCH_REGISTER"); return e && !strcmp(e, "0"); }();
        if (off) return;
        hipPointerAttribute_t a;
        if (hipPointerGetAttributes(&a, p) == hipSuccess && a.type == hipMemoryTypeHost) return;   // pinned already
        (void)hipGetLastError();
        const uintptr_t pg = 4096, lo = reinterpret_cast<uintptr_t>(p) & ~(pg - 1),
                        hi = (reinterpret_cast<uintptr_t>(p) + n + pg - 1) & ~(pg - 1);
        if (hipHostRegister(reinterpret_cast<void*>(lo), hi - lo, writable ? hipHostRegisterDefault
                                                                          : hipHostRegisterReadOnly) == hipSuccess)
            base = reinterpret_cast<void*>(lo);
        else
            (void)hipGetLastError();
    }
    ~HostRegistration()
    {
        if (base) (void)hipHostUnregister(base);
    }
    bool ok() const { return base != nullptr; }
    HostRegistration(const HostRegistration&) = delete;
    HostRegistration& operator=(const HostRegistration&) = delete;
};

// A growable host byte buffer that is never zero-filled (std::vector's
// resize zero-fills: ~0.1 s per GB of output that is then overwritten).
struct RawBytes {
    std::unique_ptr<uint8_t[]> p;
    size_t n = 0, cap = 0;
    void resize(size_t k)                       // contents up to min(n, k) kept
    {
        if (k > cap) {
            const size_t c = k + k / 2 + 4096;
            std::unique_ptr<uint8_t[]> q(new uint8_t[c]);
            if (n) memcpy(q.get(), p.get(), n < k ? n : k);
            p.swap(q);
            cap = c;
        }
        n = k;
    }
    uint8_t* data() { return p.get(); }
    const uint8_t* data() const { return p.get(); }
    size_t size() const { return n; }
    void clear() { n = 0; }
    void release() { p.reset(); n = cap = 0; }
};

// ---------------------------------------------------------------------------
// Wave / workgroup scan helpers (wave64).
// ---------------------------------------------------------------------------
template <class T>
__device__ __forceinline__ T wave_incl_scan_add(T v)
{
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        T o = __shfl_up(v, d, 64);
        if (lane >= d) v += o;
    }
    return v;
}

template <class T>
__device__ __forceinline__ T wave_incl_scan_max(T v)
{
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        T o = __shfl_up(v, d, 64);
        if (lane >= d) v = (o > v) ? o : v;
    }
    return v;
}

template <class T>
__device__ __forceinline__ T wave_reduce_add(T v)
{
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

// Block-wide exclusive sum; `sh` must hold blockDim.x/64 + 1 elements.
// Returns the exclusive prefix for this thread; *total gets the block sum.
// 32-bit versions on DPP row shifts and row broadcasts (VALU, no LDS
// round trip; gfx9 family): Hillis-Steele inside each 16-lane row, then
// row_bcast:15 / row_bcast:31 carry row totals upward.  Every lane of the wave
// must be active (same contract as the shuffle forms).
__device__ __forceinline__ uint32_t dpp_up(uint32_t v, int ctrl_shr)   // 0 where the source is out of row
{
    switch (ctrl_shr) {
    case 1: return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);
    case 2: return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);
    case 4: return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);
    default: return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true);
    }
}
__device__ __forceinline__ uint32_t dpp_bc15(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);
}
__device__ __forceinline__ uint32_t dpp_bc31(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);
}

template <>
__device__ __forceinline__ uint32_t wave_incl_scan_add<uint32_t>(uint32_t v)
{
    v += dpp_up(v, 1);
    v += dpp_up(v, 2);
    v += dpp_up(v, 4);
    v += dpp_up(v, 8);
    v += dpp_bc15(v);
    v += dpp_bc31(v);
    return v;
}

template <>
__device__ __forceinline__ uint32_t wave_incl_scan_max<uint32_t>(uint32_t v)
{
    uint32_t t;
    t = dpp_up(v, 1); v = t > v ? t : v;
    t = dpp_up(v, 2); v = t > v ? t : v;
    t = dpp_up(v, 4); v = t > v ? t : v;
    t = dpp_up(v, 8); v = t > v ? t : v;
    t = dpp_bc15(v); v = t > v ? t : v;
    t = dpp_bc31(v); v = t > v ? t : v;
    return v;
}

__device__ __forceinline__ uint32_t wave_incl_scan_or(uint32_t v)
{
    v |= dpp_up(v, 1);
    v |= dpp_up(v, 2);
    v |= dpp_up(v, 4);
    v |= dpp_up(v, 8);
    v |= dpp_bc15(v);
    v |= dpp_bc31(v);
    return v;
}

template <>
__device__ __forceinline__ uint32_t wave_reduce_add<uint32_t>(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan_add<uint32_t>(v), 63);
}

__device__ __forceinline__ uint64_t wave_reduce_or64(uint64_t v)
{
    const uint32_t lo = wave_incl_scan_or((uint32_t)v), hi = wave_incl_scan_or((uint32_t)(v >> 32));
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)hi, 63) << 32) |
           (uint32_t)__builtin_amdgcn_readlane((int)lo, 63);
}

__device__ __forceinline__ uint32_t wave_reduce_max(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan_max<uint32_t>(v), 63);
}

template <class T>
__device__ __forceinline__ T block_excl_scan_add(T v, T* sh, T* total)
{
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    T inc = wave_incl_scan_add(v);
    if (lane == 63) sh[wid] = inc;
    __syncthreads();
    if (wid == 0) {
        T s = (lane < nw) ? sh[lane] : T(0);
        T si = wave_incl_scan_add(s);
        if (lane < nw) sh[lane] = si - s;
        if (lane == nw - 1) sh[nw] = si;
    }
    __syncthreads();
    T res = sh[wid] + inc - v;
    if (total) *total = sh[nw];
    __syncthreads();
    return res;
}

template <class T>
__device__ __forceinline__ T block_incl_scan_max(T v, T* sh)
{
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    T inc = wave_incl_scan_max(v);
    if (lane == 63) sh[wid] = inc;
    __syncthreads();
    if (wid == 0) {
        T s = (lane < nw) ? sh[lane] : T(0);
        T si = wave_incl_scan_max(s);
        if (lane < nw) sh[lane] = si;   // inclusive max up to wave lane
    }
    __syncthreads();
    T prev = (wid > 0) ? sh[wid - 1] : T(0);
    T res = (prev > inc) ? prev : inc;
    __syncthreads();
    return res;
}

// ---------------------------------------------------------------------------
// Device-wide exclusive scans (reduce -> scan partials -> downsweep).
// ---------------------------------------------------------------------------
namespace scan {
constexpr int kThreads = 256;
constexpr int kItems = 16;                   // elements per thread
constexpr int kTile = kThreads * kItems;     // 4096 per tile

// Exclusive prefix sum of in[0..n) into out (may alias), 64-bit accumulation.
// Returns nothing; *total_dev (optional) receives the grand total.
void excl_sum_u64(const uint64_t* in, uint64_t* out, uint64_t n, uint64_t* total_dev,
                  DevBuf& tmp, hipStream_t st);
void excl_sum_u32_to_u64(const uint32_t* in, uint64_t* out, uint64_t n, uint64_t* total_dev,
                         DevBuf& tmp, hipStream_t st);
// In-place inclusive max-scan of u64 (used for "index of last valid" propagation).
void incl_max_u64(uint64_t* data, uint64_t n, DevBuf& tmp, hipStream_t st);
}  // namespace scan

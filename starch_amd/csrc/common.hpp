// starch_amd/csrc/common.hpp -- shared device/host helpers for the MI355X
// (gfx950, CDNA4) Starch pipeline.  wave64 throughout; all arithmetic integer.
#pragma once
#include <hip/hip_runtime.h>

#include <stdlib.h>
#include <string.h>

#include <map>
#include <memory>
#include <mutex>
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

// Process-wide record of the host ranges the library may DMA from: ranges the
// caller page-locked through starch_host_register (permanent until
// starch_host_unregister) and the library's own temporary registrations
// (HostRegistration, refcounted: two threads coding from one shared input see
// one registration, which is dropped when the last of them is done -- a
// registration owned by one thread and merely "found pinned" by another was
// unregistered under the other's in-flight copy).
struct PinRegistry {
    struct Range {
        uintptr_t hi;
        int refs;        // temporary registrations: users; permanent: 0
        bool temp;
    };
    std::mutex mu;
    std::map<uintptr_t, Range> m;   // lo -> range (ranges never overlap)
    // the range holding address a (lock held), or end()
    std::map<uintptr_t, Range>::iterator holding(uintptr_t a)
    {
        auto it = m.upper_bound(a);
        if (it == m.begin()) return m.end();
        --it;
        return a < it->second.hi ? it : m.end();
    }
    bool overlaps(uintptr_t lo, uintptr_t hi)   // (lock held)
    {
        auto it = m.lower_bound(lo);
        if (it != m.end() && it->first < hi) return true;
        if (it == m.begin()) return false;
        --it;
        return it->second.hi > lo;
    }
};
inline PinRegistry& pin_registry()
{
    static PinRegistry* r = new PinRegistry;   // (never destroyed: used until exit)
    return *r;
}

// Host memory the runtime can DMA from directly for the duration of one call
// (an mmap'ed file, a caller's buffer): registering a page-cached 2.4 GB
// mapping took ~28 ms and its copies then ran at the pinned rate
// (tools/probes/h2d_file_probe.cpp), against ~0.2 s per GB to pin fresh memory
// or ~0.1 s per GB to copy through a staging buffer.  Only the whole pages
// inside [p, p + n) are registered -- a page shared with a neighbouring
// allocation (malloc'ed buffers next to each other) stays as it was, so
// another thread's copies into that neighbour are not disturbed (a
// page-rounded registration made them fail with "invalid argument").  Copies
// go through h2d(): the DMA-able middle directly, the rest around it as
// pageable copies.  Read-only.  Where the range starts:
//   * in a range the caller registered (starch_host_register): DMA up to that
//     range's end, never past it;
//   * in a temporary registration of another call: shared (refcounted);
//   * in memory pinned by other means (hipHostMalloc, a framework's pinned
//     allocator): DMA up to the end of that allocation as the runtime reports
//     it (hipMemGetAddressRange), else nothing is DMA'd directly;
//   * elsewhere: its whole pages are registered for the call, unless they
//     overlap another recorded range (then pageable copies only).
// STARCH_REGISTER=0: off.
struct HostRegistration {
    uintptr_t lo = 0, hi = 0;                  // the DMA-able part [lo, hi)
    uintptr_t temp = 0;                        // the temporary registration this call holds a reference on
    HostRegistration(const void* p, uint64_t n, uint64_t min_bytes)
    {
        if (!p || n < min_bytes) return;
        static const bool off = [] { const char* e = getenv("STARCH_REGISTER"); return e && !strcmp(e, "0"); }();
        if (off) return;
        const uintptr_t b0 = reinterpret_cast<uintptr_t>(p), e0 = b0 + n;
        PinRegistry& R = pin_registry();
        std::lock_guard<std::mutex> lk(R.mu);
        auto it = R.holding(b0);
        if (it != R.m.end()) {                 // caller-registered, or another call's registration
            lo = b0;
            hi = e0 < it->second.hi ? e0 : it->second.hi;
            if (it->second.temp) { ++it->second.refs; temp = it->first; }
            return;
        }
        hipPointerAttribute_t a;
        const bool pinned = hipPointerGetAttributes(&a, p) == hipSuccess && a.type == hipMemoryTypeHost;
        (void)hipGetLastError();
        if (pinned) {                          // pinned outside the library: its allocation bounds the DMA
            void* base = nullptr;
            size_t sz = 0;
            if (hipMemGetAddressRange(&base, &sz, const_cast<void*>(p)) == hipSuccess && base && sz) {
                const uintptr_t ah = reinterpret_cast<uintptr_t>(base) + sz;
                if (reinterpret_cast<uintptr_t>(base) <= b0 && ah > b0) {
                    lo = b0;
                    hi = e0 < ah ? e0 : ah;
                }
            }
            (void)hipGetLastError();
            return;
        }
        const uintptr_t pg = 4096;
        const uintptr_t l = (b0 + pg - 1) & ~(pg - 1), h = e0 & ~(pg - 1);
        if (h <= l || h - l < min_bytes / 2) return;
        if (R.overlaps(l, h)) return;
        if (hipHostRegister(reinterpret_cast<void*>(l), h - l, hipHostRegisterReadOnly | hipHostRegisterPortable) == hipSuccess) {
            R.m[l] = PinRegistry::Range{h, 1, true};
            temp = l;
            lo = l;
            hi = h;
        } else {
            (void)hipGetLastError();
        }
    }
    ~HostRegistration()
    {
        if (!temp) return;
        PinRegistry& R = pin_registry();
        std::lock_guard<std::mutex> lk(R.mu);
        auto it = R.m.find(temp);
        if (it == R.m.end() || !it->second.temp || --it->second.refs > 0) return;
        (void)hipHostUnregister(reinterpret_cast<void*>(temp));
        (void)hipGetLastError();
        R.m.erase(it);
    }
    bool ok() const { return hi > lo; }   // (registered here, or pinned by the caller)
    // host [src, src + n) -> dst on stream st, splitting around the DMA-able part
    void h2d(void* dst, const void* src, uint64_t n, hipStream_t st) const
    {
        uint8_t* d = static_cast<uint8_t*>(dst);
        const uintptr_t s = reinterpret_cast<uintptr_t>(src), e = s + n;
        if (hi <= lo || e <= lo || s >= hi) {
            if (n) HIP_CHECK(hipMemcpyAsync(d, src, n, hipMemcpyHostToDevice, st));
            return;
        }
        const uintptr_t a = s > lo ? s : lo, b = e < hi ? e : hi;
        if (a > s) HIP_CHECK(hipMemcpyAsync(d, src, a - s, hipMemcpyHostToDevice, st));
        HIP_CHECK(hipMemcpyAsync(d + (a - s), reinterpret_cast<const void*>(a), b - a, hipMemcpyHostToDevice, st));
        if (e > b) HIP_CHECK(hipMemcpyAsync(d + (b - s), reinterpret_cast<const void*>(b), e - b, hipMemcpyHostToDevice, st));
    }
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

// starch_amd/csrc/scan.hip -- device-wide scans used by the transform and the
// bzip2 stages: reduce-then-scan over 4096-element tiles (256 threads x 16
// items, coalesced per-thread strips), a single-workgroup scan of the tile
// partials, and a downsweep.  HBM-bound: 2 reads + 1 write per element.
#include "common.hpp"

namespace scan {
namespace {

struct OpAdd {
    template <class T> __device__ static T id() { return T(0); }
    template <class T> __device__ static T op(T a, T b) { return a + b; }
};
struct OpMax {
    template <class T> __device__ static T id() { return T(0); }
    template <class T> __device__ static T op(T a, T b) { return a > b ? a : b; }
};

template <class Op, class T>
__device__ __forceinline__ T wave_incl(T v)
{
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        T o = __shfl_up(v, d, 64);
        if (lane >= d) v = Op::op(o, v);
    }
    return v;
}

// exclusive block scan with operator; sh: kThreads/64 + 1 entries
template <class Op, class T>
__device__ __forceinline__ T block_excl(T v, T* sh, T* total)
{
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    T inc = wave_incl<Op>(v);
    T exc = __shfl_up(inc, 1, 64);
    if (lane == 0) exc = Op::template id<T>();
    if (lane == 63) sh[wid] = inc;
    __syncthreads();
    if (wid == 0) {
        T s = (lane < nw) ? sh[lane] : Op::template id<T>();
        T si = wave_incl<Op>(s);
        T se = __shfl_up(si, 1, 64);
        if (lane == 0) se = Op::template id<T>();
        if (lane < nw) sh[lane] = se;
        if (lane == nw - 1) sh[nw] = si;
    }
    __syncthreads();
    T res = Op::op(sh[wid], exc);
    if (total) *total = sh[nw];
    __syncthreads();
    return res;
}

template <class Op, class Tin, class T>
__global__ void __launch_bounds__(kThreads) k_reduce(const Tin* __restrict__ in, uint64_t n, T* __restrict__ part)
{
    __shared__ T sh[kThreads / 64 + 1];
    const uint64_t base = (uint64_t)blockIdx.x * kTile + (uint64_t)threadIdx.x * kItems;
    T acc = Op::template id<T>();
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
        uint64_t i = base + k;
        if (i < n) acc = Op::op(acc, (T)in[i]);
    }
    T tot;
    (void)block_excl<Op>(acc, sh, &tot);
    if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

// single workgroup: exclusive scan of part[0..m) in place; total to *total
template <class Op, class T>
__global__ void __launch_bounds__(1024) k_scan_parts(T* __restrict__ part, uint64_t m, T* __restrict__ total)
{
    __shared__ T sh[1024 / 64 + 1];
    T carry = Op::template id<T>();
    for (uint64_t b = 0; b < m; b += 1024) {
        uint64_t i = b + threadIdx.x;
        T v = (i < m) ? part[i] : Op::template id<T>();
        T tot;
        T e = block_excl<Op>(v, sh, &tot);
        if (i < m) part[i] = Op::op(carry, e);
        carry = Op::op(carry, tot);
    }
    if (threadIdx.x == 0 && total) *total = carry;
}

template <class Op, bool Inclusive, class Tin, class T>
__global__ void __launch_bounds__(kThreads) k_down(const Tin* in, T* out, uint64_t n,
                                                   const T* __restrict__ part)
{
    __shared__ T sh[kThreads / 64 + 1];
    const uint64_t base = (uint64_t)blockIdx.x * kTile + (uint64_t)threadIdx.x * kItems;
    T v[kItems];
    T acc = Op::template id<T>();
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
        uint64_t i = base + k;
        v[k] = (i < n) ? (T)in[i] : Op::template id<T>();
        acc = Op::op(acc, v[k]);
    }
    T pre = block_excl<Op>(acc, sh, (T*)nullptr);
    T run = Op::op(part[blockIdx.x], pre);
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
        uint64_t i = base + k;
        T nx = Op::op(run, v[k]);
        if (i < n) out[i] = Inclusive ? nx : run;
        run = nx;
    }
}

template <class Op, bool Inclusive, class Tin, class T>
void run_scan(const Tin* in, T* out, uint64_t n, T* total_dev, DevBuf& tmp, hipStream_t st)
{
    if (n == 0) {
        if (total_dev) HIP_CHECK(hipMemsetAsync(total_dev, 0, sizeof(T), st));
        return;
    }
    uint64_t nb = ceil_div(n, kTile);
    T* part = tmp.as<T>(nb + 1);
    hipLaunchKernelGGL((k_reduce<Op, Tin, T>), dim3((unsigned)nb), dim3(kThreads), 0, st, in, n, part);
    hipLaunchKernelGGL((k_scan_parts<Op, T>), dim3(1), dim3(1024), 0, st, part, nb, total_dev);
    hipLaunchKernelGGL((k_down<Op, Inclusive, Tin, T>), dim3((unsigned)nb), dim3(kThreads), 0, st, in, out, n,
                       (const T*)part);
    HIP_CHECK(hipGetLastError());
}
}  // namespace

void excl_sum_u64(const uint64_t* in, uint64_t* out, uint64_t n, uint64_t* total_dev, DevBuf& tmp, hipStream_t st)
{
    run_scan<OpAdd, false, uint64_t, uint64_t>(in, out, n, total_dev, tmp, st);
}
void excl_sum_u32_to_u64(const uint32_t* in, uint64_t* out, uint64_t n, uint64_t* total_dev, DevBuf& tmp,
                         hipStream_t st)
{
    run_scan<OpAdd, false, uint32_t, uint64_t>(in, out, n, total_dev, tmp, st);
}
void incl_max_u64(uint64_t* data, uint64_t n, DevBuf& tmp, hipStream_t st)
{
    run_scan<OpMax, true, uint64_t, uint64_t>(data, data, n, (uint64_t*)nullptr, tmp, st);
}
}  // namespace scan

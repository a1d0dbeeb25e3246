// starch_amd/csrc/bz2_mtf.hip -- move-to-front and RUNA/RUNB coding on MI355X
// (restates makeMaps_e + generateMTFValues, bz:compress.c:105-231).
//
// Input: the block's last column as sequence symbols (makeMaps_e ranks of
// block[(ptr[i]-1) mod n]), BwtScratch::LL, written by the block sort next
// to SA (k_last_col below for blocks sorted by the fallback).
//
// One 1024-thread workgroup per block, the block split into 1024 contiguous
// chunks of 128-byte lines.  MTF is made parallel by the chunk decomposition
//     state(c+1) = local(c) ++ (state(c) \ local(c)),
// where local(c) lists chunk c's symbols by last occurrence (most recent
// first); the map composes associatively, so every chunk's start state is an
// exclusive scan.  Alphabets of <= 16 symbols (BED3 transforms) keep the list
// as 16 nibbles of a u64 in a register: finding a symbol is a SWAR zero-nibble
// search and the move-to-front three masks and a shift.  Each lane reads its
// chunk as whole 128-byte lines (8 x 16-B loads), so every line is fetched
// once; the backward pass that builds local(c) stops as soon as all symbols
// of the block have been seen.  Zero runs may cross chunks; the
// (leading zeros, trailing zeros, inner outputs) summaries form a monoid whose
// scan places every chunk's output, and the MTF is simply re-run to emit
// (cheaper than storing the index stream).  Larger alphabets (nInUse > 16)
// keep byte lists in LDS (256 chunks, sequential start states).
#include "bz2_bwt.hpp"

namespace bz {

constexpr int MT = 1024;
constexpr int NCH_BIG = 256;
constexpr uint32_t LINE = 128;

__device__ __forceinline__ uint32_t nsym_run(uint32_t z) { return z ? (31 - __clz(z + 1)) : 0; }

// zero-run summary of a symbol range (monoid, applied left to right)
struct RunSum {
    uint32_t nz;      // has a non-zero MTF index
    uint32_t lz;      // leading zeros (all zeros: the length)
    uint32_t tz;      // trailing zeros
    uint32_t inner;   // outputs after the first non-zero symbol, trailing run excluded
};

__device__ __forceinline__ RunSum run_compose(const RunSum& a, const RunSum& b)
{
    RunSum r;
    if (!a.nz) {
        r.nz = b.nz; r.lz = a.lz + b.lz; r.tz = b.tz; r.inner = b.inner;
    } else if (!b.nz) {
        r.nz = 1; r.lz = a.lz; r.tz = a.tz + b.lz; r.inner = a.inner;
    } else {
        r.nz = 1; r.lz = a.lz; r.tz = b.tz; r.inner = a.inner + nsym_run(a.tz + b.lz) + 1 + b.inner;
    }
    return r;
}

__device__ __forceinline__ RunSum shfl_up_rs(const RunSum& v, int d)
{
    RunSum r;
    r.nz = __shfl_up(v.nz, d, 64);
    r.lz = __shfl_up(v.lz, d, 64);
    r.tz = __shfl_up(v.tz, d, 64);
    r.inner = __shfl_up(v.inner, d, 64);
    return r;
}

// Visit the bytes of one 128-byte line (all eight 16-B loads issued first, so
// the line is fetched once) as f(offset, byte); eight explicit pieces keep
// every index a compile-time constant (no scratch arrays).
template <bool FWD, class F>
__device__ __forceinline__ void piece(const uint4 v, int base, F& f)
{
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
        const int k = FWD ? kk : 15 - kk;
        f(base + k, (w[k >> 2] >> (8 * (k & 3))) & 0xffu);
    }
}

template <bool FWD, class F>
__device__ __forceinline__ void visit_line(const uint8_t* p, F&& f)
{
    const uint4* q = reinterpret_cast<const uint4*>(p);
    const uint4 v0 = q[0], v1 = q[1], v2 = q[2], v3 = q[3], v4 = q[4], v5 = q[5], v6 = q[6], v7 = q[7];
    if (FWD) {
        piece<FWD>(v0, 0, f); piece<FWD>(v1, 16, f); piece<FWD>(v2, 32, f); piece<FWD>(v3, 48, f);
        piece<FWD>(v4, 64, f); piece<FWD>(v5, 80, f); piece<FWD>(v6, 96, f); piece<FWD>(v7, 112, f);
    } else {
        piece<FWD>(v7, 112, f); piece<FWD>(v6, 96, f); piece<FWD>(v5, 80, f); piece<FWD>(v4, 64, f);
        piece<FWD>(v3, 48, f); piece<FWD>(v2, 32, f); piece<FWD>(v1, 16, f); piece<FWD>(v0, 0, f);
    }
}

// MTF values of alphabets <= 32 are stored as u8 (every value <= nInUse + 1
// <= 31; k_tables32 and k_emit_data read bytes for those blocks, k_mtf_big's
// larger alphabets stay u16), through a 128-bit shift register: one 16-byte
// store per 16 symbols once a window is wholly the chunk's; the partial
// windows at the chunk's two ends are written as 8/4/2/1-byte pieces
// (neighbouring chunks own the other bytes).  (u16 values took twice the
// stores: MTF stage 2.57 -> 2.40 ms on cfg2.  OR-ing a run's RUNA/RUNB
// symbols and the index into the window as one branch-free insertion
// measured slower, 2.80 ms.)
struct Out8 {
    uint8_t* base;
    uint32_t o;       // next index
    uint32_t s;       // the chunk's first output index
    uint64_t lo, hi;  // window byte j at register byte j once the window is complete
    __device__ __forceinline__ void init(uint8_t* b, uint32_t start)
    {
        base = b; o = start; s = start; lo = 0; hi = 0;
    }
    // store register bytes [p, q) of the window at w (register byte j = window byte j)
    __device__ __forceinline__ void store_range(uint32_t w, uint32_t p, uint32_t q, uint64_t rl, uint64_t rh)
    {
#pragma unroll 1
        while (p < q) {
            const uint64_t x = p >= 8 ? rh >> (8 * (p - 8)) : ((rl >> (8 * p)) | (p ? rh << (64 - 8 * p) : 0ull));
            uint8_t* d = base + w + p;
            if ((p & 7u) == 0 && p + 8 <= q) { *reinterpret_cast<uint64_t*>(d) = x; p += 8; }
            else if ((p & 3u) == 0 && p + 4 <= q) { *reinterpret_cast<uint32_t*>(d) = (uint32_t)x; p += 4; }
            else if ((p & 1u) == 0 && p + 2 <= q) { *reinterpret_cast<uint16_t*>(d) = (uint16_t)x; p += 2; }
            else { *d = (uint8_t)x; p += 1; }
        }
    }
    __device__ __forceinline__ void put(uint32_t sym)
    {
        lo = (lo >> 8) | (hi << 56);
        hi = (hi >> 8) | ((uint64_t)sym << 56);
        if ((o & 15u) == 15u) {
            const uint32_t w = o - 15u;
            if (w >= s) *reinterpret_cast<uint4*>(base + w) =
                make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
            else store_range(w, s - w, 16u, lo, hi);
        }
        ++o;
    }
    __device__ __forceinline__ void flush()
    {
        const uint32_t k = o & 15u;               // bytes of the open window: the top k of the register
        if (!k) return;
        const uint32_t w = o - k, p = s > w ? s - w : 0u;
        const uint32_t sh = 8u * (16u - k);       // align window byte 0 to register byte 0
        const uint64_t rl = sh >= 64 ? hi >> (sh - 64) : ((lo >> sh) | (sh ? hi << (64 - sh) : 0ull));
        const uint64_t rh = sh >= 64 ? 0ull : hi >> sh;
        store_range(w, p, k, rl, rh);
    }
};

__device__ __forceinline__ void put_run(Out8& out, uint32_t z)   // bijective base 2: RUNA = 0, RUNB = 1
{
    while (z) {
        const uint32_t d = ((z - 1) & 1u) ? 1u : 0u;
        out.put(d);
        z = (z - (d + 1)) >> 1;
    }
}

// ---- alphabets <= 32: five launches over (block, 512-symbol chunk) ----
// Per-chunk state lives in the (free) key scratch of the block's batch slot:
//   [0, SW*C)          local recency list + set    (k_mtf_local)
//   [SW*C, (SW+LW)*C)  start list of the chunk     (k_mtf_scan_lists)
//   then RunSum (2 words) and (zeros carried in, output offset) (1 word)
// (u64 words, C = chunks per slot).  The three chunk passes are flat grids,
// so every CU has work whatever the block count; the two scans are one
// workgroup per block over <= 2 chunks per thread.  The list lives in
// registers: 16 nibbles of a u64 for <= 16 symbols (NibP, BED3 text), 32
// bytes in three / four u64 for 17..24 / 25..30 symbols (ByteP<3> / ByteP<4>, narrowPeak and other BED6+
// text); both do the move-to-front branch-free with SWAR compares.
constexpr uint32_t MCS = 512;                 // symbols per chunk (4 lines); batches of few blocks
                                              // use shorter chunks (mtf_chunk)
constexpr int MCT = 256;                      // threads of the chunk kernels
constexpr int MST = 1024;                     // threads of the scan kernels

struct NibP {
    using State = NibState;
    using List = uint64_t;
    static constexpr uint32_t LO = 1, HI = 16;        // nInUse range handled
    static constexpr uint32_t SW = 2, LW = 1;         // u64 words per State / List
    static constexpr uint32_t IXB = 4;                // bits per stored MTF index (k_mtf_runs -> k_mtf_emit)
    // nibble MTF is cheap: k_mtf_emit re-runs it from the last column (storing
    // the indices measured slower: the stores queue behind the chunk's loads)
#ifndef STARCH_NIB_SIX
#define STARCH_NIB_SIX 0
#endif
    static constexpr bool SIX = STARCH_NIB_SIX != 0;
    __device__ static State empty() { State r; r.list = 0; r.set = 0; r.cnt = 0; return r; }
    __device__ static void add(State& st, uint32_t s)
    {
        if (!((st.set >> s) & 1u)) { st.set |= 1u << s; st.list |= (uint64_t)s << (4 * st.cnt); ++st.cnt; }
    }
    __device__ static State compose(const State& c, const State& d) { return nib_compose(c, d); }
    __device__ static State identity(uint32_t nin)
    {
        State st;
        st.list = 0;
        for (uint32_t i = 0; i < nin; ++i) st.list |= (uint64_t)i << (4 * i);
        st.set = nin >= 32 ? ~0u : (1u << nin) - 1u;
        st.cnt = nin;
        return st;
    }
    __device__ static List list_of(const State& st) { return st.list; }
    __device__ static uint32_t mtf(List& L, uint32_t s) { return nib_mtf(L, s); }
};

struct ByteState {        // transform L -> list ++ (L \ set); list byte i = i-th symbol, unused bytes 0xFF
    uint64_t w[4];
    uint32_t set;         // 32-bit symbol set
    uint32_t cnt;
};
struct ByteList { uint64_t w[4]; };

// NW list words: 3 for 17..24 symbols (narrowPeak's 17..20), 4 for 25..30
template <int NW>
struct ByteP {
    static_assert(NW == 3 || NW == 4, "ByteP: 3 or 4 list words");
    using State = ByteState;
    using List = ByteList;
    // <= 30 symbols: the alphabet (nInUse + 2) stays within k_tables32, which
    // counts mtfFreq itself (k_tables reads the counts k_mtf_big leaves)
    static constexpr uint32_t LO = NW == 3 ? 17 : 25, HI = NW == 3 ? 24 : 30;
    static constexpr uint32_t SW = 5, LW = 4;
    static constexpr uint32_t IXB = 8;
    // the zero runs from neighbour compares (k_mtf_runs) and the byte-list MTF
    // run once, in k_mtf_emit (STARCH_BYTE_SIX=1: k_mtf_runs runs the MTF and
    // stores the indices, k_mtf_emit reads them)
#ifndef STARCH_BYTE_SIX
#define STARCH_BYTE_SIX 0
#endif
    static constexpr bool SIX = STARCH_BYTE_SIX != 0;
    __device__ static void put(uint64_t* w, uint32_t i, uint32_t s)
    {
        const uint32_t j = i >> 3, sh = 8 * (i & 7);
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q)
            if (q == j) w[q] = (w[q] & ~(0xFFull << sh)) | ((uint64_t)s << sh);
    }
    __device__ static uint32_t get(const uint64_t* w, uint32_t i)
    {
        const uint32_t j = i >> 3;
        const uint64_t x = j == 0 ? w[0] : j == 1 ? w[1] : j == 2 ? w[2] : w[3];
        return (uint32_t)(x >> (8 * (i & 7))) & 0xFFu;
    }
    __device__ static State empty()
    {
        State r;
        r.w[0] = r.w[1] = r.w[2] = r.w[3] = ~0ull;
        r.set = 0;
        r.cnt = 0;
        return r;
    }
    __device__ static void add(State& st, uint32_t s)
    {
        if (!((st.set >> s) & 1u)) { st.set |= 1u << s; put(st.w, st.cnt, s); ++st.cnt; }
    }
    __device__ static State compose(const State& c, const State& d)   // apply c, then d
    {
        State r = d;
        for (uint32_t i = 0; i < c.cnt; ++i) {
            const uint32_t sym = get(c.w, i);
            if (!((d.set >> sym) & 1u)) { put(r.w, r.cnt, sym); ++r.cnt; }
        }
        r.set = c.set | d.set;
        return r;
    }
    __device__ static State identity(uint32_t nin)
    {
        State st = empty();
        for (uint32_t i = 0; i < nin; ++i) put(st.w, i, i);
        st.set = nin >= 32 ? ~0u : (1u << nin) - 1u;
        st.cnt = nin;
        return st;
    }
    __device__ static List list_of(const State& st)
    {
        List l;
        l.w[0] = st.w[0]; l.w[1] = st.w[1]; l.w[2] = st.w[2]; l.w[3] = st.w[3];
        return l;
    }
    // one MTF step: index of s (s must be in the list); zero-byte search per
    // word (the lowest flagged byte is exact), then bytes 0..k-1 move up one
    __device__ static uint32_t mtf(List& L, uint32_t s)
    {
        const uint64_t pat = (uint64_t)s * 0x0101010101010101ull;
        uint64_t z[4] = {0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < NW; ++j) {
            const uint64_t x = L.w[j] ^ pat;
            z[j] = (x - 0x0101010101010101ull) & ~x & 0x8080808080808080ull;
        }
        const uint32_t k = z[0] ? ((uint32_t)__builtin_ctzll(z[0]) >> 3)
                         : z[1] ? 8u + ((uint32_t)__builtin_ctzll(z[1]) >> 3)
                         : (NW == 3 || z[2]) ? 16u + ((uint32_t)__builtin_ctzll(z[2]) >> 3)
                                : 24u + ((uint32_t)__builtin_ctzll(z[3]) >> 3);
        const uint32_t jk = k >> 3, kb = k & 7u;
        const uint64_t m = kb == 7u ? ~0ull : ((1ull << (8u * kb + 8u)) - 1ull);   // bytes [0, kb]
        uint64_t carry = s;
#pragma unroll
        for (uint32_t j = 0; j < (uint32_t)NW; ++j) {
            const uint64_t nv = (L.w[j] << 8) | carry;
            carry = L.w[j] >> 56;
            L.w[j] = j < jk ? nv : (j == jk ? ((nv & m) | (L.w[j] & ~m)) : L.w[j]);
        }
        return k;
    }
};

template <class P>
struct MtfScr {
    uint64_t* base;
    uint32_t C;
    __device__ typename P::State* st() const { return reinterpret_cast<typename P::State*>(base); }
    __device__ typename P::List* l0() const { return reinterpret_cast<typename P::List*>(base + (uint64_t)P::SW * C); }
    __device__ RunSum* rs() const { return reinterpret_cast<RunSum*>(base + (uint64_t)(P::SW + P::LW) * C); }
    __device__ uint2* zo() const { return reinterpret_cast<uint2*>(base + (uint64_t)(P::SW + P::LW + 2) * C); }
    // the MTF indices of the whole block (P::IXB bits each, chunk c at c * cs symbols)
    __device__ uint8_t* ix() const { return reinterpret_cast<uint8_t*>(base + (uint64_t)(P::SW + P::LW + 3) * C); }
};

template <class P>
__device__ __forceinline__ MtfScr<P> mtf_scr(uint64_t* K, uint64_t kstride, uint32_t slot, uint32_t C)
{
    MtfScr<P> m;
    m.base = K + (uint64_t)slot * kstride;
    m.C = C;
    return m;
}

template <class P>
__device__ __forceinline__ bool mtf_mine(uint32_t nin) { return nin >= P::LO && nin <= P::HI; }

// visit symbols [a, e) of a chunk in order: 16-byte pieces, the next piece's
// load issued before the current one is processed (one load in flight, few
// registers: the per-symbol chains stay short-lived); the final partial
// piece is bounds-tested
template <class F>
__device__ __forceinline__ void visit_chunk(const uint8_t* ll, uint32_t a, uint32_t e, F&& f)
{
    const uint4* q = reinterpret_cast<const uint4*>(ll + a);
    const uint32_t np = (e - a + 15) / 16;
    uint4 cur = q[0];
#pragma unroll 1
    for (uint32_t i = 0; i < np; ++i) {
        const uint4 nxt = q[i + 1 < np ? i + 1 : i];
        const uint32_t lim = e - a - 16 * i;
        if (lim >= 16) {
            auto all = [&](int, uint32_t s) { f(s); };
            piece<true>(cur, 0, all);
        } else {
            auto some = [&](int k, uint32_t s) { if ((uint32_t)k < lim) f(s); };
            piece<true>(cur, 0, some);
        }
        cur = nxt;
    }
}

// the same, whole 128-byte lines at a time (eight loads in flight): faster
// for the emit pass, whose branchy per-symbol code keeps few values live
template <class F>
__device__ __forceinline__ void visit_chunk_lines(const uint8_t* ll, uint32_t a, uint32_t e, F&& f)
{
    const uint32_t full = a + ((e - a) & ~(LINE - 1));
#pragma unroll 1
    for (uint32_t j0 = a; j0 < full; j0 += LINE) visit_line<true>(ll + j0, [&](int, uint32_t s) { f(s); });
    if (full < e) {
        const uint32_t lim = e - full;
        visit_line<true>(ll + full, [&](int k, uint32_t s) { if ((uint32_t)k < lim) f(s); });
    }
}

template <class P>
__global__ void __launch_bounds__(MCT) k_mtf_local(const BlockDesc* __restrict__ blocks, uint32_t b0,
                                                   const uint8_t* __restrict__ LL, uint64_t ll_stride,
                                                   uint64_t* __restrict__ K, uint64_t kstride, uint32_t C, uint32_t cs)
{
    const uint32_t slot = blockIdx.y, b = b0 + slot;
    const uint32_t n = blocks[b].n, nin = blocks[b].n_in_use;
    const uint32_t ch = blockIdx.x * MCT + threadIdx.x;
    const uint32_t a = ch * cs;
    if (!mtf_mine<P>(nin) || a >= n) return;
    const uint32_t e = a + cs < n ? a + cs : n;
    const uint8_t* ll = LL + (uint64_t)slot * ll_stride;
    // local(c): the chunk's symbols by last occurrence, most recent first;
    // backward, line by line, until every symbol of the block has been seen
    typename P::State loc = P::empty();
    const uint32_t full = a + ((e - a) & ~(LINE - 1));
    auto add = [&](uint32_t s) { P::add(loc, s); };
    if (full < e) {
        const uint32_t lim = e - full;
        visit_line<false>(ll + full, [&](int k, uint32_t s) { if ((uint32_t)k < lim) add(s); });
    }
#pragma unroll 1
    for (uint32_t j0 = full; j0 > a && loc.cnt < nin;) {
        j0 -= LINE;
        visit_line<false>(ll + j0, [&](int, uint32_t s) { add(s); });
    }
    mtf_scr<P>(K, kstride, slot, C).st()[ch] = loc;
}

// start list of every chunk: exclusive scan of the local-list composition
template <class P>
__global__ void __launch_bounds__(MST) k_mtf_scan_lists(const BlockDesc* __restrict__ blocks, uint32_t b0,
                                                        uint64_t* __restrict__ K, uint64_t kstride, uint32_t C,
                                                        uint32_t cs)
{
    __shared__ typename P::State sh[MST];
    const int tid = threadIdx.x;
    const uint32_t slot = blockIdx.x, b = b0 + slot;
    const uint32_t n = blocks[b].n, nin = blocks[b].n_in_use;
    if (!mtf_mine<P>(nin)) return;
    const uint32_t nch = (n + cs - 1) / cs;
    const uint32_t per = (nch + MST - 1) / MST;          // <= 2 for 900 KB blocks at 512-symbol chunks
    const MtfScr<P> ms = mtf_scr<P>(K, kstride, slot, C);
    const uint32_t c0 = tid * per;
    typename P::State agg = P::empty();
    for (uint32_t q = 0; q < per; ++q)
        if (c0 + q < nch) agg = P::compose(agg, ms.st()[c0 + q]);
    sh[tid] = agg;
    __syncthreads();
    for (int d = 1; d < MST; d <<= 1) {                 // inclusive scan of the composition
        const typename P::State v = (tid >= d) ? P::compose(sh[tid - d], sh[tid]) : sh[tid];
        __syncthreads();
        sh[tid] = v;
        __syncthreads();
    }
    typename P::State st = P::identity(nin);
    if (tid) st = P::compose(st, sh[tid - 1]);
    for (uint32_t q = 0; q < per; ++q) {
        if (c0 + q >= nch) break;
        ms.l0()[c0 + q] = P::list_of(st);
        st = P::compose(st, ms.st()[c0 + q]);
    }
}

// MTF of each chunk: its indices, stored for k_mtf_emit (P::IXB bits each,
// one store per 16 symbols), and their zero-run summary (branch-free per symbol)
template <class P>
__global__ void __launch_bounds__(MCT) k_mtf_runs(const BlockDesc* __restrict__ blocks, uint32_t b0,
                                                  const uint8_t* __restrict__ LL, uint64_t ll_stride,
                                                  uint64_t* __restrict__ K, uint64_t kstride, uint32_t C, uint32_t cs)
{
    const uint32_t slot = blockIdx.y, b = b0 + slot;
    const uint32_t n = blocks[b].n, nin = blocks[b].n_in_use;
    const uint32_t ch = blockIdx.x * MCT + threadIdx.x;
    const uint32_t a = ch * cs;
    if (!mtf_mine<P>(nin) || a >= n) return;
    const uint32_t e = a + cs < n ? a + cs : n;
    const MtfScr<P> ms = mtf_scr<P>(K, kstride, slot, C);
    uint32_t z = 0, nz = 0, lz = 0, inner = 0;
    if constexpr (!P::SIX) {
        // An MTF index is 0 exactly when the symbol equals the one before it
        // (the list's front is the last symbol coded; the block's first symbol
        // meets the initial list, whose front is symbol 0), so the zero runs --
        // all the run summary needs -- come from comparing neighbours, without
        // the move-to-front chain (k_mtf_emit runs that once)
        const uint8_t* ll = LL + (uint64_t)slot * ll_stride;
        uint32_t prev = a ? ll[a - 1] : 0u;
        visit_chunk_lines(ll, a, e, [&](uint32_t s) {
            const uint32_t nzf = s != prev ? 1u : 0u;
            prev = s;
            inner += (nzf & nz) ? 1u + (31u - __clz(z + 1u)) : 0u;
            lz = (nzf & (nz ^ 1u)) ? z : lz;
            nz |= nzf;
            z = nzf ? 0u : z + 1u;
        });
        RunSum r;
        r.nz = nz;
        r.lz = nz ? lz : z;
        r.tz = nz ? z : 0u;
        r.inner = inner;
        ms.rs()[ch] = r;
        return;
    }
    typename P::List L = ms.l0()[ch];
    uint8_t* ixp = ms.ix() + (uint64_t)a * P::IXB / 8;     // 16 symbols = 8 (IXB 4) or 16 (IXB 8) bytes
    // indices enter at the top of a 64-bit (IXB 4) / 128-bit (IXB 8) shift
    // register; after 16 symbols the first sits in the lowest bits
    uint64_t lo = 0, hi = 0;
    uint32_t k16 = 0, piece_no = 0;
    visit_chunk(LL + (uint64_t)slot * ll_stride, a, e, [&](uint32_t s) {
        const uint32_t x = P::mtf(L, s);
        if constexpr (P::IXB == 4) {
            lo = (lo >> 4) | ((uint64_t)x << 60);
        } else {
            lo = (lo >> 8) | (hi << 56);
            hi = (hi >> 8) | ((uint64_t)x << 56);
        }
        if (P::SIX && ++k16 == 16) {
            if constexpr (P::IXB == 4) reinterpret_cast<uint64_t*>(ixp)[piece_no] = lo;
            else reinterpret_cast<uint4*>(ixp)[piece_no] = make_uint4((uint32_t)lo, (uint32_t)(lo >> 32),
                                                                      (uint32_t)hi, (uint32_t)(hi >> 32));
            k16 = 0;
            ++piece_no;
        }
        const uint32_t nzf = x != 0 ? 1u : 0u;
        inner += (nzf & nz) ? 1u + (31u - __clz(z + 1u)) : 0u;
        lz = (nzf & (nz ^ 1u)) ? z : lz;
        nz |= nzf;
        z = nzf ? 0u : z + 1u;
    });
    if (P::SIX && k16) {                                 // partial last piece: align its first symbol to bit 0
        const uint32_t sh = (16 - k16) * P::IXB;
        if constexpr (P::IXB == 4) {
            reinterpret_cast<uint64_t*>(ixp)[piece_no] = lo >> sh;
        } else {
            const uint64_t l2 = sh >= 64 ? hi >> (sh - 64) : ((lo >> sh) | (hi << (64 - sh)));
            const uint64_t h2 = sh >= 64 ? 0 : hi >> sh;
            reinterpret_cast<uint4*>(ixp)[piece_no] = make_uint4((uint32_t)l2, (uint32_t)(l2 >> 32), (uint32_t)h2,
                                                                 (uint32_t)(h2 >> 32));
        }
    }
    RunSum r;
    r.nz = nz;
    r.lz = nz ? lz : z;
    r.tz = nz ? z : 0u;
    r.inner = inner;
    ms.rs()[ch] = r;
}

// exclusive scan of the run summaries: zeros carried into each chunk and its
// first output index; the block's trailing run, EOB and n_mtf
template <class P>
__global__ void __launch_bounds__(MST) k_mtf_scan_runs(BlockDesc* __restrict__ blocks, uint32_t b0,
                                                       uint64_t* __restrict__ K, uint64_t kstride, uint32_t C,
                                                       uint32_t cs, uint16_t* __restrict__ mtfv_all, uint64_t mtf_stride)
{
    __shared__ RunSum sh[MST];
    const int tid = threadIdx.x;
    const uint32_t slot = blockIdx.x, b = b0 + slot;
    const uint32_t n = blocks[b].n, nin = blocks[b].n_in_use;
    if (!mtf_mine<P>(nin)) return;
    const uint32_t nch = (n + cs - 1) / cs;
    const uint32_t per = (nch + MST - 1) / MST;
    const MtfScr<P> ms = mtf_scr<P>(K, kstride, slot, C);
    const uint32_t c0 = tid * per;
    RunSum agg;
    agg.nz = 0; agg.lz = 0; agg.tz = 0; agg.inner = 0;
    for (uint32_t q = 0; q < per; ++q)
        if (c0 + q < nch) agg = run_compose(agg, ms.rs()[c0 + q]);
    sh[tid] = agg;
    __syncthreads();
    for (int d = 1; d < MST; d <<= 1) {
        const RunSum v = (tid >= d) ? run_compose(sh[tid - d], sh[tid]) : sh[tid];
        __syncthreads();
        sh[tid] = v;
        __syncthreads();
    }
    RunSum ex;
    ex.nz = 0; ex.lz = 0; ex.tz = 0; ex.inner = 0;
    if (tid) ex = sh[tid - 1];
    for (uint32_t q = 0; q < per; ++q) {
        if (c0 + q >= nch) break;
        const uint32_t zin = ex.nz ? ex.tz : ex.lz;
        const uint32_t obase = ex.nz ? nsym_run(ex.lz) + 1 + ex.inner : 0;
        ms.zo()[c0 + q] = make_uint2(zin, obase);
        ex = run_compose(ex, ms.rs()[c0 + q]);
    }
    if (tid == MST - 1) {
        const RunSum T = sh[MST - 1];
        uint8_t* mtfv = reinterpret_cast<uint8_t*>(mtfv_all + (uint64_t)b * mtf_stride);   // u8 values
        uint32_t z = T.nz ? T.tz : T.lz;
        uint32_t o = T.nz ? nsym_run(T.lz) + 1 + T.inner : 0;
        while (z) {
            const uint32_t d = ((z - 1) & 1u) ? 1u : 0u;
            mtfv[o++] = (uint8_t)d;
            z = (z - (d + 1)) >> 1;
        }
        mtfv[o++] = (uint8_t)(nin + 1);        // EOB
        blocks[b].n_mtf = o;
    }
}

// emit each chunk's RUNA/RUNB + symbols at its offset, from the MTF indices
// k_mtf_runs stored
template <class P>
__global__ void __launch_bounds__(MCT) k_mtf_emit(const BlockDesc* __restrict__ blocks, uint32_t b0,
                                                  const uint8_t* __restrict__ LL, uint64_t ll_stride,
                                                  const uint64_t* __restrict__ K, uint64_t kstride, uint32_t C,
                                                  uint32_t cs, uint16_t* __restrict__ mtfv_all, uint64_t mtf_stride)
{
    const uint32_t slot = blockIdx.y, b = b0 + slot;
    const uint32_t n = blocks[b].n, nin = blocks[b].n_in_use;
    const uint32_t ch = blockIdx.x * MCT + threadIdx.x;
    const uint32_t a = ch * cs;
    if (!mtf_mine<P>(nin) || a >= n) return;
    const uint32_t e = a + cs < n ? a + cs : n;
    const MtfScr<P> ms = mtf_scr<P>(const_cast<uint64_t*>(K), kstride, slot, C);
    const uint2 zo = ms.zo()[ch];
    Out8 out;
    out.init(reinterpret_cast<uint8_t*>(mtfv_all + (uint64_t)b * mtf_stride), zo.y);
    uint32_t z = zo.x;
    auto f = [&](uint32_t x) {
        if (x == 0) {
            ++z;
        } else {
            put_run(out, z);
            out.put(x + 1);
            z = 0;
        }
    };
    if constexpr (!P::SIX) {                           // re-run the MTF from the chunk's start list
        typename P::List L = ms.l0()[ch];
        visit_chunk_lines(LL + (uint64_t)slot * ll_stride, a, e, [&](uint32_t s) { f(P::mtf(L, s)); });
        out.flush();
        return;
    }
    // one 16-B piece (32 or 16 indices) at a time, the next piece's load in flight
    constexpr uint32_t SPP = 128 / P::IXB;             // symbols per 16-B piece
    const uint4* q = reinterpret_cast<const uint4*>(ms.ix() + (uint64_t)a * P::IXB / 8);
    const uint32_t cnt = e - a, np = (cnt + SPP - 1) / SPP;
    uint4 cur = q[0];
#pragma unroll 1
    for (uint32_t i = 0; i < np; ++i) {
        const uint4 nxt = q[i + 1 < np ? i + 1 : i];
        const uint32_t wv[4] = {cur.x, cur.y, cur.z, cur.w};
        const uint32_t lim = cnt - i * SPP;
        if (lim >= SPP) {
#pragma unroll
            for (uint32_t k = 0; k < SPP; ++k)
                f(P::IXB == 4 ? (wv[k >> 3] >> (4 * (k & 7))) & 15u : (wv[k >> 2] >> (8 * (k & 3))) & 255u);
        } else {
#pragma unroll
            for (uint32_t k = 0; k < SPP; ++k)
                if (k < lim) f(P::IXB == 4 ? (wv[k >> 3] >> (4 * (k & 7))) & 15u : (wv[k >> 2] >> (8 * (k & 3))) & 255u);
        }
        cur = nxt;
    }
    out.flush();
}

// ---- alphabets > 16: byte lists in LDS, 256 chunks; also produces mtfFreq ----
__global__ void __launch_bounds__(MT) k_mtf_big(BlockDesc* __restrict__ blocks, uint32_t b0,
                                                 const uint8_t* __restrict__ LL, uint64_t ll_stride,
                                                 uint8_t* __restrict__ scratch, uint64_t scratch_stride,
                                                 uint16_t* __restrict__ mtfv_all, uint64_t mtf_stride,
                                                 Tables* __restrict__ tabs)
{
    constexpr uint32_t C = NCH_BIG;
    constexpr int NF = 4;
    __shared__ RunSum cs_sh[C];
    __shared__ uint32_t freq[NF][258];
    __shared__ uint32_t scan_sh[MT / 64 + 1];
    __shared__ uint32_t tail[2];
    __shared__ uint8_t lst[256 * NCH_BIG];   // [pos][chunk]
    __shared__ uint32_t seen[NCH_BIG][8];
    __shared__ uint8_t st[256], st2[256], fl[256];
    __shared__ uint32_t lcnt[NCH_BIG];
    __shared__ uint32_t zin_sh[C], out_sh[C];

    const int tid = threadIdx.x;
    const uint32_t slot = blockIdx.x;
    const uint32_t b = b0 + slot;
    const uint32_t n = blocks[b].n;
    const uint32_t nin = blocks[b].n_in_use;
    if (nin <= ByteP<4>::HI) return;                 // <= 30 symbols: the register-list kernels
    for (int i = tid; i < NF * 258; i += MT) (&freq[0][0])[i] = 0;
    const uint8_t* ll = LL + (uint64_t)slot * ll_stride;
    uint8_t* idx = scratch + (uint64_t)slot * scratch_stride;            // MTF indices
    uint8_t* locl = idx + ((n + 255u) & ~255u);                          // per-chunk local lists
    uint8_t* sstate = locl + 256ull * C;                                 // per-chunk start states
    uint16_t* mtfv = mtfv_all + (uint64_t)b * mtf_stride;
    const uint32_t csz = (n + C - 1) / C;
    const uint32_t a = tid * csz;
    uint32_t e = a + csz;
    if (e > n) e = n;
    const bool mine = (uint32_t)tid < C && a < e;
    if (tid < NCH_BIG) for (int j = 0; j < 8; ++j) seen[tid][j] = 0;
    __syncthreads();
    if ((uint32_t)tid < C) {
        uint32_t cnt = 0;
        uint8_t* out = locl + (uint64_t)tid * 256;
        for (uint32_t j = e; j > a && a < e; --j) {
            uint32_t s = ll[j - 1];
            uint32_t bit = 1u << (s & 31);
            if (!(seen[tid][s >> 5] & bit)) { seen[tid][s >> 5] |= bit; out[cnt++] = (uint8_t)s; }
            if (cnt == nin) break;
        }
        lcnt[tid] = cnt;
    }
    if (tid < 256) { st[tid] = (uint8_t)tid; fl[tid] = 0; }
    __syncthreads();
    for (uint32_t c = 0; c < C; ++c) {   // list state at each chunk start (sequential)
        const uint32_t cnt = lcnt[c];
        const uint8_t* lc = locl + (uint64_t)c * 256;
        if (tid < (int)nin) sstate[(uint64_t)c * 256 + tid] = st[tid];
        if (tid < (int)cnt) fl[lc[tid]] = 1;
        __syncthreads();
        uint32_t keep = (tid < (int)nin && !fl[st[tid]]) ? 1u : 0u;
        uint32_t pre = block_excl_scan_add<uint32_t>(keep, scan_sh, (uint32_t*)nullptr);
        if (keep) st2[cnt + pre] = st[tid];
        if (tid < (int)cnt) st2[tid] = lc[tid];
        __syncthreads();
        if (tid < (int)nin) st[tid] = st2[tid];
        if (tid < (int)cnt) fl[lc[tid]] = 0;
        __syncthreads();
    }
    RunSum cs;
    cs.nz = 0; cs.lz = 0; cs.tz = 0; cs.inner = 0;
    if (mine) {
        for (uint32_t k = 0; k < nin; ++k) lst[k * NCH_BIG + tid] = sstate[(uint64_t)tid * 256 + k];
        uint32_t z = 0;
        for (uint32_t j = a; j < e; ++j) {
            uint8_t s = ll[j];
            uint8_t cur = lst[tid];
            uint32_t k = 0;
            if (cur != s) {   // bz:compress.c:197-211
                uint8_t carry_v = cur;
                k = 1;
                for (;;) {
                    uint8_t nxt = lst[k * NCH_BIG + tid];
                    lst[k * NCH_BIG + tid] = carry_v;
                    if (nxt == s || k >= 255) break;
                    carry_v = nxt;
                    ++k;
                }
                lst[tid] = s;
            }
            idx[j] = (uint8_t)k;
            if (k == 0) { ++z; continue; }
            if (!cs.nz) { cs.lz = z; cs.nz = 1; } else { cs.inner += 1 + nsym_run(z); }
            z = 0;
        }
        if (!cs.nz) cs.lz = z; else cs.tz = z;
    }
    if ((uint32_t)tid < C) cs_sh[tid] = cs;
    __syncthreads();
    if (tid == 0) {
        RunSum p;
        p.nz = 0; p.lz = 0; p.tz = 0; p.inner = 0;
        for (uint32_t c = 0; c < C; ++c) {
            zin_sh[c] = p.nz ? p.tz : p.lz;
            out_sh[c] = p.nz ? nsym_run(p.lz) + 1 + p.inner : 0;
            p = run_compose(p, cs_sh[c]);
        }
        tail[0] = p.nz ? p.tz : p.lz;
        tail[1] = p.nz ? nsym_run(p.lz) + 1 + p.inner : 0;
    }
    __syncthreads();
    const int wv = (tid >> 6) & (NF - 1);
    if (mine) {
        uint32_t o = out_sh[tid];
        uint32_t z = zin_sh[tid];
        for (uint32_t j = a; j < e; ++j) {
            const uint32_t v = idx[j];
            if (v == 0) { ++z; continue; }
            while (z) {
                uint32_t d = ((z - 1) & 1u) ? 1u : 0u;       // RUNB : RUNA
                mtfv[o++] = (uint16_t)d;
                atomicAdd(&freq[wv][d], 1u);
                z = (z - (d + 1)) >> 1;
            }
            mtfv[o++] = (uint16_t)(v + 1);
            atomicAdd(&freq[wv][v + 1], 1u);
        }
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t z = tail[0], o = tail[1];
        while (z) {
            uint32_t d = ((z - 1) & 1u) ? 1u : 0u;
            mtfv[o++] = (uint16_t)d;
            freq[0][d]++;
            z = (z - (d + 1)) >> 1;
        }
        mtfv[o++] = (uint16_t)(nin + 1);      // EOB
        freq[0][nin + 1]++;
        blocks[b].n_mtf = o;
    }
    __syncthreads();
    if (tid < 258) {
        uint32_t f = 0;
        for (int w = 0; w < NF; ++w) f += freq[w][tid];
        tabs[b].freq[tid] = f;
    }
}

// Last column L[j] = unseqToSeq[block[(SA[j] - 1) mod n]] (bz:compress.c:166-168) for the
// listed batch slots (which == nullptr: slots 0..nwhich-1).  The text gather is
// random within the block, so all tiles of a block run on one XCD (workgroup L
// -> slot L mod 8 inside groups of 8; round-robin XCD dealing) and small tiles
// keep ~2 blocks per XCD in flight: the 900 KB block text stays in that XCD's
// 4 MB L2 instead of costing an HBM line per byte.
constexpr uint32_t LC_PER = 16;                    // elements per lane, all loads in flight
constexpr uint32_t LC_TILE = 256 * LC_PER;

__global__ void __launch_bounds__(256) k_last_col(const BlockDesc* __restrict__ blocks, uint32_t b0,
                                                   const uint32_t* __restrict__ which, uint32_t nwhich,
                                                   uint32_t ntile, const uint8_t* __restrict__ blkbytes,
                                                   uint64_t stride, BwtScratch scr)
{
    __shared__ uint8_t seq[256];
    const uint32_t L = blockIdx.x;
    const uint32_t grp = L / (8u * ntile), r = L % (8u * ntile);
    const uint32_t k = grp * 8u + (r & 7u), tile = r >> 3;
    if (k >= nwhich) return;
    const uint32_t slot = which ? which[k] : k;
    const uint32_t b = b0 + slot;
    const uint32_t n = blocks[b].n;
    {                                                // makeMaps_e: unseqToSeq
        const uint32_t c = threadIdx.x;
        uint32_t below = __popc(blocks[b].in_use[c >> 5] & ((1u << (c & 31)) - 1u));
        for (uint32_t j = 0; j < (c >> 5); ++j) below += __popc(blocks[b].in_use[j]);
        seq[c] = (uint8_t)below;
    }
    __syncthreads();
    const uint8_t* blk = blkbytes + (uint64_t)b * stride;
    const uint64_t so = (uint64_t)slot * scr.stride;
    const uint32_t j = tile * LC_TILE + threadIdx.x * LC_PER;
    if (j >= n) return;
    if (j + LC_PER <= n) {
        const uint4* sp = reinterpret_cast<const uint4*>(scr.SA + so + j);
        const uint4 p0 = sp[0], p1 = sp[1], p2 = sp[2], p3 = sp[3];
        const uint32_t p[16] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w,
                                p2.x, p2.y, p2.z, p2.w, p3.x, p3.y, p3.z, p3.w};
        uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
        for (int t = 0; t < 16; ++t) w[t >> 2] |= (uint32_t)seq[blk[p[t] ? p[t] - 1 : n - 1]] << (8 * (t & 3));
        *reinterpret_cast<uint4*>(scr.LL + so + j) = make_uint4(w[0], w[1], w[2], w[3]);
    } else {
        for (uint32_t t = j; t < n; ++t) {
            const uint32_t pp = scr.SA[so + t];
            scr.LL[so + t] = seq[blk[pp ? pp - 1 : n - 1]];
        }
    }
}

void launch_last_col(const BlockDesc* blocks, uint32_t b0, const uint32_t* which, uint32_t nwhich,
                     const uint8_t* blkbytes, uint64_t stride, const BwtScratch& scr, hipStream_t st)
{
    if (!nwhich) return;
    const uint32_t ntile = (uint32_t)((scr.stride + LC_TILE - 1) / LC_TILE);
    const uint32_t grid = ntile * ((nwhich + 7) / 8 * 8);
    hipLaunchKernelGGL(k_last_col, dim3(grid), dim3(256), 0, st, blocks, b0, which, nwhich, ntile, blkbytes, stride,
                       scr);
    HIP_CHECK(hipGetLastError());
}

void launch_mtf(BlockDesc* blocks, uint32_t b0, uint32_t nb, const uint8_t* blkbytes, uint64_t stride,
                const BwtScratch& scr, uint16_t* mtfv, uint64_t mtf_stride, Tables* tabs, hipStream_t st,
                uint32_t need)
{
    (void)blkbytes;
    (void)stride;
    // alphabets <= 32: chunk passes over the key scratch (free after the sort)
    // chunk length: 512 symbols when the batch fills the GPU; a few blocks
    // take shorter chunks (more lanes, shorter serial MTF chains per lane)
    const uint32_t cs = nb >= 256 ? MCS : nb >= 64 ? 256u : nb >= 8 ? 128u : 64u;
    const uint32_t C = (uint32_t)((scr.stride + cs - 1) / cs);
    const uint64_t kstride = scr.stride;                     // u64 words per slot
    const dim3 gch((C + MCT - 1) / MCT, nb);
    auto run = [&](auto pol) {
        using P = decltype(pol);
        hipLaunchKernelGGL(k_mtf_local<P>, gch, dim3(MCT), 0, st, blocks, b0, scr.LL, scr.stride, scr.K, kstride, C, cs);
        hipLaunchKernelGGL(k_mtf_scan_lists<P>, dim3(nb), dim3(MST), 0, st, blocks, b0, scr.K, kstride, C, cs);
        hipLaunchKernelGGL(k_mtf_runs<P>, gch, dim3(MCT), 0, st, blocks, b0, scr.LL, scr.stride, scr.K, kstride, C,
                           cs);
        hipLaunchKernelGGL(k_mtf_scan_runs<P>, dim3(nb), dim3(MST), 0, st, blocks, b0, scr.K, kstride, C, cs, mtfv,
                           mtf_stride);
        hipLaunchKernelGGL(k_mtf_emit<P>, gch, dim3(MCT), 0, st, blocks, b0, scr.LL, scr.stride, scr.K, kstride, C,
                           cs, mtfv, mtf_stride);
    };
    // need (mtf_need): the alphabet classes present in the batch; the other
    // classes' kernels are not launched
    if (need & kMtfNib) run(NibP{});
    if (need & kMtfByte3) run(ByteP<3>{});
    if (need & kMtfByte4) run(ByteP<4>{});
    // large alphabets: index bytes + per-chunk lists in the (free) key scratch
    if (need & kMtfBig)
        hipLaunchKernelGGL(k_mtf_big, dim3(nb), dim3(MT), 0, st, blocks, b0, scr.LL, scr.stride,
                           reinterpret_cast<uint8_t*>(scr.K), scr.stride * sizeof(uint64_t), mtfv, mtf_stride, tabs);
    HIP_CHECK(hipGetLastError());
}

}  // namespace bz

// starch_amd/csrc/bz2_encoder.hip -- host orchestration of the GPU bzip2
// pipeline (the work bzip2's handle_compress / BZ2_compressBlock loop does
// serially, bz:bzlib.c:369-412, bz:compress.c:602-667).  All byte work runs
// in the kernels of bz2_rle / bz2_bwt / bz2_mtf / bz2_tables / bz2_emit; the
// host only sizes buffers, reads back per-stream / per-block counters and
// lays out offsets.
#include "bz2_bwt.hpp"

#include <string.h>

#include <algorithm>

namespace bz {

// stage timer: an event pair queued on the encoder, read by resolve_timers()
// after the caller's synchronisation (no host wait per stage)
struct EvTimer {
    hipEvent_t a = nullptr;
    hipStream_t st;
    std::vector<Encoder::PendTimer>* q;
    int stage;
    EvTimer(hipStream_t s, Stats* stats, std::vector<Encoder::PendTimer>* pq, int stg) : st(s), q(pq), stage(stg)
    {
        if (!stats) return;
        HIP_CHECK(hipEventCreate(&a));
        HIP_CHECK(hipEventRecord(a, st));
    }
    void stop()
    {
        if (!a) return;
        hipEvent_t b = nullptr;
        HIP_CHECK(hipEventCreate(&b));
        HIP_CHECK(hipEventRecord(b, st));
        q->push_back(Encoder::PendTimer{a, b, stage});
        a = nullptr;
    }
    ~EvTimer() { if (a) stop(); }
};

void Encoder::resolve_timers(Stats* stats)
{
    for (auto& t : pend_) {
        float ms = 0;
        if (stats) {
            HIP_CHECK(hipEventSynchronize(t.b));
            HIP_CHECK(hipEventElapsedTime(&ms, t.a, t.b));
            float* f[5] = {&stats->rle, &stats->bwt, &stats->mtf, &stats->tables, &stats->emit};
            *f[t.stage] += ms;
        }
        (void)hipEventDestroy(t.a);
        (void)hipEventDestroy(t.b);
    }
    pend_.clear();
}

void Encoder::take_intervals(hipEvent_t ref, std::vector<Interval>& out)
{
    for (auto& t : pend_) {
        float a = 0, b = 0;
        HIP_CHECK(hipEventSynchronize(t.b));
        HIP_CHECK(hipEventElapsedTime(&a, ref, t.a));
        HIP_CHECK(hipEventElapsedTime(&b, ref, t.b));
        out.push_back(Interval{t.stage, a, b});
        (void)hipEventDestroy(t.a);
        (void)hipEventDestroy(t.b);
    }
    pend_.clear();
}

void Encoder::release_device()
{
    for (DevBuf* b : {&b_streams, &b_tiles, &b_tile_sum, &b_tile_carry, &b_tile_w, &b_tile_wpre, &b_tile_block, &b_cut_tab, &b_seg_tile0, &b_seg_nblk, &b_blk_tmp, &b_blk, &b_blkbytes, &b_scal, &b_tmp, &b_bwt, &b_mtfv, &b_freq, &b_sel, &b_tabs, &b_gbits, &b_souts, &b_fallback, &b_bwt3, &b_crc, &b_dedupe, &b_rep_bytes, &b_rep_blk, &b_last})
        b->release();
}

static uint64_t round_up(uint64_t x, uint64_t m) { return (x + m - 1) / m * m; }

uint32_t* Encoder::PinnedCtr::get()
{
    if (!p) HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&p), 64 * sizeof(uint32_t), hipHostMallocDefault));
    return p;
}

Encoder::PinnedCtr::~PinnedCtr()
{
    if (p) (void)hipHostFree(p);
}

void Encoder::plan(const uint8_t* d_text, const std::vector<StreamIn>& streams, int bs100k, hipStream_t st,
                   std::vector<StreamOut>& outs, Stats* stats)
{
    if (bs100k < 1 || bs100k > 9) throw StarchError(-2, "blockSize100k must be 1..9");
    upload_crc_constants();
    resolve_timers(nullptr);
    text_ = d_text;
    bs100k_ = bs100k;
    streams_ = streams;
    nstreams_ = (uint32_t)streams.size();
    const uint32_t nblock_max = 100000u * (uint32_t)bs100k - 19u;     // bz:bzlib.c:194
    blk_stride_ = round_up(100000ull * bs100k + 64, 256);
    ngroups_ = 0;
    for (uint32_t s = 0; s < nstreams_; ++s) {
        if (streams[s].group < ngroups_ - (ngroups_ ? 1u : 0u) || streams[s].group > ngroups_)
            throw StarchError(-2, "stream pieces must be grouped consecutively");
        ngroups_ = std::max(ngroups_, streams[s].group + 1);
    }
    outs.assign(ngroups_, StreamOut());
    nblocks_ = 0;
    if (nstreams_ == 0) return;

    EvTimer t_rle(st, stats, &pend_, 0);
    StreamIn* d_streams = b_streams.as<StreamIn>(nstreams_);
    HIP_CHECK(hipMemcpyAsync(d_streams, streams.data(), nstreams_ * sizeof(StreamIn), hipMemcpyHostToDevice, st));
    std::vector<uint64_t> tile0(nstreams_ + 1, 0);
    uint64_t text_end = 0;
    for (uint32_t s = 0; s < nstreams_; ++s) {
        tile0[s + 1] = tile0[s] + ceil_div(streams[s].text_len, kTB);
        text_end = std::max(text_end, streams[s].text_off + streams[s].text_len);
    }
    const uint64_t ntiles = tile0[nstreams_];
    uint64_t* d_tile0 = b_seg_tile0.as<uint64_t>(nstreams_ + 1);
    HIP_CHECK(hipMemcpyAsync(d_tile0, tile0.data(), (nstreams_ + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, st));

    TileDesc* d_tiles = b_tiles.as<TileDesc>(ntiles + 1);
    TileSum* d_sums = b_tile_sum.as<TileSum>(ntiles + 1);
    uint32_t* d_carry = b_tile_carry.as<uint32_t>(ntiles + 1);
    uint32_t* d_tw = b_tile_w.as<uint32_t>(ntiles + 1);
    uint64_t* d_twpre = b_tile_wpre.as<uint64_t>(ntiles + 1);
    uint64_t* d_scal = b_scal.as<uint64_t>(nstreams_ + 16);
    HIP_CHECK(hipMemsetAsync(d_twpre, 0, (ntiles + 1) * sizeof(uint64_t), st));
    if (ntiles) {
        rle_tiles(d_tile0, d_streams, nstreams_, ntiles, d_tiles, st);
        rle_sum(d_text, d_tiles, ntiles, d_sums, st);
        rle_carry(d_tile0, nstreams_, d_sums, d_carry, d_tw, st);
        scan::excl_sum_u32_to_u64(d_tw, d_twpre, ntiles, d_twpre + ntiles, b_tmp, st);
    }
    // block-descriptor slots per stream from an upper bound on its RLE1 size
    // (<= 5/4 of its text: a 4-byte run emits 5), so no read-back is needed here
    std::vector<uint64_t> slot0(nstreams_ + 1, 0);
    for (uint32_t s = 0; s < nstreams_; ++s)
        slot0[s + 1] = slot0[s] + (streams[s].text_len + streams[s].text_len / 4 + 1) / nblock_max + 2;
    const uint64_t nb_max = slot0[nstreams_];
    if (nb_max > 0xFFFFFFFFull) throw StarchError(-2, "too many blocks");
    uint64_t* d_slot0 = b_seg_nblk.as<uint64_t>(2 * nstreams_ + 2);
    uint32_t* d_nblk = reinterpret_cast<uint32_t*>(d_slot0 + nstreams_ + 1);
    HIP_CHECK(hipMemcpyAsync(d_slot0, slot0.data(), (nstreams_ + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    BlockDesc* d_btmp = b_blk_tmp.as<BlockDesc>(nb_max + 1);
    uint64_t max_slots = 0;
    for (uint32_t s = 0; s < nstreams_; ++s) max_slots = std::max<uint64_t>(max_slots, slot0[s + 1] - slot0[s]);
    rle_cut(d_streams, d_tile0, d_twpre, d_text, d_carry, nstreams_, nblock_max, d_slot0, nb_max, max_slots,
            b_cut_tab.get(rle_cut_tab_bytes(nb_max)), d_btmp, d_nblk, st);
    // first block of every stream and the block count, on the device; the
    // block arrays are sized by the bound, the counts read back once below
    uint32_t* d_first = reinterpret_cast<uint32_t*>(b_souts.as<uint64_t>(nstreams_ + 2));
    uint32_t* d_nb = d_first + nstreams_;
    rle_block_first(d_nblk, nstreams_, d_first, d_nb, st);
    BlockDesc* d_blocks = b_blk.as<BlockDesc>(nb_max + 1);
    // tile -> block of its first byte
    uint32_t* d_tile_block = b_tile_block.as<uint32_t>(ntiles + 1);
    rle_compact(d_btmp, d_slot0, d_nblk, d_first, nstreams_, d_blocks, d_streams, d_tile0, d_tile_block, st);
    uint8_t* d_blkbytes = b_blkbytes.as<uint8_t>(nb_max * blk_stride_ + 64);
    if (ntiles) {
        rle_emit(d_text, d_tiles, ntiles, d_twpre, d_tile0, d_carry, d_streams, d_first, d_nblk, d_tile_block, d_blocks,
                 d_blkbytes, blk_stride_, st);
    }
    rle_crc(d_text, d_blocks, (uint32_t)nb_max, d_nb, b_crc.as<uint32_t>(nb_max * kCrcMaxChunks), st);
    HIP_CHECK(hipGetLastError());
    // one read-back: per-stream block counts, the total and every block's descriptor
    uint32_t* nblk = h_nblk_.as<uint32_t>(nstreams_ + 1);
    BlockDesc* hbp = h_blocks_.as<BlockDesc>(nb_max + 1);
    HIP_CHECK(hipMemcpyAsync(nblk, d_nblk, nstreams_ * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipMemcpyAsync(nblk + nstreams_, d_nb, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipMemcpyAsync(hbp, d_blocks, nb_max * sizeof(BlockDesc), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    t_rle.stop();
    uint32_t nb = 0;
    for (uint32_t s = 0; s < nstreams_; ++s) {
        if (streams[s].open && s + 1 != nstreams_) throw StarchError(-2, "only the last piece may be open");
        StreamOut& g = outs[streams[s].group];
        if (g.n_blocks == 0) g.first_block = nb;
        g.n_blocks += nblk[s];
        nb += nblk[s];
    }
    if (nb != nblk[nstreams_]) throw StarchError(-10, "block count mismatch");
    open_rest_ = 0;
    if (streams.back().open) {   // the open piece's last block waits for more text
        const StreamIn& o = streams.back();
        open_rest_ = o.text_off + o.text_len;
        if (nblk[nstreams_ - 1]) {
            open_rest_ = hbp[nb - 1].in_beg;
            --nb;
            --outs[o.group].n_blocks;
        }
    }
    nblocks_ = nb;
    if (stats) stats->n_blocks += nb;
    // frame of each output stream (whole stream: header + trailer, phase 0)
    for (uint32_t s = 0; s < nstreams_; ++s) {
        StreamOut& g = outs[streams[s].group];
        const bool first = s == 0 || streams[s - 1].group != streams[s].group;
        const bool last = s + 1 == nstreams_ || streams[s + 1].group != streams[s].group;
        if (first) {
            g.frame = (streams[s].cont ? 0u : 1u) | ((streams[s].phase & 7u) << 8);
            g.combined_crc = streams[s].comb_in;
        }
        if (last && !streams[s].open) g.frame |= 2u;
    }
    auto frame_bits = [](const StreamOut& o) {
        return (uint64_t)((o.frame >> 8) & 7u) + ((o.frame & 1u) ? 32u : 0u) + ((o.frame & 2u) ? 80u : 0u);
    };
    if (nb == 0) {
        for (uint32_t g = 0; g < ngroups_; ++g) {   // header + trailer (bz:compress.c:622-666)
            outs[g].block_bits = 0;
            outs[g].bytes = (frame_bits(outs[g]) + 7) / 8;
        }
        uint64_t off = 0;
        for (uint32_t g = 0; g < ngroups_; ++g) { outs[g].out_off = off; off += outs[g].bytes; }
        return;
    }

    // ---- exact block reuse (bz2_dedupe.hip) ------------------------------------
    // Group candidate duplicates by (nblock, blockCRC, inUse), confirm each with a
    // byte compare against its representative, and run the block sort, MTF and
    // tables once per distinct block.  STARCH_DEDUPE=0 disables it.
    std::vector<BlockDesc> hb(hbp, hbp + nb);
    const char* env_d = getenv("STARCH_DEDUPE");
    const bool dedupe_on = !(env_d && !strcmp(env_d, "0"));
    // STARCH_DEDUPE_KEY=n groups by nblock only (tests: forces byte-compare rejections)
    const char* env_k = getenv("STARCH_DEDUPE_KEY");
    const bool key_n_only = env_k && !strcmp(env_k, "n");
    std::vector<uint32_t> rep_of(nb);
    uint32_t ndup = 0;
    for (uint32_t b = 0; b < nb; ++b) rep_of[b] = b;
    if (dedupe_on && nb > 1) {
        std::vector<uint32_t> order(nb);
        for (uint32_t b = 0; b < nb; ++b) order[b] = b;
        auto key_less = [&](uint32_t x, uint32_t y) {
            const BlockDesc &a = hb[x], &c = hb[y];
            if (a.n != c.n) return a.n < c.n;
            if (!key_n_only) {
                if (a.crc != c.crc) return a.crc < c.crc;
                int m = memcmp(a.in_use, c.in_use, sizeof(a.in_use));
                if (m) return m < 0;
            }
            return x < y;
        };
        auto key_eq = [&](uint32_t x, uint32_t y) {
            const BlockDesc &a = hb[x], &c = hb[y];
            return a.n == c.n && (key_n_only || (a.crc == c.crc && !memcmp(a.in_use, c.in_use, sizeof(a.in_use))));
        };
        std::sort(order.begin(), order.end(), key_less);
        std::vector<uint32_t> pairs;
        for (uint32_t i = 1, r = order[0]; i < nb; ++i) {
            if (key_eq(order[i], r)) { pairs.push_back(order[i]); pairs.push_back(r); }
            else r = order[i];
        }
        const uint32_t npairs = (uint32_t)(pairs.size() / 2);
        if (npairs) {
            uint32_t* d_pairs = b_dedupe.as<uint32_t>(3ull * npairs + 2 * nb + 16);
            uint32_t* d_mis = d_pairs + 2ull * npairs;
            HIP_CHECK(hipMemcpyAsync(d_pairs, pairs.data(), pairs.size() * sizeof(uint32_t), hipMemcpyHostToDevice,
                                     st));
            launch_block_equal(d_blkbytes, blk_stride_, d_pairs, npairs, d_blocks, d_mis, st);
            std::vector<uint32_t> mis(npairs);
            HIP_CHECK(hipMemcpyAsync(mis.data(), d_mis, npairs * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
            HIP_CHECK(hipStreamSynchronize(st));
            for (uint32_t p = 0; p < npairs; ++p)
                if (!mis[p]) { rep_of[pairs[2 * p]] = pairs[2 * p + 1]; ++ndup; }
        }
    }
    // data index space: the distinct blocks, in block order
    const bool reuse = ndup > 0;
    std::vector<uint32_t> reps, src_of(nb);
    for (uint32_t b = 0; b < nb; ++b)
        if (rep_of[b] == b) { src_of[b] = (uint32_t)reps.size(); reps.push_back(b); }
    for (uint32_t b = 0; b < nb; ++b) src_of[b] = src_of[rep_of[b]];
    const uint32_t nr = (uint32_t)reps.size();
    BlockDesc* d_bl = d_blocks;              // blocks the sort / MTF / tables run over
    const uint8_t* d_bytes = d_blkbytes;
    src_of_dev_ = nullptr;
    src_of_host_.clear();
    if (reuse) {
        src_of_host_ = src_of;
        uint32_t* d_idx = b_dedupe.as<uint32_t>(2ull * nb + 16);
        HIP_CHECK(hipMemcpyAsync(d_idx, reps.data(), nr * sizeof(uint32_t), hipMemcpyHostToDevice, st));
        HIP_CHECK(hipMemcpyAsync(d_idx + nb, src_of.data(), nb * sizeof(uint32_t), hipMemcpyHostToDevice, st));
        src_of_dev_ = d_idx + nb;
        uint8_t* d_rbytes = b_rep_bytes.as<uint8_t>((uint64_t)nr * blk_stride_ + 64);
        launch_gather_blocks(d_blkbytes, blk_stride_, d_idx, nr, d_rbytes, st);
        std::vector<BlockDesc> hr(nr);
        for (uint32_t k = 0; k < nr; ++k) hr[k] = hb[reps[k]];
        d_bl = b_rep_blk.as<BlockDesc>(nr + 1);
        HIP_CHECK(hipMemcpyAsync(d_bl, hr.data(), nr * sizeof(BlockDesc), hipMemcpyHostToDevice, st));
        HIP_CHECK(hipStreamSynchronize(st));    // hr leaves scope
        d_bytes = d_rbytes;
        if (stats) stats->dedup_blocks += ndup;
    }

    // ---- per-batch: block sort, MTF, tables (over the distinct blocks) -------
    size_t free_b = 0, total_b = 0;
    const uint64_t mtf_stride = blk_stride_ + 16;
    uint16_t* d_mtfv = b_mtfv.as<uint16_t>((uint64_t)nr * mtf_stride);
    Tables* d_tabs = b_tabs.as<Tables>(nr);
    uint8_t* d_sel = b_sel.as<uint8_t>((uint64_t)nr * 2 * kMaxSelectors);
    // group sizes (one row per distinct block), then their prefixes (one row per block, emit)
    uint32_t* d_gbits = b_gbits.as<uint32_t>((uint64_t)(nr + nb) * kMaxSelectors);
    gpre_off_ = (uint64_t)nr * kMaxSelectors;
    HIP_CHECK(hipMemGetInfo(&free_b, &total_b));
    const bool kmat = bwt_kmat();
    const uint64_t per_slot = blk_stride_ * (kmat ? 59ull : 41ull);   // sort scratch + 1 B last column
    // (mem_share_: the part of the free HBM this encoder may take -- encoder
    // lanes planning at once all see the same free memory)
    uint64_t max_batch = std::max<uint64_t>(1, (uint64_t)(free_b * 0.45 * mem_share_) / per_slot);
#ifndef STARCH_BATCH_MAX
#define STARCH_BATCH_MAX 2048
#endif
    uint32_t batch = (uint32_t)std::min<uint64_t>({(uint64_t)nr, max_batch, (uint64_t)STARCH_BATCH_MAX});
    // STARCH_BWT_BATCH=k caps the batch (tests: exercises batches after the first)
    static const uint64_t batch_cap = [] { const char* e = getenv("STARCH_BWT_BATCH"); return e ? (uint64_t)atoll(e) : 0ull; }();
    if (batch_cap) batch = (uint32_t)std::min<uint64_t>(batch, batch_cap);
    if (b_bwt.cap < batch * per_slot) {
        // allocate the whole batch scratch once
        b_bwt.get(batch * per_slot + 4096);
    }
    BwtScratch scr;
    {
        uint8_t* base = static_cast<uint8_t*>(b_bwt.get(batch * per_slot + 4096));   // + tail pad for line reads
        uint64_t S = blk_stride_;
        scr.stride = S;
        scr.K = reinterpret_cast<uint64_t*>(base);
        scr.K2 = scr.K + S * batch;
        scr.V = reinterpret_cast<uint32_t*>(scr.K2 + S * batch);
        scr.V2 = scr.V + S * batch;
        scr.SA = scr.V2 + S * batch;
        scr.RK = scr.SA + S * batch;
        scr.U = scr.RK + S * batch;
        scr.U2 = scr.U + S * batch;
        if (kmat) {
            scr.KM0 = reinterpret_cast<uint64_t*>(scr.U2 + S * batch);
            scr.KM1 = scr.KM0 + S * batch;
            scr.LS0 = reinterpret_cast<uint8_t*>(scr.KM1 + S * batch);
            scr.LS1 = scr.LS0 + S * batch;
            scr.LL = scr.LS1 + S * batch;
        } else {
            scr.KM0 = scr.KM1 = nullptr;
            scr.LS0 = scr.LS1 = nullptr;
            scr.LL = reinterpret_cast<uint8_t*>(scr.U2 + S * batch);
        }
    }
    unsigned long long* d_stats = reinterpret_cast<unsigned long long*>(d_scal);
    HIP_CHECK(hipMemsetAsync(d_stats, 0, 4 * sizeof(uint64_t), st));
    BlockDesc* hr = h_hr_.as<BlockDesc>(nr);
    uint32_t* d_which = reinterpret_cast<uint32_t*>(b_fallback.as<uint32_t>(batch + 1));
    for (uint32_t b0 = 0; b0 < nr; b0 += batch) {
        uint32_t cnt = std::min(batch, nr - b0);
        uint32_t mtf_need = kMtfAll;
        {
            EvTimer tb(st, stats, &pend_, 1);
            // STARCH_BWT=lsd selects the one-workgroup-per-block prefix-doubling sort of
            // bz2_bwt.hip (kept as an independent implementation for cross-checks)
            static const bool lsd = [] { const char* e = getenv("STARCH_BWT"); return e && !strcmp(e, "lsd"); }();
            // blocks of 17..20 symbols take the 8192-bin mixed-radix top-level digit
            // (STARCH_WIDE=0: binary 12-bit digit everywhere; tests compare the two)
            static const bool wide_off = [] { const char* e = getenv("STARCH_WIDE"); return e && !strcmp(e, "0"); }();
            bool wide = false;
            mtf_need = 0;                  // alphabet classes of the batch (launch_mtf / launch_tables)
            for (uint32_t k = 0; k < cnt; ++k) {
                const BlockDesc& bd = hb[reuse ? reps[b0 + k] : b0 + k];
                uint32_t nin = 0;
                for (int j = 0; j < 8; ++j) nin += (uint32_t)__builtin_popcount(bd.in_use[j]);
                wide = wide || (!wide_off && nin >= 17 && nin <= 20);
                mtf_need |= mtf_class(nin);
            }
            bool doubled = true;
            if (lsd) launch_bwt(d_bl, b0, cnt, d_bytes, blk_stride_, scr, d_stats, st);
            else doubled = launch_bwt3(d_bl, b0, cnt, d_bytes, blk_stride_, scr, b_bwt3, h_ctr_.get(), d_stats, st, wide);
            std::vector<uint32_t> which, wn;
            if (doubled) {   // periodic blocks are found by the doubling rounds only
                HIP_CHECK(hipMemcpyAsync(hr + b0, d_bl + b0, cnt * sizeof(BlockDesc), hipMemcpyDeviceToHost, st));
                HIP_CHECK(hipStreamSynchronize(st));
                for (uint32_t k = 0; k < cnt; ++k)
                    if (hr[b0 + k].flags & 1u) { which.push_back(k); wn.push_back(hr[b0 + k].n); }
            }
            if (!which.empty()) {
                HIP_CHECK(hipMemcpyAsync(d_which, which.data(), which.size() * sizeof(uint32_t),
                                         hipMemcpyHostToDevice, st));
                launch_fallback(d_bl, b0, which.data(), wn.data(), (uint32_t)which.size(), d_bytes, blk_stride_, scr,
                                fb_pool_, st);
                if (stats) stats->periodic_blocks += which.size();
            }
            // the v3 sort writes the last column next to SA; the v1 sort and the
            // fallback (periodic blocks) leave it to the gather kernel
            if (lsd) launch_last_col(d_bl, b0, nullptr, cnt, d_bytes, blk_stride_, scr, st);
            else if (!which.empty())
                launch_last_col(d_bl, b0, d_which, (uint32_t)which.size(), d_bytes, blk_stride_, scr, st);
        }
        {
            EvTimer tm(st, stats, &pend_, 2);
            launch_mtf(d_bl, b0, cnt, d_bytes, blk_stride_, scr, d_mtfv, mtf_stride, d_tabs, st, mtf_need);
        }
        {
            EvTimer tt(st, stats, &pend_, 3);
            launch_tables(d_bl, b0, cnt, d_mtfv, mtf_stride, d_tabs, d_sel, d_gbits, scr, st, mtf_need);
        }
    }
    HIP_CHECK(hipMemcpyAsync(hr, d_bl, nr * sizeof(BlockDesc), hipMemcpyDeviceToHost, st));
    uint64_t* hstats = reinterpret_cast<uint64_t*>(h_wtot_.as<uint64_t>(std::max<uint64_t>(nstreams_, 4)));
    HIP_CHECK(hipMemcpyAsync(hstats, d_stats, 4 * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    // every block takes the sort / MTF / table results of its data block; its
    // position fields (text range, stream, RLE offset) stay its own
    if (!reuse) memcpy(hb.data(), hr, nb * sizeof(BlockDesc));
    else {
        for (uint32_t b = 0; b < nb; ++b) {
            BlockDesc o = hr[src_of[b]];
            o.in_beg = hb[b].in_beg;
            o.in_end = hb[b].in_end;
            o.w_beg = hb[b].w_beg;
            o.bit_off = hb[b].bit_off;
            o.stream = hb[b].stream;
            hb[b] = o;
        }
        HIP_CHECK(hipMemcpyAsync(d_blocks, hb.data(), nb * sizeof(BlockDesc), hipMemcpyHostToDevice, st));
        HIP_CHECK(hipStreamSynchronize(st));
    }
    if (stats) {
        stats->bwt_rounds += hstats[0];
        stats->bwt_tied += hstats[2];
        for (auto& b : hb) stats->rle_bytes += b.n;
    }
    // stream sizes: (phase) + 32 header bits + blocks + 80 trailer bits, padded to a byte
    uint64_t off = 0;
    for (uint32_t s = 0; s < ngroups_; ++s) {
        uint64_t bits = 0;
        for (uint32_t k = 0; k < outs[s].n_blocks; ++k) bits += hb[outs[s].first_block + k].bits;
        outs[s].block_bits = bits;
        bits += frame_bits(outs[s]);
        outs[s].bytes = (bits + 7) / 8;
        outs[s].out_off = off;
        off += outs[s].bytes;
    }
    host_blocks_.swap(hb);
}

void Encoder::emit(uint8_t* d_out, uint64_t out_cap, uint64_t out_base, std::vector<StreamOut>& outs,
                   hipStream_t st, Stats* stats)
{
    EvTimer te(st, stats, &pend_, 4);
    uint64_t total = 0;
    for (auto& o : outs) total = std::max(total, o.out_off + o.bytes);
    if (((uintptr_t)d_out & 3u) != 0) throw StarchError(-2, "output buffer must be 4-byte aligned");
    if (out_base + total + 4 > out_cap) throw StarchError(-3, "output buffer too small");
    if (total == 0) return;
    HIP_CHECK(hipMemsetAsync(d_out + out_base, 0, total, st));
    // absolute bit offsets of every block
    for (uint32_t s = 0; s < ngroups_; ++s) {
        uint64_t pos = (out_base + outs[s].out_off) * 8 + ((outs[s].frame >> 8) & 7u) + ((outs[s].frame & 1u) ? 32u : 0u);
        for (uint32_t k = 0; k < outs[s].n_blocks; ++k) {
            BlockDesc& b = host_blocks_[outs[s].first_block + k];
            b.bit_off = pos;
            pos += b.bits;
        }
    }
    BlockDesc* d_blocks = static_cast<BlockDesc*>(b_blk.p);
    if (nblocks_) {
        HIP_CHECK(hipMemcpyAsync(d_blocks, host_blocks_.data(), nblocks_ * sizeof(BlockDesc), hipMemcpyHostToDevice,
                                 st));
    }
    StreamOut* d_souts = b_souts.as<StreamOut>(ngroups_ + 1);
    HIP_CHECK(hipMemcpyAsync(d_souts, outs.data(), ngroups_ * sizeof(StreamOut), hipMemcpyHostToDevice, st));
    uint32_t* out32 = reinterpret_cast<uint32_t*>(d_out);
    const uint64_t mtf_stride = blk_stride_ + 16;
    uint32_t* gbits = static_cast<uint32_t*>(b_gbits.p);
    launch_emit_blocks(d_blocks, nblocks_, static_cast<uint16_t*>(b_mtfv.p), mtf_stride,
                       static_cast<Tables*>(b_tabs.p), static_cast<uint8_t*>(b_sel.p), gbits, gbits + gpre_off_,
                       src_of_dev_, out32, st);
    launch_stream_frame(d_souts, d_blocks, ngroups_, bs100k_, out_base, out32, st);
    for (uint32_t s = 0; s < ngroups_; ++s) {
        uint32_t comb = outs[s].combined_crc;      // the CRC entering the piece (0: a whole stream)
        for (uint32_t k = 0; k < outs[s].n_blocks; ++k) {
            uint32_t c = host_blocks_[outs[s].first_block + k].crc;
            comb = ((comb << 1) | (comb >> 31)) ^ c;
        }
        outs[s].combined_crc = comb;
    }
    te.stop();
}

uint32_t Encoder::last_write_bits(uint32_t g, const StreamOut& so, hipStream_t st)
{
    (void)g;
    if (so.n_blocks == 0) return 0;
    const uint32_t b = so.first_block + so.n_blocks - 1;
    const BlockDesc& bd = host_blocks_[b];
    const uint32_t src = src_of_host_.empty() ? b : src_of_host_[b];
    const uint8_t* d_sel = static_cast<const uint8_t*>(b_sel.p) + (uint64_t)src * 2 * kMaxSelectors + (bd.n_sel - 1);
    uint8_t t = 0, len = 0;
    HIP_CHECK(hipMemcpyAsync(&t, d_sel, 1, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    const Tables* tab = static_cast<const Tables*>(b_tabs.p) + src;
    HIP_CHECK(hipMemcpyAsync(&len, &tab->len[t][bd.n_in_use + 1], 1, hipMemcpyDeviceToHost, st));   // EOB = nInUse + 1
    HIP_CHECK(hipStreamSynchronize(st));
    return len;
}

// EOB code length of every block (bz:compress.c:580-593: the last symbol of
// the last group): its table is the last selector's
__global__ void k_last_bits(const BlockDesc* __restrict__ blocks, uint32_t nb, const uint8_t* __restrict__ sel,
                            const Tables* __restrict__ tabs, const uint32_t* __restrict__ src_of,
                            uint32_t* __restrict__ out)
{
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    const BlockDesc& bd = blocks[b];
    const uint32_t src = src_of ? src_of[b] : b;
    const uint32_t t = sel[(uint64_t)src * 2 * kMaxSelectors + (bd.n_sel - 1)];
    out[b] = tabs[src].len[t][bd.n_in_use + 1];
}

void Encoder::block_results(std::vector<BlockOut>& out, hipStream_t st)
{
    out.assign(nblocks_, BlockOut{});
    if (!nblocks_) return;
    uint32_t* d_last = b_last.as<uint32_t>(nblocks_ + 16);
    hipLaunchKernelGGL(k_last_bits, dim3((nblocks_ + 255) / 256), dim3(256), 0, st, static_cast<BlockDesc*>(b_blk.p),
                       nblocks_, static_cast<const uint8_t*>(b_sel.p), static_cast<const Tables*>(b_tabs.p),
                       src_of_dev_, d_last);
    HIP_CHECK(hipGetLastError());
    uint32_t* h = static_cast<uint32_t*>(h_last_.get((nblocks_ + 16) * sizeof(uint32_t)));
    HIP_CHECK(hipMemcpyAsync(h, d_last, nblocks_ * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    for (uint32_t b = 0; b < nblocks_; ++b) {
        const BlockDesc& bd = host_blocks_[b];
        out[b] = BlockOut{bd.in_beg, bd.in_end, bd.bit_off, bd.bits, bd.crc, h[b]};
    }
}

uint64_t Encoder::plan_and_encode(const uint8_t* d_text, const std::vector<StreamIn>& streams, int bs100k,
                                  uint8_t* d_out, uint64_t out_cap, uint64_t out_base, std::vector<StreamOut>& outs,
                                  hipStream_t st, Stats* stats)
{
    plan(d_text, streams, bs100k, st, outs, stats);
    emit(d_out, out_cap, out_base, outs, st, stats);
    HIP_CHECK(hipStreamSynchronize(st));
    resolve_timers(stats);
    uint64_t total = 0;
    for (auto& o : outs) total = std::max(total, o.out_off + o.bytes);
    return total;
}

}  // namespace bz

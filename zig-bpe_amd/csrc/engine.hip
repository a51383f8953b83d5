// Host orchestration of the MI355X BPE trainer: device buffers, the per-merge launch sequence,
// Zig-order tie resolution, compaction, encode. One Engine per process and GPU.
//
// Per merge (BasicTokenizer.expandVocabulary loop, basic_tokenizer.zig:183-204):
//   [argmax of the previous update is already on the host]
//   tie? -> zbpe_tie_occupy, zbpe_tie_resolve (+ exact emulation if undecided)
//   zbpe_scan_pairs | (compact, zbpe_self_tiles, zbpe_self_carry, zbpe_scan_self) for (a, a)
//   zbpe_replace (apply + count update), zbpe_select (argmax + resets) -> one D2H + sync
#include "engine.hpp"

#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include <hipcub/hipcub.hpp>

#include "kernels.hpp"
#include "zig_order.hpp"

namespace zbpe {

// Device allocations. ZBPE_POISON=1 (diagnostics) fills every new buffer with 0xA5 bytes, so that a read of
// memory no kernel wrote fails the same way on every run instead of depending on what the allocator hands back.
static hipError_t dev_alloc_raw(void **p, size_t bytes) {
    // (ZBPE_POISON=1: 0xA5 bytes, 2: 0xFF, 3: 0x01)
    static const int poison = getenv("ZBPE_POISON") ? atoi(getenv("ZBPE_POISON")) : 0;
    hipError_t e = hipMalloc(p, bytes);
    if (e == hipSuccess && poison) {
        e = hipMemset(*p, poison == 2 ? 0xFF : poison == 3 ? 0x01 : 0xA5, bytes);
        if (e == hipSuccess) e = hipDeviceSynchronize();
    }
    return e;
}
template <class T_>
static hipError_t dev_alloc(T_ **p, size_t bytes) {
    return dev_alloc_raw(reinterpret_cast<void **>(p), bytes);
}

#define HIP_OK(expr)                                                                       \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess) return fail(ZBPE_DEVICE_ERROR, "%s: %s (%s:%d)", #expr,     \
                                          hipGetErrorString(e_), __FILE__, __LINE__);      \
    } while (0)
#define LAUNCH_OK() HIP_OK(hipGetLastError())
#define CHECK(expr)                       \
    do {                                  \
        zbpe_status s_ = (expr);          \
        if (s_ != ZBPE_OK) return s_;     \
    } while (0)

static double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static inline uint64_t round_up(uint64_t x, uint64_t m) { return (x + m - 1) / m * m; }

zbpe_status Engine::fail(zbpe_status s, const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    err = buf;
    return s;
}

Engine::~Engine() { release(); }

void Engine::release() {
    auto f = [](void *p) { if (p) (void)hipFree(p); };
    f(d_text); f(d_tok[0]); f(d_tok[1]);
    f(T.ht); f(T.id_key); f(T.id_cnt); f(T.hpos); f(T.hcnt);
    f(d_delta); f(d_st); f(d_rec); f(d_partial); f(d_hist); f(d_bnd_mine); f(d_bnd_all); f(d_x0); f(d_shard_fn); f(d_fns_all);
    f(d_tile_cnt); f(d_tile_off); f(d_tile_fn); f(d_carry); f(d_bitmap); f(d_tie_list);
    f(d_first); f(d_gather); f(d_recount); f(T.hot); f(T.home_cnt); f(d_summ); f(d_count_hist); f(T.home_dirty); f(d_sup); f(d_pres); f(T.tok_cnt); f(d_log); f(d_halo); f(T.lst_off); f(T.lst_len); f(d_list_total); f(d_lists); f(d_list_cnt); f(d_cand); f(d_cs); f(d_rtk); f(d_sizes);
    f(d_enc_cnt); f(d_enc_ctr); f(d_nb); f(d_ord_pos); f(d_ord_ent); f(d_sort_tmp); f(d_rdelta); f(d_rlog);
    d_rdelta = d_rlog = nullptr;
    f(d_dir); f(d_dir_row); f(d_row_tok); f(d_dir_tmp); f(d_sort_hist);
    d_dir = d_dir_row = d_row_tok = d_sort_hist = nullptr; d_dir_tmp = nullptr;
    dir_cap = dir_row_cap = row_tok_cap = dir_tmp_cap = sort_hist_cap = 0;
    dirs_built = false;
    d_ord_pos = nullptr; d_ord_ent = nullptr; d_sort_tmp = nullptr; ord_pos_cap = ord_ent_cap = sort_tmp_cap = 0;
    if (h_ord) (void)hipHostFree(h_ord);
    h_ord = nullptr; h_ord_cap = 0;
    d_nb = nullptr; nb_cap = 0;
    d_enc_cnt = nullptr; d_enc_ctr = nullptr; enc_cnt_cap = enc_ctr_cap = 0;
    for (auto &e : bev) if (e) (void)hipEventDestroy(e);
    bev.clear();
    if (h_st) (void)hipHostFree(h_st);
    if (h_count_hist) (void)hipHostFree(h_count_hist);
    for (auto &e : ev) if (e) (void)hipEventDestroy(e);
    if (stream) (void)hipStreamDestroy(stream);
    d_text = nullptr; d_tok[0] = d_tok[1] = nullptr; T = Tables{};
    d_delta = nullptr; d_st = nullptr; d_rec = nullptr; d_partial = nullptr; d_hist = nullptr;
    d_bnd_mine = d_bnd_all = nullptr; d_x0 = nullptr; d_shard_fn = d_fns_all = nullptr;
    if (h_bnd) (void)hipHostFree(h_bnd);
    h_bnd = nullptr;
    comm.reset();
    d_tile_cnt = nullptr; d_tile_off = nullptr; d_tile_fn = d_carry = nullptr; d_bitmap = nullptr; d_cand = nullptr; d_cs = nullptr; d_rtk = nullptr; cs_cap = 0; d_sizes = nullptr; sizes_cap = 0;
    d_tie_list = nullptr; d_first = nullptr; d_gather = nullptr; d_recount = nullptr; h_st = nullptr; stream = nullptr;
    d_summ = nullptr; d_count_hist = nullptr; h_count_hist = nullptr; hot_cap_alloc = home_words_cap = 0; home_slots = 0;
    dirty_bits_cap = 0; d_sup = nullptr; sup_cap = 0; d_pres = nullptr; pres_cap = 0;
    for (auto &e : ev) e = nullptr;
}

zbpe_status Engine::init(int dev) {
    device = dev;
    int ndev = 0;
    HIP_OK(hipGetDeviceCount(&ndev));
    if (dev < 0 || dev >= ndev) return fail(ZBPE_INVALID_ARGUMENT, "device %d out of range (%d devices)", dev, ndev);
    HIP_OK(hipSetDevice(dev));
    HIP_OK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    HIP_OK(hipHostMalloc((void **)&h_st, sizeof(DevState), hipHostMallocDefault));
    HIP_OK(dev_alloc(&d_st, sizeof(DevState)));
    HIP_OK(dev_alloc(&d_delta, 2 * DELTA_WORDS * sizeof(uint32_t)));  // two: merges alternate (delta_of)
    HIP_OK(hipMemset(d_delta, 0, 2 * DELTA_WORDS * sizeof(uint32_t)));
    HIP_OK(dev_alloc(&d_rdelta, (size_t)ROUND_MAX * DELTA_WORDS * sizeof(uint32_t)));
    HIP_OK(hipMemset(d_rdelta, 0, (size_t)ROUND_MAX * DELTA_WORDS * sizeof(uint32_t)));
    HIP_OK(dev_alloc(&d_rlog, MAX_BATCH * sizeof(uint32_t)));
    h_rlog.resize(MAX_BATCH);
    HIP_OK(dev_alloc(&d_hist, 65536 * sizeof(uint32_t)));
    HIP_OK(dev_alloc(&T.tok_cnt, 65536 * sizeof(int32_t)));
    HIP_OK(dev_alloc(&d_log, 65536 * sizeof(MergeLog)));
    HIP_OK(dev_alloc(&T.lst_off, 65536 * sizeof(uint32_t)));
    HIP_OK(dev_alloc(&T.lst_len, 65536 * sizeof(uint32_t)));
    HIP_OK(dev_alloc(&d_list_total, 65536 * sizeof(uint32_t)));
    HIP_OK(hipFuncSetAttribute((const void *)zbpe_list_hist, hipFuncAttributeMaxDynamicSharedMemorySize, PRES_MAX_VP * 4));
    HIP_OK(hipFuncSetAttribute((const void *)zbpe_list_scatter, hipFuncAttributeMaxDynamicSharedMemorySize, PRES_MAX_VP * 4));
    HIP_OK(dev_alloc(&d_halo, sizeof(Halo)));
    h_log.resize(65536);
    bev.resize(BEV_PER_MERGE * MAX_BATCH + 2);  // per timed merge + the batch's first and last
    for (auto &e : bev) HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));  // timing only: no L2 writeback
    HIP_OK(dev_alloc(&d_partial, ARGMAX_MAX_BLOCKS * sizeof(MaxRec)));
    HIP_OK(dev_alloc(&d_cand, ((size_t)NEXT_MAX_SEL * (NEXT_CAND + 1) + 64) * sizeof(uint32_t)));  // keys | pkey | lastpair
    HIP_OK(dev_alloc(&d_rtk, RTK_WORDS * sizeof(uint32_t)));
    HIP_OK(dev_alloc(&d_count_hist, COUNT_BINS * sizeof(uint32_t)));
    HIP_OK(hipHostMalloc((void **)&h_count_hist, COUNT_BINS * sizeof(uint32_t), hipHostMallocDefault));
    for (auto &e : ev) HIP_OK(hipEventCreate(&e));
    // the initial byte-pair histogram keeps 128 KiB of bins in LDS
    HIP_OK(hipFuncSetAttribute((const void *)zbpe_count_byte_pairs, hipFuncAttributeMaxDynamicSharedMemorySize, 32768 * 4));
    HIP_OK(hipFuncSetAttribute((const void *)zbpe_pres_build, hipFuncAttributeMaxDynamicSharedMemorySize, PRES_MAX_VP * 4));
    HIP_OK(hipFuncSetAttribute((const void *)zbpe_pair_hist, hipFuncAttributeMaxDynamicSharedMemorySize, PH_SLOTS * 8));
    HIP_OK(hipFuncSetAttribute((const void *)zbpe_pair_hist_bytes, hipFuncAttributeMaxDynamicSharedMemorySize, 32768 * 4));
    CHECK(set_scan_variant(0));
    hipDeviceProp_t prop;
    HIP_OK(hipGetDeviceProperties(&prop, dev));
    num_cus = prop.multiProcessorCount;
    return ZBPE_OK;
}

template <typename T_>
zbpe_status Engine::ensure(T_ **p, size_t &cap, size_t need, const char *what) {
    if (*p && cap >= need) return ZBPE_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    size_t c = std::max(need, cap * 2);
    if (dev_alloc((void **)p, c * sizeof(T_)) != hipSuccess) {
        (void)hipGetLastError();
        *p = nullptr;
        cap = 0;
        return fail(ZBPE_OUT_OF_MEMORY, "device allocation of %zu x %zu B for %s failed", c, sizeof(T_), what);
    }
    cap = c;
    return ZBPE_OK;
}

// Stage this rank's shard [s, e) of the corpus in HBM (the whole corpus on one GPU or when
// shard == false). The first byte after the shard feeds the boundary pair of the initial histogram;
// the bytes around it are the initial halo.
zbpe_status Engine::upload(const uint8_t *text, size_t n, bool shard) {
    const size_t s = shard ? (size_t)((unsigned __int128)n * rank / world) : 0;
    const size_t e = shard ? (size_t)((unsigned __int128)n * (rank + 1) / world) : n;
    // positions are u32 within a shard (the occurrence arena, records, tiles); the corpus may exceed
    // 2^32 bytes when it is sharded over enough GPUs
    if (e - s >= (size_t)0xFFFFFFF0u)
        return fail(ZBPE_INVALID_ARGUMENT, "corpus shard of %zu bytes exceeds 2^32 tokens (shard it over more GPUs)", e - s);
    HIP_OK(hipSetDevice(device));
    CHECK(ensure(&d_text, text_cap, round_up(e - s + 64, 64), "corpus"));
    if (e > s) HIP_OK(hipMemcpyAsync(d_text, text + s, e - s, hipMemcpyHostToDevice, stream));
    HIP_OK(hipStreamSynchronize(stream));
    n_text = e - s;
    n_total = n;
    shard_offset = (uint64_t)s;
    next_byte = e < n && shard ? (int)text[e] : -1;
    Halo H = halo_empty();
    if (shard) {
        for (size_t i = s; i > 0 && H.nleft < 2; i--) halo_push_left(H, text[i - 1]);
        for (size_t i = e; i < n && H.nright < 3; i++) halo_push_right(H, text[i]);
    }
    halo0 = H;
    sharded = shard;
    uploaded = true;
    return ZBPE_OK;
}

zbpe_status Engine::init_dist(int r, int w, std::unique_ptr<Comm> c) {
    rank = r;
    world = w;
    comm = std::move(c);
    HIP_OK(hipSetDevice(device));
    HIP_OK(dev_alloc(&d_bnd_mine, sizeof(Boundary)));
    HIP_OK(dev_alloc(&d_bnd_all, (size_t)w * sizeof(Boundary)));
    HIP_OK(hipHostMalloc((void **)&h_bnd, (size_t)w * sizeof(Boundary), hipHostMallocDefault));
    HIP_OK(dev_alloc(&d_x0, 16));
    HIP_OK(dev_alloc(&d_shard_fn, 16));
    HIP_OK(dev_alloc(&d_fns_all, (size_t)w * 4 + 16));
    return ZBPE_OK;
}

zbpe_status Engine::sync_state() {
    HIP_OK(hipMemcpyAsync(h_st, d_st, sizeof(DevState), hipMemcpyDeviceToHost, stream));
    HIP_OK(hipStreamSynchronize(stream));
    if (h_st->error & 512u)
        return fail(ZBPE_INVALID_ARGUMENT, "a byte pair occurs 2^32 times or more in the corpus: pair counts are u32 on the device");
    if (h_st->error)
        return fail(ZBPE_INTERNAL, "device consistency check failed (flags 0x%x: 1 id overflow, 2 count underflow, 4 missing key, 8 record overflow, 16 home count range, 32 dirty list overflow, 64 occurrences != count, 128 tie collection, 1024 select wait timed out)%s",
                    h_st->error,
                    (h_st->error & 64u) ? (" [first 64: merge " + std::to_string(h_st->err_x) + " found " + std::to_string(h_st->err_occ) +
                                           " occurrences of (" + std::to_string(h_st->err_key & 0xFFFF) + "," + std::to_string(h_st->err_key >> 16) +
                                           ") counted " + std::to_string(h_st->err_cnt) + ", " + (h_st->err_mode ? "list" : "stream") +
                                           " scan" + (h_st->err_light ? ", a pair select" : "") + ", rank " + std::to_string(rank) + "]").c_str()
                                        : (h_st->error & 4u) ? (" [first 4: pair (" + std::to_string(h_st->err4_key & 0xFFFF) + "," +
                                                                 std::to_string(h_st->err4_key >> 16) + ") at site " +
                                                                 std::to_string(h_st->err4_site) + "]").c_str()
                                                              : "");
    return ZBPE_OK;
}

// tables sized for `need_ids`; rebuild keeps live ids only
zbpe_status Engine::alloc_tables(size_t id_cap_new) {
    size_t ht_cap_new = 1;
    while (ht_cap_new < 2 * id_cap_new || ht_cap_new < 64) ht_cap_new <<= 1;  // >= 8 buckets of 8
    Tables N{};
    N.hot = T.hot; N.hot_cap = T.hot_cap; N.hcnt = T.hcnt; N.home_cnt = T.home_cnt; N.home_mask = T.home_mask;
    N.home_dirty = T.home_dirty;
    N.tok_cnt = T.tok_cnt; N.lst_off = T.lst_off; N.lst_len = T.lst_len;
    N.id_cap = (uint32_t)id_cap_new;
    N.ht_mask = (uint32_t)(ht_cap_new - 1);
    if (dev_alloc(&N.ht, ht_cap_new * 8) != hipSuccess || dev_alloc(&N.id_key, id_cap_new * 4) != hipSuccess ||
        dev_alloc(&N.id_cnt, id_cap_new * 4) != hipSuccess || dev_alloc(&N.hpos, id_cap_new * 4) != hipSuccess) {
        (void)hipGetLastError();
        for (void *p : {(void *)N.ht, (void *)N.id_key, (void *)N.id_cnt, (void *)N.hpos}) if (p) (void)hipFree(p);
        return fail(ZBPE_OUT_OF_MEMORY, "pair table allocation (%zu ids) failed", id_cap_new);
    }
    HIP_OK(hipMemsetAsync(N.ht, 0xFF, ht_cap_new * 8, stream));
    HIP_OK(hipMemsetAsync(N.hpos, 0xFF, id_cap_new * 4, stream));  // no id listed (the hot list is rebuilt)
    if (T.id_key) {  // rebuild from the old tables
        uint32_t old_n = h_st->num_ids;
        HIP_OK(hipMemsetAsync(&d_st->num_ids, 0, 4, stream));
        zbpe_rebuild<<<std::min<uint32_t>(2048, (old_n + 255) / 256 + 1), 256, 0, stream>>>(T.id_key, T.id_cnt, old_n, N, d_st);
        LAUNCH_OK();
        HIP_OK(hipStreamSynchronize(stream));
        (void)hipFree(T.ht); (void)hipFree(T.id_key); (void)hipFree(T.id_cnt); (void)hipFree(T.hpos);
        stats_rebuilds++;
    }
    T = N;
    hot_stale = true;  // ids were renumbered
    return ZBPE_OK;
}

// room for the new ids of `k` merges starting at X (each adds at most 2X + 1 pairs), and a rebuild
// when dead ids dominate
zbpe_status Engine::maybe_grow_tables(uint32_t X, uint32_t k) {
    const uint64_t per = 2ull * (X + k) + 8;
    const uint64_t need = (uint64_t)h_st->num_ids + per * k;
    const uint64_t live = (uint64_t)std::max(h_st->live, 0);
    const uint64_t dead = h_st->num_ids - live;
    if (need <= T.id_cap && !(dead > std::max<uint64_t>(live, 1u << 20))) return ZBPE_OK;
    uint64_t cap = T.id_cap;
    while (live + per * k > cap / 2) cap *= 2;
    CHECK(alloc_tables(cap));
    return sync_state();
}

zbpe_status Engine::compact() {
    layout_gen++;
    const int64_t ntiles = (n_slots + COMPACT_TILE - 1) / COMPACT_TILE;
    if (ntiles == 0) return ZBPE_OK;
    CHECK(ensure(&d_tile_cnt, tile_cnt_cap, ntiles, "compaction tiles"));
    CHECK(ensure(&d_tile_off, tile_off_cap, ntiles + 1, "compaction offsets"));
    uint16_t *src = d_tok[cur], *dst = d_tok[cur ^ 1];
    zbpe_compact_count<<<ntiles, 256, 0, stream>>>(src, n_slots, d_tile_cnt);
    LAUNCH_OK();
    zbpe_scan_u32<<<1, 1024, 0, stream>>>(d_tile_cnt, ntiles, d_tile_off, d_tile_off + ntiles);
    LAUNCH_OK();
    zbpe_compact_scatter<<<ntiles, 256, 0, stream>>>(src, n_slots, d_tile_off, dst);
    LAUNCH_OK();
    const int64_t pad_end = (int64_t)round_up(n_live + 1, 64) + 64;
    zbpe_fill_u16<<<64, 256, 0, stream>>>(dst, n_live, pad_end, HOLE);
    LAUNCH_OK();
    cur ^= 1;
    n_slots = n_live;
    if (dist()) global_slots = global_live;  // every rank compacts together (holes_over)
    stats.compactions++;
    CHECK(build_presence());
    if (debug_checks) {
        uint64_t total = 0;
        HIP_OK(hipMemcpyAsync(&total, d_tile_off + ntiles, 8, hipMemcpyDeviceToHost, stream));
        HIP_OK(hipStreamSynchronize(stream));
        if ((int64_t)total != n_live) return fail(ZBPE_INTERNAL, "compaction kept %llu tokens, expected %lld",
                                                  (unsigned long long)total, (long long)n_live);
    }
    return ZBPE_OK;
}

// Compaction during training: positions move, so the occurrence lists are rebuilt (once they are
// on, or once pair counts have become small against the stream), else the arena is emptied.
// Hole-ratio compaction trigger. One GPU (and replicas): this stream's holes. Sharded: the holes of all
// shards from replicated totals, so every rank compacts at the same merge -- a compaction resets the
// arena fill (arena_rep) and may rebuild the lists, both of which gate halts and collectives
// (a rank-local trigger let one rank's arena_rep drift from the others').
bool Engine::holes_over() const {
    const uint64_t den = lists_on ? compact_den_lists : compact_den;
    // one GPU or replicas, once the merges only walk lists (the last batch did): holes cost the list walks little,
    // a compaction rebuilds the lists (~11 ms at C4) -- compact later (sharded: the ranks' scan forms may differ,
    // so the replicated rule above stays)
    if (!dist() && lists_on && list_streak) return (uint64_t)(n_slots - n_live) * compact_den_walks > (uint64_t)n_slots;
    if (!dist()) return (uint64_t)(n_slots - n_live) * den > (uint64_t)n_slots;
    return (global_slots - global_live) * den > global_slots;
}

zbpe_status Engine::compact_train(uint32_t X) {
    CHECK(sync_state());  // the arena fill logged is the device's now, whatever the caller last synced
    compact_log.push_back(X);
    compact_log.push_back(h_st->arena_rep);
    HIP_OK(hipEventRecord(ev[3], stream));
    CHECK(compact());
    // sharded: on replicated quantities (every rank compacts here, at the same merge)
    const uint64_t live_ref = dist() ? global_live : (uint64_t)n_live, ranks = dist() ? (uint64_t)world : 1;
    const bool want = list_mode && pres_vp <= PRES_MAX_VP && (uint64_t)n_slots < 0xF0000000ull &&
                      (lists_on || list_start == 0 || (uint64_t)h_st->top_count * list_start * ranks < live_ref);
    if (want && !(dist() && replicate_late)) {  // sharded: lists come with the replication (run_batch)
        CHECK(build_lists(X, list_ratio, true));
    } else {
        HIP_OK(hipMemsetAsync(&d_st->arena_top, 0, 4, stream));
        HIP_OK(hipMemsetAsync(&d_st->arena_rep, 0, 4, stream));
        HIP_OK(hipMemsetAsync(&d_st->lists_valid, 0, 4, stream));
    }
    HIP_OK(hipEventRecord(ev[4], stream));
    HIP_OK(hipEventSynchronize(ev[4]));
    float ms;
    HIP_OK(hipEventElapsedTime(&ms, ev[3], ev[4]));
    run.ev_replace += ms * 1e-3;
    return sync_state();
}

// Multi-GPU, late phase: gather the compacted shards into the whole stream on every rank (one
// all-gather of max-shard-sized pieces, padded with holes, then a compaction) and continue as
// replicas. The pair table is already identical on every rank, so from here each rank computes
// the same merges with no collective; the halo is empty and positions are global.
zbpe_status Engine::replicate() {
    layout_gen++;
    CHECK(ensure(&d_sizes, sizes_cap, 2 * (size_t)world + 2, "shard sizes"));
    const uint32_t mine = (uint32_t)n_live;
    HIP_OK(hipMemcpyAsync(d_sizes, &mine, 4, hipMemcpyHostToDevice, stream));
    if (!comm->allgather(d_sizes, d_sizes + world, 4, stream)) return fail(ZBPE_COMM_ERROR, "all-gather of shard sizes failed");
    std::vector<uint32_t> sz(world);
    HIP_OK(hipMemcpyAsync(sz.data(), d_sizes + world, 4 * (size_t)world, hipMemcpyDeviceToHost, stream));
    HIP_OK(hipStreamSynchronize(stream));
    uint64_t total = 0, M = 0;
    for (uint32_t v : sz) { total += v; M = std::max<uint64_t>(M, v); }
    M = round_up(std::max<uint64_t>(M, 1), 64);  // whole 16-B vectors per piece
    const size_t need = round_up((size_t)M * world + 1, 64) + 64;
    if (need > 0xFFFFFFF0u) return fail(ZBPE_INVALID_ARGUMENT, "replicated stream of %zu slots exceeds 2^32", need);
    // this rank's piece: its live tokens, then holes up to M (the shard buffer holds >= M + 64 slots)
    if ((size_t)M > std::min(tok_cap0, tok_cap1)) return fail(ZBPE_INTERNAL, "shard buffer smaller than the gather piece");
    zbpe_fill_u16<<<64, 256, 0, stream>>>(d_tok[cur], n_live, (int64_t)M, HOLE);
    LAUNCH_OK();
    uint16_t *full = nullptr;
    if (dev_alloc(&full, need * 2) != hipSuccess) { (void)hipGetLastError(); return fail(ZBPE_OUT_OF_MEMORY, "replicated stream (%zu slots)", need); }
    zbpe_fill_u16<<<256, 256, 0, stream>>>(full, 0, (int64_t)need, HOLE);
    LAUNCH_OK();
    if (!comm->allgather(d_tok[cur], full, (size_t)M * 2, stream)) { (void)hipFree(full); return fail(ZBPE_COMM_ERROR, "all-gather of the shards failed"); }
    // the gathered stream becomes the current buffer; the compaction target grows to match
    (void)hipFree(d_tok[cur]);
    d_tok[cur] = full;
    (cur == 0 ? tok_cap0 : tok_cap1) = need;
    CHECK(ensure(&d_tok[cur ^ 1], cur == 0 ? tok_cap1 : tok_cap0, need, "token stream (compaction buffer)"));
    replicated = true;
    n_slots = (int64_t)M * world;
    n_live = (int64_t)total;
    const long long lt = (long long)total;
    HIP_OK(hipMemcpyAsync(&d_st->live_tokens, &lt, sizeof(lt), hipMemcpyHostToDevice, stream));
    halo = halo_empty();
    shard_offset = 0;
    CHECK(compact());  // squeeze the padding: the stream is the whole corpus's, in shard order
    // the occurrence arena was sized for the shard: lists of the whole stream + later records
    // (its contents are rebuilt by build_lists right after)
    CHECK(ensure(&d_lists, lists_cap, std::min<size_t>(0xFFFFFFF0u, total + total / 2 + (16u << 20)), "occurrence arena"));
    stats.replications++;
    return ZBPE_OK;
}

// occurrence lists of the compacted stream (no holes): counting sort of positions by token
// a larger occurrence arena, keeping [0, arena_top) (the lists and this batch's records); sharded, the
// new limit follows from replicated values only
zbpe_status Engine::grow_arena(uint64_t need) {
    if (need > 0xFFFFFFF0u) return fail(ZBPE_OUT_OF_MEMORY, "occurrence arena of %llu entries exceeds 2^32", (unsigned long long)need);
    if (need > lists_cap) {
        uint32_t *grown = nullptr;
        if (dev_alloc(&grown, need * 4) != hipSuccess) {
            (void)hipGetLastError();
            return fail(ZBPE_OUT_OF_MEMORY, "occurrence arena (%llu entries)", (unsigned long long)need);
        }
        CHECK(sync_state());
        if (h_st->arena_top) HIP_OK(hipMemcpyAsync(grown, d_lists, (size_t)h_st->arena_top * 4, hipMemcpyDeviceToDevice, stream));
        HIP_OK(hipStreamSynchronize(stream));
        (void)hipFree(d_lists);
        d_lists = grown;
        lists_cap = need;
    }
    if (dist()) arena_cap_rep = std::max<uint64_t>(arena_cap_rep, need);
    return ZBPE_OK;
}

// max over the ranks of a u32 (an all-reduce(min) of its complement); the value itself on one GPU
zbpe_status Engine::max_over_ranks(uint32_t v, uint32_t *out) {
    if (!dist()) { *out = v; return ZBPE_OK; }
    uint32_t *d_w = d_delta + DELTA_WORDS - 8;  // scratch words past the delta layout
    const uint32_t c = ~v;
    HIP_OK(hipMemcpyAsync(d_w, &c, 4, hipMemcpyHostToDevice, stream));
    if (!comm->allreduce_u32(d_w, 1, COMM_MIN_U32, stream)) return fail(ZBPE_COMM_ERROR, "all-reduce(min) failed");
    uint32_t r = 0;
    HIP_OK(hipMemcpyAsync(&r, d_w, 4, hipMemcpyDeviceToHost, stream));
    HIP_OK(hipStreamSynchronize(stream));
    HIP_OK(hipMemsetAsync(d_w, 0, 4, stream));
    *out = ~r;
    return ZBPE_OK;
}

zbpe_status Engine::build_lists(uint32_t lists_x, uint32_t ratio, bool ranges) {
    layout_gen++;
    const int64_t n = n_slots;
    if (dist()) {  // (sharded, replicate_late off) the arena limit stays replicated: grown from the largest shard
        uint32_t nmax = 0;
        CHECK(max_over_ranks((uint32_t)n, &nmax));
        if ((uint64_t)nmax + (1u << 20) > arena_cap_rep) CHECK(grow_arena((uint64_t)nmax + (16u << 20)));
    } else if ((uint64_t)n + (1u << 20) > lists_cap) {
        CHECK(grow_arena((uint64_t)n + (16u << 20)));  // lists <= n entries
    }
    const uint32_t nchunks = (uint32_t)std::max<int64_t>(1, (n + LIST_CHUNK - 1) / LIST_CHUNK);
    CHECK(ensure(&d_list_cnt, list_cnt_cap, (size_t)nchunks * pres_vp, "list chunk histograms"));
    zbpe_list_hist<<<nchunks, LIST_THREADS, pres_vp * 4, stream>>>(d_tok[cur], n, pres_vp, d_list_cnt);
    LAUNCH_OK();
    zbpe_list_colscan<<<(pres_vp + 255) / 256, 256, 0, stream>>>(d_list_cnt, nchunks, pres_vp, d_list_total);
    LAUNCH_OK();
    const uint32_t max_len = (uint32_t)std::min<uint64_t>(0xFFFFFFFEu, (uint64_t)n / ratio);
    zbpe_list_offsets<<<1, 1024, 0, stream>>>(d_list_total, pres_vp, max_len, T.lst_off, T.lst_len, d_st, lists_x);
    LAUNCH_OK();
    // the build-time neighbours of every list entry (the filtered list walk). Sharded, the successor of the shard's
    // last token is the next shard's first live token (the halo): an occurrence across the edge is this shard's,
    // found from a's list; the predecessor of its first token stays HOLE (that occurrence is the left shard's)
    if (list_nb) {
        CHECK(ensure(&d_nb, nb_cap, (size_t)n + 64, "list neighbours"));
    }
    const uint32_t tail_succ = dist() && halo.nright > 0 ? halo_right(halo, 0) : (uint32_t)HOLE;
    zbpe_list_scatter<<<nchunks, LIST_THREADS, pres_vp * 4, stream>>>(d_tok[cur], n, pres_vp, d_list_cnt, T.lst_off,
                                                                       T.lst_len, d_lists, list_nb ? d_nb : nullptr, tail_succ);
    LAUNCH_OK();
    // successor ranges: training on one stream (a shard's edge entries have no successor in it)
    dirs_built = false;
    if (ranges && list_ranges && list_nb && (!dist() || replicated) && lists_x + 1 <= DIR_MAX_TOK && range_max_rows) {
        dir_w = lists_x + 2;
        CHECK(ensure(&d_dir_row, dir_row_cap, 65536, "list directory rows"));
        CHECK(ensure(&d_row_tok, row_tok_cap, 2 * (size_t)range_max_rows + 4, "list directory tokens"));
        CHECK(ensure(&d_dir, dir_cap, (size_t)range_max_rows * dir_w, "list directory"));
        CHECK(ensure(&d_dir_tmp, dir_tmp_cap, (size_t)n + 64, "list sort copy"));
        // chunks: at most one partial chunk per row beyond the entries' whole chunks; a row is a list of
        // >= range_min_len entries, so there are at most n / range_min_len of them
        const uint64_t rows_bound = std::min<uint64_t>(range_max_rows, (uint64_t)n / std::max<uint32_t>(range_min_len, 1) + 1);
        const uint64_t max_chunks = (uint64_t)n / SORT_CHUNK + rows_bound + 1;
        CHECK(ensure(&d_sort_hist, sort_hist_cap, (size_t)max_chunks * (lists_x + 1), "list sort chunk histograms"));
        uint32_t *row_ch0 = d_row_tok + range_max_rows, *rows = row_ch0 + range_max_rows + 1;
        zbpe_dir_rows<<<1, 1024, 0, stream>>>(T.lst_len, lists_x, range_min_len, range_max_len, range_max_rows, d_dir_row, d_row_tok,
                                              row_ch0, rows);
        LAUNCH_OK();
        zbpe_list_sort_hist<<<(unsigned)max_chunks, DIR_THREADS, 0, stream>>>(d_lists, d_nb, d_dir_tmp, T.lst_off, T.lst_len, rows, d_row_tok,
                                                                               row_ch0, lists_x, d_sort_hist);
        LAUNCH_OK();
        zbpe_list_sort_cols<<<dim3((lists_x + 1 + 255) / 256, std::min<uint32_t>(range_max_rows, 64)), 256, 0, stream>>>(d_sort_hist, rows, row_ch0, lists_x,
                                                                                                  d_dir, dir_w);
        LAUNCH_OK();
        zbpe_list_sort_row<<<std::min<uint32_t>(range_max_rows, 1024), DIR_THREADS, 0, stream>>>(T.lst_off, T.lst_len, rows, d_row_tok, lists_x, d_dir, dir_w);
        LAUNCH_OK();
        zbpe_list_sort_scatter<<<(unsigned)max_chunks, DIR_THREADS, 0, stream>>>(d_lists, d_nb, d_dir_tmp, T.lst_off, T.lst_len, rows,
                                                                                  d_row_tok, row_ch0, lists_x, d_sort_hist, d_dir, dir_w);
        LAUNCH_OK();
        dirs_built = true;
    }
    if (dist()) {  // arena_rep (the replicated fill that halts are decided on) >= every rank's arena_top
        CHECK(sync_state());
        uint32_t top_max = 0;
        CHECK(max_over_ranks(h_st->arena_top, &top_max));
        const uint32_t rep = std::max(top_max, h_st->arena_rep);
        HIP_OK(hipMemcpyAsync(&d_st->arena_rep, &rep, 4, hipMemcpyHostToDevice, stream));
    }
    lists_on = true;
    nb_built = list_nb;
    pres_on = false;  // block skipping is not maintained once scans can bypass the stream
    stats.list_builds++;
    return ZBPE_OK;
}

// list scans may filter list entries by their build-time neighbours (kernels.hpp scan_dispatch)
void Engine::set_list_nb(ScanArgs &A) const {
    A.nb = lists_on && nb_built ? d_nb : nullptr;
    A.dir_row = lists_on && dirs_built && A.nb && A.count_deltas ? d_dir_row : nullptr;
    A.dir = d_dir;
    A.dir_w = dir_w;
}

static uint32_t count_bin_lo(int b) {
    if (b < 64) return (uint32_t)b;
    const int e = (b - 64) / 32 + 6, m = (b - 64) % 32;
    return (uint32_t)(32 + m) << (e - 5);
}

// Hot list rebuild: choose theta so that about hot_target live ids have count >= theta.
zbpe_status Engine::rebuild_hot() {
    const uint32_t nid = h_st->num_ids;
    HIP_OK(hipMemsetAsync(d_count_hist, 0, COUNT_BINS * 4, stream));
    zbpe_count_hist<<<std::min<uint32_t>(2048, nid / 256 + 1), 256, 0, stream>>>(T, d_st, d_count_hist);
    LAUNCH_OK();
    HIP_OK(hipMemcpyAsync(h_count_hist, d_count_hist, COUNT_BINS * 4, hipMemcpyDeviceToHost, stream));
    HIP_OK(hipStreamSynchronize(stream));
    uint64_t cum = 0;
    uint32_t theta = 1;
    for (int b = COUNT_BINS - 1; b >= 1; b--) {
        const uint64_t h = h_count_hist[b];
        if (!h) continue;
        if (cum > 0 && cum + h > hot_target) break;
        cum += h;
        theta = count_bin_lo(b);
    }
    const size_t need = std::max<size_t>(4 * hot_target, 2 * cum + 4096);
    if (T.hot) {  // the current list's ids unlisted (Tables::hpos) before the list is rebuilt
        zbpe_hot_clear<<<64, 256, 0, stream>>>(T, d_st);
        LAUNCH_OK();
    }
    if (!T.hot || hot_cap_alloc < need) {
        if (T.hot) (void)hipFree(T.hot);
        if (T.hcnt) (void)hipFree(T.hcnt);
        T.hot = nullptr;
        T.hcnt = nullptr;
        if (dev_alloc(&T.hot, need * 8) != hipSuccess || dev_alloc(&T.hcnt, need * 4) != hipSuccess) {
            (void)hipGetLastError();
            hot_cap_alloc = 0;
            return fail(ZBPE_OUT_OF_MEMORY, "hot list allocation (%zu ids) failed", need);
        }
        hot_cap_alloc = need;
    }
    T.hot_cap = (uint32_t)hot_cap_alloc;
    uint32_t th[2] = {theta, 0};  // DevState.theta, DevState.hot_len
    HIP_OK(hipMemcpyAsync(&d_st->theta, th, 8, hipMemcpyHostToDevice, stream));
    zbpe_hot_build<<<std::min<uint32_t>(2048, nid / 256 + 1), 256, 0, stream>>>(T, d_st);
    LAUNCH_OK();
    HIP_OK(hipStreamSynchronize(stream));
    hot_stale = false;
    hot_rebuilds++;
    return ZBPE_OK;
}

int Engine::argmax_blocks(uint32_t X) const {
    const uint64_t work = std::max<uint64_t>(T.hot_cap / 4, X);
    const int blocks = (int)std::min<uint64_t>(ARGMAX_MAX_BLOCKS, (work + ARGMAX_THREADS - 1) / ARGMAX_THREADS);
    return std::max(blocks, 1);
}

zbpe_status Engine::launch_argmax(uint32_t X, int roll) {
    if (hot_stale) CHECK(rebuild_hot());
    const int blocks = argmax_blocks(X);
    zbpe_select<<<blocks, ARGMAX_THREADS, 0, stream>>>(T, d_st, d_partial, d_tok[cur], n_slots, delta_of(X), X, roll, d_bnd_all,
                                                       dist() ? world : 1);
    LAUNCH_OK();
    return ZBPE_OK;
}

// After an argmax + sync: if the hot list overflowed or no listed id still reaches theta, the
// result is not the global max: rebuild the list (lower theta) and select again.
zbpe_status Engine::select_ready() {
    for (int tries = 0; tries < 4; tries++) {
        const bool overflow = h_st->hot_len > T.hot_cap;
        const bool exhausted = h_st->live > 0 && h_st->top_count == 0;
        if (!overflow && !exhausted) {
            if (debug_checks) {  // cross-check the hot list against a full argmax over every id
                DevState *dbg = nullptr;
                HIP_OK(dev_alloc(&dbg, sizeof(DevState)));
                HIP_OK(hipMemcpyAsync(dbg, d_st, sizeof(DevState), hipMemcpyDeviceToDevice, stream));
                const uint32_t nid = h_st->num_ids;
                const int blocks = (int)std::min<uint64_t>(ARGMAX_MAX_BLOCKS, nid / (4 * ARGMAX_THREADS) + 1);
                zbpe_argmax_partial<<<blocks, ARGMAX_THREADS, 0, stream>>>(T.id_cnt, T.id_cap, dbg, d_partial);
                zbpe_argmax_final<<<1, 256, 0, stream>>>(d_partial, blocks, T, d_tok[cur], n_slots, dbg);
                DevState h{};
                HIP_OK(hipMemcpyAsync(&h, dbg, sizeof(DevState), hipMemcpyDeviceToHost, stream));
                HIP_OK(hipStreamSynchronize(stream));
                (void)hipFree(dbg);
                if (h.top_count != h_st->top_count || h.tie_count != h_st->tie_count)
                    return fail(ZBPE_INTERNAL, "hot-list argmax (%u x%u) != full argmax (%u x%u)", h_st->top_count,
                                h_st->tie_count, h.top_count, h.tie_count);
            }
            return ZBPE_OK;
        }
        hot_stale = true;
        CHECK(launch_argmax(0, 0));
        CHECK(sync_state());
    }
    return fail(ZBPE_INTERNAL, "hot list rebuild did not converge (live %d, hot_len %u, theta %u)", h_st->live, h_st->hot_len,
                h_st->theta);
}

zbpe_status Engine::rebuild_home(uint64_t cap) {
    // whole 4096-slot blocks (the tie kernels read a block's slots as 16-B vectors)
    const auto words_for = [](uint64_t c) { return (std::max<uint64_t>(c, SUMM_SLOTS) + SUMM_SLOTS - 1) / SUMM_SLOTS * (SUMM_SLOTS / 4); };
    const size_t words = words_for(cap);
    if (!T.home_cnt || home_words_cap < words) {
        if (T.home_cnt) (void)hipFree(T.home_cnt);
        T.home_cnt = nullptr;
        // room for two more doublings: a capacity step halts the batch, and a free + allocation took most of
        // its host path (~4 ms each at C4 merges 500-2000, profiles/r05_c4_merge_timeline.json)
        const size_t alloc = words_for(std::min<uint64_t>(cap * 4, 1ull << 31));
        if (dev_alloc(&T.home_cnt, alloc * 4) != hipSuccess) {
            (void)hipGetLastError();
            home_words_cap = 0;
            home_slots = 0;
            return fail(ZBPE_OUT_OF_MEMORY, "home histogram allocation (%llu slots) failed", (unsigned long long)cap);
        }
        home_words_cap = alloc;
    }
    const size_t nb = (cap + SUMM_SLOTS - 1) / SUMM_SLOTS, nsb = (nb + SUPER_BLOCKS - 1) / SUPER_BLOCKS;
    if (summ_cap < nb) CHECK(ensure(&d_summ, summ_cap, 4 * nb, "home summaries"));  // (headroom as above)
    if (sup_cap < nsb) CHECK(ensure(&d_sup, sup_cap, 4 * nsb, "home super-block summaries"));
    if (dirty_bits_cap < 2 * nsb) CHECK(ensure(&T.home_dirty, dirty_bits_cap, 8 * nsb, "home dirty bits"));
    HIP_OK(hipMemsetAsync(T.home_cnt, 0, words * 4, stream));
    HIP_OK(hipMemsetAsync(T.home_dirty, 0, 2 * nsb * 4, stream));
    T.home_mask = (uint32_t)(cap - 1);
    const uint32_t nid = h_st->num_ids;
    zbpe_home_build<<<std::min<uint32_t>(4096, nid / 256 + 1), 256, 0, stream>>>(T, d_st);
    LAUNCH_OK();
    HIP_OK(hipMemsetAsync(T.home_dirty, 0, 2 * nsb * 4, stream));
    zbpe_home_summary<<<(unsigned)std::min<size_t>(nb, 4096), 256, 0, stream>>>(T, d_st, (uint32_t)cap, (uint32_t)nb, d_summ);
    LAUNCH_OK();
    zbpe_super_summary<<<(unsigned)(nsb + 3) / 4, 256, 0, stream>>>(d_summ, (uint32_t)nb, d_sup, d_st, 0);
    LAUNCH_OK();
    home_slots = cap;
    home_rebuilds++;
    return ZBPE_OK;
}

// Zig-order winner among the pairs sharing the top count
zbpe_status Engine::resolve_tie(uint32_t top, uint32_t ties, uint32_t *winner) {
    stats.tie_iterations++;
    const uint64_t D = (uint64_t)h_st->live;
    const bool call_after = h_st->lastpair_count >= 2;
    const uint64_t cap = zig_final_capacity(D, call_after);
    if (cap > (1ull << 31)) return fail(ZBPE_INTERNAL, "Zig map capacity %llu out of range", (unsigned long long)cap);
    if (cap != home_slots) CHECK(rebuild_home(cap));
    CHECK(ensure(&d_tie_list, tie_list_cap, ties, "tie list"));
    HIP_OK(hipMemsetAsync(&d_st->tie_len, 0, 4, stream));
    const uint32_t hl = std::min<uint32_t>(h_st->hot_len, T.hot_cap);
    zbpe_tie_collect<<<std::min<uint32_t>(1024, hl / 256 + 1), 256, 0, stream>>>(T, d_st, top, (uint32_t)(cap - 1), d_tie_list,
                                                                                  (uint32_t)tie_list_cap, 0, BeginArgs{});
    LAUNCH_OK();
    const uint32_t nb = (uint32_t)((cap + SUMM_SLOTS - 1) / SUMM_SLOTS), nsb = (nb + SUPER_BLOCKS - 1) / SUPER_BLOCKS;
    zbpe_home_refresh<<<nsb, REFRESH_THREADS, 0, stream>>>(T, d_st, (uint32_t)cap, nb, d_summ, d_sup, 0);
    LAUNCH_OK();
    HomeView V{T.home_cnt, d_summ, d_sup, (uint32_t)cap, nb, nsb};
    zbpe_tie_decide<<<1, DECIDE_THREADS, 0, stream>>>(d_st, d_tie_list, (uint32_t)tie_list_cap, V, d_log, 0);
    LAUNCH_OK();
    CHECK(sync_state());
    if (h_st->tie_len != ties)
        return fail(ZBPE_INTERNAL, "tie collection found %u pairs at count %u, argmax said %u", h_st->tie_len, top, ties);
    if (h_st->tie_verdict == 0 && !exact_now) {
        *winner = h_st->tie_winner;
        return ZBPE_OK;
    }
    const uint32_t nid = h_st->num_ids;
    // exact emulation from first-occurrence order
    stats.tie_fallbacks++;
    CHECK(ensure(&d_first, first_cap, nid, "first occurrences"));
    HIP_OK(hipMemsetAsync(d_first, 0xFF, (size_t)nid * 4, stream));
    const double tp0 = now_s();
    HIP_OK(hipMemsetAsync(&d_st->gather_len, 0, 4, stream));
    {
        ScanArgs A{d_tok[cur], n_slots, 0, 0, nullptr, nullptr, d_st, nullptr, 0, 0, nullptr, nullptr, halo};
        zbpe_first_occ<<<2048, 256, 0, stream>>>(A, T, d_first, d_st);  // shard-local positions
        LAUNCH_OK();
    }
    if (!dist()) {
        // one GPU: sort the live pairs by first occurrence on the device (positions are unique per pair),
        // copy the ordered emulation entries to pinned host memory, replay the Zig map on the host
        CHECK(ensure(&d_ord_pos, ord_pos_cap, 2 * (size_t)D + 2, "tie emulation positions"));
        CHECK(ensure(&d_ord_ent, ord_ent_cap, 2 * (size_t)D + 2, "tie emulation entries"));
        uint32_t *pos_in = d_ord_pos, *pos_out = d_ord_pos + D + 1;
        unsigned long long *ent_in = d_ord_ent, *ent_out = d_ord_ent + D + 1;
        zbpe_gather_order<<<std::min<uint32_t>(4096, nid / 256 + 1), 256, 0, stream>>>(T, d_first, d_st, top, pos_in, ent_in,
                                                                                        (uint32_t)(D + 1));
        LAUNCH_OK();
        CHECK(sync_state());
        const double tp1 = now_s();
        const uint32_t g = h_st->gather_len;
        if (g != D) return fail(ZBPE_INTERNAL, "gathered %u live pairs, expected %llu", g, (unsigned long long)D);
        int end_bit = 1;
        while (end_bit < 32 && ((uint64_t)n_slots >> end_bit)) end_bit++;
        size_t tmp_bytes = 0;
        HIP_OK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, pos_in, pos_out, ent_in, ent_out, (int)g, 0, end_bit, stream));
        CHECK(ensure(&d_sort_tmp, sort_tmp_cap, tmp_bytes + 16, "tie emulation sort scratch"));
        HIP_OK(hipcub::DeviceRadixSort::SortPairs(d_sort_tmp, tmp_bytes, pos_in, pos_out, ent_in, ent_out, (int)g, 0, end_bit, stream));
        if (h_ord_cap < g) {
            if (h_ord) (void)hipHostFree(h_ord);
            h_ord = nullptr;
            h_ord_cap = 0;
            HIP_OK(hipHostMalloc((void **)&h_ord, (size_t)g * 8 + 8, hipHostMallocDefault));
            h_ord_cap = g;
        }
        HIP_OK(hipMemcpyAsync(h_ord, ent_out, (size_t)g * 8, hipMemcpyDeviceToHost, stream));
        HIP_OK(hipStreamSynchronize(stream));
        const double tp2 = now_s();
        if (!zig_emulate_first_tied(h_ord, g, call_after, winner, emu_work))
            return fail(ZBPE_INTERNAL, "exact tie emulation found no pair with count %u", top);
        if (tie_prof)
            fprintf(stderr, "tie_prof: %u live pairs, %u tied: first occurrences + gather %.1f ms, sort + copy %.1f ms, "
                            "host emulation %.1f ms\n", g, ties, (tp1 - tp0) * 1e3, (tp2 - tp1) * 1e3, (now_s() - tp2) * 1e3);
    } else {
    CHECK(ensure(&d_gather, gather_cap, (size_t)D, "live pairs"));
    zbpe_gather_live<<<std::min<uint32_t>(4096, nid / 256 + 1), 256, 0, stream>>>(T, d_first, d_st, d_gather, (uint32_t)gather_cap);
    LAUNCH_OK();
    CHECK(sync_state());
    const uint32_t g = h_st->gather_len;
    if (g != D || g > gather_cap) return fail(ZBPE_INTERNAL, "gathered %u live pairs, expected %llu", g, (unsigned long long)D);
    std::vector<LiveRec> recs(g);
    HIP_OK(hipMemcpyAsync(recs.data(), d_gather, (size_t)g * sizeof(LiveRec), hipMemcpyDeviceToHost, stream));
    HIP_OK(hipStreamSynchronize(stream));
    std::vector<uint64_t> order(g);
    for (uint32_t i = 0; i < g; i++) order[i] = recs[i].first_pos;
    if (dist()) {
        // every rank holds the same live keys: in key order the ranks' entries line up. The global first
        // occurrence of a pair is in the lowest rank holding one (shards are contiguous, in rank order),
        // at that rank's local position: one all-reduce(min) of the holding rank, one of the position
        // offered by that rank only -- u32 collectives, whatever the corpus size
        std::sort(recs.begin(), recs.end(), [](const LiveRec &x, const LiveRec &y) { return x.key < y.key; });
        std::vector<uint32_t> w(g);
        for (uint32_t i = 0; i < g; i++) w[i] = recs[i].first_pos != 0xFFFFFFFFu ? (uint32_t)rank : 0xFFFFFFFFu;
        CHECK(ensure(&d_first, first_cap, std::max<size_t>(g, nid), "first occurrences"));
        HIP_OK(hipMemcpyAsync(d_first, w.data(), (size_t)g * 4, hipMemcpyHostToDevice, stream));
        if (!comm->allreduce_u32(d_first, g, COMM_MIN_U32, stream)) return fail(ZBPE_COMM_ERROR, "all-reduce(min) failed");
        std::vector<uint32_t> lowest(g);
        HIP_OK(hipMemcpyAsync(lowest.data(), d_first, (size_t)g * 4, hipMemcpyDeviceToHost, stream));
        HIP_OK(hipStreamSynchronize(stream));
        for (uint32_t i = 0; i < g; i++) w[i] = lowest[i] == (uint32_t)rank ? recs[i].first_pos : 0xFFFFFFFFu;
        HIP_OK(hipMemcpyAsync(d_first, w.data(), (size_t)g * 4, hipMemcpyHostToDevice, stream));
        if (!comm->allreduce_u32(d_first, g, COMM_MIN_U32, stream)) return fail(ZBPE_COMM_ERROR, "all-reduce(min) failed");
        HIP_OK(hipMemcpyAsync(w.data(), d_first, (size_t)g * 4, hipMemcpyDeviceToHost, stream));
        HIP_OK(hipStreamSynchronize(stream));
        for (uint32_t i = 0; i < g; i++) order[i] = ((uint64_t)lowest[i] << 32) | w[i];
    }
    std::vector<ZigOrderInput> in(g);
    for (uint32_t i = 0; i < g; i++) in[i] = ZigOrderInput{order[i], recs[i].key, recs[i].count};
    if (!zig_order_winner(std::move(in), top, call_after, winner))
        return fail(ZBPE_INTERNAL, "exact tie emulation found no pair with count %u", top);
    }
    if (h_st->tie_verdict == 0) {
        if (*winner != h_st->tie_winner)
            return fail(ZBPE_INTERNAL, "tie fast path chose 0x%08x, exact emulation 0x%08x", h_st->tie_winner, *winner);
        stats.tie_crosschecks++;  // both paths decided this tie, alike
    }
    return ZBPE_OK;
}

using ScanFn = void (*)(const DevState *, ScanArgs);
// 0 is the default: unroll 4, non-temporal loads, two-token-window candidate test, candidates
// compacted per wave and resolved one per lane on the LDS-staged tile. The others for A/B runs
// (tools/scan_density.py): 2 resolves per vector in its lane (slower at every density measured:
// 4.8 vs 5.2 TB/s for a rare pair with a frequent first token, 1.7 vs 2.9 TB/s for (e, ' ')).
static const ScanFn kScanVariants[] = {zbpe_scan_pairs_t<4, true, true, true, true>, zbpe_scan_pairs_t<8, true, true, true, true>,
                                       zbpe_scan_pairs_t<4, true, true>, zbpe_scan_pairs_t<4, true, false>,
                                       zbpe_scan_pairs_t<2, true, true, true, true>, zbpe_scan_pairs_t<4, true, true, false, true>,
                                       zbpe_scan_pairs_t<4, false, true, true, true>,
                                       zbpe_scan_pairs_t<4, true, true, true, true, false, true>};
static const int kScanUnroll[] = {4, 8, 4, 4, 2, 4, 4, 4};
static constexpr int kScanBlocksPerCuMax = 4;

zbpe_status Engine::set_scan_variant(int v) {
    if (v < 0 || v >= (int)(sizeof(kScanVariants) / sizeof(kScanVariants[0])))
        return fail(ZBPE_INVALID_ARGUMENT, "scan variant %d out of range", v);
    int nb = 0;
    HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void *)kScanVariants[v], SCAN_THREADS, 0));
    scan_variant = v;
    // at most four per CU: the occupancy query reports 8, but a grid past four workgroups per CU ran long list walks
    // in two dispatch rounds (C4: 8 per CU 17.4k merges/s, 4 per CU 17.8k, profiles/r02_ab_knobs.jsonl)
    scan_blocks_per_cu = std::max(1, std::min(nb, kScanBlocksPerCuMax));
    return ZBPE_OK;
}

// Variant 0 by default; its batching twin (variant 7) once the pair is known to be sparse: count_hint
// (a bound on the pair's count: the top count when the merges were enqueued, which never rises) times
// SCAN_BATCH_DENSITY below the stream's slots. (Batching resolves a sparse tile's few candidates with
// those of other tiles; since its windows move by DPP it is ahead at every density below 3e-2,
// tools/scan_bands.py, profiles/r06_scan_bands_dpp.jsonl.)
static constexpr int kScanBatchVariant = 7;
zbpe_status Engine::launch_scan(const ScanArgs &A, int grid, uint64_t count_hint) {
    int v = scan_variant;
    if (v == 0 && !A.prof &&
        (scan_batch == 2 || (scan_batch == 1 && count_hint && count_hint * SCAN_BATCH_DENSITY < (uint64_t)A.n)))
        v = kScanBatchVariant;
    // option sel_prof: the probed instantiation of the default variant
    const ScanFn f = A.prof && v == 0 ? zbpe_scan_pairs_t<4, true, true, true, true, true> : kScanVariants[v];
    ScanArgs B = A;
    B.batch = scan_batch;
    hipLaunchKernelGGL(f, dim3(grid > 0 ? grid : scan_grid(A.n)), dim3(SCAN_THREADS), 0, stream, (const DevState *)B.st, B);
    LAUNCH_OK();
    return ZBPE_OK;
}

// scan-kernel microbenchmark on the current stream: `reps` launches for pair (a, b)
zbpe_status Engine::bench_scan(uint32_t a, uint32_t b, int reps, double *avg_ms, double *gbps) {
    if (!uploaded) return fail(ZBPE_INVALID_ARGUMENT, "no corpus uploaded");
    HIP_OK(hipSetDevice(device));
    if (!stream_ready) {
        CHECK(alloc_stream(n_text));
        stream_ready = true;
    }
    CHECK(ensure(&d_rec, rec_cap, (size_t)n_slots / 2 + 1, "occurrence records"));
    uint32_t *tail = d_delta + DELTA_WORDS - 32;
    ScanArgs A{d_tok[cur], n_slots, a, b, d_delta, d_delta + 65536, d_st, d_rec, (uint32_t)rec_cap, 1, tail, tail + 1, Halo{}};
    double total = 0;
    for (int r = 0; r < reps; r++) {
        HIP_OK(hipMemsetAsync(d_st, 0, sizeof(DevState), stream));
        HIP_OK(hipEventRecord(ev[0], stream));
        CHECK(launch_scan(A));
        HIP_OK(hipEventRecord(ev[1], stream));
        zbpe_reset_merge<<<256, 256, 0, stream>>>(d_st, d_delta, d_delta + 65536, 65536);
        LAUNCH_OK();
        HIP_OK(hipEventSynchronize(ev[1]));
        float ms;
        HIP_OK(hipEventElapsedTime(&ms, ev[0], ev[1]));
        if (r) total += ms;  // first launch warms up
    }
    *avg_ms = reps > 1 ? total / (reps - 1) : 0;
    *gbps = *avg_ms > 0 ? 2.0 * (double)n_slots / (*avg_ms * 1e-3) / 1e9 : 0;
    return ZBPE_OK;
}

// Late-phase scan microbenchmark on a trained context: `reps` launches of the pair scan for the pair
// at the top of the current selection, exactly as training would launch it for the next merge (list
// form when its list is short), with the per-merge counters and deltas reset between launches. The
// stream, the lists and the counts are left as they were (records land past the arena top).
zbpe_status Engine::bench_train_scan(int reps, int grid, double *avg_us, uint32_t *pair, uint32_t *list_len, int *mode) {
    if (!trained || multi()) return fail(ZBPE_INVALID_ARGUMENT, "bench_train_scan needs a trained single-GPU context");
    HIP_OK(hipSetDevice(device));
    CHECK(sync_state());
    const uint32_t key = h_st->top_key, a = key & 0xFFFF, b = key >> 16, X = 256 + (uint32_t)run.merges;
    if (a == b || !h_st->top_count || X >= 65536) return fail(ZBPE_INVALID_ARGUMENT, "no scannable pair (self pair or exhausted)");
    uint32_t *left = delta_of(X), *right = left + X, *tail = left + 2 * X;
    ScanArgs A{d_tok[cur], n_slots, a, b, left, right, d_st, d_lists, (uint32_t)lists_cap, 1, tail, tail + 1, halo,
               nullptr, pres_vp, X, T.tok_cnt, 0, nullptr, lists_on ? d_lists : nullptr, T.lst_off, T.lst_len, list_ratio, 1,
               d_log, nullptr, 0};
    set_list_nb(A);
    double total = 0;
    for (int r = 0; r <= reps; r++) {
        zbpe_reset_merge<<<(X + 255) / 256, 256, 0, stream>>>(d_st, left, right, X);
        LAUNCH_OK();
        HIP_OK(hipMemsetAsync(tail, 0, 8, stream));
        HIP_OK(hipEventRecord(ev[0], stream));
        CHECK(launch_scan(A, grid, h_st->top_count));  // the variant training picks for this pair
        HIP_OK(hipEventRecord(ev[1], stream));
        HIP_OK(hipEventSynchronize(ev[1]));
        float ms;
        HIP_OK(hipEventElapsedTime(&ms, ev[0], ev[1]));
        if (r) total += ms;  // the first launch warms up
    }
    zbpe_reset_merge<<<(X + 255) / 256, 256, 0, stream>>>(d_st, left, right, X);
    LAUNCH_OK();
    HIP_OK(hipMemsetAsync(tail, 0, 8, stream));
    CHECK(sync_state());
    MergeLog L{};
    HIP_OK(hipMemcpy(&L, d_log + (X - 256), sizeof L, hipMemcpyDeviceToHost));
    *avg_us = reps ? total * 1e3 / reps : 0;
    *pair = key;
    *mode = (int)h_st->scan_mode;
    *list_len = h_st->scan_mode ? L.list_len : 0;
    if (h_st->scan_mode) fprintf(stderr, "bench_train_scan: pair (%u,%u) count %u: walked list %u entries, %u live\n", a, b,
                                 h_st->top_count, L.list_len, L.key_live);
    return ZBPE_OK;
}

// a self pair (a, a) walks a's occurrence list when the lists describe the stream, no shard edge
// is involved and the list is short against the stream (self_list_ratio; the stream form costs
// three passes over it)
bool Engine::self_list_ok(uint32_t a, bool training) {
    if (!lists_on || dist() || self_list_ratio == 0 || (training && !h_st->lists_valid)) return false;
    uint32_t len = NO_LIST;
    if (hipMemcpyAsync(&len, T.lst_len + a, 4, hipMemcpyDeviceToHost, stream) != hipSuccess ||
        hipStreamSynchronize(stream) != hipSuccess)
        return false;
    return len != NO_LIST && (uint64_t)len * self_list_ratio < (uint64_t)n_slots;
}

// persistent grid: as many blocks as are resident at once, fewer for short streams
int Engine::scan_grid(int64_t slots) const {
    const int unroll = kScanUnroll[scan_variant];
    const int64_t wave_tiles = (slots / 8 + 64 * unroll - 1) / (64 * unroll);
    const int64_t blocks = (wave_tiles + SCAN_THREADS / 64 - 1) / (SCAN_THREADS / 64);
    return (int)std::max<int64_t>(1, std::min<int64_t>(blocks, (int64_t)num_cus * scan_blocks_per_cu));
}

// (re)build the token -> block presence bitmap from the current stream (block skipping)
zbpe_status Engine::build_presence() {
    if (!pres_on) return ZBPE_OK;
    const uint64_t groups = std::max<uint64_t>(1, ((uint64_t)n_slots + (uint64_t)PRES_BLK * PRES_GROUP - 1) /
                                                      ((uint64_t)PRES_BLK * PRES_GROUP));
    CHECK(ensure(&d_pres, pres_cap, groups * pres_vp, "presence bitmap"));
    pres_groups = (uint32_t)groups;
    zbpe_pres_build<<<(unsigned)groups, PRES_THREADS, pres_vp * 4, stream>>>(d_tok[cur], n_slots, pres_vp, d_pres);
    LAUNCH_OK();
    stats_pres_builds++;
    return ZBPE_OK;
}

zbpe_status Engine::alloc_stream(size_t n) {
    const size_t need = round_up(n + 1, 64) + 64;
    CHECK(ensure(&d_tok[0], tok_cap0, need, "token stream"));
    CHECK(ensure(&d_tok[1], tok_cap1, need, "token stream (compaction buffer)"));
    cur = 0;
    zbpe_fill_u16<<<256, 256, 0, stream>>>(d_tok[0], 0, (int64_t)need, HOLE);
    LAUNCH_OK();
    const uint64_t n_pad16 = round_up(n, 16);
    if (n) {
        zbpe_widen<<<(int)std::min<uint64_t>(4096, n_pad16 / 16 / 256 + 1), 256, 0, stream>>>(d_text, d_tok[0], n, n_pad16);
        LAUNCH_OK();
    }
    n_slots = (int64_t)n;
    n_live = (int64_t)n;
    stream_ready = false;
    return ZBPE_OK;
}

// generateInitialTokens (basic_tokenizer.zig:155-170): the u8 -> u16 stream (alloc_stream's widen), timed
// with events; like the reference it prints its runtime line to stderr (:156-160; train and encode both
// call it, :150 and :72), on rank 0, unless option "print_runtime" is 0
zbpe_status Engine::generate_initial_tokens(size_t n) {
    HIP_OK(hipEventRecord(ev[6], stream));
    CHECK(alloc_stream(n));
    HIP_OK(hipEventRecord(ev[7], stream));
    HIP_OK(hipEventSynchronize(ev[7]));
    float ms = 0;
    HIP_OK(hipEventElapsedTime(&ms, ev[6], ev[7]));
    gen_tokens_s = ms * 1e-3;
    if (print_runtime && rank == 0) fprintf(stderr, "generateInitialTokens runtime: %.3f seconds\n", gen_tokens_s);
    return ZBPE_OK;
}

// halo of this rank from the gathered boundary records (walks past shards with too few live tokens)
void Engine::halo_from_boundaries() {
    Halo H = halo_empty();
    for (int r = rank - 1; r >= 0 && H.nleft < 2; r--)
        for (int k = 0; k < h_bnd[r].nlast && H.nleft < 2; k++) halo_push_left(H, h_bnd[r].last[k]);
    for (int r = rank + 1; r < world && H.nright < 3; r++)
        for (int k = 0; k < h_bnd[r].nfirst && H.nright < 3; k++) halo_push_right(H, h_bnd[r].first[k]);
    halo = H;
}

zbpe_status Engine::comm_sum(uint32_t *d, size_t n) {
    if (dist() && n && !comm->allreduce_u32(d, n, COMM_SUM_U32, stream))
        return fail(ZBPE_COMM_ERROR, "all-reduce of %zu u32 failed", n);
    return ZBPE_OK;
}

zbpe_status Engine::train(uint16_t vocab_size, int verbose, uint16_t *out_triples, uint64_t *out_counts,
                          size_t *out_n_merges, zbpe_stats *out_stats) {
    const double t_start = now_s();
    stats = zbpe_stats{};
    *out_n_merges = 0;
    if (vocab_size < 256) return fail(ZBPE_INVALID_VOCAB_SIZE, "vocabSize %u < 256", vocab_size);
    if (!uploaded) return fail(ZBPE_INVALID_ARGUMENT, "no corpus uploaded");
    if (!sharded && multi()) return fail(ZBPE_INVALID_ARGUMENT, "distributed context: upload the corpus with zbpe_upload");
    HIP_OK(hipSetDevice(device));
    const size_t n = n_text;
    double ev_count = 0, ev_select = 0, ev_replace = 0;

    // ---- generateInitialTokens + initial histogram ------------------------------------------------
    CHECK(generate_initial_tokens(n));
    stats.generate_tokens_s = gen_tokens_s;
    pres_vp = ((uint32_t)vocab_size + 63) & ~63u;
    pres_on = block_skip && pres_vp <= PRES_MAX_VP;
    CHECK(build_presence());
    // arena: the occurrence lists (<= live tokens) + the records appended until the next compaction
    {
        const auto arena_for = [&](uint64_t m) -> uint64_t {
            const uint64_t c = std::min<uint64_t>(0xFFFFFFF0u, m + m / 2 + (16u << 20));
            return arena_cap_opt ? std::min<uint64_t>(c, arena_cap_opt) : c;
        };
        CHECK(ensure(&d_lists, lists_cap, arena_for(n), "occurrence arena"));
        // the smallest shard's arena: a limit every rank computes alike
        arena_cap_rep = std::min<uint64_t>(lists_cap, arena_for(sharded ? n_total / world : n));
    }
    lists_on = false;
    list_streak = false;
    if (!T.id_key || T.id_cap < (1u << 20)) {
        if (T.id_key) {
            (void)hipFree(T.ht); (void)hipFree(T.id_key); (void)hipFree(T.id_cnt); (void)hipFree(T.hpos);
            T.ht = nullptr; T.id_key = T.id_cnt = T.hpos = nullptr;
        }
        CHECK(alloc_tables(1u << 20));
    } else {
        HIP_OK(hipMemsetAsync(T.ht, 0xFF, ((size_t)T.ht_mask + 1) * 8, stream));
        HIP_OK(hipMemsetAsync(T.hpos, 0xFF, (size_t)T.id_cap * 4, stream));  // ids restart at 0
    }
    HIP_OK(hipMemsetAsync(d_st, 0, sizeof(DevState), stream));
    {
        const long long lt = (long long)n;
        HIP_OK(hipMemcpyAsync(&d_st->live_tokens, &lt, sizeof(lt), hipMemcpyHostToDevice, stream));
        HIP_OK(hipStreamSynchronize(stream));
    }
    home_slots = 0;
    T.home_mask = 0;
    replicated = false;
    sum_tokens_rep = 0;
    global_live = sharded ? n_total : n;
    global_slots = global_live;
    if (T.home_cnt) { (void)hipFree(T.home_cnt); T.home_cnt = nullptr; home_words_cap = 0; }
    if (T.home_dirty) { (void)hipFree(T.home_dirty); T.home_dirty = nullptr; dirty_bits_cap = 0; }
    hot_stale = true;
    halo = halo0;
    HIP_OK(hipMemsetAsync(d_delta, 0, 2 * DELTA_WORDS * 4, stream));
    // the rounds' member buffers: each round's select clears them, but a train that failed between a round's
    // replace and its select (e.g. a hot-list rebuild's error) left them dirty for the next train on this engine
    HIP_OK(hipMemsetAsync(d_rdelta, 0, (size_t)ROUND_MAX * DELTA_WORDS * 4, stream));
    HIP_OK(hipMemsetAsync(d_hist, 0, 65536 * 4, stream));
    HIP_OK(hipEventRecord(ev[0], stream));
    if (n + (next_byte >= 0 ? 1 : 0) >= 2) {
        const int hb = std::max(1, num_cus);
        for (uint32_t lo : {0u, 128u}) {
            zbpe_count_byte_pairs<<<hb, HIST_THREADS, 32768 * 4, stream>>>(d_text, n, next_byte, lo, d_hist);
            LAUNCH_OK();
        }
    }
    if (dist()) {  // every rank builds the same table from the summed histogram (16-bit limbs: exact)
        uint32_t *limbs = d_delta;  // scratch: the merge loop clears it below
        zbpe_hist_split<<<256, 256, 0, stream>>>(d_hist, limbs);
        LAUNCH_OK();
        CHECK(comm_sum(limbs, 2 * 65536));
        zbpe_hist_join<<<256, 256, 0, stream>>>(limbs, d_hist, d_st);
        LAUNCH_OK();
        HIP_OK(hipMemsetAsync(d_delta, 0, 2 * 65536 * 4, stream));
    }
    if (multi()) {  // boundary tokens of every shard (the first select needs the stream's last pair)
        zbpe_boundary<<<1, 1, 0, stream>>>(d_tok[cur], n_slots, n_live, d_bnd_mine, nullptr);
        LAUNCH_OK();
        if (!comm->allgather(d_bnd_mine, d_bnd_all, sizeof(Boundary), stream))
            return fail(ZBPE_COMM_ERROR, "all-gather of shard boundaries failed");
    }
    HIP_OK(hipMemsetAsync(T.tok_cnt, 0, 65536 * sizeof(int32_t), stream));
    zbpe_hist_to_table<<<256, 256, 0, stream>>>(d_hist, T, d_st);
    LAUNCH_OK();
    HIP_OK(hipEventRecord(ev[1], stream));
    CHECK(sync_state());
    CHECK(launch_argmax(0, 0));
    HIP_OK(hipEventRecord(ev[2], stream));
    CHECK(sync_state());
    CHECK(select_ready());
    {
        float ms;
        HIP_OK(hipEventElapsedTime(&ms, ev[0], ev[1])); ev_count += ms * 1e-3;
        HIP_OK(hipEventElapsedTime(&ms, ev[1], ev[2])); ev_select += ms * 1e-3;
        stats.count_pairs_calls++;
    }
    run = RunCtx{};
    begun = false;
    run.out_triples = out_triples;
    run.out_counts = out_counts;
    run.verbose = verbose;
    run.vocab = vocab_size;
    trace.clear();
    compact_log.clear();
    halt_log.clear();
    scan_log.clear();
    std::fill(h_log.begin(), h_log.end(), MergeLog{});
    uint32_t X = 256;
    while (X < vocab_size) {
        if (h_st->live <= 0) {  // sortedCodePointPairs.len == 0 (basic_tokenizer.zig:188-191)
            if (rank == 0) fprintf(stderr, "No more pairs to merge. Stopping early.\n");
            break;
        }
        if (merge_batch > 1 && !debug_checks && !exact_at(X) && vocab_size - X > 1) {
            uint32_t done = 0;
            bool halted = false;
            const bool was_sharded = dist();
            const double t_b = now_s();
            CHECK(run_batch(X, &done, &halted));
            if (batch_checks && X + done > batch_checks) CHECK(table_check(X, X + done, "batch"));
            // (a batch that replicated at its start ran its merges as a replica)
            const bool batch_sharded = was_sharded && dist();
            (batch_sharded ? stats.sharded_s : stats.replicated_s) += now_s() - t_b;
            if (batch_sharded) stats.sharded_merges += done;
            X += done;
            if (!halted) continue;
            // the device stopped at merge X: clear the flag, make the selection valid, finish X here
            const uint32_t reason = h_st->halt;
            const double t_h = now_s();
            HIP_OK(hipMemsetAsync(&d_st->halt, 0, 4, stream));
            CHECK(sync_state());
            CHECK(select_ready());
            if (h_st->live <= 0) continue;
            const double t_m = now_s();
            CHECK(merge_sync(X));
            if (batch_checks && X + 1 > batch_checks) CHECK(table_check(X, X + 1, "halted merge"));
            (batch_sharded ? stats.sharded_s : stats.replicated_s) += now_s() - t_m;
            if (batch_sharded) stats.sharded_merges++;
            halt_log.insert(halt_log.end(), {X, reason, (uint32_t)std::min(4e9, (now_s() - t_h) * 1e6)});
            X++;
            continue;
        }
        const bool was_sharded = dist();
        const double t_m = now_s();
        CHECK(merge_sync(X));
        if (batch_checks && X + 1 > batch_checks) CHECK(table_check(X, X + 1, "merge"));
        (was_sharded ? stats.sharded_s : stats.replicated_s) += now_s() - t_m;
        if (was_sharded) stats.sharded_merges++;
        X++;
    }
    const size_t merges = run.merges;
    {  // device time of the batches, split into the stages by the shares of the timed merges
        const double tm = run.tm_count + run.tm_select + run.tm_replace;
        if (tm > 0) {
            ev_count += run.batch_s * run.tm_count / tm;
            ev_select += run.batch_s * run.tm_select / tm;
            ev_replace += run.batch_s * run.tm_replace / tm;
            stats.comm_s = run.batch_s * run.tm_comm / tm;
        }
    }
    ev_count += run.ev_count;
    ev_select += run.ev_select;
    ev_replace += run.ev_replace;
    HIP_OK(hipStreamSynchronize(stream));
    *out_n_merges = merges;
    stats.scan_read_bytes = 2ull * h_st->scanned_slots;
    stats.count_pairs_s = ev_count;
    stats.sort_pairs_s = ev_select;
    stats.replace_pair_s = ev_replace;
    stats.final_tokens = (uint64_t)n_live;
    if (multi()) {  // stream lengths are per shard: sum them (scan bytes stay per rank, like scan time)
        // the replicated phase counted the whole stream on every rank: rank 0 contributes it once
        uint64_t v[2] = {replicated ? (rank == 0 ? stats.final_tokens : 0) : stats.final_tokens,
                         stats.sum_tokens - sum_tokens_rep + (rank == 0 ? sum_tokens_rep : 0)};
        uint32_t w[8] = {0};
        for (int i = 0; i < 2; i++) {  // exact u64 sums from 16-bit limbs (<= 2^16 ranks)
            w[4 * i] = (uint32_t)(v[i] & 0xFFFF);
            w[4 * i + 1] = (uint32_t)((v[i] >> 16) & 0xFFFF);
            w[4 * i + 2] = (uint32_t)((v[i] >> 32) & 0xFFFF);
            w[4 * i + 3] = (uint32_t)(v[i] >> 48);
        }
        uint32_t *d_w = d_delta + DELTA_WORDS - 16;
        HIP_OK(hipMemcpyAsync(d_w, w, 32, hipMemcpyHostToDevice, stream));
        if (!comm->allreduce_u32(d_w, 8, COMM_SUM_U32, stream)) return fail(ZBPE_COMM_ERROR, "all-reduce of the stream statistics failed");
        HIP_OK(hipMemcpyAsync(w, d_w, 32, hipMemcpyDeviceToHost, stream));
        HIP_OK(hipStreamSynchronize(stream));
        for (int i = 0; i < 2; i++)
            v[i] = (uint64_t)w[4 * i] + ((uint64_t)w[4 * i + 1] << 16) + ((uint64_t)w[4 * i + 2] << 32) + ((uint64_t)w[4 * i + 3] << 48);
        stats.final_tokens = v[0];
        stats.sum_tokens = v[1];
        HIP_OK(hipMemsetAsync(d_w, 0, 32, stream));
    }
    if (sel_prof) {  // wall_clock64 runs at 100 MHz
        HIP_OK(hipMemcpy(h_st, d_st, sizeof(DevState), hipMemcpyDeviceToHost));
        const unsigned long long *P = h_st->sel_prof;
        const double calls = std::max(1.0, (double)P[7]), us = 0.01;
        fprintf(stderr, "sel_prof: %llu last-block calls; avg us: argmax+ticket %.2f, reduce %.2f, finish+begin %.2f, "
                        "tie gather %.2f, decide %.2f; argmax blocks done %.2f\n",
                P[7], P[0] * us / calls, P[1] * us / calls, P[2] * us / calls, P[3] * us / calls, P[4] * us / calls,
                P[5] * us / calls);
        const double nd = std::max(1.0, (double)P[8]), nr = std::max(1.0, (double)P[13]), np = std::max(1.0, (double)P[14]);
        fprintf(stderr, "sel_prof: %llu tie decisions; avg us per decision: gather %.2f, refresh wait %.2f, carries %.2f, "
                        "decision total %.2f; latest refresh block done %.2f (%llu samples); refresh prefix start %.2f, end %.2f "
                        "(%llu samples; all from the first argmax block's start)\n", P[8],
                P[3] * us / nd, P[10] * us / nd, P[9] * us / nd, P[4] * us / nd, P[12] * us / nr, P[13], P[6] * us / np,
                P[11] * us / np, P[14]);
        fprintf(stderr, "sel_prof: refresh workgroups: %llu, average duration %.2f us (start to its summaries stored)\n", P[16],
                P[15] * us / std::max(1.0, (double)P[16]));
        fprintf(stderr, "sel_prof: argmax block 0 (from its start): hot counts in %.2f us, block max %.2f us; hot list %.0f ids on average\n",
                P[17] * us / calls, P[18] * us / calls, P[19] / calls);
        fprintf(stderr, "sel_prof: pair selects %llu, average %.2f us from the first argmax block's start to their commit\n", P[20],
                P[21] * us / std::max(1.0, (double)P[20]));
        const uint32_t *W = h_st->rd_why;
        fprintf(stderr, "sel_prof: rounds with named keys ended by: all walked %u, a merged member's pair at the top count %u, not walked %u, "
                        "touch %u, records %u, vocabulary end %u, arena %u, free slots %u, capacity %u, junction counts differ %u\n",
                W[0], W[1], W[2], W[3], W[4], W[5], W[6], W[7], W[8], W[9]);
        fprintf(stderr, "sel_prof: merged members with a junction to an earlier one %u; members skipped (decremented by a merged member) %u; "
                        "ending flags: a new pair (or junction pair) at the top count %u, only adjacent occurrences %u\n",
                W[10], W[13], W[14], W[15]);
        const uint32_t *U = W + 16;  // (kernels.hpp RW_U)
        fprintf(stderr, "sel_prof: untied rounds with named keys %u, members merged beyond the first %u; ended by: all walked %u, "
                        "a merged member's pair at the member's count %u, not walked %u, decremented %u, records %u, vocabulary end %u, "
                        "arena %u, junction counts differ %u\n",
                U[10], U[11], U[0], U[1], U[2], U[3], U[4], U[5], U[6], U[9]);
        const unsigned long long nw = (P[23] & 0xFFFFFFFFull) + (P[23] >> 32);
        fprintf(stderr, "sel_prof: round member walks %llu (%llu with the decision's plan), average %.2f us from the workgroup's state words in (round_scan) to the walk's start\n",
                nw, P[23] & 0xFFFFFFFFull, P[22] * us / std::max(1.0, (double)nw));
        static const char *bucket[3] = {"merges < 7936", "merges 7936-19743", "merges >= 19744"};
        for (int k = 0; k < 3; k++) {
            const unsigned long long *Q = h_st->pipe_prof[k];
            const double nl = std::max(1.0, (double)Q[4]), nr = std::max(1.0, (double)Q[7]), ns = std::max(1.0, (double)Q[9]);
            fprintf(stderr, "pipe_prof %s: list scans %llu: avg us from the launch's block-0 start: LDS clear done %.2f, walk "
                            "done %.2f, flush done %.2f, replace starts %.2f; replace (%llu): work done %.2f, select starts %.2f; "
                            "select's commit -> next scan's block-0 start, in-batch (%llu) %.2f; round scans' bound "
                            "workgroups done %.2f\n",
                    bucket[k], Q[4], Q[0] * us / nl, Q[1] * us / nl, Q[2] * us / nl, Q[3] * us / nl, Q[7], Q[5] * us / nr,
                    Q[6] * us / nr, Q[9], Q[8] * us / ns, Q[15] * us / nl);
            fprintf(stderr, "pipe_prof %s: replace phases, avg us from its block-0 start (latest block): deltas in %.2f, "
                            "gathered %.2f, ids/hot reserved %.2f, table updated %.2f; apply blocks done %.2f\n",
                    bucket[k], Q[10] * us / nr, Q[11] * us / nr, Q[12] * us / nr, Q[13] * us / nr, Q[14] * us / nr);
        }
    }
    stats.replicated_s = std::max(0.0, stats.replicated_s - stats.replicate_s);  // (the replicating batch's wall held it)
    stats.total_s = now_s() - t_start;
    stats.other_s = std::max(0.0, stats.total_s - ev_count - ev_select - ev_replace);
    stats.distinct_pairs = (uint64_t)std::max(h_st->live, 0);
    stats.pair_selects = h_st->pr_hits;
    stats.round_merges = h_st->rd_merges;
    stats.pair_ids = h_st->num_ids;
    trained = true;
    if (out_stats) *out_stats = stats;
    return ZBPE_OK;
}

// Device-resident batch: enqueue up to merge_batch merges without a host sync. Every kernel
// reads the merge's pair from DevState; zbpe_merge_begin / zbpe_tie_decide halt the batch at a
// merge the device cannot finish alone (self pair, undecided tie, capacity change, hot-list
// rebuild), after which every remaining kernel of the batch returns at once. One sync per batch.
zbpe_status Engine::run_batch(uint32_t X0, uint32_t *done, bool *halted) {
    uint32_t K = std::min<uint32_t>(merge_batch, run.vocab - X0);
    if (X0 < exact_lo && exact_lo < exact_hi) K = std::min<uint32_t>(K, exact_lo - X0);  // stop at the exact-tie window
    *done = 0;
    *halted = false;
    // multi-GPU: once pair counts are small against the stream (the single-GPU criterion for
    // occurrence lists, on replicated quantities so every rank decides alike), gather the stream
    // and continue as replicas
    uint64_t wfac = 1;
    for (int i = 0; i < handover; i++) wfac *= (uint64_t)world;
    if (dist() && replicate_late && list_mode && pres_vp <= PRES_MAX_VP &&
        (uint64_t)h_st->top_count * list_start * wfac < global_live &&
        global_live + 64ull * world + (64u << 20) < 0xF0000000ull) {  // the gathered stream must fit u32 positions
        const double t_rep = now_s();
        HIP_OK(hipEventRecord(ev[3], stream));
        CHECK(compact());  // this shard's live tokens, contiguous
        CHECK(replicate());
        CHECK(build_lists(X0, list_ratio, true));
        // merge X0 was begun by the last sharded select (begun): its log row holds the shard's live tokens; it runs as a
        // replica, on the whole stream (sum_tokens and the scan bytes count the row's live tokens, rank 0 once replicated)
        if (begun) {
            const uint32_t lt = (uint32_t)n_live;
            HIP_OK(hipMemcpyAsync(&d_log[X0 - 256].live, &lt, 4, hipMemcpyHostToDevice, stream));
            HIP_OK(hipStreamSynchronize(stream));
        }
        HIP_OK(hipEventRecord(ev[4], stream));
        HIP_OK(hipEventSynchronize(ev[4]));
        float ms;
        HIP_OK(hipEventElapsedTime(&ms, ev[3], ev[4]));
        run.ev_replace += ms * 1e-3;
        CHECK(sync_state());
        stats.replicate_s += now_s() - t_rep;  // (inside this batch's wall, taken out of replicated_s in train)
    }
    // option sel_prof: the select -> scan gap probe counts in-batch transitions only (a batch's first scan follows a
    // host window: a halt's rebuild, a compaction or the host's own turn, not a launch gap)
    if (sel_prof) HIP_OK(hipMemsetAsync(&d_st->pp_t[7], 0, 8, stream));
    const uint64_t C = home_slots;
    const uint32_t nb = (uint32_t)((C + SUMM_SLOTS - 1) / SUMM_SLOTS), nsb = (nb + SUPER_BLOCKS - 1) / SUPER_BLOCKS;
    const HomeView V{T.home_cnt, d_summ, d_sup, (uint32_t)C, nb, nsb};
    // the tie decision's carries, precomputed by the select's last refresh workgroup (one thread per super-block)
    uint32_t *cs = nullptr;
    if (C && fused_select && refresh_prefix && nsb <= (uint32_t)NEXT_THREADS) {
        CHECK(ensure(&d_cs, cs_cap, nsb + 1, "home carries"));
        cs = d_cs;
    }
    // multi-merge rounds: once the merges walk occurrence lists (the last batch only did),
    // one GPU or replicas, with the naming decisions of the pair selects; a launch triple then does 1 .. round_k
    // merges, which the device decides (round_valid), so the kernels take the merge index from the state and
    // the batch's merges are counted after it
    // (and in tie streaks: a round of one costs more than a plain merge -- the members' walks, the full selects)
    // (untied rounds, option round_untied: in every list streak -- the mid phase's merges are mostly untied)
    // (round_streak 0: also in batches that follow stream scans, while the batch's bound on its records -- round_k merges
    // per launch triple, each at most the top count -- is a sixteenth of the arena: else every batch would compact)
    const bool streak_ok = list_streak || (!round_streak && (uint64_t)K * round_k * h_st->top_count * 16 < arena_limit());
    const bool rounds = round_k >= 2 && !dist() && fused_select && pair_select && refresh_prefix && lists_on && streak_ok &&
                        (round_untied || last_tied_pct >= round_ties) && !replace_split && cs && C >= (uint64_t)SUMM_SLOTS * SUPER_BLOCKS;
    uint32_t KM = rounds ? std::min<uint32_t>(K * (uint32_t)round_k, run.vocab - X0) : K;  // merges the batch may do
    if (X0 < exact_lo && exact_lo < exact_hi) KM = std::min<uint32_t>(KM, exact_lo - X0);      // (no round past the exact-tie window's start)
    // headroom for KM merges: ids, occurrence records (counts never grow), tie list; compaction
    CHECK(maybe_grow_tables(X0, KM));
    if (hot_stale) CHECK(rebuild_hot());  // a table rebuild renumbered the ids the tie kernels read
    const uint32_t top0 = h_st->top_count;
    if (holes_over() || arena_used() + (uint64_t)KM * top0 > arena_limit()) CHECK(compact_train(X0));
    CHECK(ensure(&d_tie_list, tie_list_cap, 1u << 16, "tie list"));
    // the refresh counts of zbpe_select_next: each launch zeroes the next one's (by X's parity, or the rounds'
    // launch parity), unless this batch does not continue the last one's launches in the same form
    if (fused_select && (!begun || rounds != last_rounds)) {
        HIP_OK(hipMemsetAsync(d_rtk, 0, RTK_WORDS * sizeof(uint32_t), stream));
        rpar = 0;
    }
    last_rounds = rounds;
    if (rounds) HIP_OK(hipMemsetAsync(d_rlog, 0, K * sizeof(uint32_t), stream));
    if (dist()) HIP_OK(hipMemcpyAsync(d_halo, &halo, sizeof(Halo), hipMemcpyHostToDevice, stream));
    // rounds: the kernels' bound on the merge index (delta clearing, update grids)
    const uint32_t Xmax = X0 + KM;
    // self pairs the batch takes: those self_list_ok would walk (a's list shorter than self_lim), tested by the
    // merge's begin on the device; the others halt to the host path
    const bool sb = self_batch && lists_on && !dist() && self_list_ratio && h_st->lists_valid;
    const uint32_t *self_len = sb ? T.lst_len : nullptr;
    const uint32_t self_lim = sb ? (uint32_t)std::min<uint64_t>(0xFFFFFFFFull, ((uint64_t)n_slots + self_list_ratio - 1) / self_list_ratio) : 0u;
    const uint32_t ab = (uint32_t)std::min<uint64_t>(2048, top0 / 256 + 1);
    const int64_t slots = n_slots;
    const double t0 = now_s();
    lists_at_batch = list_streak;  // the last batch only walked lists: sample this one
    if (merge_timing) HIP_OK(hipEventRecord(bev[BEV_PER_MERGE * MAX_BATCH], stream));
    for (uint32_t i = 0; i < K; i++) {
        if (rounds) {
            CHECK(launch_round(i, X0, Xmax, K, top0, V, cs, self_len, self_lim));
            continue;
        }
        const uint32_t X = X0 + i;
        const bool timed = merge_timed(X);
        if (timed) HIP_OK(hipEventRecord(bev[BEV_PER_MERGE * i], stream));
        uint32_t *left = delta_of(X), *right = left + X, *tail = left + 2 * X;
        // merge start (halt checks, tie_on, ties): done by the previous merge's zbpe_select_next,
        // else fused into the tie collection + refresh + decide
        if (!fused_select || (i == 0 && !begun)) {
            zbpe_tie_collect<<<64, 256, 0, stream>>>(T, d_st, 0, (uint32_t)(C ? C - 1 : 0), d_tie_list, (uint32_t)tie_list_cap, 1,
                                                     BeginArgs{X, C, (uint32_t)arena_limit(), d_log, dist() ? 1 : 0});
            LAUNCH_OK();
            if (C) {
                zbpe_home_refresh<<<nsb, REFRESH_THREADS, 0, stream>>>(T, d_st, (uint32_t)C, nb, d_summ, d_sup, 1);
                LAUNCH_OK();
                zbpe_tie_decide<<<1, DECIDE_THREADS, 0, stream>>>(d_st, d_tie_list, (uint32_t)tie_list_cap, V, d_log, 1);
                LAUNCH_OK();
            }
        }
        if (timed) HIP_OK(hipEventRecord(bev[BEV_PER_MERGE * i + 1], stream));
        ScanArgs A{d_tok[cur], slots, 0, 0, left, right, d_st, d_lists, (uint32_t)lists_cap, 1, tail, tail + 1, halo,
                   pres_on ? d_pres : nullptr, pres_vp, X, T.tok_cnt, 1, dist() ? d_halo : nullptr,
                   lists_on ? d_lists : nullptr, T.lst_off, T.lst_len, list_ratio, 1, d_log, nullptr, (int)sel_prof};
        set_list_nb(A);
        A.gen = layout_gen;
        // a batch that follows one of list scans only launches a smaller grid (fewer idle workgroups
        // to dispatch); a stream scan still completes on it, only slower
        CHECK(launch_scan(A, list_streak ? list_grid : 0, top0));
        if (timed) HIP_OK(hipEventRecord(bev[BEV_PER_MERGE * i + 2], stream));
        CHECK(comm_sum(left, 2ull * X + 2));
        if (timed) HIP_OK(hipEventRecord(bev[BEV_PER_MERGE * i + 3], stream));
        const int pair_blk = fused_select && pair_select && cs && C >= (uint64_t)SUMM_SLOTS * SUPER_BLOCKS ? 1 : 0;
        ReplaceArgs R{d_tok[cur], slots, d_lists, (uint32_t)lists_cap, left, right, tail, 0, 0, X, 0, ab, halo, nullptr,
                      1, dist() ? d_halo : nullptr, 1, (int)sel_prof, pair_blk, d_summ, d_sup, (uint32_t)C, nb, nsb, cs,
                      A.dir_row, A.dir, A.dir_w, layout_gen, scan_plan && lists_on ? 1 : 0};
        if (!replace_split) {
            zbpe_replace<<<ab + update_blocks(X, update_per(X)) + pair_blk, 256, 0, stream>>>(d_st, R.left, R.X, R.apply_blocks, R, T);
        } else {  // profiling: apply and count update as two launches (no pair-select bound)
            R.pair_blk = 0;
            zbpe_replace<<<ab, 256, 0, stream>>>(d_st, R.left, R.X, R.apply_blocks, R, T);
            R.apply_blocks = 0;
            zbpe_replace<<<update_blocks(X, update_per(X)), 256, 0, stream>>>(d_st, R.left, R.X, R.apply_blocks, R, T);
        }
        LAUNCH_OK();
        if (dist()) {
            zbpe_boundary<<<1, 1, 0, stream>>>(d_tok[cur], slots, 0, d_bnd_mine, d_st);
            LAUNCH_OK();
            if (!comm->allgather(d_bnd_mine, d_bnd_all, sizeof(Boundary), stream))
                return fail(ZBPE_COMM_ERROR, "all-gather of shard boundaries failed");
            zbpe_halo_build<<<1, 1, 0, stream>>>(d_bnd_all, rank, world, d_halo, d_st);
            LAUNCH_OK();
        }
        if (timed) HIP_OK(hipEventRecord(bev[BEV_PER_MERGE * i + 4], stream));
        if (fused_select) {
            if (hot_stale) CHECK(rebuild_hot());
            // about four hot entries per thread (the list grows by the new ids of the batch), and
            // the delta words to clear
            // (the grid only sets the parallelism: the argmax loops over whatever the hot list holds at run time)
            const uint64_t hot_est = std::min<uint64_t>(T.hot_cap, (uint64_t)h_st->hot_len + (uint64_t)K * sel_growth + sel_margin);
            const uint64_t work = std::max<uint64_t>(hot_est / SEL_U, C ? 0ull : 2ull * X / 4);  // refresh blocks clear the deltas
            const uint32_t sel = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(NEXT_MAX_SEL, (work + NEXT_THREADS - 1) / NEXT_THREADS));
            NextArgs N{BeginArgs{X + 1, C, (uint32_t)arena_limit(), d_log, dist() ? 1 : 0, self_len, self_lim}, run.vocab, V, d_tie_list, (uint32_t)tie_list_cap, sel, d_cand,
                       d_cand + (size_t)NEXT_MAX_SEL * NEXT_CAND, d_cand + (size_t)NEXT_MAX_SEL * (NEXT_CAND + 1), d_bnd_all,
                       dist() ? world : 1, (int)sel_prof, cs, d_rtk, A.dir_row, A.dir, A.dir_w, layout_gen,
                       scan_plan && lists_on ? 1 : 0, lp_lazy, pair_select, pair_refresh ? 0 : 1, pair_m3w, pair_chain};
            const uint32_t nref = C ? (refresh_wgs ? std::min<uint32_t>(nsb, refresh_wgs) : nsb) : 0u;
            zbpe_select_next<<<sel + nref, NEXT_THREADS, 0, stream>>>(d_st, T.hot, T.hcnt, T.hot_cap, nref, sel,
                                                                                 d_tok[cur], slots, T, d_partial, left, X, N);
            LAUNCH_OK();
        } else {
            CHECK(launch_argmax(X, 1));
        }
        if (timed) HIP_OK(hipEventRecord(bev[BEV_PER_MERGE * i + 5], stream));
    }
    if (merge_timing) HIP_OK(hipEventRecord(bev[BEV_PER_MERGE * MAX_BATCH + 1], stream));
    if (dist()) HIP_OK(hipMemcpyAsync(h_bnd, d_bnd_all, world * sizeof(Boundary), hipMemcpyDeviceToHost, stream));
    CHECK(sync_state());
    const double wall = now_s() - t0;
    batches++;
    // rounds: the merges the batch did follow from the state (the last select began cur_x); a round that reached the
    // vocabulary's end halted the launches after it (HALT_DONE at the end: not a halt of the merge loop)
    // (and one that reached the batch's bound Xmax -- the vocabulary's end, the exact-tie window's start, or K
    // launch triples' worth of merges: the merge there is not started; the next batch or the host path starts it)
    bool at_bound = false;
    if (rounds && h_st->halt == HALT_DONE && h_st->halt_at == Xmax) {
        h_st->halt = 0;
        h_st->cur_x = Xmax;
        at_bound = true;
        HIP_OK(hipMemsetAsync(&d_st->halt, 0, 4, stream));
    }
    const uint32_t m = h_st->halt ? h_st->halt_at - X0 : rounds ? h_st->cur_x - X0 : K;
    if (rounds) HIP_OK(hipMemcpy(h_rlog.data(), d_rlog, K * sizeof(uint32_t), hipMemcpyDeviceToHost));
    if (merge_timing) {
        float ms = 0;
        HIP_OK(hipEventElapsedTime(&ms, bev[BEV_PER_MERGE * MAX_BATCH], bev[BEV_PER_MERGE * MAX_BATCH + 1]));
        run.batch_s += ms * 1e-3;
    }
    begun = fused_select && !h_st->halt && !at_bound;  // the last select started merge X0 + K
    if (h_st->halt) {
        *halted = true;
        batch_halts++;
        if (m > KM) return fail(ZBPE_INTERNAL, "batch halted at merge %u outside [%u, %u)", h_st->halt_at, X0, X0 + KM);
    }
    if (m) HIP_OK(hipMemcpy(h_log.data() + (X0 - 256), d_log + (X0 - 256), m * sizeof(MergeLog), hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < m; i++) {
        const MergeLog &L = h_log[X0 - 256 + i];
        const uint32_t X = X0 + i, a = L.key & 0xFFFF, b = L.key >> 16;
        if (run.verbose && rank == 0)
            fprintf(stderr, "merge %u/%u: (%u,%u) -> %u had %u occurrences\n", X - 256 + 1, run.vocab - 256u, a, b, X, L.count);
        run.out_triples[3 * run.merges + 0] = (uint16_t)a;
        run.out_triples[3 * run.merges + 1] = (uint16_t)b;
        run.out_triples[3 * run.merges + 2] = (uint16_t)X;
        if (run.out_counts) run.out_counts[run.merges] = L.count;
        run.merges++;
        if (a == b) stats.self_pair_merges++;  // (its occurrences are fewer than its count: live tokens below)
        else global_live -= L.count;           // one token per occurrence
        stats.sum_tokens += L.live;
        if (replicated) sum_tokens_rep += L.live;
        stats.scan_alg_bytes += 2ull * L.live;
        stats.scan_launches++;
        stats.sort_pairs_calls++;
        stats.count_pairs_calls++;
        stats.replace_pair_calls++;
        if (L.ties > 1) stats.tie_iterations++;
        if (L.mode) stats.list_scans++;
        float ms_sel = 0, ms_scan = 0, ms_rep = 0, ms_begin = 0, ms_comm = 0;
        if (!rounds && merge_timed(X)) {
            const hipEvent_t *E = &bev[BEV_PER_MERGE * i];
            const double w = merge_weight();  // the merges this one stands for
            HIP_OK(hipEventElapsedTime(&ms_begin, E[0], E[1]));
            HIP_OK(hipEventElapsedTime(&ms_scan, E[1], E[2]));
            HIP_OK(hipEventElapsedTime(&ms_comm, E[2], E[3]));
            HIP_OK(hipEventElapsedTime(&ms_rep, E[3], E[4]));
            HIP_OK(hipEventElapsedTime(&ms_sel, E[4], E[5]));
            ms_sel += ms_begin;  // argmax + Zig-order tie decision: sortCodePointPairs + [0]
            if (!L.mode) {  // the roofline covers stream scans (a list scan reads no stream)
                stats.scan_kernel_s += ms_scan * 1e-3;
                stats.scan_timed_launches++;
                stats.scan_timed_alg_bytes += 2ull * L.live;
            }
            // the sampled merges give the shares of the stages; the batch's measured span is split by them
            run.tm_count += w * (ms_scan + ms_comm) * 1e-3;  // the exchange of the count deltas is counting
            if (dist()) run.tm_comm += w * ms_comm * 1e-3;  // world 1 or replicas: no collective, only an event gap
            run.tm_select += w * ms_sel * 1e-3;
            run.tm_replace += w * ms_rep * 1e-3;
        }
        if (trace_on) {
            const float row[ZBPE_TRACE_COLS] = {(float)(X - 256), (float)L.count, (float)L.live, (float)slots,
                                                L.mode ? (float)L.list_len : 0.f, ms_scan,
                                                ms_rep, ms_sel, (float)(wall * 1e3 / K), 0.f, (float)L.ties};
            trace.insert(trace.end(), row, row + ZBPE_TRACE_COLS);
        }
    }
    if (rounds) {
        // launch i's round (rlog: first merge | members << 16; 0: the launch returned at once after a halt); its
        // events time the whole round, whose merges share them for the stage split
        for (uint32_t i = 0; i < K; i++) {
            const uint32_t r = h_rlog[i], x = r & 0xFFFF;
            scan_log.push_back(r ? (int32_t)(2 * (x - 256) + (h_log[x - 256].mode ? 1 : 0)) : -1);
            if (r && merge_timing && i % merge_timing == 0) {
                const hipEvent_t *E = &bev[BEV_PER_MERGE * i];
                float ms_b = 0, ms_s = 0, ms_r = 0, ms_x = 0;
                HIP_OK(hipEventElapsedTime(&ms_b, E[0], E[1]));
                HIP_OK(hipEventElapsedTime(&ms_s, E[1], E[2]));
                HIP_OK(hipEventElapsedTime(&ms_r, E[3], E[4]));
                HIP_OK(hipEventElapsedTime(&ms_x, E[4], E[5]));
                const double w = merge_timing;
                run.tm_count += w * ms_s * 1e-3;
                run.tm_replace += w * ms_r * 1e-3;
                run.tm_select += w * (ms_x + ms_b) * 1e-3;
                if (!h_log[x - 256].mode) {
                    stats.scan_kernel_s += ms_s * 1e-3;
                    stats.scan_timed_launches++;
                    stats.scan_timed_alg_bytes += 2ull * h_log[x - 256].live;
                }
            }
        }
    } else {
        for (uint32_t i = 0; i < K; i++)  // every merge of the batch launched one scan; those past a halt returned at once
            scan_log.push_back(i < m ? (int32_t)(2 * (X0 + i - 256) + (h_log[X0 - 256 + i].mode ? 1 : 0)) : -1);
    }
    uint32_t nlist = 0;
    for (uint32_t i = 0; i < m; i++) nlist += h_log[X0 - 256 + i].mode;
    list_streak = m > 0 && nlist == m;
    uint32_t ntied = 0;
    for (uint32_t i = 0; i < m; i++) ntied += h_log[X0 - 256 + i].ties > 1 ? 1u : 0u;
    last_tied_pct = m ? 100u * ntied / m : 0u;
    n_live = h_st->live_tokens;
    if (sb) global_live = (uint64_t)n_live;  // (self pairs only run here on one GPU or replicas: the stream is whole)
    if (dist()) halo_from_boundaries();
    *done = m;
    return ZBPE_OK;
}

// Launch triple i of a batch of multi-merge rounds (run_batch): the round scan, the round replace and the
// select, each reading the round's first merge from the state; X0: the batch's first merge (begun by the last
// batch's select, else here), Xmax: the bound on every merge index of the batch (delta clearing, update grids).
zbpe_status Engine::launch_round(uint32_t i, uint32_t X0, uint32_t Xmax, uint32_t K, uint32_t top0, const HomeView &V, uint32_t *cs,
                                 const uint32_t *self_len, uint32_t self_lim) {
    const uint64_t C = V.C;
    const bool timed = merge_timing && i % merge_timing == 0;
    if (timed) HIP_OK(hipEventRecord(bev[BEV_PER_MERGE * i], stream));
    if (i == 0 && !begun) {  // merge X0's start (its select did not run on the device: a halt or a host-path merge)
        zbpe_tie_collect<<<64, 256, 0, stream>>>(T, d_st, 0, (uint32_t)(C - 1), d_tie_list, (uint32_t)tie_list_cap, 1,
                                                 BeginArgs{X0, C, (uint32_t)arena_limit(), d_log, 0});
        LAUNCH_OK();
        zbpe_home_refresh<<<V.nsb, REFRESH_THREADS, 0, stream>>>(T, d_st, (uint32_t)C, V.nb, d_summ, d_sup, 1);
        LAUNCH_OK();
        zbpe_tie_decide<<<1, DECIDE_THREADS, 0, stream>>>(d_st, d_tie_list, (uint32_t)tie_list_cap, V, d_log, 1);
        LAUNCH_OK();
    }
    if (timed) HIP_OK(hipEventRecord(bev[BEV_PER_MERGE * i + 1], stream));
    uint32_t *base = d_rdelta;
    ScanArgs A{d_tok[cur], n_slots, 0, 0, base, base + 65536, d_st, d_lists, (uint32_t)lists_cap, 1, base + 2 * 65536,
               base + 2 * 65536 + 1, halo, pres_on ? d_pres : nullptr, pres_vp, Xmax, T.tok_cnt, 1, nullptr,
               lists_on ? d_lists : nullptr, T.lst_off, T.lst_len, list_ratio, 1, d_log, nullptr, 0};
    set_list_nb(A);
    A.gen = layout_gen;
    A.batch = scan_batch;
    A.round = round_k;
    A.x_end = Xmax;  // (the rounds' delta layouts and update grids hold merges below Xmax)
    A.hv = HomeView{nullptr, d_summ, d_sup, (uint32_t)C, V.nb, V.nsb};
    A.cs = cs;
    const int g = list_streak && list_grid > 0 ? list_grid : scan_grid(n_slots);
    A.prof = (int)sel_prof;
    if (sel_prof)  // (the probed instantiation)
        hipLaunchKernelGGL((zbpe_scan_pairs_t<4, true, true, true, true, true, false, true>), dim3(g + RD_FREE_WGS), dim3(SCAN_THREADS),
                           RD_QUEUE * sizeof(uint32_t), stream, (const DevState *)d_st, A);
    else
        hipLaunchKernelGGL((zbpe_scan_pairs_t<4, true, true, true, true, false, false, true>), dim3(g + RD_FREE_WGS), dim3(SCAN_THREADS),
                           RD_QUEUE * sizeof(uint32_t), stream, (const DevState *)d_st, A);  // (dynamic LDS: rd_queue)
    LAUNCH_OK();
    if (timed) {
        HIP_OK(hipEventRecord(bev[BEV_PER_MERGE * i + 2], stream));
        HIP_OK(hipEventRecord(bev[BEV_PER_MERGE * i + 3], stream));
    }
    const uint32_t ab = (uint32_t)std::min<uint64_t>(2048, top0 / 256 + 1);
    const uint32_t pm = ab + update_blocks(Xmax, update_per(Xmax));
    ReplaceArgs R{d_tok[cur], n_slots, d_lists, (uint32_t)lists_cap, base, base + 65536, base + 2 * 65536, 0, 0, Xmax, 0, ab, halo,
                  nullptr, 1, nullptr, 1, (int)sel_prof, 0, d_summ, d_sup, (uint32_t)C, V.nb, V.nsb, cs, nullptr, nullptr, 0, layout_gen, 0};
    R.round = round_k;
    R.per_member = pm;
    R.x_end = Xmax;
    zbpe_replace_round<<<(uint32_t)round_k * pm, 256, 0, stream>>>(d_st, base, Xmax, ab, R, T);
    LAUNCH_OK();
    if (timed) HIP_OK(hipEventRecord(bev[BEV_PER_MERGE * i + 4], stream));
    if (hot_stale) CHECK(rebuild_hot());
    const uint64_t hot_est = std::min<uint64_t>(T.hot_cap, (uint64_t)h_st->hot_len + (uint64_t)K * round_k * sel_growth + sel_margin);
    const uint64_t work = hot_est / SEL_U;
    const uint32_t sel = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(NEXT_MAX_SEL, (work + NEXT_THREADS - 1) / NEXT_THREADS));
    // the naming decision must name every member the rounds take: chains up to round_k - 1 further keys
    const int chain = std::min(3, std::max(pair_chain, round_k - 2));
    NextArgs N{BeginArgs{Xmax, C, (uint32_t)arena_limit(), d_log, 0, self_len, self_lim}, Xmax, V, d_tie_list, (uint32_t)tie_list_cap, sel, d_cand,
               d_cand + (size_t)NEXT_MAX_SEL * NEXT_CAND, d_cand + (size_t)NEXT_MAX_SEL * (NEXT_CAND + 1), d_bnd_all, 1,
               (int)sel_prof, cs, d_rtk, A.dir_row, A.dir, A.dir_w, layout_gen, scan_plan && lists_on ? 1 : 0, lp_lazy, pair_select,
               1, 1, chain};
    N.round = round_k;
    N.untied = round_untied;
    N.par = rpar;
    N.seq = launch_seq++;
    N.rlog_i = i;
    N.rlog = d_rlog;
    rpar ^= 1u;
    const uint32_t nref = refresh_wgs ? std::min<uint32_t>(V.nsb, refresh_wgs) : V.nsb;
    zbpe_select_next<<<sel + nref, NEXT_THREADS, 0, stream>>>(d_st, T.hot, T.hcnt, T.hot_cap, nref, sel, d_tok[cur], n_slots, T,
                                                              d_partial, base, Xmax, N);
    LAUNCH_OK();
    if (timed) HIP_OK(hipEventRecord(bev[BEV_PER_MERGE * i + 5], stream));
    return ZBPE_OK;
}

// One merge on the synchronous path: the host reads the selection, resolves a tie (exact
// fallback included), handles self pairs, and syncs once at the end.
zbpe_status Engine::merge_sync(uint32_t X) {
    const double t_merge = now_s();
    const uint64_t slots_before = h_st->scanned_slots;
    const int64_t live_before = n_live, slots_now = n_slots;
    const uint32_t top = h_st->top_count, ties = h_st->tie_count;
    uint32_t key = h_st->top_key;
    const double t_sel = now_s();
    exact_now = exact_at(X);
    begun = false;  // this merge's select (zbpe_select) does not start the next merge on the device
    if (ties > 1) CHECK(resolve_tie(top, ties, &key));
    stats.sort_pairs_calls++;
    if (ties > 1) run.ev_select += now_s() - t_sel;
    const uint32_t a = key & 0xFFFF, b = key >> 16;
    if (run.verbose && rank == 0)
        fprintf(stderr, "merge %u/%u: (%u,%u) -> %u had %u occurrences\n", X - 256 + 1, run.vocab - 256u, a, b, X, top);
    run.out_triples[3 * run.merges + 0] = (uint16_t)a;
    run.out_triples[3 * run.merges + 1] = (uint16_t)b;
    run.out_triples[3 * run.merges + 2] = (uint16_t)X;
    if (run.out_counts) run.out_counts[run.merges] = top;
    run.merges++;
    stats.sum_tokens += (uint64_t)n_live;
    if (replicated) sum_tokens_rep += (uint64_t)n_live;

    CHECK(maybe_grow_tables(X, 1));
    const bool self = a == b;
    // records need room in the arena (self pairs treat holes as transparent: no compaction needed)
    // (sharded: replicated quantities only, so every rank compacts / grows alike and the ranks' collectives stay in step)
    if (arena_used() + top > arena_limit()) CHECK(compact_train(X));
    if (arena_used() + top > arena_limit()) CHECK(grow_arena(arena_used() + top + (16u << 20)));
    // delta layout for this merge: left[0, X) | right[X, 2X) | xx | occurrences
    uint32_t *left = delta_of(X), *right = left + X, *tail = left + 2 * X;
    // ---- count: scan the stream for (a, b) -----------------------------------------------------
    ScanArgs A{d_tok[cur], n_slots, a, b, left, right, d_st, d_lists, (uint32_t)lists_cap, 1, tail, tail + 1, halo,
               pres_on ? d_pres : nullptr, pres_vp, X, T.tok_cnt, 0, nullptr, lists_on ? d_lists : nullptr, T.lst_off,
               T.lst_len, list_ratio, 1, nullptr};
    set_list_nb(A);
    HIP_OK(hipEventRecord(ev[0], stream));
    if (!self) {
        CHECK(launch_scan(A, 0, top));
        stats.scan_launches++;
    } else {
        stats.self_pair_merges++;
        if (self_list_ok(a, true)) {
            zbpe_scan_self_list<<<scan_grid(n_slots), SCAN_THREADS, 0, stream>>>(A);
            LAUNCH_OK();
            stats.list_scans++;
        } else {
        const int64_t ntiles = std::max<int64_t>(1, (n_slots + SELF_TILE - 1) / SELF_TILE);
        CHECK(ensure(&d_tile_fn, tile_fn_cap, ntiles, "self tiles"));
        CHECK(ensure(&d_carry, carry_cap, ntiles, "self carry"));
        zbpe_self_tiles<<<ntiles, SELF_THREADS, 0, stream>>>(d_tok[cur], n_slots, a, d_tile_fn);
        LAUNCH_OK();
        if (dist()) {  // parity of the run of a's entering this shard from the ranks to the left
            zbpe_self_carry<<<1, 1024, 0, stream>>>(d_tile_fn, ntiles, d_carry, nullptr, d_shard_fn);
            LAUNCH_OK();
            if (!comm->allgather(d_shard_fn, d_fns_all, 4, stream)) return fail(ZBPE_COMM_ERROR, "all-gather of run carries failed");
            zbpe_self_x0<<<1, 1, 0, stream>>>(d_fns_all, rank, d_x0);
            LAUNCH_OK();
        }
        zbpe_self_carry<<<1, 1024, 0, stream>>>(d_tile_fn, ntiles, d_carry, dist() ? d_x0 : nullptr, nullptr);
        LAUNCH_OK();
        zbpe_scan_self<<<std::min(ntiles, SELF_GRID), SELF_THREADS, 0, stream>>>(A, d_carry);
        LAUNCH_OK();
        }
    }
    HIP_OK(hipEventRecord(ev[1], stream));
    // ---- exchange: sum the count deltas of all shards (one RCCL all-reduce per merge) ---------------
    CHECK(comm_sum(left, 2ull * X + 2));
    // ---- replace: apply + count update ---------------------------------------------------------
    {
        const uint32_t ab = (uint32_t)std::min<uint64_t>(2048, top / 256 + 1);
        ReplaceArgs R{d_tok[cur], n_slots, d_lists, (uint32_t)lists_cap, left, right, tail, a, b, X, key, ab, halo,
                      (self && dist()) ? d_x0 : nullptr, 0, nullptr, 1};
        zbpe_replace<<<ab + update_blocks(X, update_per(X)), 256, 0, stream>>>(d_st, R.left, R.X, R.apply_blocks, R, T);
        LAUNCH_OK();
    }
    if (dist()) {  // boundary tokens of every shard for the next merge's halos
        zbpe_boundary<<<1, 1, 0, stream>>>(d_tok[cur], n_slots, n_live, d_bnd_mine, nullptr);
        LAUNCH_OK();
        if (!comm->allgather(d_bnd_mine, d_bnd_all, sizeof(Boundary), stream))
            return fail(ZBPE_COMM_ERROR, "all-gather of shard boundaries failed");
    }
    HIP_OK(hipEventRecord(ev[2], stream));
    // ---- select for the next merge (also clears the deltas, rolls the counters) ----------------------
    CHECK(launch_argmax(X, 1));
    if (dist()) HIP_OK(hipMemcpyAsync(h_bnd, d_bnd_all, world * sizeof(Boundary), hipMemcpyDeviceToHost, stream));
    HIP_OK(hipEventRecord(ev[3], stream));
    CHECK(sync_state());
    CHECK(select_ready());
    {
        float ms;
        float ms_r, ms_s;
        HIP_OK(hipEventElapsedTime(&ms, ev[0], ev[1])); run.ev_count += ms * 1e-3;
        h_log[X - 256] = MergeLog{key, top, (uint32_t)live_before, ties, self ? 0u : h_st->scan_mode, 0, 0, 0};  // (zbpe_merge_log)
        if (!self) {
            scan_log.push_back((int32_t)(2 * (X - 256) + (h_st->scan_mode ? 1 : 0)));
            stats.scan_alg_bytes += 2ull * (uint64_t)n_live;
            if (h_st->scan_mode) {
                stats.list_scans++;
            } else {
                stats.scan_kernel_s += ms * 1e-3;
                stats.scan_timed_launches++;
                stats.scan_timed_alg_bytes += 2ull * (uint64_t)n_live;
            }
        }
        HIP_OK(hipEventElapsedTime(&ms_r, ev[1], ev[2])); run.ev_replace += ms_r * 1e-3;
        HIP_OK(hipEventElapsedTime(&ms_s, ev[2], ev[3])); run.ev_select += ms_s * 1e-3;
        if (trace_on) {
            const float row[ZBPE_TRACE_COLS] = {(float)(X - 256), (float)top, (float)live_before, (float)slots_now,
                                                (float)(h_st->scanned_slots - slots_before), ms, ms_r, ms_s,
                                                (float)((now_s() - t_merge) * 1e3), self ? 1.f : 0.f, (float)ties};
            trace.insert(trace.end(), row, row + ZBPE_TRACE_COLS);
        }
        stats.count_pairs_calls++;
        stats.replace_pair_calls++;
    }
    if (dist()) halo_from_boundaries();
    if (debug_checks) {
        uint64_t bad = 0;
        uint32_t info[3] = {0, 0, 0};
        CHECK(recount_check(&bad, info));
        if (bad)
            return fail(ZBPE_INTERNAL, "merge %u (%u,%u): %llu pair counts differ from a full recount (first: key (%u,%u) table %u, recount %u)",
                        X, a, b, (unsigned long long)bad, info[0] & 0xFFFF, info[0] >> 16, info[1], info[2]);
    }
    const uint32_t gocc = h_st->last_gocc;
    global_live -= gocc;
    if (!self && gocc != top)
        return fail(ZBPE_INTERNAL, "merge %u: scan found %u occurrences of (%u,%u), count was %u", X, gocc, a, b, top);
    const uint64_t gone = h_st->last_holes;  // slots of this shard that became holes
    n_live -= gone;
    (void)gone;
    if (holes_over()) CHECK(compact_train(X + 1));
    return ZBPE_OK;
}

zbpe_status Engine::verify_counts(uint64_t *mismatches) {
    if (!trained) return fail(ZBPE_INVALID_ARGUMENT, "verify_counts needs a trained context");
    return recount_check(mismatches, nullptr);
}

// the live tokens of the current stream, holes squeezed out, into the spare stream buffer (the current
// buffer, its holes and the occurrence lists stay as they are); *total: their number
zbpe_status Engine::compact_to_spare(uint64_t *total) {
    *total = 0;
    const int64_t ntiles = (n_slots + COMPACT_TILE - 1) / COMPACT_TILE;
    if (ntiles <= 0) return ZBPE_OK;
    CHECK(ensure(&d_tile_cnt, tile_cnt_cap, ntiles, "compaction tiles"));
    CHECK(ensure(&d_tile_off, tile_off_cap, ntiles + 1, "compaction offsets"));
    uint16_t *src = d_tok[cur], *dst = d_tok[cur ^ 1];
    zbpe_compact_count<<<ntiles, 256, 0, stream>>>(src, n_slots, d_tile_cnt);
    LAUNCH_OK();
    zbpe_scan_u32<<<1, 1024, 0, stream>>>(d_tile_cnt, ntiles, d_tile_off, d_tile_off + ntiles);
    LAUNCH_OK();
    zbpe_compact_scatter<<<ntiles, 256, 0, stream>>>(src, n_slots, d_tile_off, dst);
    LAUNCH_OK();
    HIP_OK(hipMemcpyAsync(total, d_tile_off + ntiles, 8, hipMemcpyDeviceToHost, stream));
    HIP_OK(hipStreamSynchronize(stream));
    return ZBPE_OK;
}

// Diagnostic download of the live token stream (holes squeezed out) into the spare stream buffer,
// leaving the current buffer, its holes and the occurrence lists as they are. out == nullptr or a
// short cap: only *n_tokens.
zbpe_status Engine::tokens(uint16_t *out, size_t cap, size_t *n_tokens) {
    if (!stream_ready && !trained && n_slots == 0) { *n_tokens = 0; return ZBPE_OK; }
    HIP_OK(hipSetDevice(device));
    uint64_t total = 0;
    CHECK(compact_to_spare(&total));
    *n_tokens = (size_t)total;
    if (out && cap >= total && total) {
        HIP_OK(hipMemcpyAsync(out, d_tok[cur ^ 1], (size_t)total * 2, hipMemcpyDeviceToHost, stream));
        HIP_OK(hipStreamSynchronize(stream));
    }
    return ZBPE_OK;
}

// Full recount of the current stream against the incremental table. Multi-GPU: each shard
// recounts the pairs it owns; ids differ between ranks but the key sets are identical, so the
// per-rank recounts line up in key order and one all-reduce sums them.
// option batch_checks (diagnostics): the pair table against a full recount of the stream after merges [x0, x1)
zbpe_status Engine::table_check(uint32_t x0, uint32_t x1, const char *what) {
    uint64_t bad = 0;
    uint32_t info[3] = {0, 0, 0};
    CHECK(recount_check(&bad, info));
    if (bad || h_st->error)
        return fail(ZBPE_INTERNAL, "after the %s of merges [%u, %u): %llu pair counts differ from a full recount (first: key (%u,%u) "
                                   "table %u, recount %u), error flags 0x%x",
                    what, x0, x1, (unsigned long long)bad, info[0] & 0xFFFF, info[0] >> 16, info[1], info[2], h_st->error);
    return ZBPE_OK;
}
zbpe_status Engine::recount_check(uint64_t *mismatches, uint32_t *first_bad_key) {
    HIP_OK(hipSetDevice(device));
    CHECK(sync_state());
    const uint32_t nid = h_st->num_ids;
    CHECK(ensure(&d_recount, recount_cap, std::max<uint32_t>(nid, 1), "recount"));
    HIP_OK(hipMemsetAsync(d_recount, 0, (size_t)std::max<uint32_t>(nid, 1) * 4, stream));
    HIP_OK(hipMemsetAsync(&d_st->mismatches, 0, 4, stream));
    uint64_t total = 0;
    CHECK(compact_to_spare(&total));
    CHECK(launch_pair_hist(total));
    if (!dist()) {
        zbpe_recount_compare<<<std::min<uint32_t>(4096, nid / 256 + 1), 256, 0, stream>>>(T, d_recount, d_st);
        LAUNCH_OK();
        CHECK(sync_state());
        *mismatches = h_st->mismatches;
        return ZBPE_OK;
    }
    uint32_t *d_dump = nullptr;
    HIP_OK(dev_alloc(&d_dump, (size_t)nid * 12 + 16));
    zbpe_recount_dump<<<std::min<uint32_t>(4096, nid / 256 + 1), 256, 0, stream>>>(T, d_recount, d_st, d_dump);
    LAUNCH_OK();
    std::vector<uint32_t> dump((size_t)nid * 3);
    HIP_OK(hipMemcpyAsync(dump.data(), d_dump, (size_t)nid * 12, hipMemcpyDeviceToHost, stream));
    HIP_OK(hipStreamSynchronize(stream));
    std::vector<uint32_t> order(nid);
    for (uint32_t i = 0; i < nid; i++) order[i] = i;
    std::sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) { return dump[3 * x] < dump[3 * y]; });
    std::vector<uint32_t> rc(nid + 1);
    for (uint32_t i = 0; i < nid; i++) rc[i] = dump[3 * order[i] + 2];
    rc[nid] = h_st->mismatches;
    HIP_OK(hipMemcpyAsync(d_dump, rc.data(), (size_t)(nid + 1) * 4, hipMemcpyHostToDevice, stream));
    if (!comm->allreduce_u32(d_dump, nid + 1, COMM_SUM_U32, stream)) { (void)hipFree(d_dump); return fail(ZBPE_COMM_ERROR, "recount all-reduce failed"); }
    HIP_OK(hipMemcpyAsync(rc.data(), d_dump, (size_t)(nid + 1) * 4, hipMemcpyDeviceToHost, stream));
    HIP_OK(hipStreamSynchronize(stream));
    (void)hipFree(d_dump);
    uint64_t bad = rc[nid];
    for (uint32_t i = 0; i < nid; i++) {
        const uint32_t id = order[i];
        if (rc[i] != dump[3 * id + 1]) {
            if (!bad && first_bad_key) { first_bad_key[0] = dump[3 * id]; first_bad_key[1] = dump[3 * id + 1]; first_bad_key[2] = rc[i]; }
            bad++;
        }
    }
    *mismatches = bad;
    return ZBPE_OK;
}

// the full pair histogram (zbpe_pair_hist) of the compacted stream in the spare buffer into d_recount
zbpe_status Engine::launch_pair_hist(uint64_t total) {
    const int32_t next_tok = dist() && halo.nright > 0 ? (int32_t)halo_right(halo, 0) : -1;  // the pair leaving the shard
    // a stream of bytes (no merge yet on this context): every byte pair in a fixed 16-bit LDS bin
    if (run.merges == 0 && dense_hist && (next_tok < 256))  // (next_tok: a byte or -1)
        zbpe_pair_hist_bytes<<<std::max(1, num_cus), PH_THREADS, 32768 * 4, stream>>>(d_tok[cur ^ 1], (int64_t)total, next_tok, T,
                                                                                       d_recount, d_st);
    else
        zbpe_pair_hist<<<std::max(1, num_cus), PH_THREADS, PH_SLOTS * 8, stream>>>(d_tok[cur ^ 1], (int64_t)total, next_tok, T,
                                                                                    d_recount, d_st);
    LAUNCH_OK();
    return ZBPE_OK;
}

// Benchmark diagnostic: `reps` launches of the full pair histogram over the current stream (compacted
// into the spare buffer first, untimed), HIP events around each launch; checks the last one against the
// incremental counts.
zbpe_status Engine::bench_recount(int reps, double *avg_us, double *gbps, uint64_t *n_tokens, uint64_t *mismatches) {
    if (!trained) return fail(ZBPE_INVALID_ARGUMENT, "bench_recount needs a trained context");
    if (dist()) return fail(ZBPE_INVALID_ARGUMENT, "bench_recount is a single-GPU diagnostic");
    HIP_OK(hipSetDevice(device));
    CHECK(sync_state());
    const uint32_t nid = h_st->num_ids;
    CHECK(ensure(&d_recount, recount_cap, std::max<uint32_t>(nid, 1), "recount"));
    uint64_t total = 0;
    CHECK(compact_to_spare(&total));
    double sum = 0;
    for (int r = 0; r <= reps; r++) {
        HIP_OK(hipMemsetAsync(d_recount, 0, (size_t)std::max<uint32_t>(nid, 1) * 4, stream));
        HIP_OK(hipMemsetAsync(&d_st->mismatches, 0, 4, stream));
        HIP_OK(hipEventRecord(ev[0], stream));
        CHECK(launch_pair_hist(total));
        HIP_OK(hipEventRecord(ev[1], stream));
        HIP_OK(hipEventSynchronize(ev[1]));
        float ms;
        HIP_OK(hipEventElapsedTime(&ms, ev[0], ev[1]));
        if (r) sum += ms;  // the first launch warms up
    }
    zbpe_recount_compare<<<std::min<uint32_t>(4096, nid / 256 + 1), 256, 0, stream>>>(T, d_recount, d_st);
    LAUNCH_OK();
    CHECK(sync_state());
    *mismatches = h_st->mismatches;
    *avg_us = reps ? sum * 1e3 / reps : 0;
    *gbps = *avg_us > 0 ? 2.0 * (double)total / (*avg_us * 1e-6) / 1e9 : 0;
    *n_tokens = total;
    return ZBPE_OK;
}

// encode (basic_tokenizer.zig:71-88): replay merges in rank order on the device
zbpe_status Engine::encode(const uint16_t *triples_in, size_t n_merges, const uint8_t *text, size_t n, uint16_t *out,
                           size_t *out_len) {
    // Token 65535 is the stream's hole marker on the device. A merge table may still hold it (the reference
    // parses any u16, deserializeMerges :342-344; a trained table never does: vocabSize is a u16, so new
    // tokens stop at 65534): the table is encoded with 65535 renamed to a token id that no merge uses (it
    // can then neither be in the input -- bytes are < 256 -- nor come from another merge, so the result is
    // the same up to the name) and renamed back in the output.
    const uint16_t *triples = triples_in;
    std::vector<uint16_t> renamed;
    uint32_t alias = 0;
    {
        bool uses_hole = false;
        for (size_t i = 0; i < 3 * n_merges && !uses_hole; i++) uses_hole = triples_in[i] == HOLE;
        if (uses_hole) {
            std::vector<uint8_t> used(65536, 0);
            for (size_t i = 0; i < 3 * n_merges; i++) used[triples_in[i]] = 1;
            for (uint32_t t = 256; t < HOLE && !alias; t++)
                if (!used[t]) alias = t;
            if (!alias) return fail(ZBPE_INVALID_ARGUMENT, "merge table uses every token id 256..65535: no id to stand for 65535");
            renamed.assign(triples_in, triples_in + 3 * n_merges);
            for (auto &t : renamed)
                if (t == HOLE) t = (uint16_t)alias;
            triples = renamed.data();
        }
    }
    CHECK(upload(text, n, false));
    trained = false;
    CHECK(generate_initial_tokens(n));
    HIP_OK(hipMemsetAsync(d_st, 0, sizeof(DevState), stream));
    // token occurrence lists (as in train): a merge's scan walks the shorter of its tokens' lists
    // when that is short; every merge's records become the list of its new token. Needs distinct
    // new tokens that are not bytes (they would overwrite a list) and vocab ids that fit the build.
    uint32_t max_tok = 255;
    bool distinct = true;
    {
        std::vector<uint8_t> seen(65536, 0);
        for (size_t k = 0; k < n_merges; k++) {
            const uint32_t X = triples[3 * k + 2];
            max_tok = std::max<uint32_t>(max_tok, std::max<uint32_t>(X, std::max(triples[3 * k], triples[3 * k + 1])));
            if (X < 256 || seen[X] || X == triples[3 * k]) distinct = false;  // (X == first would overwrite first's list)
            seen[X] = 1;
        }
    }
    const uint32_t vp = (max_tok + 1 + 63) & ~63u;
    const bool use_lists = list_mode && distinct && vp <= PRES_MAX_VP && n < 0x70000000u && n_merges > 0;
    pres_on = false;
    if (use_lists) {
        CHECK(ensure(&d_lists, lists_cap, 2 * n + 1024, "occurrence arena"));  // lists <= n, records <= n
        pres_vp = vp;
        CHECK(build_lists(256, enc_list_ratio));  // the byte tokens exist at the build; every merge makes a new token >= 256
    } else {
        lists_on = false;
        CHECK(ensure(&d_rec, rec_cap, std::max<size_t>(n / 2 + 1, 1), "occurrence records"));
    }
    uint32_t *recbuf = use_lists ? d_lists : d_rec;
    const uint32_t reccap = (uint32_t)(use_lists ? lists_cap : rec_cap);
    uint32_t *tail = d_delta + DELTA_WORDS - 32;  // scratch: encode keeps no counts
    uint64_t holes = 0;
    // batched path (with lists): live token counts (exact after the list build of the fresh stream),
    // one record counter per merge of a batch, a scratch region of n records
    const bool batched = use_lists && enc_batch > 1;
    if (batched) {
        CHECK(ensure(&d_rec, rec_cap, (size_t)n + 1, "encode scratch"));
        CHECK(ensure(&d_enc_cnt, enc_cnt_cap, 65536, "token counts"));
        CHECK(ensure(&d_enc_ctr, enc_ctr_cap, ENC_MAX_BATCH, "batch counters"));
        HIP_OK(hipMemsetAsync(d_enc_cnt, 0, 65536 * sizeof(int32_t), stream));
        HIP_OK(hipMemcpyAsync(d_enc_cnt, d_list_total, vp * sizeof(uint32_t), hipMemcpyDeviceToDevice, stream));
        HIP_OK(hipMemsetAsync(d_enc_ctr, 0, ENC_MAX_BATCH * sizeof(uint32_t), stream));
    }
    const uint32_t maxb = std::min<uint32_t>(enc_batch, ENC_MAX_BATCH);
    enc_batches = 0;
    for (size_t k = 0; k < n_merges;) {
        if (batched && triples[3 * k] != triples[3 * k + 1]) {
            // greedy batch: the next merges while none uses a token an earlier one of the batch uses or makes
            EncBatch E{};
            uint32_t used[3 * ENC_MAX_BATCH];
            uint32_t nused = 0;
            auto is_used = [&](uint32_t t) { return std::find(used, used + nused, t) != used + nused; };
            while (k < n_merges && E.nb < maxb) {
                const uint32_t a = triples[3 * k], b = triples[3 * k + 1], X = triples[3 * k + 2];
                if (a == b || is_used(a) || is_used(b)) break;
                E.a[E.nb] = a;
                E.b[E.nb] = b;
                E.X[E.nb] = X;
                E.nb++;
                used[nused++] = a;
                used[nused++] = b;
                used[nused++] = X;
                k++;
            }
            ScanArgs A{d_tok[cur], n_slots, 0, 0, d_delta, d_delta + 65536, d_st, d_rec, 0, 0, tail, tail + 1, Halo{},
                       nullptr, vp, 0, nullptr, 0, nullptr, d_lists, T.lst_off, T.lst_len, enc_list_ratio, 0, nullptr};
            set_list_nb(A);
            hipLaunchKernelGGL(zbpe_encode_scan_batch, dim3(scan_grid(n_slots), E.nb), dim3(SCAN_THREADS), 0, stream, A, E,
                               (const int32_t *)d_enc_cnt, d_enc_ctr, d_rec);
            LAUNCH_OK();
            zbpe_encode_apply_batch<<<dim3(std::max<uint32_t>(8, 512 / E.nb), E.nb), 256, 0, stream>>>(
                d_tok[cur], n_slots, E, d_rec, d_enc_cnt, d_enc_ctr, d_lists, d_st, T);
            LAUNCH_OK();
            enc_batches++;
            continue;
        }
        const uint32_t a = triples[3 * k], b = triples[3 * k + 1], X = triples[3 * k + 2];
        k++;
        // X == a: the reference re-tests position i after a merge there (it does not advance), so an a
        // absorbs the whole run of b's after it (a == b: a run of a's collapses to one a). Each pass
        // of the merge below absorbs one b per a (halves an a-run): repeat until a pass finds none.
        const bool chain = X == a;
        uint64_t occ_seen = 0;
        if (chain) {
            CHECK(sync_state());
            occ_seen = h_st->total_occ;
        }
        for (;;) {
        ScanArgs A{d_tok[cur], n_slots, a, b, d_delta, d_delta + 65536, d_st, recbuf, reccap, 0, tail, tail + 1, Halo{},
                   nullptr, vp, X, nullptr, 0, nullptr, use_lists ? d_lists : nullptr, T.lst_off, T.lst_len, enc_list_ratio,
                   use_lists ? 1 : 0, nullptr};
        set_list_nb(A);
        if (a != b) {
            CHECK(launch_scan(A));
        } else if (use_lists && self_list_ok(a, false)) {
            zbpe_scan_self_list<<<scan_grid(n_slots), SCAN_THREADS, 0, stream>>>(A);
            LAUNCH_OK();
        } else {  // holes are transparent to the self-pair path
            const int64_t ntiles = std::max<int64_t>(1, (n_slots + SELF_TILE - 1) / SELF_TILE);
            CHECK(ensure(&d_tile_fn, tile_fn_cap, ntiles, "self tiles"));
            CHECK(ensure(&d_carry, carry_cap, ntiles, "self carry"));
            zbpe_self_tiles<<<ntiles, SELF_THREADS, 0, stream>>>(d_tok[cur], n_slots, a, d_tile_fn);
            LAUNCH_OK();
            zbpe_self_carry<<<1, 1024, 0, stream>>>(d_tile_fn, ntiles, d_carry, nullptr, nullptr);
            LAUNCH_OK();
            zbpe_scan_self<<<std::min(ntiles, SELF_GRID), SELF_THREADS, 0, stream>>>(A, d_carry);
            LAUNCH_OK();
        }
        zbpe_encode_apply<<<512, 256, 0, stream>>>(d_tok[cur], n_slots, recbuf, reccap, use_lists ? 1 : 0, X, d_st, T, tail,
                                                   batched ? d_enc_cnt : nullptr, a, b);
        LAUNCH_OK();
        enc_batches++;
        if (!chain) break;
        CHECK(sync_state());
        if (h_st->total_occ == occ_seen) break;
        occ_seen = h_st->total_occ;
        }
        if (!use_lists && (k & 255) == 0) {  // without lists: squeeze the holes now and then
            CHECK(sync_state());
            holes += h_st->total_occ;
            n_live -= h_st->total_occ;
            HIP_OK(hipMemsetAsync(&d_st->total_occ, 0, 4, stream));
            if (holes * compact_den > (uint64_t)n_slots) { CHECK(compact()); holes = 0; }
        }
    }
    CHECK(sync_state());
    n_live -= h_st->total_occ;
    HIP_OK(hipMemsetAsync(&d_st->total_occ, 0, 4, stream));
    CHECK(compact());
    // the engine stream is non-blocking: copy on it (a null-stream hipMemcpy would not wait for compact())
    if (n_live) HIP_OK(hipMemcpyAsync(out, d_tok[cur], (size_t)n_live * 2, hipMemcpyDeviceToHost, stream));
    HIP_OK(hipStreamSynchronize(stream));
    *out_len = (size_t)n_live;
    if (alias)
        for (int64_t i = 0; i < n_live; i++)
            if (out[i] == alias) out[i] = HOLE;
    return ZBPE_OK;
}

}  // namespace zbpe

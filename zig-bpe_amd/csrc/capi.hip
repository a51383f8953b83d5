// extern "C" entry points declared in include/zbpe.h.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <new>

#include "engine.hpp"
#include "zig_order.hpp"
#include <vector>
#include <string>

struct zbpe_ctx {
    zbpe::Engine eng;
};

static const char *env_or(const char *k) { const char *v = getenv(k); return v && *v ? v : nullptr; }

extern "C" {

const char *zbpe_version(void) { return "zbpe-mi355x 0.3 (gfx950, zbpe_stats v3)"; }

size_t zbpe_stats_size(void) { return sizeof(zbpe_stats); }

zbpe_status zbpe_create(int device, zbpe_ctx **out) {
    if (!out) return ZBPE_INVALID_ARGUMENT;
    *out = nullptr;
    zbpe_ctx *c = new (std::nothrow) zbpe_ctx();
    if (!c) return ZBPE_OUT_OF_MEMORY;
    zbpe_status s = c->eng.init(device);
    if (s != ZBPE_OK) {
        *out = c;  // keep it so zbpe_last_error() can report; caller destroys
        return s;
    }
    if (env_or("ZBPE_DEBUG")) c->eng.debug_checks = true;
    if (env_or("ZBPE_EXACT_TIES")) c->eng.force_exact_ties = true;
    if (env_or("ZBPE_TIE_PROF")) c->eng.tie_prof = true;
    if (const char *v = env_or("ZBPE_COMPACT_DEN")) c->eng.compact_den = strtoull(v, nullptr, 10);
    if (const char *v = env_or("ZBPE_SCAN_BLOCKS_PER_CU")) c->eng.scan_blocks_per_cu = atoi(v);
    *out = c;
    return ZBPE_OK;
}

zbpe_status zbpe_comm_unique_id(void *out128) {
    if (!out128) return ZBPE_INVALID_ARGUMENT;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return ZBPE_COMM_ERROR;
    memcpy(out128, &id, sizeof(id));
    return ZBPE_OK;
}

static zbpe_status finish_dist(zbpe_ctx *c, int rank, int world, std::unique_ptr<zbpe::Comm> comm, zbpe_ctx **out) {
    zbpe_status s = c->eng.init_dist(rank, world, std::move(comm));
    *out = c;
    return s;
}

zbpe_status zbpe_create_dist(int device, int rank, int world, const void *unique_id128, zbpe_ctx **out) {
    if (!out || world < 1 || rank < 0 || rank >= world || (world > 1 && !unique_id128)) return ZBPE_INVALID_ARGUMENT;
    zbpe_status s = zbpe_create(device, out);
    if (s != ZBPE_OK || (world == 1 && !unique_id128)) return s;
    auto comm = std::make_unique<zbpe::RcclComm>();
    if (!comm->init(rank, world, unique_id128)) return (*out)->eng.fail(ZBPE_COMM_ERROR, "ncclCommInitRank failed (rank %d of %d)", rank, world);
    (*out)->eng.force_shard = world == 1;  // a one-rank communicator: the sharded path, over one rank
    return finish_dist(*out, rank, world, std::move(comm), out);
}

zbpe_status zbpe_create_dist_host(int device, int rank, int world, zbpe_collective_fn fn, void *user, zbpe_ctx **out) {
    if (!out || !fn || world < 1 || rank < 0 || rank >= world) return ZBPE_INVALID_ARGUMENT;
    zbpe_status s = zbpe_create(device, out);
    if (s != ZBPE_OK) return s;
    auto comm = std::make_unique<zbpe::HostComm>();
    comm->fn = fn;
    comm->user = user;
    comm->rank = rank;
    comm->world = world;
    (*out)->eng.force_shard = world == 1;
    return finish_dist(*out, rank, world, std::move(comm), out);
}

void zbpe_destroy(zbpe_ctx *ctx) { delete ctx; }

const char *zbpe_last_error(const zbpe_ctx *ctx) { return ctx ? ctx->eng.err.c_str() : "null context"; }

zbpe_status zbpe_upload(zbpe_ctx *ctx, const uint8_t *text, size_t n) {
    if (!ctx || (!text && n)) return ZBPE_INVALID_ARGUMENT;
    return ctx->eng.upload(text, n, ctx->eng.multi());
}

zbpe_status zbpe_train_resident(zbpe_ctx *ctx, uint16_t vocab_size, int verbose, uint16_t *out_triples,
                                uint64_t *out_counts, size_t *out_n_merges, zbpe_stats *stats) {
    if (!ctx || !out_n_merges || (!out_triples && vocab_size > 256)) return ZBPE_INVALID_ARGUMENT;
    return ctx->eng.train(vocab_size, verbose, out_triples, out_counts, out_n_merges, stats);
}

zbpe_status zbpe_train(zbpe_ctx *ctx, const uint8_t *text, size_t n, uint16_t vocab_size, int verbose,
                       uint16_t *out_triples, uint64_t *out_counts, size_t *out_n_merges, zbpe_stats *stats) {
    if (!ctx || !out_n_merges || (!text && n)) return ZBPE_INVALID_ARGUMENT;
    *out_n_merges = 0;
    if (vocab_size < 256) return ctx->eng.fail(ZBPE_INVALID_VOCAB_SIZE, "vocabSize %u < 256", vocab_size);
    zbpe_status s = ctx->eng.upload(text, n, ctx->eng.multi());
    if (s != ZBPE_OK) return s;
    return zbpe_train_resident(ctx, vocab_size, verbose, out_triples, out_counts, out_n_merges, stats);
}

zbpe_status zbpe_encode(zbpe_ctx *ctx, const uint16_t *triples, size_t n_merges, const uint8_t *text, size_t n,
                        uint16_t *out, size_t *out_len) {
    if (!ctx || !out_len || (!text && n) || (!triples && n_merges) || (!out && n)) return ZBPE_INVALID_ARGUMENT;
    return ctx->eng.encode(triples, n_merges, text, n, out, out_len);
}

zbpe_status zbpe_verify_counts(zbpe_ctx *ctx, uint64_t *mismatches) {
    if (!ctx || !mismatches) return ZBPE_INVALID_ARGUMENT;
    return ctx->eng.verify_counts(mismatches);
}

zbpe_status zbpe_tokens(zbpe_ctx *ctx, uint16_t *out, size_t cap, size_t *n_tokens) {
    if (!ctx || !n_tokens || (!out && cap)) return ZBPE_INVALID_ARGUMENT;
    return ctx->eng.tokens(out, cap, n_tokens);
}

zbpe_status zbpe_set_option(zbpe_ctx *ctx, const char *name, int64_t value) {
    if (!ctx || !name) return ZBPE_INVALID_ARGUMENT;
    std::string k(name);
    zbpe::Engine &e = ctx->eng;
    if (k == "debug_checks") e.debug_checks = value != 0;
    else if (k == "batch_checks" && value >= 0 && value < 65536) e.batch_checks = value ? (uint32_t)value + 256 : 0u;
    else if (k == "exact_ties") e.force_exact_ties = value != 0;
    else if (k == "exact_ties_from" && value >= 0 && value < 65536) e.exact_lo = (uint32_t)value + 256;
    else if (k == "exact_ties_to" && value >= 0 && value < 65536) e.exact_hi = (uint32_t)value + 256;
    else if (k == "compact_den" && value > 0) e.compact_den = (uint64_t)value;
    else if (k == "compact_den_walks" && value > 0) e.compact_den_walks = (uint64_t)value;
    else if (k == "scan_blocks_per_cu" && value > 0) e.scan_blocks_per_cu = (int)value;
    else if (k == "scan_variant") return e.set_scan_variant((int)value);
    else if (k == "scan_batch") {
        if (value < 0 || value > 2) return e.fail(ZBPE_INVALID_ARGUMENT, "scan_batch is 0, 1 or 2");
        e.scan_batch = (int)value;
    }
    else if (k == "list_ranges") e.list_ranges = value != 0;
    else if (k == "scan_plan") e.scan_plan = value != 0;
    else if (k == "range_min_len" && value >= 1 && value < (1ll << 32)) e.range_min_len = (uint32_t)value;
    else if (k == "range_max_rows" && value >= 0 && value <= 65536) e.range_max_rows = (uint32_t)value;
    else if (k == "range_max_len" && value >= 1 && value < (1ll << 32)) e.range_max_len = (uint32_t)value;
    else if (k == "block_skip") e.block_skip = value != 0;
    else if (k == "trace") e.trace_on = value != 0;
    else if (k == "merge_batch" && value >= 1) e.merge_batch = (uint32_t)std::min<int64_t>(value, zbpe::MAX_BATCH);
    else if (k == "merge_timing" && value >= 0) e.merge_timing = (uint32_t)value;
    else if (k == "sel_prof" && value >= 0) e.sel_prof = (uint32_t)value;
    else if (k == "timing_full") e.timing_full = value != 0;
    else if (k == "list_nb") e.list_nb = value != 0;
    else if (k == "arena_cap" && value >= 0) e.arena_cap_opt = (uint64_t)value;
    else if (k == "replace_split") e.replace_split = value != 0;
    else if (k == "fused_select") e.fused_select = value != 0;
    else if (k == "refresh_prefix") e.refresh_prefix = value != 0;
    else if (k == "replicate_late") e.replicate_late = value != 0;
    else if (k == "handover" && value >= 1 && value <= 3) e.handover = (int)value;
    else if (k == "list_mode" && value >= 0 && value <= 1) e.list_mode = (int)value;
    else if (k == "compact_den_lists" && value >= 1) e.compact_den_lists = (uint64_t)value;
    else if (k == "list_grid" && value >= 0) e.list_grid = (int)value;
    else if (k == "list_ratio" && value >= 1) e.list_ratio = (uint32_t)value;
    else if (k == "dense_hist" && (value == 0 || value == 1)) e.dense_hist = (int)value;
    else if (k == "refresh_wgs" && value >= 0) e.refresh_wgs = (uint32_t)value;
    else if (k == "lp_lazy" && (value == 0 || value == 1)) e.lp_lazy = (int)value;
    else if (k == "pair_select" && (value == 0 || value == 1)) e.pair_select = (int)value;
    else if (k == "pair_refresh" && (value == 0 || value == 1)) e.pair_refresh = (int)value;
    else if (k == "pair_m3w" && (value == 0 || value == 1)) e.pair_m3w = (int)value;
    else if (k == "pair_chain" && value >= 0 && value <= 3) e.pair_chain = (int)value;
    else if (k == "round_k" && value >= 1 && value <= zbpe::ROUND_MAX) e.round_k = (int)value;
    else if (k == "round_ties" && value >= 0 && value <= 100) e.round_ties = (uint32_t)value;
    else if (k == "round_untied" && (value == 0 || value == 1)) e.round_untied = (int)value;
    else if (k == "round_streak" && (value == 0 || value == 1)) e.round_streak = (int)value;
    else if (k == "encode_list_ratio" && value >= 1) e.enc_list_ratio = (uint32_t)value;
    else if (k == "list_start" && value >= 0) e.list_start = (uint64_t)value;
    else if (k == "hot_target" && value > 0) e.hot_target = (uint64_t)value;
    else if (k == "sel_growth" && value >= 0) e.sel_growth = (uint32_t)value;
    else if (k == "sel_margin" && value >= 0 && value < (1ll << 31)) e.sel_margin = (uint32_t)value;
    else if (k == "print_runtime") e.print_runtime = value != 0;
    else if (k == "encode_batch" && value >= 1) e.enc_batch = (uint32_t)value;
    else if (k == "self_list_ratio" && value >= 0) e.self_list_ratio = (uint32_t)value;
    else if (k == "self_batch" && (value == 0 || value == 1)) e.self_batch = (int)value;
    else return e.fail(ZBPE_INVALID_ARGUMENT, "unknown option %s", name);
    return ZBPE_OK;
}

// printTimeStats (time_statistics.zig:36-60): the reference's lines for the GPU buckets. The device
// never materialises the pair array (the scan reads pairs in place), so generateCodePointPairs takes
// 0 s over the count calls.
zbpe_status zbpe_format_time_stats(const zbpe_stats *st, char *buf, size_t cap, size_t *len) {
    if (!st || !len || (!buf && cap)) return ZBPE_INVALID_ARGUMENT;
    std::string out = "\nTime statistics:\n";
    auto line = [&](const char *name, double t, uint64_t calls) {
        char b[256], avg[64];
        if (calls) snprintf(avg, sizeof avg, "%.3f", t / (double)calls);
        else snprintf(avg, sizeof avg, "nan");  // Zig prints 0.0 / 0.0 as nan
        snprintf(b, sizeof b, "%s: %.3fs total, %llu calls, %ss avg\n", name, t, (unsigned long long)calls, avg);
        out += b;
    };
    line("sortCodePointPairs", st->sort_pairs_s, st->sort_pairs_calls);
    line("replaceTopPairWithIndex", st->replace_pair_s, st->replace_pair_calls);
    line("generateCodePointPairs", 0.0, st->count_pairs_calls);
    line("countPointPairs", st->count_pairs_s, st->count_pairs_calls);
    char b[128];
    snprintf(b, sizeof b, "Other operations: %.3fs\n",
             st->total_s - st->sort_pairs_s - st->replace_pair_s - st->count_pairs_s);
    out += b;
    *len = out.size();
    if (buf && cap) {
        const size_t k = std::min(cap - 1, out.size());
        memcpy(buf, out.data(), k);
        buf[k] = 0;
    }
    return ZBPE_OK;
}

zbpe_status zbpe_bench_scan(zbpe_ctx *ctx, uint16_t a, uint16_t b, int reps, double *avg_ms, double *gbps) {
    if (!ctx || !avg_ms || !gbps || reps < 1 || a == b) return ZBPE_INVALID_ARGUMENT;
    return ctx->eng.bench_scan(a, b, reps, avg_ms, gbps);
}

zbpe_status zbpe_bench_train_scan(zbpe_ctx *ctx, int reps, int grid, double *avg_us, uint32_t *pair, uint32_t *list_len,
                                  int *mode) {
    if (!ctx || !avg_us || !pair || !list_len || !mode || reps < 0 || grid < 0) return ZBPE_INVALID_ARGUMENT;
    return ctx->eng.bench_train_scan(reps, grid, avg_us, pair, list_len, mode);
}

zbpe_status zbpe_bench_recount(zbpe_ctx *ctx, int reps, double *avg_us, double *gbps, uint64_t *n_tokens,
                               uint64_t *mismatches) {
    if (!ctx || !avg_us || !gbps || !n_tokens || !mismatches || reps < 0) return ZBPE_INVALID_ARGUMENT;
    return ctx->eng.bench_recount(reps, avg_us, gbps, n_tokens, mismatches);
}

zbpe_status zbpe_merge_log(zbpe_ctx *ctx, uint32_t *rows, size_t cap_rows, size_t *n_rows) {
    if (!ctx || !n_rows || (!rows && cap_rows)) return ZBPE_INVALID_ARGUMENT;
    const auto &L = ctx->eng.h_log;
    *n_rows = std::min(ctx->eng.run.merges, L.size());
    const size_t k = std::min(cap_rows, *n_rows);
    for (size_t i = 0; i < k; i++) {
        const zbpe::MergeLog &m = L[i];
        const uint32_t r[ZBPE_MERGE_LOG_COLS] = {m.key, m.count, m.live, m.ties, m.mode, m.list_len, m.key_live, m.range};
        memcpy(rows + i * ZBPE_MERGE_LOG_COLS, r, sizeof r);
    }
    return ZBPE_OK;
}

zbpe_status zbpe_trace(zbpe_ctx *ctx, float *rows, size_t cap_rows, size_t *n_rows) {
    if (!ctx || !n_rows || (!rows && cap_rows)) return ZBPE_INVALID_ARGUMENT;
    const auto &t = ctx->eng.trace;
    *n_rows = t.size() / ZBPE_TRACE_COLS;
    const size_t k = std::min(cap_rows, *n_rows);
    if (k) memcpy(rows, t.data(), k * ZBPE_TRACE_COLS * sizeof(float));
    return ZBPE_OK;
}

zbpe_status zbpe_scan_log(zbpe_ctx *ctx, int32_t *out, size_t cap, size_t *n) {
    if (!ctx || !n || (!out && cap)) return ZBPE_INVALID_ARGUMENT;
    const auto &l = ctx->eng.scan_log;
    *n = l.size();
    const size_t k = std::min(cap, *n);
    if (k) memcpy(out, l.data(), k * sizeof(int32_t));
    return ZBPE_OK;
}

zbpe_status zbpe_compaction_log(zbpe_ctx *ctx, uint32_t *rows, size_t cap_rows, size_t *n_rows) {
    if (!ctx || !n_rows || (!rows && cap_rows)) return ZBPE_INVALID_ARGUMENT;
    const auto &l = ctx->eng.compact_log;
    *n_rows = l.size() / 2;
    const size_t k = std::min(cap_rows, *n_rows);
    if (k) memcpy(rows, l.data(), k * 2 * sizeof(uint32_t));
    return ZBPE_OK;
}

zbpe_status zbpe_halt_log(zbpe_ctx *ctx, uint32_t *rows, size_t cap_rows, size_t *n_rows) {
    if (!ctx || !n_rows || (!rows && cap_rows)) return ZBPE_INVALID_ARGUMENT;
    const auto &l = ctx->eng.halt_log;
    *n_rows = l.size() / 3;
    const size_t k = std::min(cap_rows, *n_rows);
    if (k) memcpy(rows, l.data(), k * 3 * sizeof(uint32_t));
    return ZBPE_OK;
}

zbpe_status zbpe_zig_order_winner(const uint32_t *first_pos, const uint32_t *keys, const uint32_t *counts, size_t n,
                                  uint32_t top, int call_after_last_insert, uint32_t *winner) {
    if ((!first_pos || !keys || !counts) && n) return ZBPE_INVALID_ARGUMENT;
    if (!winner) return ZBPE_INVALID_ARGUMENT;
    std::vector<zbpe::ZigOrderInput> in(n);
    for (size_t i = 0; i < n; i++) in[i] = zbpe::ZigOrderInput{(uint64_t)first_pos[i], keys[i], counts[i]};
    return zbpe::zig_order_winner(std::move(in), top, call_after_last_insert != 0, winner) ? ZBPE_OK : ZBPE_INTERNAL;
}

}  // extern "C"

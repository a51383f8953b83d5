// Engine: one MI355X, one process. See engine.hip for the per-merge launch sequence.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <memory>
#include <string>
#include <vector>

#include "../../include/zbpe.h"
#include "comm.hpp"
#include "types.hpp"
#include "zig_order.hpp"

namespace zbpe { struct ScanArgs; }

namespace zbpe {

constexpr int ARGMAX_MAX_BLOCKS = 1024;
constexpr size_t DELTA_WORDS = 2 * 65536 + 64;  // left | right | xx | occurrences (+ scratch)
constexpr uint32_t MAX_BATCH = 256;              // merges per device-resident batch (option "merge_batch")
constexpr uint32_t BEV_PER_MERGE = 6;  // events of a timed batch merge: start, begun, scanned, exchanged, replaced, selected
constexpr uint32_t PRES_MAX_VP = 32768;          // presence bitset of a block group fits one workgroup LDS (128 KiB)

struct Engine {
    int device = 0;
    int num_cus = 256;
    hipStream_t stream = nullptr;
    std::string err;

    // corpus (this rank's shard) and token stream
    uint8_t *d_text = nullptr;
    size_t text_cap = 0, n_text = 0;
    bool uploaded = false, trained = false, stream_ready = false;
    int scan_variant = 0;
    int scan_batch = 1;  // ScanArgs::batch of stream-form launches (option scan_batch)
    uint16_t *d_tok[2] = {nullptr, nullptr};
    size_t tok_cap0 = 0, tok_cap1 = 0;
    int cur = 0;
    int64_t n_slots = 0;  // live tokens + holes
    int64_t n_live = 0;

    // pair table and per-merge scratch
    Tables T{};
    // per-merge neighbour deltas, two buffers of DELTA_WORDS: merge X uses delta_of(X) (a select may then
    // scan merge X + 1 into the other buffer while its own merge's words are still being cleared)
    uint32_t *d_delta = nullptr, *d_hist = nullptr;
    uint32_t *delta_of(uint32_t X) const { return d_delta + (size_t)(X & 1) * DELTA_WORDS; }
    // multi-merge rounds (option round_k): the members' delta buffers (ROUND_MAX of
    // DELTA_WORDS, fixed layout: left at +0, right at +65536, tail at +131072), the rounds' log of a batch
    // (d_rlog[i] = the first merge of launch i's round | members << 16), the refresh counters' parity of the
    // next round select and a launch id (ref_noprefix) that no merge index equals
    uint32_t *d_rdelta = nullptr, *d_rlog = nullptr;
    std::vector<uint32_t> h_rlog;
    uint32_t rpar = 0, launch_seq = 1u << 20;
    bool last_rounds = false;
    int round_k = 5;            // option "round_k": members of a multi-merge round (1: no rounds; at most ROUND_MAX)
    uint32_t round_ties = 50;   // option "round_ties": rounds once this many percent of the last batch's merges were tied
    int round_untied = 1;       // option "round_untied": untied rounds (the next distinct counts' pairs), in every list streak
    int round_streak = 1;       // option "round_streak": 1 rounds only in list streaks; 0 in any batch once the lists are on
                                // and the batch's records fit the arena with room to spare (a stream scan is a round of one)
    uint32_t last_tied_pct = 0; // (the last batch's)

    // multi-GPU: this rank's shard and its neighbours' boundary tokens
    int rank = 0, world = 1;
    std::unique_ptr<Comm> comm;
    bool sharded = false;
    // multi-GPU, late phase: once the occurrence lists take over (scans stop streaming the shards),
    // every rank gathers the whole stream and runs the remaining merges as a replica, with no
    // per-merge collective (option "replicate_late")
    bool replicate_late = true, replicated = false;
    // option "handover": the ranks replicate once top count * list_start * world^handover < live tokens (1: the round-5
    // rule; 2, default: later for more ranks -- a sharded merge's stream scan and replace shrink with the world while
    // its two collectives and the select do not, so the sharded form stays cheaper for longer)
    int handover = 2;
    uint64_t sum_tokens_rep = 0;     // stats.sum_tokens accumulated while replicated (counted once)
    uint64_t n_total = 0;            // corpus bytes over all ranks
    uint64_t global_live = 0;        // live tokens over all ranks (host-tracked from the merged counts)
    uint64_t global_slots = 0;       // stream slots over all ranks (changes at compactions, which are global)
    uint32_t *d_sizes = nullptr;     // [2 * world + 2] live-token counts of the shards
    size_t sizes_cap = 0;
    // a one-rank communicator (zbpe_create_dist with world 1 and a unique id, or a host callback) runs the
    // sharded code path too: every collective of a multi-GPU run executes, over one rank
    bool force_shard = false;
    bool multi() const { return world > 1 || force_shard; }
    bool dist() const { return multi() && !replicated; }
    uint64_t shard_offset = 0;  // global position of the shard's first byte
    int next_byte = -1;         // first byte of the next shard (-1: none)
    Halo halo0{}, halo{};
    Boundary *d_bnd_mine = nullptr, *d_bnd_all = nullptr, *h_bnd = nullptr;
    uint8_t *d_x0 = nullptr;
    uint32_t *d_shard_fn = nullptr, *d_fns_all = nullptr;
    DevState *d_st = nullptr, *h_st = nullptr;
    uint32_t *d_rec = nullptr;
    size_t rec_cap = 0;
    MaxRec *d_partial = nullptr;
    uint32_t *d_tile_cnt = nullptr;
    size_t tile_cnt_cap = 0;
    uint64_t *d_tile_off = nullptr;
    size_t tile_off_cap = 0;
    uint8_t *d_tile_fn = nullptr, *d_carry = nullptr;
    size_t tile_fn_cap = 0, carry_cap = 0;
    uint32_t *d_bitmap = nullptr;
    size_t bitmap_cap = 0;
    uint64_t *d_tie_list = nullptr;
    size_t tie_list_cap = 0;
    uint32_t *d_first = nullptr;
    size_t first_cap = 0;
    LiveRec *d_gather = nullptr;
    size_t gather_cap = 0;
    // exact tie emulation on one GPU: live pairs sorted by first occurrence on the device
    uint32_t *d_ord_pos = nullptr;
    unsigned long long *d_ord_ent = nullptr;
    uint8_t *d_sort_tmp = nullptr;
    size_t ord_pos_cap = 0, ord_ent_cap = 0, sort_tmp_cap = 0;
    uint64_t *h_ord = nullptr;  // pinned
    size_t h_ord_cap = 0;
    ZigEmuWork emu_work;        // the host emulation's tables, kept between ties
    bool tie_prof = false;      // env ZBPE_TIE_PROF: phase times of every exact tie emulation on stderr
    uint32_t *d_recount = nullptr;
    size_t recount_cap = 0;
    uint32_t *d_count_hist = nullptr, *h_count_hist = nullptr;
    size_t hot_cap_alloc = 0;
    size_t home_words_cap = 0, dirty_bits_cap = 0;
    uint64_t home_slots = 0;    // Zig capacity the home histogram is kept for (0: none)
    Summ *d_summ = nullptr, *d_sup = nullptr;
    size_t summ_cap = 0, sup_cap = 0;
    bool hot_stale = true;
    // block skipping
    uint32_t *d_pres = nullptr;
    size_t pres_cap = 0;
    uint32_t pres_vp = 0, pres_groups = 0;
    bool pres_on = false, block_skip = true;
    uint64_t stats_pres_builds = 0;
    // token occurrence lists + this merge's records, in one arena (see kernels.hpp list kernels)
    uint32_t *d_lists = nullptr;
    size_t lists_cap = 0;
    // sharded: the arena limit every rank decides halts and compactions on (from the smallest shard,
    // the same on every rank; each rank's lists_cap is at least this) -- with DevState::arena_rep
    uint64_t arena_cap_rep = 0;
    uint64_t arena_cap_opt = 0;  // option "arena_cap": arena entries to allocate (tests; 0 = 1.5 n + 16 Mi)
    uint64_t arena_limit() const { return dist() ? arena_cap_rep : lists_cap; }
    uint64_t arena_used() const { return dist() ? h_st->arena_rep : h_st->arena_top; }
    uint32_t *d_list_cnt = nullptr, *d_list_total = nullptr;
    size_t list_cnt_cap = 0;
    bool lists_on = false;
    // build-time neighbours of the list entries (the filtered list walk; option "list_nb")
    uint32_t *d_nb = nullptr;  // pred << 16 | succ of every list entry at the build
    size_t nb_cap = 0;
    // successor ranges of the long lists (zbpe_list_sort_succ): rows, the token of each row, the sort's copy
    uint32_t *d_dir = nullptr, *d_dir_row = nullptr, *d_row_tok = nullptr, *d_sort_hist = nullptr;
    uint2 *d_dir_tmp = nullptr;
    size_t dir_cap = 0, dir_row_cap = 0, row_tok_cap = 0, dir_tmp_cap = 0, sort_hist_cap = 0;
    uint32_t dir_w = 0;
    bool dirs_built = false;
    uint32_t list_ranges = 1;            // option "list_ranges": successor-sorted long lists (0: off)
    uint32_t scan_plan = 1;              // option "scan_plan": the select stores the next merge's list plan (0: off)
    uint32_t layout_gen = 1;             // bumped by every list build / compaction / replication (a stored scan plan of another is stale)
    uint32_t range_min_len = 1u << 14;   // option "range_min_len": lists that get a directory row
    uint32_t range_max_rows = 4096;      // option "range_max_rows"
    uint32_t range_max_len = 0xFFFFFFFEu;  // option "range_max_len": longer lists keep the filtered walk
    bool list_nb = true, nb_built = false;
    bool list_streak = false;   // the last batch used list scans only
    int list_grid = 0;          // scan grid after such a batch (option "list_grid"; 0 = the full grid)
    int list_mode = 1;          // 0: never build lists, 1: once pair counts are small against the stream
    uint32_t refresh_wgs = 256;   // option "refresh_wgs": home-refresh workgroups of zbpe_select_next (0: one per super-block)
    int pair_select = 1;        // option "pair_select": a tied merge's decision qualifies the next merge's winner (DevState::pr_*)
    int pair_refresh = 0;       // option "pair_refresh": 1 = a pair select's refresh workgroups still refresh the dirty home blocks
    int pair_m3w = 1;           // option "pair_m3w": the decision's third-smallest tied home by a wave of its own
    int pair_chain = 2;         // option "pair_chain": a pair select names the next merge's candidate too (1: three merges per decision, 2: four)
    int lp_lazy = 1;            // option "lp_lazy": the select looks the stream's last pair up only when a tie's capacity needs it
    int dense_hist = 1;         // option "dense_hist": the full pair histogram of a byte stream counts every byte pair in a fixed 16-bit LDS bin
    uint32_t list_ratio = 96;   // training: list scan when list length * ratio < stream slots
    uint32_t enc_list_ratio = 48;   // the same for encode (option "encode_list_ratio")
    uint32_t self_list_ratio = 8;  // self pair from a's list when length * ratio < stream slots (0: never)
    int self_batch = 1;            // batches take the self pairs self_list_ratio walks (0: they halt to the host path)
    uint64_t list_start = 64;   // build lists at a compaction once top count * list_start < live tokens (0: always)
    // per-merge trace (option "trace"), ZBPE_TRACE_COLS floats per merge
    bool trace_on = false;
    std::vector<float> trace;
    std::vector<int32_t> scan_log;  // per pair-scan launch of the last train (zbpe_scan_log)
    std::vector<uint32_t> compact_log;  // per training compaction: merge X, arena_rep (zbpe_compaction_log)
    // per halted device-resident batch of the last train (zbpe_halt_log): merge X, HaltReason, host-path
    // microseconds (from the batch's return to the end of the synchronous merge that finished X)
    std::vector<uint32_t> halt_log;
    // encode: merges applied per launch pair (option "encode_batch"; 1 = one merge at a time)
    uint32_t enc_batch = 32;
    uint64_t enc_batches = 0;       // launch pairs of the last encode
    int32_t *d_enc_cnt = nullptr;   // live count per token
    size_t enc_cnt_cap = 0;
    uint32_t *d_enc_ctr = nullptr;  // records per merge of the batch
    size_t enc_ctr_cap = 0;
    // device-resident merge loop
    uint32_t merge_batch = 32;      // merges enqueued per host sync (1: synchronous loop)
    uint32_t sel_prof = 0;          // phase timestamps inside zbpe_select_next (printed to stderr after train)
    // HIP events around every merge_timing-th merge of a batch (0: none); with timing_full also around
    // every merge of a batch that follows one with stream-form scans (those take 100s of us: the
    // roofline then sees nearly every stream scan; each event adds ~1 us of gap, so the bench's timed
    // steps sample and a separate probe train sets timing_full)
    uint32_t merge_timing = 8;
    bool timing_full = false;
    bool lists_at_batch = false;    // the batch being enqueued follows a list-only batch
    bool merge_timed(uint32_t X) const {
        return merge_timing && ((timing_full && !lists_at_batch) || X % merge_timing == 0);
    }
    double merge_weight() const { return timing_full && !lists_at_batch ? 1.0 : (double)merge_timing; }
    bool replace_split = false;     // profiling: apply and count update as separate launches
    bool fused_select = true;       // zbpe_select_next: the select of merge X also starts merge X+1 (ties included)
    bool refresh_prefix = true;     // zbpe_select_next: the last refresh workgroup precomputes the tie decision's carries
    bool begun = false;             // the next batch's first merge was started by the last batch's final select
    uint32_t *d_cand = nullptr;     // zbpe_select_next: keys at each argmax block's max
    uint32_t *d_cs = nullptr;       // zbpe_select_next: carries into the home super-blocks (refresh_prefix)
    size_t cs_cap = 0;
    uint32_t *d_rtk = nullptr;      // zbpe_select_next: refresh arrival counters (RTK_WORDS)
    MergeLog *d_log = nullptr;
    std::vector<MergeLog> h_log;
    Halo *d_halo = nullptr;
    std::vector<hipEvent_t> bev;
    uint64_t batches = 0, batch_halts = 0;
    struct RunCtx {
        uint16_t *out_triples = nullptr;
        uint64_t *out_counts = nullptr;
        size_t merges = 0;
        int verbose = 0;
        uint16_t vocab = 0;
        double ev_count = 0, ev_select = 0, ev_replace = 0;  // measured directly (sync path, compactions)
        double tm_count = 0, tm_select = 0, tm_replace = 0, tm_comm = 0;  // stage times of the timed batch merges
        double batch_s = 0;                                   // device span of the batches
    } run;
    uint64_t hot_target = 1u << 11;  // ids the hot list aims to hold after a rebuild (short: one argmax
                                     // workgroup, no ticket; a rebuild every few hundred merges)
    uint32_t sel_growth = 16;        // hot-list growth per merge assumed when sizing zbpe_select_next's argmax grid
    uint32_t sel_margin = 0;         // + this many entries (option "sel_margin")
    uint64_t hot_rebuilds = 0, home_rebuilds = 0;
    hipEvent_t ev[8] = {};
    bool print_runtime = true;  // generateInitialTokens' runtime line on stderr (option "print_runtime")
    double gen_tokens_s = 0;

    // policy knobs
    uint64_t compact_den = 8;     // compact when holes > slots / compact_den
    uint64_t compact_den_lists = 8;  // the same once occurrence lists are on (a compaction also rebuilds them)
    uint64_t compact_den_walks = 4;  // option "compact_den_walks": the same while the merges only walk lists (one GPU)
    int scan_blocks_per_cu = 4;  // set by set_scan_variant: occupancy, at most four (one dispatch round)
    bool debug_checks = false;    // extra syncs + consistency checks
    uint32_t batch_checks = 0;    // option batch_checks m (> 0): the table against a recount after every batch / host merge past merge m
    bool force_exact_ties = false;  // resolve every tie by the exact emulation and cross-check the fast path
    // the same for the merges X in [exact_lo, exact_hi) only (options "exact_ties_from" / "exact_ties_to", merge
    // indices X - 256): those run on the synchronous path, the others in device-resident batches
    uint32_t exact_lo = 0xFFFFFFFFu, exact_hi = 0;
    bool exact_at(uint32_t X) const { return force_exact_ties || (X >= exact_lo && X < exact_hi); }
    bool exact_now = false;         // the merge being finished on the synchronous path is in the exact window

    zbpe_stats stats{};
    uint64_t stats_rebuilds = 0;

    ~Engine();
    zbpe_status init(int device);
    void release();
    zbpe_status fail(zbpe_status s, const char *fmt, ...);
    template <typename T_>
    zbpe_status ensure(T_ **p, size_t &cap, size_t need, const char *what);
    zbpe_status upload(const uint8_t *text, size_t n, bool shard);
    zbpe_status init_dist(int rank, int world, std::unique_ptr<Comm> comm);
    zbpe_status train(uint16_t vocab_size, int verbose, uint16_t *out_triples, uint64_t *out_counts,
                      size_t *out_n_merges, zbpe_stats *out_stats);
    zbpe_status encode(const uint16_t *triples, size_t n_merges, const uint8_t *text, size_t n, uint16_t *out,
                       size_t *out_len);
    zbpe_status verify_counts(uint64_t *mismatches);
    zbpe_status tokens(uint16_t *out, size_t cap, size_t *n_tokens);
    zbpe_status set_scan_variant(int v);
    zbpe_status bench_scan(uint32_t a, uint32_t b, int reps, double *avg_ms, double *gbps);
    zbpe_status bench_train_scan(int reps, int grid, double *avg_us, uint32_t *pair, uint32_t *list_len, int *mode);
    zbpe_status bench_recount(int reps, double *avg_us, double *gbps, uint64_t *n_tokens, uint64_t *mismatches);

   private:
    zbpe_status sync_state();
    zbpe_status alloc_tables(size_t id_cap);
    zbpe_status maybe_grow_tables(uint32_t X, uint32_t k);
    zbpe_status merge_sync(uint32_t X);
    zbpe_status run_batch(uint32_t X0, uint32_t *done, bool *halted);
    zbpe_status launch_round(uint32_t i, uint32_t X0, uint32_t Xmax, uint32_t K, uint32_t top0, const HomeView &V, uint32_t *cs,
                             const uint32_t *self_len, uint32_t self_lim);
    zbpe_status alloc_stream(size_t n);
    zbpe_status generate_initial_tokens(size_t n);
    zbpe_status build_presence();
    zbpe_status compact();
    zbpe_status compact_train(uint32_t X);
    bool holes_over() const;
    zbpe_status max_over_ranks(uint32_t v, uint32_t *out);
    zbpe_status grow_arena(uint64_t need);
    zbpe_status build_lists(uint32_t lists_x, uint32_t ratio, bool ranges = false);
    void set_list_nb(ScanArgs &A) const;
    zbpe_status replicate();
    zbpe_status launch_argmax(uint32_t X, int roll);
    int argmax_blocks(uint32_t X) const;
    int scan_grid(int64_t slots) const;
    zbpe_status launch_scan(const ScanArgs &A, int grid = 0, uint64_t count_hint = 0);
    bool self_list_ok(uint32_t a, bool training);
    zbpe_status rebuild_hot();
    zbpe_status rebuild_home(uint64_t cap);
    zbpe_status select_ready();
    void halo_from_boundaries();
    zbpe_status table_check(uint32_t x0, uint32_t x1, const char *what);
    zbpe_status comm_sum(uint32_t *d, size_t n);
    zbpe_status recount_check(uint64_t *mismatches, uint32_t *first_bad_key);
    zbpe_status compact_to_spare(uint64_t *total);
    zbpe_status launch_pair_hist(uint64_t total);
    zbpe_status resolve_tie(uint32_t top, uint32_t ties, uint32_t *winner);
};

}  // namespace zbpe

/*
 * zbpe.h -- C ABI of the MI355X BPE trainer (libzbpe.so, built from zig-bpe_amd/csrc).
 *
 * Drop-in boundary for the hot path of dbtreasure/zig-bpe: BasicTokenizer.train's pair
 * count + merge loop (src/basic_tokenizer.zig:140-306) and its encode (:71-88). The Zig
 * struct API (init/deinit/train/encode/decode/serializeMerges/deserializeMerges) stays on
 * the host; it calls these entry points through `extern "C"` (see INTEGRATION.md for the
 * Zig, ctypes and C++ bindings). Plain pointers and sizes only; no torch types.
 *
 * Ownership: inputs are borrowed for the duration of a call; outputs go to caller-allocated
 * buffers sized from the arguments; device memory is owned by the context.
 * Threading: one call at a time per context (the reference is single-threaded too).
 * Errors: every entry point returns a zbpe_status; zbpe_last_error() gives the message.
 */
#ifndef ZBPE_H
#define ZBPE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum zbpe_status {
    ZBPE_OK = 0,
    ZBPE_INVALID_VOCAB_SIZE = 1, /* TrainError.InvalidVocabSize (basic_tokenizer.zig:6-10,147-149) */
    ZBPE_OUT_OF_MEMORY = 2,      /* TrainError.OutOfMemory (host or device allocation failed) */
    ZBPE_DEVICE_ERROR = 3,       /* a HIP call or kernel failed; the Zig shim maps it to OutOfMemory */
    ZBPE_COMM_ERROR = 4,         /* an RCCL collective failed */
    ZBPE_INVALID_ARGUMENT = 5,   /* null pointer, size out of range, unsupported merge table */
    ZBPE_INVALID_TOKEN = 6,      /* decode: token with no merge (error.InvalidToken, :101,125,135) */
    ZBPE_INTERNAL = 7            /* an internal consistency check failed (bug) */
} zbpe_status;

typedef struct zbpe_ctx zbpe_ctx;

/* Timing buckets mirror the reference's TimeStats (src/utils/time_statistics.zig:4-13) so the CPU
 * and GPU breakdowns line up; the remaining fields are measurement counters. Times in seconds. */
typedef struct zbpe_stats {
    double count_pairs_s;     /* generateCodePointPairs + countCodePointPairs: initial histogram + per-merge scan */
    double sort_pairs_s;      /* sortCodePointPairs + [0]: argmax over pair counts + Zig-order tie-break */
    double replace_pair_s;    /* replaceTopPairWithNewToken: apply + count update + compaction */
    double other_s;           /* upload, widen, host bookkeeping, synchronisation */
    double total_s;           /* wall time of the call */
    uint64_t count_pairs_calls, sort_pairs_calls, replace_pair_calls;
    /* dominant kernel (zbpe_scan_pairs) measured with HIP events on the engine's stream */
    uint64_t scan_launches;
    double scan_kernel_s;     /* sum of the timed scan kernel durations (see scan_timed_launches) */
    uint64_t scan_alg_bytes;  /* algorithmic bytes of every scan: 2 B per live token */
    uint64_t scan_read_bytes; /* bytes the scan actually streamed (live tokens + holes) */
    uint64_t tie_iterations;  /* merges whose top count was shared by >1 pair */
    uint64_t tie_fallbacks;   /* ties resolved by the exact first-occurrence emulation */
    uint64_t compactions;
    uint64_t self_pair_merges;
    uint64_t final_tokens;    /* token-stream length after training (all ranks) */
    uint64_t distinct_pairs;  /* live pairs after the last merge */
    uint64_t pair_ids;        /* pair-table ids allocated (live + dead) */
    uint64_t sum_tokens;      /* sum over merges of the stream length n_t */
    /* scan launches timed with HIP events (every merge_timing-th merge of a device-resident batch,
     * every merge on the synchronous path) and their algorithmic bytes: scan_kernel_s covers these */
    uint64_t scan_timed_launches;
    uint64_t scan_timed_alg_bytes;
    uint64_t list_scans;      /* pair scans that walked a token occurrence list instead of the stream */
    uint64_t list_builds;     /* occurrence-list rebuilds (after compactions) */
    uint64_t replications;    /* multi-GPU: 1 once the ranks gathered the whole stream for the late phase */
    /* multi-GPU phase split (wall, host clock): merges while the stream is sharded (per-merge
     * collectives), the one-time replication (compaction + all-gather of the shards + list build), the
     * merges after it (replicas, no collective); comm_s: device time of the per-merge count-delta
     * all-reduce, from the HIP events of the timed merges, split like the stage buckets */
    double sharded_s, replicate_s, replicated_s, comm_s;
    uint64_t sharded_merges;
    /* ties decided by both the device's cluster test and the exact emulation, with the same winner
     * (options "exact_ties", "exact_ties_from" / "exact_ties_to"); a disagreement fails the train */
    uint64_t tie_crosschecks;
    /* generateInitialTokens (basic_tokenizer.zig:155-170): the u8 -> u16 widening of the resident corpus
     * (device time); train prints it like the reference, "generateInitialTokens runtime: S seconds" */
    double generate_tokens_s;
    /* merges whose winner the previous merge's tie decision qualified (option "pair_select"): their select
     * skipped the argmax and the Zig-order decision */
    uint64_t pair_selects;
    /* merges applied by multi-merge rounds beyond each round's first (option "round_k"): their scan,
     * replace and select launches were shared with the round's first merge */
    uint64_t round_merges;
} zbpe_stats;

/* Layout version of zbpe_stats. The struct is caller-allocated and has grown across versions: a
 * consumer compares zbpe_stats_size() with the size of the zbpe_stats of the header it was built against
 * before passing a zbpe_stats: the library writes zbpe_stats_size() bytes.
 *   1: up to tie_fallbacks ... list_builds;  2: + replications, phase split, sharded_merges;
 *   3: + tie_crosschecks, generate_tokens_s;  4: + pair_selects, pair_scans;
 *   5: pair_scans -> round_merges (same size and offset: merges applied by rounds beyond their first members). */
#define ZBPE_STATS_VERSION 5
size_t zbpe_stats_size(void);

/* Create a single-GPU context on HIP device `device`. */
zbpe_status zbpe_create(int device, zbpe_ctx **out);

/* Multi-GPU: one process per GPU. Rank 0 calls zbpe_comm_unique_id() and broadcasts the 128 bytes
 * (e.g. with torch.distributed); every rank then calls zbpe_create_dist. The token stream is split
 * into `world` contiguous shards; pair-count deltas are summed with an RCCL all-reduce each merge
 * while scans stream the shards. When the occurrence lists take over, the ranks all-gather the
 * whole stream once and finish as replicas (no per-merge collective; option "replicate_late").
 * world == 1 with a unique id: a one-rank RCCL communicator, and the sharded code path with every
 * collective (all-reduce of the count deltas, boundary all-gathers) runs over that one rank. */
zbpe_status zbpe_comm_unique_id(void *out128);
zbpe_status zbpe_create_dist(int device, int rank, int world, const void *unique_id128, zbpe_ctx **out);

/* Same, with the collectives done by a host callback instead of RCCL (e.g. torch.distributed with
 * gloo; lets several ranks share one GPU in tests). op 0: in-place sum of `count` u32 in buf;
 * op 1: in-place min of `count` u32; op 2: all-gather, buf holds world * count bytes and this
 * rank's count bytes are at rank * count. Return 0 on success. */
typedef int (*zbpe_collective_fn)(void *user, int op, void *buf, size_t count);
zbpe_status zbpe_create_dist_host(int device, int rank, int world, zbpe_collective_fn fn, void *user, zbpe_ctx **out);

void zbpe_destroy(zbpe_ctx *ctx);
const char *zbpe_last_error(const zbpe_ctx *ctx);

/* BasicTokenizer.train (basic_tokenizer.zig:140-153): learn up to vocab_size-256 merges from `text`.
 * out_triples: caller buffer of 3*(vocab_size-256) u16 {first, second, new_token} in training order.
 * out_counts:  optional, vocab_size-256 u64 top counts ("had N occurrences", :309).
 * verbose:     print the reference's per-merge line to stderr (:308-317).
 * n == 0 or 1 yields zero merges ("No more pairs to merge. Stopping early.", :188-191).
 * In a distributed context every rank passes the same full text. */
zbpe_status zbpe_train(zbpe_ctx *ctx, const uint8_t *text, size_t n, uint16_t vocab_size, int verbose,
                       uint16_t *out_triples, uint64_t *out_counts, size_t *out_n_merges, zbpe_stats *stats);

/* Split form of zbpe_train for benchmarks: zbpe_upload stages this rank's shard of `text` in HBM;
 * zbpe_train_resident trains from the resident bytes (inputs already in HBM when timing starts). */
zbpe_status zbpe_upload(zbpe_ctx *ctx, const uint8_t *text, size_t n);
zbpe_status zbpe_train_resident(zbpe_ctx *ctx, uint16_t vocab_size, int verbose, uint16_t *out_triples,
                                uint64_t *out_counts, size_t *out_n_merges, zbpe_stats *stats);

/* BasicTokenizer.encode (basic_tokenizer.zig:71-88): apply `n_merges` merges in order, left-greedy.
 * out: caller buffer of n u16; *out_len receives the encoded length. Any u16 may appear in the table
 * (as deserializeMerges allows, :342-344), 65535 included. Prints the generateInitialTokens runtime
 * line like the reference's encode (:72). */
zbpe_status zbpe_encode(zbpe_ctx *ctx, const uint16_t *triples, size_t n_merges, const uint8_t *text, size_t n,
                        uint16_t *out, size_t *out_len);

/* Diagnostics used by the parity tests: recount every pair of the current token stream with the
 * full-histogram kernel and compare with the incrementally maintained counts. Returns ZBPE_OK and
 * *mismatches = 0 when they agree. Valid after zbpe_train*. */
zbpe_status zbpe_verify_counts(zbpe_ctx *ctx, uint64_t *mismatches);

/* Diagnostic used by the parity tests: the current token stream (the `currentTokens` of
 * expandVocabulary after the last zbpe_train*, basic_tokenizer.zig:173-204, or the result of the
 * last zbpe_encode), holes removed. *n_tokens receives its length; the tokens are copied to `out`
 * when cap >= *n_tokens (pass out = NULL, cap = 0 to query the length). In a sharded context
 * this is the rank's shard (the whole stream once the ranks replicated). No training state changes. */
zbpe_status zbpe_tokens(zbpe_ctx *ctx, uint16_t *out, size_t cap, size_t *n_tokens);

/* Tuning / test options: "debug_checks" (0/1), "exact_ties" (resolve every tie by the exact
 * first-occurrence emulation and cross-check the GPU cluster test), "exact_ties_from" / "exact_ties_to"
 * (the same for merge indices k in [from, to) only; the other merges stay device-resident), "compact_den" (compact when
 * holes > slots/den), "scan_blocks_per_cu", "scan_variant" (0..7: unroll, load kind, phase-2 form;
 * see engine.hip kScanVariants), "dense_hist" (0/1: the full pair histogram of a byte stream counts every byte pair in a fixed 16-bit LDS bin),
 * "scan_batch" (stream form, variants with cross-tile candidate batching:
 * 0 off, 1 for sparse pairs -- count * 32 < slots --, 2 always), "hot_target" (ids kept by the argmax hot list),
 * "block_skip" (0/1: stream only the 8192-slot blocks that hold the pair's rarer token),
 * "trace" (0/1: record per-merge timings, see zbpe_trace), "merge_batch" (merges enqueued per host
 * sync, 1 = synchronous loop), "merge_timing" (HIP events around every N-th merge of a batch; 0 =
 * none), "timing_full" (0/1: also around every merge of a batch that follows one with stream-form
 * scans, so the scan roofline covers nearly every stream scan), "arena_cap" (tests: occurrence-arena entries to allocate;
 * the arena grows when a merge needs more), "list_nb" (0/1: list entries carry their build-time
 * neighbours and a list scan gathers the stream only at entries whose neighbour is the pair's other
 * token), "sel_prof" (in-kernel wall-clock
 * probes of the merge pipeline, printed to stderr after train), "replace_split" (profiling: apply and count update as separate launches), "list_mode"
 * (0: always stream the token stream; 1: token occurrence lists once counts are small), "list_ratio"
 * (train: list scan when list length * ratio < stream slots), "encode_list_ratio" (the same for encode), "list_start" (build the lists at a compaction
 * once top count * list_start < live tokens; 0: at the first compaction), "compact_den_lists" (compact_den
 * once lists are on), "compact_den_walks" (default 4: the same once the merges only walk lists, one GPU), "print_runtime" (0: no generateInitialTokens
 * runtime line on stderr), "pair_select" (0/1, default 1: a tied merge's decision qualifies the next
 * merge's winner, whose select then skips the argmax and the decision), "pair_chain"
 * (0-3, default 2: a pair select passes that on to up to this many further merges), "pair_refresh"
 * (0/1, default 0: a pair select's home refresh is left to the next full select; 1 disables chains),
 * "pair_m3w" (0/1: the decision's further tied homes by a wave of their own), "round_k" (1-5, default 5:
 * members of a multi-merge round -- a tied merge and the tied keys its decision named, applied in one scan,
 * replace and select launch when the reference's loop would merge them next; 1: no rounds), "round_ties" (0-100,
 * default 50: rounds in batches after one with at least this many percent tied merges), "round_untied" (0/1, default 1:
 * untied rounds -- an untied merge and the pairs of the next distinct counts, each held by one pair, merged in one
 * launch triple while no pair the merged members made reaches the next member's count; rounds in every list streak), "lp_lazy" (0/1,
 * default 1: the stream's last pair is looked up only for a tie whose Zig capacity depends on it),
 * "refresh_wgs" (home refresh workgroups of a select), "self_batch" (0/1, default 1: a self pair (a, a) whose
 * list the host path would walk runs inside a batch instead of halting it), "round_streak" (0/1, default 1: rounds
 * only in list streaks; 0: also in batches with stream-form scans when the arena holds their records), "handover"
 * (1-3, default 2: sharded ranks replicate once top count * list_start * world^handover < live tokens). */
zbpe_status zbpe_set_option(zbpe_ctx *ctx, const char *name, int64_t value);

/* printTimeStats (src/utils/time_statistics.zig:36-60): the reference's "Time statistics" text for
 * `stats` (sortCodePointPairs / replaceTopPairWithIndex / generateCodePointPairs / countPointPairs /
 * Other operations). Writes up to cap-1 bytes + NUL to buf; *len receives the full length. The
 * reference prints this to stderr at the end of every train (:141-145); the host shims do the same. */
zbpe_status zbpe_format_time_stats(const zbpe_stats *stats, char *buf, size_t cap, size_t *len);

/* Benchmark diagnostic: time `reps` launches of the pair-scan kernel for pair (a, b), a != b, over
 * the stream of the uploaded corpus (zbpe_upload) as it stands; the first launch is not timed.
 * *gbps = 2 B per stream slot / average launch time. */
zbpe_status zbpe_bench_scan(zbpe_ctx *ctx, uint16_t a, uint16_t b, int reps, double *avg_ms, double *gbps);

/* Benchmark diagnostic, after zbpe_train*: `reps` launches of the pair scan for the pair at the top of
 * the current selection (the next merge's argmax, ties not broken), as training would launch it
 * (the occurrence-list form when its list is short), on a grid of `grid` workgroups (0: training's).
 * The per-merge counters are reset between launches; stream, lists and counts stay as they were.
 * *avg_us: average launch time (HIP events); *pair: first | second << 16; *mode: 1 list, 0 stream;
 * *list_len: entries of the walked list. */
zbpe_status zbpe_bench_train_scan(zbpe_ctx *ctx, int reps, int grid, double *avg_us, uint32_t *pair, uint32_t *list_len,
                                  int *mode);

/* Benchmark diagnostic, after zbpe_train* (one GPU): `reps` launches of the full pair-histogram kernel
 * (the recount behind zbpe_verify_counts: every adjacent pair of the current stream, counted in LDS
 * tables per workgroup, the rest by global lookups) over the stream compacted into the spare buffer;
 * the first launch is not timed. *avg_us: average launch time (HIP events); *gbps = 2 B per token /
 * *avg_us; *n_tokens: the stream's live tokens; *mismatches: pair counts of the last launch that differ
 * from the incremental table (0 expected). */
zbpe_status zbpe_bench_recount(zbpe_ctx *ctx, int reps, double *avg_us, double *gbps, uint64_t *n_tokens,
                               uint64_t *mismatches);

/* Profiling diagnostic: with option "trace" = 1, train records one row of ZBPE_TRACE_COLS floats per
 * merge: {merge index, count, live tokens, stream slots, slots streamed by the scan (a list scan in a
 * device-resident batch: entries of the walked list), scan ms,
 * replace ms, select ms, wall ms of the merge, self pair (0/1), ties}. Copies up to `cap_rows`
 * rows of the last train into `rows`; returns the number of rows recorded in *n_rows. */
#define ZBPE_TRACE_COLS 11
zbpe_status zbpe_trace(zbpe_ctx *ctx, float *rows, size_t cap_rows, size_t *n_rows);

/* Profiling diagnostic: the device's per-merge log of the last train, ZBPE_MERGE_LOG_COLS u32 per merge:
 * {pair (first | second << 16), count, live tokens, tied pairs, scan form (1 list), walked list entries,
 * live occurrences of the list's token, 1 when the walk read only the pair's successor range}. Rows of merges the synchronous path finished are zero
 * beyond what it logs. Copies up to cap_rows rows; *n_rows = merges of the last train. */
#define ZBPE_MERGE_LOG_COLS 8
zbpe_status zbpe_merge_log(zbpe_ctx *ctx, uint32_t *rows, size_t cap_rows, size_t *n_rows);

/* Profiling diagnostic: one entry per pair-scan kernel launch (zbpe_scan_pairs_t) of the last
 * train, in launch order: 2 * (merge index) + form (0 stream scan, 1 list scan), or -1 for a launch
 * that returned at once (its batch had halted before it). Lets a rocprofv3 per-dispatch trace (PMC
 * counters) be matched to merges. Copies up to `cap` entries; *n = entries recorded. */
zbpe_status zbpe_scan_log(zbpe_ctx *ctx, int32_t *out, size_t cap, size_t *n);

/* Diagnostic: one row {merge token X, arena_rep} per stream compaction of the last train (X: the merge it
 * preceded; arena_rep: the replicated occurrence-arena fill it was decided on). Sharded ranks must agree
 * on every row (compactions are decided on replicated quantities). Copies up to cap_rows rows of 2 u32. */
zbpe_status zbpe_compaction_log(zbpe_ctx *ctx, uint32_t *rows, size_t cap_rows, size_t *n_rows);

/* Profiling diagnostic: one row {merge token X, reason, host microseconds} per device-resident batch of the
 * last train that halted (the device could not finish merge X alone and the host's synchronous path did).
 * reason: 2 hot-list argmax to rebuild, 3 Zig map capacity changed (home histogram rebuild), 4 tie the
 * cluster test left undecided (exact emulation), 5 self pair, 6 occurrence arena too small. Host
 * microseconds: from the batch's return to the end of that synchronous merge. Copies up to cap_rows rows. */
zbpe_status zbpe_halt_log(zbpe_ctx *ctx, uint32_t *rows, size_t cap_rows, size_t *n_rows);

/* Host-only diagnostic (no device work): the Zig 0.13 pair-map iteration order emulation used by
 * the exact tie fallback. Given every live pair's first-occurrence position, key (first |
 * second << 16) and count, returns the first pair in slot order whose count == top. */
zbpe_status zbpe_zig_order_winner(const uint32_t *first_pos, const uint32_t *keys, const uint32_t *counts, size_t n,
                                  uint32_t top, int call_after_last_insert, uint32_t *winner);

/* Library version string. */
const char *zbpe_version(void);

#ifdef __cplusplus
}
#endif
#endif /* ZBPE_H */

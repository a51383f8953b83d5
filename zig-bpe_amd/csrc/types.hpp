// Types and constants shared by the device code (kernels.hpp) and the host engine.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace zbpe {


constexpr uint16_t HOLE = 0xFFFF;
constexpr uint32_t EMPTY_KEY = 0xFFFFFFFFu;  // (0xFFFF, 0xFFFF) is never a real pair
constexpr uint32_t NO_ID = 0xFFFFFFFFu;
constexpr int WAVE = 64;
constexpr int SCAN_THREADS = 256;
constexpr int SCAN_UNROLL = 4;                                       // 16-B vectors per lane per wave-tile
constexpr int SCAN_TILE = SCAN_THREADS * SCAN_UNROLL * 8;            // tokens per tile (8192)
constexpr int SCAN_REC_CAP = SCAN_TILE / 2;                          // occurrences per tile (non-overlapping)
constexpr int LDS_BINS = 1024;                                       // neighbour tokens counted in LDS
constexpr int COMPACT_TILE = 8192;                                   // tokens per compaction tile
constexpr int PRES_BLK = 8192;       // stream slots per presence block (a multiple of every wave-tile)
constexpr int PRES_GROUP = 32;       // presence blocks per bitmap word

__host__ __device__ constexpr inline uint32_t pair_key(uint32_t first, uint32_t second) { return first | (second << 16); }

// Multi-merge rounds (option round_k). A round applies a merge and up to ROUND_MAX - 1
// named keys in one scan, one replace and one select launch. The keys are named two ways:
//   - tied rounds: a tied merge's decision names the next tied keys by home slot order (DevState::ph, pr_key2 ..
//     pr_key4); member j >= 1 merges when it is still tied and first in Zig slot order;
//   - untied rounds (option round_untied): the select that begins an untied merge (its count T_0 unique) names
//     the pairs of the next distinct counts T_1 > T_2 > .. below it, each held by one pair (DevState::ur);
//     member j merges when no merged member decremented it and no pair a merged member made reaches T_j (then
//     it holds the unique top count, as the reference's loop would see it).
// The round's scan walks every member's occurrences (member j -> merge cur_x + j, new token cur_x + j) into
// its own delta buffer and records; the replace applies the longest valid prefix of members, one after the
// other, with no occurrence touching an earlier member's; the select rolls them all and starts the merge after
// the round.
constexpr int ROUND_MAX = 5;
// RoundHead::top bits (member j's walk)
constexpr uint32_t RT_XX = 2u;        // adjacent occurrences: (X, X) is new, (b, a) falls
constexpr uint32_t RT_JUNCTION = 16u; // the walk counted junction sides (DevState::rd_jn)
constexpr uint32_t RT_WALKED = 32u;   // member j >= 1 walked by a list form (a stream scan is never a member)
struct RoundHead {
    uint32_t n;                  // members the scan took (1 .. ROUND_MAX; written by its block 0)
    uint32_t ties;               // tied keys at the decision that named them (PairHead ties; 0: an untied round)
    int32_t live0;               // live pairs at the round's start (DevState::live as the scan saw it)
    uint32_t ties0;              // merge cur_x's tied pairs (DevState::tie_count as the scan saw it; 1: untied round)
    uint32_t key[ROUND_MAX];     // member keys (key[0] = cur_key)
    uint32_t touch[ROUND_MAX];   // an occurrence of member j touches one of an earlier member's
    uint32_t top[ROUND_MAX];     // RT_XX | RT_JUNCTION | RT_WALKED
    uint32_t birth[ROUND_MAX];   // new pairs of member j: its distinct neighbour tokens
    uint32_t rec[ROUND_MAX];     // records of member j >= 1 (member 0's: DevState::rec_count)
    int32_t freeb[ROUND_MAX];    // tied rounds: free Zig-map slots: [0] after the largest tied home's block, [j] after
                                 // member j's home block and before the next tied home (j >= 1); -1: no bound
    uint32_t dec[ROUND_MAX];     // tied pairs member j decremented first (the replace), for the tie counts
    uint32_t nmax[ROUND_MAX];    // the largest count a new pair of member j's neighbour deltas reaches
    uint32_t cnt[ROUND_MAX];     // member j's count: the top count (tied), the j-th distinct count (untied)
};
static_assert(sizeof(RoundHead) == 4 * (4 + 9 * ROUND_MAX), "round head: packed words");
// Untied rounds: the select that began untied merge x named the pairs of the next n distinct counts (each the
// only pair with its count, at least the hot list's threshold, not a self pair), in count order
struct UntiedHead {
    uint32_t x, n;
    uint32_t key[ROUND_MAX - 1], cnt[ROUND_MAX - 1];
};
static_assert(sizeof(UntiedHead) == 4 * (2 + 2 * (ROUND_MAX - 1)), "untied head: packed words");
struct RoundPlans {
    uint32_t key[ROUND_MAX - 1];
    uint32_t gen;
    uint32_t pad[3];
    uint32_t plan[ROUND_MAX - 1][6];
};
static_assert(sizeof(RoundPlans) == 4 * (8 + 6 * (ROUND_MAX - 1)), "round plans: packed words");
// A pair select's candidate for merge x (DevState::ph): what the light test reads (the kernel entry's round trip)
struct PairHead {
    uint32_t x, key, slack, ties, births, dt, pad, plan_gen;
};
// Device-resident state. Host reads a copy after each merge (one small D2H per merge).
struct DevState {
    // ---- hot header (the first 96 B): the words the merge kernels read first, loaded together in one
    // scalar round trip at kernel entry (StateHead; a chain of dependent state loads was several
    // round trips of each late merge's launches)
    uint32_t halt;           // HaltReason; every merge-loop kernel returns at once while set
    uint32_t cur_key;        // the pair this merge replaces (after the tie-break)
    uint32_t arena_top;      // arena entries in use (lists, then this merge's records)
    uint32_t lists_valid;    // 1: token occurrence lists describe the current stream
    uint32_t lists_x;        // tokens < lists_x existed when the lists were built (their entries carry neighbours)
    uint32_t top_count;      // argmax result
    uint32_t theta;          // hot-list threshold: every live id with count >= theta is in the hot list
    uint32_t hot_len;        // ids appended to the hot list (may exceed its capacity -> rebuild); follows theta
    uint32_t rec_count;      // occurrences recorded by the last scan
    // scan plan of merge plan_x (pair plan_key), written by zbpe_select_next with cur_key: the list
    // lengths / offsets of both tokens and the successor range of (a, b) in a's sorted list (NO_LIST:
    // none), valid while the host's layout generation (lists, stream positions) is plan_gen
    uint32_t plan_x, plan_key, plan_gen;
    uint32_t plan_la, plan_lb, plan_oa, plan_ob, plan_r0, plan_r1;
    // the stream's last pair (zbpe_select_next): its key and pair id when last looked up, so that the
    // count is one load beside the tail tokens' (the key only changes when a merge reaches the tail)
    uint32_t lp_key, lp_id;
    uint32_t cur_x;          // merge token X being processed (the first member of a multi-merge round)
    uint32_t rd_v;           // multi-merge rounds: members the round's replace applied (0: not a round; RoundHead)
    uint32_t rd_mask;        // multi-merge rounds: which members the replace applied (RoundVerdict)
    uint32_t head_pad;
    // ---- the rest
    uint32_t num_ids;        // pair ids allocated
    int32_t live;            // D_t: pairs with count > 0
    uint32_t xx;             // adjacent occurrences: (b,a) -> (X,X)
    uint32_t tie_count;
    uint32_t top_id;
    uint32_t top_key;
    uint32_t lastpair_count; // count of the stream's last pair (decides the Zig map's final grow)
    uint32_t tie_len;        // tied keys collected by the tie kernel
    uint32_t tie_verdict;    // 0 = winner found by the cluster test, 1 = needs the exact emulation
    uint32_t tie_winner;
    uint32_t error;          // bit flags: 1 id overflow, 2 count underflow, 4 key missing, 8 record overflow
    uint32_t gather_len;
    uint32_t mismatches;
    uint32_t last_occ;       // occurrences merged by the last merge (copied by zbpe_reset_merge)
    uint32_t total_occ;      // running sum of last_occ (encode bookkeeping)
    uint32_t err_x;          // the first failed occurrence check (error 64): merge X, occurrences found, count
    uint32_t ticket;         // zbpe_select: blocks done (the last one reduces), reset by it
    uint32_t last_gocc;      // occurrences merged by the last merge on all ranks
    uint32_t consumed;       // 1: this shard's first live token was the b of the left rank's last occurrence
    uint32_t holes_made;     // slots of this shard turned into holes by the current merge
    uint32_t last_holes;     // holes_made of the last merge (rolled by zbpe_select)
    uint32_t err_occ, err_cnt;
    unsigned long long scanned_slots;  // stream slots the scans actually streamed (block skipping)
    // device-resident merge loop (Engine::run_batch): the host enqueues a batch of merges whose
    // kernels read the pair from here; a merge the device cannot finish alone halts the batch
    uint32_t halt_at;        // merge token X of the halted merge
    uint32_t tie_on;         // 1: this merge's top count is tied (the tie kernels run)
    long long live_tokens;   // live tokens of this shard (rolled by zbpe_select)
    uint32_t arena_rep;      // sum of the merges' global occurrence counts since the arena was emptied: the same on
                             // every rank and >= any rank's arena_top, so halts decided on it keep ranks in step
    uint32_t scan_mode;      // last pair scan: 0 streamed the token stream, 1 walked an occurrence list
    // option sel_prof: zbpe_select_next phase times (wall_clock64 ticks, summed over merges)
    unsigned long long sel_t0, sel_ta, sel_tr;  // start; latest argmax / refresh block finish
    // [0..4] last-block phases, [5] argmax blocks done, [7] last-block calls, [8] tie decisions, [9] their carries,
    // [10] refresh wait, [12] latest refresh block done (at decisions, [13] samples), [6]/[11] prefix start/end ([14] samples)
    unsigned long long sel_prof[24];  // [15]/[16]: summed refresh-workgroup durations / their count; [17]/[18] argmax: counts in / block max (last argmax block); [20]/[21] pair selects / their time
    unsigned long long sel_prof_pq, sel_prof_pp;  // refresh_prefix start / end stamps of the current launch
    // option sel_prof, whole merge pipeline (batch mode): probe stamps of the current launches and the
    // sums they fold into (Engine::train prints them): scan (list form) LDS clear / walk / flush done and
    // the next kernel's start, replace work span and the select's start, select end -> scan start
    unsigned long long pp_t[16];  // [8..12]: replace phases (update blocks: deltas in, gathered, reserved, table done; apply done)
    unsigned long long pipe_prof[3][16];  // by merge: [256, 8192), [8192, 20000), [20000, ...)
    // zbpe_select_next of merge X whose merge X+1 is not tied (its last argmax block stores X): the
    // last refresh workgroup skips the decision's carries (zeroed with the state at each train)
    uint32_t ref_noprefix;
    // Pair selects (option pair_select, zbpe_select_next): the tie decision of merge X names the tied key of
    // the second-smallest home as merge X+1's candidate (PairHead key, x = X+1); merge X's replace computes a
    // lower bound on the free Zig-map slots that keep it first (slack), counts its new pairs (births) and, in
    // dt, the tied pairs it decremented (low 16 bits) with flags above them (bit 16 the candidate was
    // decremented, bit 17 a new pair reached the top count, bit 18 adjacent occurrences); the select of merge
    // X then starts merge X+1 with the candidate and no argmax or decision when every condition holds
    // (pr_hits counts those). Loaded as PairHead (the test, at kernel entry) and PairTail,
    // and the candidate's scan plan (pr_plan, valid for layout generation plan_gen; by the replace's extra workgroup)
    // Two PairHead slots, by the candidate merge's parity: ph[x & 1] holds merge x's candidate. The select that starts
    // merge x1 evaluates the light test on ph[x1 & 1] in every workgroup at entry, and a workgroup may start after the
    // launch's committing block has moved on to merge x1 + 1: so no kernel writes ph[x1 & 1] in that launch (the
    // chain and a decision name merge x1 + 1's candidate in ph[(x1 + 1) & 1]), and every workgroup sees the words the
    // launch started with.
    alignas(128) PairHead ph[2];
    uint32_t pr_plan[6];
    // chains (option pair_refresh 0): the third-smallest home's key, candidate of merge X+2 once merge X+1 was a
    // pair select (bit 19 of dt: decremented); the tied homes the replace bounds the free slots with: the
    // candidate's and the next one's (pr_h2, pr_h3), the one after (pr_h4) and the largest (pr_hmax)
    uint32_t pr_key2, pr_key3;        // (pr_key3: merge X+3's, option pair_chain 2; bit 20 of dt: decremented)
    uint32_t pr_h2, pr_h3, pr_h4, pr_hmax, pr_h5;
    uint32_t pr_key4, pr_h6;          // (merge X+4's, option pair_chain 3; bit 21)
    // the candidate's merge as a tie decision set it (a pair select's chain shift leaves it): a multi-merge round takes the named
    // keys only from the decision itself (the chain state past a pair select counts what that merge did)
    uint32_t pr_full;
    uint32_t pr_hits;        // pair selects taken (the committing block's counter)
    uint32_t pr_pad2[7];
    // multi-merge rounds (option round_k, one GPU or replicas): see RoundHead; rd_merges counts the merges
    // rounds applied beyond their first members
    alignas(128) RoundHead rd;
    uint32_t rd_merges;
    uint32_t rd_why[32];     // rounds that walked named keys, by what ended them (RoundWhy, kernels.hpp; untied from RW_U)
    alignas(16) uint32_t rd_jn[64];  // the round's junction counts (kernels.hpp RJ, RJ_R), cleared by the roll
    // the named keys' scan plans (ScanArgs::pl), by a spare wave of the naming decision (zbpe_select_next, round
    // mode), valid for layout generation rp.gen: a member walk then starts without loading its lists' words
    alignas(16) RoundPlans rp;
    alignas(64) UntiedHead ur;  // untied rounds' named keys (zbpe_select_next, read by the next round's scan)
    uint32_t err_key, err_mode;  // (error 64: the pair, and its scan's form -- scan_mode)
    uint32_t last_light, err_light;  // the last merge a pair select started; (error 64: was the merge one)
    uint32_t err4_key, err4_site;  // (error 4: the first missing pair and where: 1 pair_dec, 2 merged pair, 3 update, 4 first occurrences)
};
struct PairTail {  // what a pair select then reads (plan, chain)
    uint32_t plan[6], key2, key3;
    uint32_t h2, h3, h4, hmax, h5;
    uint32_t key4, h6;
};
static_assert(sizeof(PairHead) == 32 && sizeof(PairTail) == 60, "pair head: 8 words, tail: 15");
// DevState's hot header as one value (StateHead load_head(st))
struct StateHead {
    uint32_t halt, cur_key, arena_top, lists_valid, lists_x, top_count, theta, hot_len, rec_count;
    uint32_t plan_x, plan_key, plan_gen, plan_la, plan_lb, plan_oa, plan_ob, plan_r0, plan_r1;
    uint32_t lp_key, lp_id;
    uint32_t cur_x, rd_v, rd_mask;
    uint32_t pad;
};
static_assert(sizeof(StateHead) == 96, "state head: 24 words");
static_assert(offsetof(DevState, rec_count) == 32 && offsetof(DevState, plan_r1) == 68 && offsetof(DevState, hot_len) == 28 &&
                  offsetof(DevState, lp_id) == 76 && offsetof(DevState, rd_v) == 84,
              "StateHead mirrors DevState's first words");
// zbpe_select_next's refresh arrival counters (a device buffer): per launch parity X & 1, eight
// per-XCD counters (workgroup i counts in i % 8) and a top counter, each on its own 128-B line. The
// select of X - 1 zeroes parity X & 1; the host zeroes both before a batch that does not continue one.
constexpr int RTK_STRIDE = 32;                     // words between counters
constexpr int RTK_SET = 10 * RTK_STRIDE;           // words per parity (counter 9: the argmax workgroups' ticket)
constexpr int RTK_WORDS = 2 * RTK_SET;
// why a device-resident batch stopped (the host finishes that merge on the synchronous path)
enum HaltReason : uint32_t {
    HALT_NONE = 0,
    HALT_DONE = 1,        // no live pairs
    HALT_SELECT = 2,      // hot-list argmax not valid (overflow / exhausted): rebuild on the host
    HALT_HOME = 3,        // the Zig map capacity changed: rebuild the home histogram
    HALT_TIE = 4,         // tie not decided by the cluster test: exact emulation on the host
    HALT_SELF = 5,        // self pair (a, a): compaction + run-parity path
    HALT_RECORDS = 6,     // occurrence buffer too small
};
// per-merge log written by the device in batch mode
struct MergeLog {
    uint32_t key, count, live, ties;
    uint32_t mode;     // 0: stream scan, 1: list scan
    uint32_t list_len; // list scan: entries of the walked occurrence list
    uint32_t key_live; // list scan: live occurrences of the list's token (the walk's useful entries)
    uint32_t range;    // list scan: 1 when it walked only the pair's successor range of a's list
};

struct Tables {
    unsigned long long *ht;  // [ht_cap] slot = key << 32 | id, ~0 = empty (one 8-B load per probe)
    uint32_t ht_mask;
    uint32_t *id_key;   // [id_cap]
    uint32_t *id_cnt;   // [id_cap]
    uint32_t id_cap;
    unsigned long long *hot;  // argmax candidates, key << 32 | id (count >= theta when appended; the key rides along)
    uint32_t hot_cap;
    // the hot entries' counts, kept beside the list (hcnt[j] == id_cnt[id of hot[j]]): the argmax reads them
    // contiguously with the entries, one round trip, instead of gathering id_cnt at random ids (4.4 us for
    // ~4096 ids from one workgroup, profiles/r04_c4_sel_prof.txt); hpos[id] = j, or NO_ID for ids not listed
    uint32_t *hcnt;     // [hot_cap]
    uint32_t *hpos;     // [id_cap]
    uint32_t *home_cnt; // u8 x 4 per word: live keys per home slot of the Zig map (nullptr: not kept)
    uint32_t home_mask; // Zig map capacity - 1 the histogram is kept for
    uint32_t *home_dirty;  // 1 bit per SUMM_SLOTS block: summary stale (2 words per super-block)
    int32_t *tok_cnt;      // [65536] live occurrences per token id (global; picks the scan's key token)
    uint32_t *lst_off, *lst_len;  // [65536] token occurrence lists in the arena (nullptr: not kept)
};

constexpr int COUNT_BINS = 64 + 26 * 32;  // count histogram for choosing theta: exact < 64, then 32 per octave
constexpr int SUMM_SLOTS = 4096;          // home-histogram slots per max-plus block summary
constexpr int SUPER_BLOCKS = 64;          // block summaries per super-block summary
// carry function c -> max(m, c + q) of a run of slots; |q|, m <= Zig capacity < 2^31, so 32-bit
// arithmetic (half the VALU chain and shuffles of the tie decision)
struct Summ { int32_t q, m; };
// the Zig-map home histogram as the tie decision reads it: per-slot counts, block and super-block summaries
struct HomeView {
    const uint32_t *hc;
    const Summ *summ, *sup;
    uint32_t C, nb, nsb;
};

// Live tokens just outside this rank's shard (multi-GPU): left token 0 is the last live token before
// the shard, left 1 the one before it; right 0..2 the first live tokens after it. Packed 16 bits per
// token so that a run-time index is a shift, not an indexed load from a private copy.
struct Halo {
    uint64_t right;  // token i in bits [16i, 16i+16)
    uint32_t left;
    uint8_t nleft, nright;
    uint16_t pad;
};
__host__ __device__ inline Halo halo_empty() { return Halo{0xFFFFFFFFFFFFull, 0xFFFFFFFFu, 0, 0, 0}; }
__host__ __device__ inline uint32_t halo_left(const Halo &h, int64_t i) { return (uint32_t)(h.left >> (16 * i)) & 0xFFFFu; }
__host__ __device__ inline uint32_t halo_right(const Halo &h, int64_t i) { return (uint32_t)(h.right >> (16 * i)) & 0xFFFFu; }
__host__ __device__ inline void halo_push_left(Halo &h, uint32_t t) {
    h.left = (h.left & ~(0xFFFFu << (16 * h.nleft))) | (t << (16 * h.nleft));
    h.nleft++;
}
__host__ __device__ inline void halo_push_right(Halo &h, uint32_t t) {
    h.right = (h.right & ~(0xFFFFull << (16 * h.nright))) | ((uint64_t)t << (16 * h.nright));
    h.nright++;
}
// Per-rank boundary record exchanged after every merge (16 B): first 3 / last 2 live tokens and
// the live-token count of the shard.
struct Boundary {
    uint16_t first[3];
    uint16_t last[2];
    uint8_t nfirst, nlast;
    uint32_t nlive;
};
static_assert(sizeof(Boundary) == 16, "Boundary is exchanged as 16 bytes");

struct MaxRec { uint32_t cnt, ties, id; };
struct LiveRec { uint32_t first_pos, key, count, pad; };

}  // namespace zbpe

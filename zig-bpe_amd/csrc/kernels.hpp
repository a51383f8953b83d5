// Device code of the MI355X (gfx950) BPE trainer. Included by engine.hip only.
//
// Token stream: u16 per token in HBM, HOLE (0xFFFF) marks a slot freed by a merge; holes are
// squeezed out by zbpe_compact_* when they exceed a fraction of the stream. Real tokens are
// < 0xFFFF because vocabSize is a u16 (basic_tokenizer.zig:140) so new tokens stop at 0xFFFE.
//
// Pair table: open addressing on u32 key = first | second << 16 -> dense id; per id a count
// (u32) and its key. Once a pair's count reaches 0 it never returns: a merge only creates pairs
// that contain the brand-new token, so table entries are never revived.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "types.hpp"
#include "wave.hpp"

namespace zbpe {
// DevState's hot header in one round trip: every word is loaded here at kernel entry, before any
// branch on them (the empty asm makes each value live at this point, so the compiler issues the
// scalar loads together and waits once instead of loading each word where it is first used)
__device__ __attribute__((always_inline)) inline StateHead load_head(const DevState *st) {
    StateHead h = *reinterpret_cast<const StateHead *>(st);
    asm volatile("" ::"s"(h.halt), "s"(h.cur_key), "s"(h.arena_top), "s"(h.lists_valid), "s"(h.lists_x), "s"(h.top_count),
                 "s"(h.theta), "s"(h.rec_count));
    asm volatile("" ::"s"(h.plan_x), "s"(h.plan_key), "s"(h.plan_gen), "s"(h.plan_la), "s"(h.plan_lb), "s"(h.plan_oa),
                 "s"(h.plan_ob), "s"(h.plan_r0), "s"(h.plan_r1), "s"(h.lp_key), "s"(h.lp_id));
    return h;
}
// ------------------------------------------------------------------------------------------
// Zig 0.13 std.hash.Wyhash(seed 0) of the 4-byte key
// ------------------------------------------------------------------------------------------
constexpr uint64_t WY_S0 = 0xa0761d6478bd642fULL, WY_S1 = 0xe7037ed1a0b428dbULL;
__host__ __device__ constexpr inline uint64_t mulhi64(uint64_t a, uint64_t b) {
    uint64_t al = a & 0xffffffffu, ah = a >> 32, bl = b & 0xffffffffu, bh = b >> 32;
    uint64_t ll = al * bl, lh = al * bh, hl = ah * bl, hh = ah * bh;
    uint64_t mid = (ll >> 32) + (lh & 0xffffffffu) + (hl & 0xffffffffu);
    return hh + (lh >> 32) + (hl >> 32) + (mid >> 32);
}
__host__ __device__ constexpr inline uint64_t wy_mix(uint64_t a, uint64_t b) { return (a * b) ^ mulhi64(a, b); }
constexpr uint64_t WY_SEED0 = 0 ^ wy_mix(0 ^ WY_S0, WY_S1);  // Wyhash.init(0).state[0]

__device__ inline uint64_t zig_pair_hash(uint32_t w) {
    uint64_t a = ((uint64_t)w << 32) | w;
    uint64_t b = a;
    a ^= WY_S1;
    b ^= WY_SEED0;
    uint64_t lo = a * b, hi = __umul64hi(a, b);
    return wy_mix(lo ^ WY_S0 ^ 4ull, hi ^ WY_S1);
}

// ------------------------------------------------------------------------------------------
// pair table
// ------------------------------------------------------------------------------------------

__device__ inline uint32_t fmix32(uint32_t h) {
    h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
    return h;
}
// Open addressing over 64-byte buckets (8 slots of key<<32 | id, ~0 = empty): a lookup reads its
// home bucket's cache line in one go (4 x 16 B loads in flight) instead of chasing slot by slot,
// and moves to the next bucket only when the home bucket is full (~2 % of buckets at the table's
// <= 1/2 load). A SIMT wave waits for its slowest lane, so the probe chain's tail is what counts.
// Buckets fill as a prefix (an insert claims the first slot it sees empty) and keys are never
// removed, so an empty slot ends a lookup.
constexpr uint32_t HT_BUCKET = 8;
__device__ inline uint32_t ht_home(const Tables &T, uint32_t key) {
    return fmix32(key) & T.ht_mask & ~(HT_BUCKET - 1);
}
__device__ inline void ht_load_bucket(const Tables &T, uint32_t s, unsigned long long (&e)[HT_BUCKET]) {
    const ulonglong2 *p = reinterpret_cast<const ulonglong2 *>(T.ht + s);
    const ulonglong2 v0 = p[0], v1 = p[1], v2 = p[2], v3 = p[3];
    e[0] = v0.x; e[1] = v0.y; e[2] = v1.x; e[3] = v1.y; e[4] = v2.x; e[5] = v2.y; e[6] = v3.x; e[7] = v3.y;
}
__device__ inline uint32_t ht_find(const Tables &T, uint32_t key) {
    uint32_t s = ht_home(T, key);
    for (uint32_t probes = 0; probes <= T.ht_mask; probes += HT_BUCKET) {
        unsigned long long e[HT_BUCKET];
        ht_load_bucket(T, s, e);
        uint32_t id = NO_ID;
        bool empty = false;
#pragma unroll
        for (uint32_t k = 0; k < HT_BUCKET; k++) {
            if ((uint32_t)(e[k] >> 32) == key) id = (uint32_t)e[k];
            empty |= e[k] == ~0ull;
        }
        if (id != NO_ID || empty) return id;
        s = (s + HT_BUCKET) & T.ht_mask;
    }
    return NO_ID;
}
__device__ inline uint32_t ht_find_count(const Tables &T, uint32_t key) {
    uint32_t id = ht_find(T, key);
    return id == NO_ID ? 0 : T.id_cnt[id];
}
// Insert a key known to be absent (callers guarantee uniqueness within a launch). A lost race
// moves to the next slot on the CAS's own answer, never re-reading the bucket: a plain re-read
// could return this XCD's stale L2 copy of the line forever.
// v: the home bucket of `key`, already loaded (ht_load_bucket(T, ht_home(T, key), v))
__device__ inline void ht_insert_loaded(const Tables &T, uint32_t key, uint32_t id, unsigned long long (&v)[HT_BUCKET]) {
    uint32_t s = ht_home(T, key);
    const unsigned long long e = ((unsigned long long)key << 32) | id;
    for (uint32_t probes = 0; probes <= T.ht_mask; probes += HT_BUCKET) {
        if (probes) ht_load_bucket(T, s, v);
        uint32_t k = HT_BUCKET;
#pragma unroll
        for (int j = HT_BUCKET - 1; j >= 0; j--)
            if (v[j] == ~0ull) k = (uint32_t)j;
        for (; k < HT_BUCKET; k++)
            if (atomicCAS(&T.ht[s + k], ~0ull, e) == ~0ull) return;
        s = (s + HT_BUCKET) & T.ht_mask;
    }
}
__device__ inline void ht_insert_new(const Tables &T, uint32_t key, uint32_t id) {
    unsigned long long v[HT_BUCKET];
    ht_load_bucket(T, ht_home(T, key), v);
    ht_insert_loaded(T, key, id, v);
}
// Live keys per home slot of the Zig map: kept incrementally once a tie
// has asked for it, so later ties need no pass over every key.
__device__ inline void home_add(const Tables &T, DevState *st, uint32_t key, bool add) {
    // fire-and-forget: the count (u8 per slot; > 255 keys on one home slot of a table loaded <= 80 %
    // has probability ~1e-500) and the block's dirty bit, both non-returning atomics
    if (!T.home_cnt) return;
    const uint32_t s = (uint32_t)(zig_pair_hash(key) & T.home_mask), sh = 8 * (s & 3);
    if (add) atomicAdd(&T.home_cnt[s >> 2], 1u << sh);
    else atomicSub(&T.home_cnt[s >> 2], 1u << sh);
    const uint32_t blk = s / SUMM_SLOTS;
    atomicOr(&T.home_dirty[blk >> 5], 1u << (blk & 31));
}
// Wave-aggregated append: one atomic per wave. Every lane of the wave must call it.
__device__ inline uint32_t wave_append(uint32_t *counter, bool flag) {
    const uint64_t m = __ballot(flag);
    if (!m) return ~0u;
    const uint32_t lane = threadIdx.x & 63;
    const int leader = __ffsll((unsigned long long)m) - 1;
    uint32_t base = 0;
    if ((int)lane == leader) base = atomicAdd(counter, (uint32_t)__popcll(m));
    base = lane_bcast(base, leader);  // (the leader lane is active: its flag is in the ballot)
    const uint64_t below = m & ((1ull << lane) - 1ull);
    return flag ? base + (uint32_t)__popcll(below) : ~0u;
}
__device__ inline unsigned long long hot_entry(uint32_t key, uint32_t id) { return ((unsigned long long)key << 32) | id; }
// hot-list slot j <- (key, id, count), or (j past the capacity: dropped) the id unlisted
__device__ inline void hot_put(const Tables &T, uint32_t j, uint32_t id, uint32_t key, uint32_t count) {
    if (j < T.hot_cap) {
        T.hot[j] = hot_entry(key, id);
        T.hcnt[j] = count;
        T.hpos[id] = j;
    } else {
        T.hpos[id] = NO_ID;
    }
}
// a listed id's count fell by d: its hot-list copy too
__device__ inline void hot_sub(const Tables &T, uint32_t id, uint32_t d) {
    const uint32_t j = T.hpos[id];
    if (j != NO_ID) atomicSub(&T.hcnt[j], d);
}
__device__ inline void pair_new(const Tables &T, DevState *st, uint32_t key, uint32_t count) {
    uint32_t id = atomicAdd(&st->num_ids, 1u);
    if (id >= T.id_cap) { atomicOr(&st->error, 1u); return; }
    T.id_key[id] = key;
    T.id_cnt[id] = count;
    ht_insert_new(T, key, id);
    atomicAdd(&st->live, 1);
    home_add(T, st, key, true);
    if (count >= st->theta) hot_put(T, atomicAdd(&st->hot_len, 1u), id, key, count);
    else T.hpos[id] = NO_ID;
}
// error 4 (a pair missing from the table): the first one's key and site, for the message
__device__ inline void key_missing(DevState *st, uint32_t key, uint32_t site) {
    if (atomicCAS(&st->err4_site, 0u, site) == 0u) st->err4_key = key;
    atomicOr(&st->error, 4u);
}
// (returns the count before the decrement, 0 for a missing key)
__device__ inline uint32_t pair_dec(const Tables &T, DevState *st, uint32_t key, uint32_t d) {
    uint32_t id = ht_find(T, key);
    if (id == NO_ID) { key_missing(st, key, 1); return 0; }
    hot_sub(T, id, d);
    uint32_t old = atomicSub(&T.id_cnt[id], d);
    if (old < d) atomicOr(&st->error, 2u);
    if (old == d) {
        atomicSub(&st->live, 1);
        home_add(T, st, key, false);
    }
    return old;
}

// ------------------------------------------------------------------------------------------
// generateInitialTokens (basic_tokenizer.zig:155-170): u8 -> u16, 16 bytes per thread
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) zbpe_widen(const uint8_t *__restrict__ text, uint16_t *__restrict__ tok,
                                                  uint64_t n, uint64_t n_pad) {
    uint64_t nv = n_pad / 16;
    for (uint64_t v = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; v < nv; v += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t base = v * 16;
        uint32_t w[8];
        if (base + 16 <= n) {
            uint4 x = *reinterpret_cast<const uint4 *>(text + base);
            uint32_t in[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
            for (int i = 0; i < 4; i++) {
                w[2 * i] = (in[i] & 0xffu) | ((in[i] & 0xff00u) << 8);
                w[2 * i + 1] = ((in[i] >> 16) & 0xffu) | ((in[i] >> 8) & 0xff0000u);
            }
        } else {
#pragma unroll
            for (int i = 0; i < 8; i++) {
                uint32_t lo = base + 2 * i < n ? text[base + 2 * i] : HOLE;
                uint32_t hi = base + 2 * i + 1 < n ? text[base + 2 * i + 1] : HOLE;
                w[i] = lo | (hi << 16);
            }
        }
        uint4 *o = reinterpret_cast<uint4 *>(tok + base);
        o[0] = make_uint4(w[0], w[1], w[2], w[3]);
        o[1] = make_uint4(w[4], w[5], w[6], w[7]);
    }
}

// ------------------------------------------------------------------------------------------
// Initial pair histogram over the byte stream (countCodePointPairs at t = 0): 65,536 possible
// byte pairs; one launch per half of the first byte so the 32,768 u32 bins fit in LDS (128 KiB).
// Pair i = (text[i], text[i+1]); pairs with i >= n-1 are absent. `next_byte` extends the shard by
// one byte (the first byte of the next shard) or is < 0 when there is none.
// ------------------------------------------------------------------------------------------
constexpr int HIST_THREADS = 1024;
__global__ void __launch_bounds__(HIST_THREADS) zbpe_count_byte_pairs(const uint8_t *__restrict__ text, uint64_t n,
                                                                      int next_byte, uint32_t lo,
                                                                      uint32_t *__restrict__ hist) {
    extern __shared__ __attribute__((aligned(16))) uint32_t h[];  // 32768
    for (int i = threadIdx.x; i < 32768; i += HIST_THREADS) h[i] = 0;
    __syncthreads();
    const uint64_t npairs = next_byte >= 0 ? n : (n ? n - 1 : 0);  // pair starts [0, npairs)
    const uint64_t per_block = ((npairs + gridDim.x - 1) / gridDim.x + 15) & ~15ull;
    const uint64_t beg = blockIdx.x * per_block;
    const uint64_t end = min(npairs, beg + per_block);
    for (uint64_t base = beg + 16ull * threadIdx.x; base < end; base += 16ull * HIST_THREADS) {
        uint8_t b[17];
        if (base + 17 <= n) {
            uint4 x = *reinterpret_cast<const uint4 *>(text + base);
            uint32_t in[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
            for (int i = 0; i < 16; i++) b[i] = (uint8_t)(in[i >> 2] >> (8 * (i & 3)));
            b[16] = text[base + 16];
        } else {
#pragma unroll
            for (int i = 0; i < 17; i++) {
                uint64_t p = base + i;
                b[i] = p < n ? text[p] : (uint8_t)(next_byte >= 0 ? next_byte : 0);
            }
        }
#pragma unroll
        for (int i = 0; i < 16; i++) {
            if (base + i < end) {
                uint32_t f = (uint32_t)b[i] - lo;
                if (f < 128) atomicAdd(&h[(f << 8) | b[i + 1]], 1u);
            }
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 32768; i += HIST_THREADS) {
        uint32_t c = h[i];
        if (c) atomicAdd(&hist[(lo << 8) + i], c);
    }
}

__device__ inline uint32_t wave_sum(uint32_t x);
// hist[first*256+second] -> pair table entries
// Multi-GPU: the byte-pair histogram is summed over the ranks in 16-bit limbs (u32 collectives cannot
// overflow for <= 2^16 ranks), and every global count must stay below 2^32: the device counts are u32,
// and no count ever exceeds the largest initial one (a new pair's count is at most the merged pair's).
__global__ void __launch_bounds__(256) zbpe_hist_split(const uint32_t *__restrict__ hist, uint32_t *__restrict__ limbs) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i < 65536) { limbs[i] = hist[i] & 0xFFFFu; limbs[65536 + i] = hist[i] >> 16; }
}
__global__ void __launch_bounds__(256) zbpe_hist_join(const uint32_t *__restrict__ limbs, uint32_t *__restrict__ hist, DevState *st) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= 65536) return;
    const uint64_t c = (uint64_t)limbs[i] + ((uint64_t)limbs[65536 + i] << 16);
    if (c > 0xFFFFFFFFull) atomicOr(&st->error, 512u);
    hist[i] = (uint32_t)c;
}
__global__ void zbpe_hist_to_table(const uint32_t *__restrict__ hist, Tables T, DevState *st) {
    // launched as <<<256, 256>>>: block = first byte
    const uint32_t k = blockIdx.x * 256 + threadIdx.x;
    uint32_t c = hist[k];
    if (c) pair_new(T, st, pair_key(k >> 8, k & 0xff), c);
    // token counts (a byte's pairs as first element; the stream's last byte is not counted)
    __shared__ uint32_t s_sum[4];
    const uint32_t w = wave_sum(c);
    if ((threadIdx.x & 63) == 0) s_sum[threadIdx.x >> 6] = w;
    __syncthreads();
    if (threadIdx.x == 0 && T.tok_cnt) T.tok_cnt[blockIdx.x] = (int32_t)(s_sum[0] + s_sum[1] + s_sum[2] + s_sum[3]);
}

// ------------------------------------------------------------------------------------------
// argmax over pair counts (sortCodePointPairs + sorted[0], basic_tokenizer.zig:280-306,:193):
// the max count, how many pairs share it, and the smallest id holding it.
// ------------------------------------------------------------------------------------------
__device__ inline MaxRec max_combine(MaxRec x, MaxRec y) {
    if (x.cnt > y.cnt) return x;
    if (y.cnt > x.cnt) return y;
    return MaxRec{x.cnt, x.ties + y.ties, min(x.id, y.id)};
}
__device__ inline MaxRec wave_max(MaxRec r) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        MaxRec o{(uint32_t)__shfl_xor((int)r.cnt, off), (uint32_t)__shfl_xor((int)r.ties, off),
                 (uint32_t)__shfl_xor((int)r.id, off)};
        r = max_combine(r, o);
    }
    return r;
}
// The same by DPP (every lane active): a butterfly inside each 16-lane row -- quad_perm [1,0,3,2] and [2,3,0,1],
// half-row mirror, row mirror; each pairs two disjoint halves, so every record is counted once -- then the four
// rows' results combined from v_readlane (wave-uniform). The select's argmax reduces on its critical path; six
// dependent ds_bpermute steps there cost ~0.25 us per reduction.
template <int CTRL>
__device__ __attribute__((always_inline)) inline MaxRec max_dpp_step(MaxRec r) {
    return max_combine(r, MaxRec{dpp_mov<CTRL>(r.cnt), dpp_mov<CTRL>(r.ties), dpp_mov<CTRL>(r.id)});
}
__device__ __attribute__((always_inline)) inline MaxRec wave_max_dpp(MaxRec r) {
    r = max_dpp_step<0xB1>(r);   // quad_perm [1,0,3,2]
    r = max_dpp_step<0x4E>(r);   // quad_perm [2,3,0,1]
    r = max_dpp_step<0x141>(r);  // row_half_mirror
    r = max_dpp_step<0x140>(r);  // row_mirror
    MaxRec q{lane_bcast(r.cnt, 0), lane_bcast(r.ties, 0), lane_bcast(r.id, 0)};
#pragma unroll
    for (int l = 16; l < 64; l += 16) q = max_combine(q, MaxRec{lane_bcast(r.cnt, l), lane_bcast(r.ties, l), lane_bcast(r.id, l)});
    return q;
}
constexpr int ARGMAX_THREADS = 256;
__global__ void __launch_bounds__(ARGMAX_THREADS) zbpe_argmax_partial(const uint32_t *__restrict__ cnt, uint32_t id_cap,
                                                                      const DevState *st, MaxRec *__restrict__ partial) {
    const uint32_t n = min(st->num_ids, id_cap);
    MaxRec r{0, 0, NO_ID};
    const uint32_t nv = n / 4;
    for (uint32_t v = blockIdx.x * ARGMAX_THREADS + threadIdx.x; v < nv; v += gridDim.x * ARGMAX_THREADS) {
        uint4 c = reinterpret_cast<const uint4 *>(cnt)[v];
        uint32_t cc[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
        for (int i = 0; i < 4; i++) r = max_combine(r, MaxRec{cc[i], cc[i] ? 1u : 0u, cc[i] ? 4 * v + i : NO_ID});
    }
    if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
        uint32_t i = nv * 4 + threadIdx.x, c = cnt[i];
        r = max_combine(r, MaxRec{c, c ? 1u : 0u, c ? i : NO_ID});
    }
    r = wave_max(r);
    __shared__ MaxRec sm[ARGMAX_THREADS / WAVE];
    if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = r;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < ARGMAX_THREADS / WAVE; w++) r = max_combine(r, sm[w]);
        partial[blockIdx.x] = r;
    }
}
// Final reduction + the count of the stream's last pair (it decides whether the Zig map grows once
// more after its last insertion) so a tie needs no extra round trip.
__global__ void __launch_bounds__(256) zbpe_argmax_final(const MaxRec *__restrict__ partial, int np, Tables T,
                                                         const uint16_t *__restrict__ tok, int64_t n, DevState *st) {
    MaxRec r{0, 0, NO_ID};
    for (int i = threadIdx.x; i < np; i += 256) r = max_combine(r, partial[i]);
    r = wave_max(r);
    __shared__ MaxRec sm[4];
    if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = r;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 4; w++) r = max_combine(r, sm[w]);
        st->top_count = r.cnt;
        st->tie_count = r.cnt ? r.ties : 0;
        st->top_id = r.id;
        st->top_key = r.id != NO_ID ? T.id_key[r.id] : EMPTY_KEY;
        if (r.ties > 1) {
            int64_t j = n - 1;
            while (j >= 0 && tok[j] == HOLE) j--;
            int64_t i = j - 1;
            while (i >= 0 && tok[i] == HOLE) i--;
            st->lastpair_count = i >= 0 ? ht_find_count(T, pair_key(tok[i], tok[j])) : 0;
        }
    }
}

// ------------------------------------------------------------------------------------------
// Stream helpers (hole skipping). Positions are signed 64-bit; -1 = none.
// (Slot by slot: a form that crossed holes 8 slots per 16-B load measured 1 % slower over a C4 train -- most runs of
// holes are one or two slots -- profiles/r06_ab_hole_walk_vector.txt.)
// ------------------------------------------------------------------------------------------
__device__ inline int64_t next_live(const uint16_t *tok, int64_t n, int64_t i) {
    for (int64_t k = i + 1; k < n; ++k)
        if (tok[k] != HOLE) return k;
    return -1;
}
__device__ inline int64_t prev_live(const uint16_t *tok, int64_t i) {
    for (int64_t k = i - 1; k >= 0; --k)
        if (tok[k] != HOLE) return k;
    return -1;
}

// LDS-privatised neighbour histograms: tokens < LDS_BINS directly in LDS; larger tokens (the merged
// ones, the common neighbours once merges are long) in a small LDS hash of (token << 16 | count)
// with a few linear probes, and only the rest straight to HBM. Contended global atomics on a few hot
// neighbour tokens cost more than the whole list walk of a late merge.
constexpr int HASH_LOG = 9;
constexpr int HASH_BINS = 1 << HASH_LOG;
struct NeighbourHist {
    uint32_t *lds_left, *lds_right;
    uint32_t *g_left, *g_right;
    uint32_t *h_left = nullptr, *h_right = nullptr;  // nullptr: no hash (large tokens go to HBM)
    // multi-merge rounds: every add to the global deltas returns the old value, so that the workgroup counts the
    // new pairs (a delta word leaving 0: one per distinct neighbour token, whichever workgroup adds first) and the
    // largest count a new pair reaches (the add that completes a word sees its final value); rd = its LDS words
    // {new pairs, largest new count, queued adds}. The walk's adds past the LDS bins and hash are queued in LDS
    // (rd_queue, the round scan's dynamic LDS) and made by the flush, all in flight together: a returning add here
    // held its thread for a memory round trip per occurrence.
    uint32_t *rd = nullptr;
    __device__ inline void gadd(uint32_t *g, uint32_t t, uint32_t v) const;
    __device__ inline void add(uint32_t *lds, uint32_t *h, uint32_t *g, uint16_t t) const {
        if (t < LDS_BINS) {
            atomicAdd(&lds[t], 1u);
            return;
        }
        if (h) {
            uint32_t s = ((uint32_t)t * 2654435761u) >> (32 - HASH_LOG);
            for (int k = 0; k < 4; k++, s = (s + 1) & (HASH_BINS - 1)) {
                uint32_t e = h[s];
                if (e == 0) {
                    e = atomicCAS(&h[s], 0u, ((uint32_t)t << 16) | 1u);
                    if (e == 0) return;
                }
                if ((e >> 16) == t) {
                    // 16-bit count: every 2^15 increments one thread moves 2^15 to HBM
                    const uint32_t old = atomicAdd(&h[s], 1u);
                    if ((old & 0xffffu) == 0x7fffu) {
                        atomicSub(&h[s], 0x8000u);
                        gadd(g, t, 0x8000u);
                    }
                    return;
                }
            }
        }
        gadd(g, t, 1u);
    }
    __device__ inline void left(uint16_t t) { add(lds_left, h_left, g_left, t); }
    __device__ inline void right(uint16_t t) { add(lds_right, h_right, g_right, t); }
};

constexpr uint32_t RD_QUEUE = 2048;  // queued adds of a round member walk's workgroup (rd_queue entries)
__device__ inline uint32_t *rd_queue() {
    extern __shared__ uint32_t rd_dyn[];
    return rd_dyn;
}
// a queued add: token | right << 16 | (v == 0x8000) << 17
__device__ inline void NeighbourHist::gadd(uint32_t *g, uint32_t t, uint32_t v) const {
    if (!rd) {
        atomicAdd(&g[t], v);
        return;
    }
    const uint32_t j = atomicAdd(&rd[2], 1u);
    if (j < RD_QUEUE) {
        rd_queue()[j] = t | (g == g_right ? 1u << 16 : 0u) | (v == 1u ? 0u : 1u << 17);
        return;
    }
    const uint32_t old = atomicAdd(&g[t], v);  // (queue full: added here)
    if (old == 0) atomicAdd(&rd[0], 1u);
    atomicMax(&rd[1], old + v);
}
// option sel_prof: merge-index bucket of the pipeline probes (DevState::pipe_prof)
__device__ inline int pp_bucket(uint32_t X) { return X < 8192 ? 0 : X < 20000 ? 1 : 2; }

struct ScanArgs {
    const uint16_t *tok;
    int64_t n;           // slots in the stream (live + holes); tok is padded with HOLE to a multiple of 8
    uint32_t a, b;       // top pair (a != b for zbpe_scan_pairs)
    uint32_t *left;      // [65536] count of (L, a) pairs destroyed == (L, X) pairs created
    uint32_t *right;     // [65536] count of (b, R) destroyed == (X, R) created
    DevState *st;
    uint32_t *rec;       // occurrence start positions
    uint32_t rec_cap;
    int count_deltas;    // 0: encode mode (records only)
    uint32_t *xx_out;    // adjacent occurrences (b,a) -> (X,X), summed over ranks
    uint32_t *occ_out;   // occurrences, summed over ranks
    Halo halo;           // live tokens beyond the shard (multi-GPU); empty on one GPU
    // block skipping: pres[(block / 32) * vp + token] bit (block % 32) = token may occur in the block
    uint32_t *pres;      // nullptr: stream every block
    uint32_t vp;         // tokens per presence row
    uint32_t X;          // the merge's new token (its presence bits are set where it is written)
    const int32_t *tokcnt;  // token counts: the rarer of a, b keys the scan (nullptr: a)
    int dyn;                // batch mode: a, b from st->cur_key, halo from *dhalo (if set); no-op when halted
    const Halo *dhalo;
    // token occurrence lists (Engine::build_lists): positions of token t at lst_off[t] .. + lst_len[t]
    // in the arena (NO_LIST: none); a scan keyed by the shorter list when it is short enough
    const uint32_t *lists;
    const uint32_t *lst_off, *lst_len;
    uint32_t list_ratio;    // list scan when list length * list_ratio < stream slots
    int rec_arena;          // records at rec + st->arena_top (they become the new token's list)
    MergeLog *log;          // batch mode: the scan records its mode in log[X - 256]
    uint32_t *rec_ctr;      // record counter (nullptr: st->rec_count); batched encode: one per merge
    int prof;               // option sel_prof: probe stamps into st->pp_t (batch mode)
    // the neighbours of every list entry when the lists were built (Engine::build_lists; nullptr:
    // none): nb[e] = pred << 16 | succ, the live tokens before / after position lists[e] at that time
    const uint32_t *nb;
    // stream form, sparse tiles' candidates batched across tiles (scan_pairs_body BATCH): 0 off, 1 when
    // the pair is sparse (count * SCAN_BATCH_DENSITY < slots; count unknown: on), 2 always
    int batch;
    // successor ranges of the long lists (Engine::build_lists, zbpe_list_sort_succ; nullptr: none):
    // dir_row[t] = t's row or NO_LIST; entries of t's list with build-time successor s (s < lists_x,
    // lists_x for the stream's end) at [dir[row * dir_w + s], dir[row * dir_w + s + 1])
    const uint32_t *dir_row, *dir;
    uint32_t dir_w;
    uint32_t gen;           // the host's layout generation (Engine::layout_gen): a scan plan of another one is stale
    // filled by scan_args_resolve from the state head (host: 0): the top count, and the scan plan
    // zbpe_select_next stored for this merge (plan_ok; pl = la, lb, oa, ob, r0, r1: DevState::plan_*)
    uint32_t top_count;
    uint32_t plan_ok;
    uint32_t pl[6];
    // multi-merge rounds (zbpe_scan_pairs_t ROUND, batch mode): rounds of up to `round` members (option round_k;
    // < 2: none) and no member at or past token x_end; the home view the naming decision saw (RoundHead::freeb)
    int round;
    uint32_t x_end;
    HomeView hv;  // (hc unused)
    const uint32_t *cs;
    // a member walk (filled by the round scan): every member's key (tk[tkj] its own; ntk members), its RoundHead
    // words and the round's junction counts (DevState::rd_jn)
    uint32_t tk[ROUND_MAX];
    uint32_t ntk, tkj;
    uint32_t *rd_touch, *rd_top, *rd_birth, *rd_jn, *rd_nmax;
};
constexpr uint32_t NO_LIST = 0xFFFFFFFFu;
// batching pays below about one occurrence per 32 slots (tools/scan_bands.py, DPP window moves: +5 % at 5e-4,
// +11 % at 2e-3, +16 % at 5e-3, +8 % at 1e-2, even at 3e-2, profiles/r06_scan_bands_dpp.jsonl; with shuffles it
// cost above 1 in 400, where most tiles are dense and each one flushed a short batch)
constexpr uint64_t SCAN_BATCH_DENSITY = 32;
// the device-held parts of the arguments: pair (batch mode), halo (batch mode, multi-GPU), record
// window in the arena
// (H: the state head, load_head at kernel entry)
// (X: the merge token, A0.X unless the state names it: a multi-merge round's first member, H.cur_x)
__device__ inline ScanArgs scan_args_resolve(const ScanArgs &A0, const StateHead &H, uint32_t X) {
    uint32_t a = A0.a, b = A0.b;
    Halo h = A0.halo;
    if (A0.dyn) {
        const uint32_t k = H.cur_key;
        a = k & 0xFFFF;
        b = k >> 16;
        if (A0.dhalo) h = *A0.dhalo;
    }
    uint32_t *rec = A0.rec;
    uint32_t cap = A0.rec_cap;
    if (A0.rec_arena) {
        const uint32_t top = H.arena_top;
        rec += top;
        cap = cap > top ? cap - top : 0;
    }
    ScanArgs A{A0.tok, A0.n, a, b, A0.left, A0.right, A0.st, rec, cap, A0.count_deltas, A0.xx_out, A0.occ_out, h,
               A0.pres, A0.vp, X, A0.tokcnt, 0, nullptr, A0.lists, A0.lst_off, A0.lst_len, A0.list_ratio, 0,
               A0.log, A0.rec_ctr ? A0.rec_ctr : &A0.st->rec_count, A0.prof, A0.nb, A0.batch,
               A0.dir_row, A0.dir, A0.dir_w, A0.gen, H.top_count, 0u, {}};
    // batch mode: the plan the select stored with this merge's pair, for the current lists
    A.plan_ok = A0.dyn && H.plan_x == X && H.plan_key == pair_key(a, b) && H.plan_gen == A0.gen ? 1u : 0u;
    A.pl[0] = H.plan_la; A.pl[1] = H.plan_lb; A.pl[2] = H.plan_oa; A.pl[3] = H.plan_ob; A.pl[4] = H.plan_r0; A.pl[5] = H.plan_r1;
    return A;
}

// Positions outside the shard address the halo: p >= n is right[p-n], p < 0 is left[-p-1].
constexpr int64_t NONE_POS = INT64_MIN;
__device__ inline uint32_t tok_h(const ScanArgs &A, int64_t p) {
    if (p >= A.n) return halo_right(A.halo, p - A.n);
    if (p < 0) return halo_left(A.halo, -p - 1);
    return A.tok[p];
}
__device__ inline int64_t next_live_h(const ScanArgs &A, int64_t p) {
    if (p < A.n) {
        const int64_t k = next_live(A.tok, A.n, p);
        if (k >= 0) return k;
        return A.halo.nright > 0 ? A.n : NONE_POS;
    }
    const int64_t i = p - A.n + 1;
    return i < A.halo.nright ? A.n + i : NONE_POS;
}
__device__ inline int64_t prev_live_h(const ScanArgs &A, int64_t p) {
    if (p >= 0) {
        const int64_t k = p > 0 ? prev_live(A.tok, p) : -1;
        if (k >= 0) return k;
        return A.halo.nleft > 0 ? -1 : NONE_POS;
    }
    const int64_t i = -p;  // p = -1 -> the token before it is left[1]
    return i < A.halo.nleft ? -(i + 1) : NONE_POS;
}

// RoundHead::touch of member j: bit e (RT_SHARED << e) an occurrence shares a token with one of earlier member e's
// (merging e decrements member j's pair: it leaves the tied set), bit 8 + e (RT_NEIGHBOUR << e) one sits next to
// one of member e's (a junction)
enum RoundTouch : uint32_t { RT_SHARED = 1u, RT_NEIGHBOUR = 1u << 8 };
// Junctions: an occurrence of member L immediately followed (holes aside) by one of member R. Merged one after the
// other they make (X_L, X_R) and their shared neighbour pair (b_L, a_R) falls once; the first of them to merge
// sees the other's original token, the second the first's new one. The walks leave a junction's side out of
// their neighbour counts and count it instead -- rd_jn[L * RJ + R] by L's walk (its right neighbour),
// rd_jn[RJ_R + L * RJ + R] by R's walk (its left neighbour) -- and the replace applies what the merged members
// make of it (round_junction_adjust; a member merged without its partner takes its side back as a neighbour).
constexpr uint32_t RJ = ROUND_MAX, RJ_R = 32;
// a round member's occurrence against the other members (tl, tll: its left neighbour and the token before it,
// tr, trn: its right neighbour and the one after it; HOLE where none): RT bits, and its junction sides
__device__ __attribute__((always_inline)) inline uint32_t round_touch(const ScanArgs &A, uint32_t tl, uint32_t tll, uint32_t tr,
                                                                      uint32_t trn, int &jl, int &jr) {
    const uint32_t j = A.tkj;
    uint32_t t = 0;
    jl = jr = -1;
#pragma unroll
    for (int e = 0; e < ROUND_MAX; e++) {
        if ((uint32_t)e < A.ntk && (uint32_t)e != j) {
            const uint32_t ta = A.tk[e] & 0xFFFFu, tb = A.tk[e] >> 16;
            // a shared token: its a is the tb after a ta, or its b the ta before a tb (an earlier e decrements it)
            if ((uint32_t)e < j) t |= ((A.a == tb && tl == ta) || (A.b == ta && tr == tb)) ? RT_SHARED << e : 0u;
            if (tl == tb && tll == ta) { jl = e; t |= RT_NEIGHBOUR << e; }
            if (tr == ta && trn == tb) { jr = e; t |= RT_NEIGHBOUR << e; }
        }
    }
    return t;
}
__device__ __attribute__((always_inline)) inline void round_touch_commit(const ScanArgs &A, uint32_t t, int jl, int jr) {
    if (t) atomicOr(A.rd_touch, t);
    if (jl >= 0) atomicAdd(&A.rd_jn[RJ_R + (uint32_t)jl * RJ + A.tkj], 1u);
    if (jr >= 0) atomicAdd(&A.rd_jn[A.tkj * RJ + (uint32_t)jr], 1u);
    if (jl >= 0 || jr >= 0) atomicOr(A.rd_top, RT_JUNCTION);  // (the roll clears rd_jn)
}
// General occurrence handler (any holes, any position, shard boundaries through the halo).
// Returns 1 if (p, next live) == (a, b).
// RD: a multi-merge round's member walk (round_touch on the exact neighbours; a junction side is not counted)
template <bool RD = false>
__device__ inline int occ_slow(const ScanArgs &A, NeighbourHist &H, int64_t p, uint32_t &xx) {
    const int64_t q = next_live_h(A, p);
    if (q == NONE_POS || tok_h(A, q) != A.b) return 0;
    int jl = -1, jr = -1;
    if (RD && A.ntk > 1) {
        const int64_t l = prev_live_h(A, p), r = next_live_h(A, q);
        const int64_t ll = l != NONE_POS ? prev_live_h(A, l) : NONE_POS, rn = r != NONE_POS ? next_live_h(A, r) : NONE_POS;
        const auto tk = [&](int64_t x) { return x != NONE_POS ? tok_h(A, x) : (uint32_t)HOLE; };
        round_touch_commit(A, round_touch(A, tk(l), tk(ll), tk(r), tk(rn), jl, jr), jl, jr);
    }
    if (A.count_deltas) {
        const int64_t l = prev_live_h(A, p);
        if (l != NONE_POS) {
            const uint32_t tl = tok_h(A, l);
            bool merged_end = false;
            if (tl == A.b) {
                const int64_t pl = prev_live_h(A, l);
                merged_end = pl != NONE_POS && tok_h(A, pl) == A.a;
            }
            if (!merged_end && jl < 0) H.left((uint16_t)tl);
        }
        const int64_t r = next_live_h(A, q);
        if (r != NONE_POS) {
            const uint32_t tr = tok_h(A, r);
            bool r_occ = false;
            if (tr == A.a) {
                const int64_t rn = next_live_h(A, r);
                r_occ = rn != NONE_POS && tok_h(A, rn) == A.b;
            }
            if (r_occ) xx++;
            else if (jr < 0) H.right((uint16_t)tr);
        }
    }
    return 1;
}

__device__ inline uint32_t wave_sum(uint32_t x) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) x += (uint32_t)__shfl_xor((int)x, off);
    return x;
}
__device__ inline uint32_t tok_at(uint4 v, int k) {
    uint32_t w = k < 2 ? v.x : k < 4 ? v.y : k < 6 ? v.z : v.w;
    return (k & 1) ? (w >> 16) : (w & 0xffffu);
}
__device__ inline uint32_t match8(uint4 v, uint32_t a) {
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) m |= (tok_at(v, k) == a ? 1u : 0u) << k;
    return m;
}

// Phase-1 candidate test of one 16-B vector (8 tokens) by two-token windows: each window is one
// 32-bit compare against (a, b) and against (a, HOLE) (by a) or (HOLE, b) (by b), so a vector
// costs ~20 VALU ops into lane masks, and per-lane bits only when some lane of the wave matched.
// By a, bit k = the window starting at token k matched; by b, the window ending at token k. `edge`
// is the neighbouring vector's word in stream order (by a: the next vector's first, by b: the
// previous vector's last), so the test is exact at every lane.
template <bool BY_B>
__device__ __attribute__((always_inline)) inline uint32_t pair_windows8(uint4 v, uint32_t edge, uint32_t P1, uint32_t P2) {
    const uint32_t ww[5] = {BY_B ? edge : v.x, BY_B ? v.x : v.y, BY_B ? v.y : v.z, BY_B ? v.z : v.w, BY_B ? v.w : edge};
    auto win = [&](int k) -> uint32_t {  // the two-token window of bit k
        const int t = k + (BY_B ? 1 : 0);
        return (t & 1) ? __builtin_amdgcn_alignbit(ww[t / 2 + 1], ww[t / 2], 16) : ww[t / 2];
    };
    auto hit = [&](int k) -> bool {
        const uint32_t x = win(k);
        return (x == P1) | (x == P2);
    };
    // the common case (no lane matches) only ORs lane masks; the bits are recomputed on a match
    bool any = false;
#pragma unroll
    for (int k = 0; k < 8; k++) any |= hit(k);
    if (!__ballot(any)) return 0;
    uint32_t bits = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) bits |= hit(k) ? (1u << k) : 0u;
    return bits;
}

// ------------------------------------------------------------------------------------------
// THE HOT KERNEL (one launch per merge): stream the token stream once, find every occurrence
// of the top pair (a, b), a != b (every occurrence is merged: non-overlapping by construction),
// and emit the pair-count deltas of replaceTopPairWithNewToken (basic_tokenizer.zig:207-232):
//   left[L]  : pair (L, a) destroyed and (L, X) created, unless L ends the previous occurrence
//   right[R] : pair (b, R) destroyed and (X, R) created, unless R starts the next occurrence
//   xx       : adjacent occurrences: (b, a) destroyed and (X, X) created
// plus the occurrence start positions.
// Layout: a wave owns wave-tiles of 64 lanes x SCAN_UNROLL 16-B vectors (2048 tokens, 4 KiB)
// and grid-strides over them with no block barrier in the loop; lanes hold 8 consecutive tokens,
// neighbours across lanes come from shuffles. Occurrence starts are staged per wave in LDS and
// flushed with one global atomic per 256*UNROLL records.
// ------------------------------------------------------------------------------------------
__device__ inline void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ inline uint32_t wave_incl_scan(uint32_t x) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        uint32_t y = (uint32_t)__shfl_up((int)x, off);
        if (lane >= off) x += y;
    }
    return x;
}
// copy the wave's staged records to the global list (one atomic)
__device__ inline void wave_flush_records(const ScanArgs &A, const uint32_t *rec, uint32_t n) {
    const int lane = threadIdx.x & 63;
    uint32_t base = 0;
    if (lane == 0) {
        base = atomicAdd(A.rec_ctr, n);
        atomicAdd(A.occ_out, n);
    }
    base = lane_bcast(base, 0);
    for (uint32_t i = lane; i < n; i += 64)
        if (base + i < A.rec_cap) A.rec[base + i] = rec[i];
    if (lane == 0 && base + n > A.rec_cap) atomicOr(&A.st->error, 8u);
}

// occurrences of (a, b) starting in vector vi (8 tokens) whose bits are set in m; returns the hit mask.
// Window = vectors vi-1, vi, vi+1 re-read from cache (they were just streamed by this wave).
// occurrences of (a, b) starting in vector vi (8 tokens) whose bits are set in m, from the window
// tok[p0-2 .. p0+11] (p0 = 8*vi) given as the previous vector's last dword pw, the vector cv and the
// next vector's first two dwords nx, ny (holes outside the stream); returns the hit mask.
// RD: a multi-merge round's member walk -- every occurrence is also tested against the earlier members' pairs
// (A.tk): does it touch one of their occurrences (share a token with one, or sit next to one)? Then A.rd_touch.
template <bool RD = false>
__device__ inline uint32_t occ_window(const ScanArgs &A, NeighbourHist &H, int64_t vi, uint32_t m, uint32_t &xx,
                                      uint32_t pw, uint4 cv, uint32_t nx, uint32_t ny);
template <bool RD = false>
__device__ inline uint32_t occ_vector(const ScanArgs &A, NeighbourHist &H, int64_t vi, int64_t nvec, uint32_t m,
                                      uint32_t &xx) {
    const uint16_t *tok = A.tok;
    const uint4 *tv = reinterpret_cast<const uint4 *>(tok);
    const uint32_t pw = vi > 0 ? tv[vi - 1].w : 0xffffffffu;
    const uint4 cv = tv[vi];
    uint32_t nx = 0xffffffffu, ny = 0xffffffffu;
    if (vi + 1 < nvec) {
        const uint4 nv = tv[vi + 1];
        nx = nv.x;
        ny = nv.y;
    }
    return occ_window<RD>(A, H, vi, m, xx, pw, cv, nx, ny);
}
template <bool RD>
__device__ inline uint32_t occ_window(const ScanArgs &A, NeighbourHist &H, int64_t vi, uint32_t m, uint32_t &xx,
                                      uint32_t pw, uint4 cv, uint32_t nx, uint32_t ny) {
    const int64_t n = A.n;
    // window of 14 tokens tok[p0-2 .. p0+11], p0 = 8*vi, in four u64 (no scratch)
    const uint64_t W0 = (uint64_t)pw | ((uint64_t)cv.x << 32);
    const uint64_t W1 = (uint64_t)cv.y | ((uint64_t)cv.z << 32);
    const uint64_t W2 = (uint64_t)cv.w | ((uint64_t)nx << 32);
    const uint64_t W3 = (uint64_t)ny;
    auto win = [&](int i) -> uint32_t {
        uint64_t q = i < 4 ? W0 : i < 8 ? W1 : i < 12 ? W2 : W3;
        return (uint32_t)(q >> ((i & 3) * 16)) & 0xffffu;
    };
    // live-slot mask of the window (bit i: window token i is not a hole); slots outside the stream
    // read as holes, so a walk that leaves the window falls back to occ_slow (halo, stream ends)
    uint32_t live = 0;
#pragma unroll
    for (int i = 0; i < 14; i++) live |= (win(i) != HOLE ? 1u : 0u) << i;
    uint32_t hits = 0;
    while (m) {
        const int k = __ffs(m) - 1;
        m &= m - 1;
        const int i = k + 2;  // window index of p
        const int64_t p = vi * 8 + k;
        // next / previous live window slots around p (14 = none)
        const uint32_t after = live >> (i + 1), before = live & ((1u << i) - 1u);
        const int q = after ? i + 1 + __builtin_ctz(after) : 14;
        int hit;
        bool fast = q < 14 && before != 0 && p >= 2 && p + 3 < n;
        int l = 0, ll = -1, r = 14, rn = 14;
        if (fast) {
            l = 31 - __builtin_clz(before);
            const uint32_t aq = live >> (q + 1);
            r = aq ? q + 1 + __builtin_ctz(aq) : 14;
            const uint32_t bl = live & ((1u << l) - 1u);
            ll = bl ? 31 - __builtin_clz(bl) : -1;
            if (r < 14) {
                const uint32_t ar = live >> (r + 1);
                rn = ar ? r + 1 + __builtin_ctz(ar) : 14;
            }
            // every token the delta rules may look at must be inside the window
            fast = r < 14 && (win(r) != A.a || rn < 14) && (win(l) != A.b || ll >= 0);
        }
        int jl = -1, jr = -1;
        if (RD && fast && A.ntk > 1 && win(q) == A.b) {
            // against every other member (round_touch); a neighbour occurrence that may reach past the window
            // sends the occurrence to the slow path
            const uint32_t tl = win(l), tr = win(r), tll = ll < 0 ? (uint32_t)HOLE : win(ll), trn = rn >= 14 ? (uint32_t)HOLE : win(rn);
            bool edge = false;
#pragma unroll
            for (int e = 0; e < ROUND_MAX; e++) {
                if ((uint32_t)e < A.ntk && (uint32_t)e != A.tkj) {
                    const uint32_t ta = A.tk[e] & 0xFFFFu, tb = A.tk[e] >> 16;
                    edge |= (tl == tb && ll < 0) || (tr == ta && rn >= 14);
                }
            }
            if (edge) fast = false;
            else round_touch_commit(A, round_touch(A, tl, tll, tr, trn, jl, jr), jl, jr);
        }
        if (fast) {
            hit = win(q) == A.b;
            if (hit && A.count_deltas) {
                const uint32_t tl = win(l), tr = win(r);
                const bool merged_end = (tl == A.b) && (win(ll < 0 ? 0 : ll) == A.a);
                if (!merged_end && jl < 0) H.left((uint16_t)tl);
                const bool r_occ = (tr == A.a) && (win(rn > 13 ? 13 : rn) == A.b);
                if (r_occ) xx++;
                else if (jr < 0) H.right((uint16_t)tr);
            }
        } else {
            hit = occ_slow<RD>(A, H, p, xx);
        }
        if (hit) hits |= 1u << k;
    }
    return hits;
}

// One candidate start p = 8 vi + k of the window tok[8 vi - 2 .. 8 vi + 11] (see occ_window): 1 if
// (p, next live) == (a, b) (deltas counted), 0 if not, -1 if the window cannot decide (occ_slow).
__device__ __attribute__((always_inline)) inline int occ_fast1(const ScanArgs &A, NeighbourHist &H, int64_t vi, int k, uint32_t &xx,
                                                               uint32_t pw, uint4 cv, uint32_t nx, uint32_t ny) {
    const uint64_t W0 = (uint64_t)pw | ((uint64_t)cv.x << 32);
    const uint64_t W1 = (uint64_t)cv.y | ((uint64_t)cv.z << 32);
    const uint64_t W2 = (uint64_t)cv.w | ((uint64_t)nx << 32);
    const uint64_t W3 = (uint64_t)ny;
    auto win = [&](int i) -> uint32_t {
        const uint64_t q = i < 4 ? W0 : i < 8 ? W1 : i < 12 ? W2 : W3;
        return (uint32_t)(q >> ((i & 3) * 16)) & 0xffffu;
    };
    uint32_t live = 0;
#pragma unroll
    for (int i = 0; i < 14; i++) live |= (win(i) != HOLE ? 1u : 0u) << i;
    const int i = k + 2;
    const int64_t p = vi * 8 + k;
    const uint32_t after = live >> (i + 1), before = live & ((1u << i) - 1u);
    if (!after || !before || p < 2 || p + 3 >= A.n) return -1;
    const int q = i + 1 + __builtin_ctz(after);
    const int l = 31 - __builtin_clz(before);
    const uint32_t aq = live >> (q + 1);
    if (!aq) return -1;
    const int r = q + 1 + __builtin_ctz(aq);
    const uint32_t bl = live & ((1u << l) - 1u), ar = live >> (r + 1);
    const int ll = bl ? 31 - __builtin_clz(bl) : -1;
    const int rn = ar ? r + 1 + __builtin_ctz(ar) : 14;
    // every token the delta rules may look at must be inside the window
    if ((win(r) == A.a && rn >= 14) || (win(l) == A.b && ll < 0)) return -1;
    if (win(q) != A.b) return 0;
    if (A.count_deltas) {
        const uint32_t tl = win(l), tr = win(r);
        const bool merged_end = (tl == A.b) && (win(ll < 0 ? 0 : ll) == A.a);
        if (!merged_end) H.left((uint16_t)tl);
        const bool r_occ = (tr == A.a) && (win(rn > 13 ? 13 : rn) == A.b);
        if (r_occ) xx++;
        else H.right((uint16_t)tr);
    }
    return 1;
}

__device__ inline void pres_set(const ScanArgs &A, int64_t pos) {
    const uint64_t blk = (uint64_t)pos / PRES_BLK;
    atomicOr(&A.pres[(blk / PRES_GROUP) * A.vp + A.X], 1u << (blk % PRES_GROUP));
}

// One candidate position p holding the scan's key token (a, or b when by_b): is it (part of) an
// occurrence of (a, b)? On a hit *pr = the occurrence's start and the deltas are counted. The
// window around p comes from one 16-B vector (+ its cached neighbours in occ_vector).
template <bool RD = false>
__device__ inline bool resolve_candidate(const ScanArgs &A, NeighbourHist &H, int64_t p, bool by_b, int64_t nvec,
                                         uint32_t &xx, uint32_t &pr) {
    const uint16_t *tok = A.tok;
    const int64_t vi = p >> 3;
    const int k = (int)(p & 7);
    if (!by_b) {
        pr = (uint32_t)p;
        return occ_vector<RD>(A, H, vi, nvec, 1u << k, xx) != 0;
    }
    const uint4 cv = reinterpret_cast<const uint4 *>(tok)[vi];
    int64_t q = -1;  // the live token before p (q < 0: the left shard's, which owns the occurrence)
    uint32_t tq = HOLE;
    for (int j = k - 1; j >= 0 && q < 0; j--) {
        const uint32_t t = tok_at(cv, j);
        if (t != HOLE) { q = vi * 8 + j; tq = t; }
    }
    if (q < 0) {
        q = prev_live_h(A, p);
        if (q >= 0) tq = tok[q];
    }
    if (q >= 0 && tq == A.a && occ_vector<RD>(A, H, q >> 3, nvec, 1u << (q & 7), xx)) {
        pr = (uint32_t)q;
        return true;
    }
    return false;
}
// LDS neighbour histograms of one scan workgroup, shared by the stream and list forms (one allocation)
// occurrence records a list walk stages per workgroup before one reservation in the arena (a counter
// shared by every walking wave saturates at ~12 ns per atomic, MI355X_MICROARCH.md fanin; sized to keep
// four scan workgroups per CU in 160 KiB of LDS)
constexpr uint32_t LREC_CAP = 440;
struct ScanLds {
    uint32_t left[LDS_BINS], right[LDS_BINS];
    uint32_t hleft[HASH_BINS], hright[HASH_BINS];
    uint32_t any;
    unsigned long long scanned;
    uint32_t lrec[LREC_CAP];
    uint32_t lrec_n, lrec_base;
    uint32_t rd[3];  // multi-merge rounds: {new pairs, the largest new-pair count, queued adds} (NeighbourHist::rd)
};
// A list walk's wave with hit lanes: stage their record starts `pr` in the workgroup's LDS buffer; lanes
// past its capacity reserve in the arena directly (one atomic per wave). Every lane of the wave calls it.
__device__ inline void lrec_stage(const ScanArgs &A, ScanLds &S, bool hit, uint32_t pr, uint64_t hm) {
    const int lane = threadIdx.x & 63;
    uint32_t lbase = 0;
    if (lane == 0) lbase = atomicAdd(&S.lrec_n, (uint32_t)__popcll(hm));
    lbase = lane_bcast(lbase, 0);
    const uint32_t j = lbase + (uint32_t)__popcll(hm & ((1ull << lane) - 1ull));
    if (hit && j < LREC_CAP) S.lrec[j] = pr;
    const uint64_t over = __ballot(hit && j >= LREC_CAP);
    if (!over) return;
    uint32_t gbase = 0;
    if (lane == 0) {
        gbase = atomicAdd(A.rec_ctr, (uint32_t)__popcll(over));
        atomicAdd(A.occ_out, (uint32_t)__popcll(over));
    }
    gbase = lane_bcast(gbase, 0);
    if (hit && j >= LREC_CAP) {
        const uint32_t jr = gbase + (uint32_t)__popcll(over & ((1ull << lane) - 1ull));
        if (jr < A.rec_cap) A.rec[jr] = pr;
        else atomicOr(&A.st->error, 8u);
    }
}
// after the walk (a barrier since the last lrec_stage): one arena reservation for the staged records,
// then the copy. Every thread calls it. It does NOT end with a barrier: a caller that reuses S.lrec or
// S.lrec_base afterwards must barrier first (today the next walk's setup does).
__device__ inline void lrec_flush(const ScanArgs &A, ScanLds &S) {
    const uint32_t n = min(S.lrec_n, LREC_CAP);
    if (threadIdx.x == 0 && n) {
        S.lrec_base = atomicAdd(A.rec_ctr, n);
        atomicAdd(A.occ_out, n);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        const uint32_t jr = S.lrec_base + i;
        if (jr < A.rec_cap) A.rec[jr] = S.lrec[i];
        else atomicOr(&A.st->error, 8u);
    }
}
// zero the workgroup's neighbour histograms (every thread calls it, then a barrier)
__device__ inline void scan_lds_clear(ScanLds &S) {
    for (int i = threadIdx.x; i < LDS_BINS; i += blockDim.x) { S.left[i] = 0; S.right[i] = 0; }
    for (int i = threadIdx.x; i < HASH_BINS; i += blockDim.x) { S.hleft[i] = 0; S.hright[i] = 0; }
}
// the same through a round member walk's returning adds (NeighbourHist::gadd), then the workgroup's counts of
// new pairs and top-count pairs into the member's RoundHead words (every thread calls it)
// (every returning add of a thread is issued before the first one's value is used: a loop that tested each
// add's return before the next add waited one memory round trip per bin)
__device__ inline void scan_lds_flush_rd(const ScanArgs &A, ScanLds &S, const NeighbourHist &H) {
    static_assert(LDS_BINS % SCAN_THREADS == 0 && HASH_BINS % SCAN_THREADS == 0, "whole bins per thread");
    constexpr int NL = LDS_BINS / SCAN_THREADS, NH = HASH_BINS / SCAN_THREADS, NB = 2 * (NL + NH);
    uint32_t *g[NB];
    uint32_t v[NB], old[NB];
#pragma unroll
    for (int k = 0; k < NL; k++) {
        const uint32_t i = threadIdx.x + k * SCAN_THREADS;
        g[2 * k] = A.left + i;
        v[2 * k] = S.left[i];
        g[2 * k + 1] = A.right + i;
        v[2 * k + 1] = S.right[i];
    }
#pragma unroll
    for (int k = 0; k < NH; k++) {
        const uint32_t i = threadIdx.x + k * SCAN_THREADS, l = S.hleft[i], r = S.hright[i];
        g[2 * NL + 2 * k] = A.left + (l >> 16);
        v[2 * NL + 2 * k] = l & 0xffffu;
        g[2 * NL + 2 * k + 1] = A.right + (r >> 16);
        v[2 * NL + 2 * k + 1] = r & 0xffffu;
    }
    // the walk's queued adds (RD_QUEUE / SCAN_THREADS per thread) join the bins' adds: every add of the thread is
    // in flight before the first value is used (one memory round trip)
    constexpr int NQ = RD_QUEUE / SCAN_THREADS;
    const uint32_t nq = min(S.rd[2], RD_QUEUE);
    const uint32_t *q = rd_queue();
    uint32_t e[NQ], oq[NQ];
#pragma unroll
    for (int k = 0; k < NQ; k++) {
        const uint32_t i = k * SCAN_THREADS + threadIdx.x;
        e[k] = i < nq ? q[i] : ~0u;
    }
#pragma unroll
    for (int k = 0; k < NB; k++) old[k] = v[k] ? atomicAdd(g[k], v[k]) : 1u;
#pragma unroll
    for (int k = 0; k < NQ; k++) {
        const uint32_t vk = (e[k] >> 17) & 1u ? 0x8000u : 1u;
        oq[k] = e[k] != ~0u ? atomicAdd(((e[k] >> 16) & 1u ? A.right : A.left) + (e[k] & 0xFFFFu), vk) : 1u;
    }
    uint32_t births = 0, top = 0;  // (top: the largest value an add of this thread left in a delta word)
#pragma unroll
    for (int k = 0; k < NB; k++) {
        births += v[k] && old[k] == 0 ? 1u : 0u;
        top = v[k] ? max(top, old[k] + v[k]) : top;
    }
#pragma unroll
    for (int k = 0; k < NQ; k++) {
        const uint32_t vk = (e[k] >> 17) & 1u ? 0x8000u : 1u;
        births += e[k] != ~0u && oq[k] == 0 ? 1u : 0u;
        top = e[k] != ~0u ? max(top, oq[k] + vk) : top;
    }
    births = wave_sum_u32(births);  // (every thread calls it)
    top = wave_max_u32(top);
    if ((threadIdx.x & 63) == 0) {
        if (births) atomicAdd(&S.rd[0], births);
        if (top) atomicMax(&S.rd[1], top);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        if (S.rd[0]) atomicAdd(A.rd_birth, S.rd[0]);
        if (S.rd[1]) atomicMax(A.rd_nmax, S.rd[1]);
    }
}
// add the workgroup's neighbour histograms to the global deltas (every thread calls it)
__device__ inline void scan_lds_flush(ScanLds &S, uint32_t *g_left, uint32_t *g_right) {
    for (int i = threadIdx.x; i < LDS_BINS; i += blockDim.x) {
        const uint32_t l = S.left[i], r = S.right[i];
        if (l) atomicAdd(&g_left[i], l);
        if (r) atomicAdd(&g_right[i], r);
    }
    for (int i = threadIdx.x; i < HASH_BINS; i += blockDim.x) {
        const uint32_t l = S.hleft[i], r = S.hright[i];
        if (l) atomicAdd(&g_left[l >> 16], l & 0xffffu);
        if (r) atomicAdd(&g_right[r >> 16], r & 0xffffu);
    }
}
template <int UNROLL, bool NT, bool FILTER, bool PIPE, bool COMPACT, bool BATCH = false>
__device__ __attribute__((always_inline)) inline void scan_pairs_body(const ScanArgs A, ScanLds &S);
template <bool PROF = false, int NT = SCAN_THREADS, bool RD = false>
__device__ __attribute__((always_inline)) inline void scan_list_body(const ScanArgs A, bool by_b, const uint32_t *L,
                                                                     uint32_t len, ScanLds &S, const uint16_t *NB,
                                                                     uint32_t vb, uint32_t vg);
template <bool PROF = false, int NT = SCAN_THREADS, bool RD = false>
__device__ __attribute__((always_inline)) inline void scan_list_filtered(const ScanArgs A, bool by_b, uint32_t off, uint32_t len,
                                                                         ScanLds &S, uint32_t vb, uint32_t vg, bool all = false);
// the list forms of one pair scan: true when it walked a list (false: the stream form is the caller's)
// (RD: a multi-merge round's member walk, round_scan)
template <bool PROF = false, bool RD = false>
__device__ __attribute__((always_inline)) inline bool scan_list_dispatch(const ScanArgs &A, ScanLds &S, const StateHead &H,
                                                                         uint32_t vb, uint32_t vg) {
    // occurrence lists: key the scan by the shorter list when it is much shorter than the stream
    const uint32_t lists_x = H.lists_x;
    if (A.lists && A.a != A.b && H.lists_valid) {
        // lengths, offsets and the successor range: from the select's plan (no load here), else two
        // round trips
        uint32_t la, lb, oa, ob, r0 = NO_LIST, r1 = NO_LIST;
        bool ranged;
        if (A.plan_ok) {
            la = A.pl[0]; lb = A.pl[1]; oa = A.pl[2]; ob = A.pl[3]; r0 = A.pl[4]; r1 = A.pl[5];
            ranged = A.dir_row && r0 != NO_LIST && A.a < lists_x && A.b < lists_x;
        } else {
            la = A.lst_len[A.a]; lb = A.lst_len[A.b]; oa = A.lst_off[A.a]; ob = A.lst_off[A.b];
            const uint32_t ra = A.dir_row ? A.dir_row[A.a] : NO_LIST;
            ranged = ra != NO_LIST && A.a < lists_x && A.b < lists_x;
            if (ranged) {
                const uint64_t rb = (uint64_t)ra * A.dir_w + A.b;
                r0 = A.dir[rb];
                r1 = A.dir[rb + 1];
            }
        }
        const bool by_b = lb < la;
        const uint32_t len = by_b ? lb : la;
        // a's list sorted by build-time successor (a long list): by the invariant below, every occurrence
        // is in the range of successor b -- about the pair's count of entries, wherever a's list is
        if (ranged) {
            if (vb == 0 && threadIdx.x == 0) {
                A.st->scan_mode = 1;
                if (A.log) {
                    A.log[A.X - 256].mode = 1;
                    A.log[A.X - 256].list_len = r1 - r0;
                    A.log[A.X - 256].key_live = A.tokcnt ? (uint32_t)A.tokcnt[A.a] : 0u;
                    A.log[A.X - 256].range = 1;
                }
                if (PROF) A.st->pp_t[4] = 1;
            }
            scan_list_filtered<PROF, SCAN_THREADS, RD>(A, false, r0, r1 - r0, S, vb, vg, true);
            return true;
        }
        // Both tokens existed when the lists were built: since then a position's successor (its
        // predecessor) has only ever changed into a token created after the build (a merge at the
        // successor turns it into the new token; a hole appears only where the position itself is
        // merged), so every occurrence of (a, b) is an entry of a's list whose successor was b at the
        // build (of b's list whose predecessor was a). The walk reads that neighbour with the entry
        // (coalesced) and gathers the stream only where it matches: ~count gathers, not ~len.
        const bool NB = A.nb && A.a < lists_x && A.b < lists_x;
        if (len != NO_LIST && (uint64_t)len * A.list_ratio < (uint64_t)A.n) {
            if (vb == 0 && threadIdx.x == 0) {
                A.st->scan_mode = 1;
                if (A.log) {
                    A.log[A.X - 256].mode = 1;
                    A.log[A.X - 256].list_len = len;
                    A.log[A.X - 256].key_live = A.tokcnt ? (uint32_t)A.tokcnt[by_b ? A.b : A.a] : 0u;
                }
                if (PROF) A.st->pp_t[4] = 1;
            }
            if (NB) scan_list_filtered<PROF, SCAN_THREADS, RD>(A, by_b, by_b ? ob : oa, len, S, vb, vg);
            else scan_list_body<PROF, SCAN_THREADS, RD>(A, by_b, A.lists + (by_b ? ob : oa), len, S, nullptr, vb, vg);
            return true;
        }
    }
    return false;
}
// Self pair (a, a) from the occurrence list of a (one GPU, or the replicas of the late phase: no
// shard edges). A thread takes an entry that still holds a and starts a live run of a's, walks the
// run and takes every other pair of it from the start (left-greedy, basic_tokenizer.zig:217-226),
// with the count deltas of zbpe_scan_self: the token before the run is the first occurrence's left
// neighbour, adjacent occurrences give (X, X), and the last one's right neighbour is the lone
// trailing a of an odd run or the token after the run. Two walks: count, then (after one atomic per
// wave for the records) emit. O(list length) instead of three passes over the stream.
// (vb, vg: this workgroup among the vg that walk the list -- zbpe_scan_self_list on the host path, or a batch
// merge's scan, scan_dispatch)
__device__ __attribute__((always_inline)) inline void self_list_walk(const ScanArgs &A, ScanLds &S, uint32_t vb, uint32_t vg) {
    const uint32_t a = A.a, len = A.lst_len[a];
    if (len == NO_LIST || (vb > 0 && (uint64_t)vb * SCAN_THREADS >= len)) return;
    const uint32_t *L = A.lists + A.lst_off[a];
    scan_lds_clear(S);
    if (threadIdx.x == 0) S.any = 0;
    __syncthreads();
    NeighbourHist H{S.left, S.right, A.left, A.right, S.hleft, S.hright};
    const uint16_t *tok = A.tok;
    const int lane = threadIdx.x & 63;
    uint32_t xx = 0, any = 0;
    const uint32_t stride = vg * SCAN_THREADS, len64 = (len + 63) & ~63u;
    for (uint32_t i = vb * SCAN_THREADS + threadIdx.x; i - lane < len64; i += stride) {
        int64_t p = -1, l = -1;
        uint32_t run = 0;
        if (i < len) {
            p = L[i];
            if (tok[p] == a) {
                l = prev_live(tok, p);
                if (l < 0 || tok[l] != a)  // the run starts here: walk it
                    for (int64_t q = p; q >= 0 && tok[q] == a; q = next_live(tok, A.n, q)) run++;
            }
        }
        const uint32_t cnt = run / 2;
        const uint32_t incl = wave_incl_scan(cnt), total = (uint32_t)__shfl((int)incl, 63);
        if (!total) continue;
        any = 1;
        uint32_t base = 0;
        if (lane == 0) {
            base = atomicAdd(A.rec_ctr, total);
            atomicAdd(A.occ_out, total);
        }
        base = (uint32_t)__shfl((int)base, 0) + incl - cnt;
        if (!cnt) continue;
        if (A.count_deltas && l >= 0) H.left((uint16_t)tok[l]);
        int64_t q = p;
        for (uint32_t k = 0; k < cnt; k++) {
            if (base + k < A.rec_cap) A.rec[base + k] = (uint32_t)q;
            else atomicOr(&A.st->error, 8u);
            q = next_live(tok, A.n, q);       // the second a of occurrence k
            q = q >= 0 ? next_live(tok, A.n, q) : -1;  // the next live token after it
        }
        if (A.count_deltas) {
            xx += cnt - 1;
            if (run & 1) H.right((uint16_t)a);  // the lone trailing a
            else if (q >= 0) H.right((uint16_t)tok[q]);
        }
    }
    xx = wave_sum_u32(xx);  // (every thread of the block)
    if (lane == 0 && xx) atomicAdd(A.xx_out, xx);
    if (lane == 0 && any) S.any = 1;
    __syncthreads();
    if (S.any) scan_lds_flush(S, A.left, A.right);
}
// one pair scan with resolved arguments: the list form when the shorter token list is short
// enough, else the stream form
// (vb, vg: this workgroup among the vg that walk a list)
template <int UNROLL, bool NT, bool FILTER, bool PIPE, bool COMPACT, bool PROF = false, bool BATCH = false>
__device__ __attribute__((always_inline)) inline void scan_dispatch(const ScanArgs &A, ScanLds &S, const StateHead &H,
                                                                    uint32_t vb, uint32_t vg) {
    if (A.a == A.b) {  // a self pair the batch took (merge_begin_eval_v: a's list is short, the lists are valid)
        if (!A.lists || !H.lists_valid) {
            if (threadIdx.x == 0) atomicOr(&A.st->error, 2048u);
            return;
        }
        if (vb == 0 && threadIdx.x == 0) {
            A.st->scan_mode = 1;
            if (A.log) {
                A.log[A.X - 256].mode = 1;
                A.log[A.X - 256].list_len = A.lst_len[A.a];
                A.log[A.X - 256].key_live = A.tokcnt ? (uint32_t)A.tokcnt[A.a] : 0u;
            }
        }
        self_list_walk(A, S, vb, vg);
        return;
    }
    if (scan_list_dispatch<PROF>(A, S, H, vb, vg)) return;
    if (blockIdx.x == 0 && threadIdx.x == 0) A.st->scan_mode = 0;
    scan_pairs_body<UNROLL, NT, FILTER, PIPE, COMPACT, BATCH>(A, S);
}
// the scan plan says this merge's scan walks a list (scan_dispatch's test, on the plan's words)
__device__ inline bool plan_is_list(const ScanArgs &A, const StateHead &H) {
    if (!A.plan_ok || !A.lists || A.a == A.b || !H.lists_valid) return false;
    const uint32_t la = A.pl[0], lb = A.pl[1], r0 = A.pl[4];
    if (A.dir_row && r0 != NO_LIST && A.a < H.lists_x && A.b < H.lists_x) return true;
    const uint32_t len = lb < la ? lb : la;
    return len != NO_LIST && (uint64_t)len * A.list_ratio < (uint64_t)A.n;
}
// ------------------------------------------------------------------------------------------
// Multi-merge rounds (option round_k; RoundHead, types.hpp). The scan of a round: the merge (member 0,
// cur_key) and the tied keys its decision named in home-slot order (DevState::ph key, pr_key2 .. pr_key4: members 1..4 for
// merges cur_x + 1 ..), each walked by its own share of the grid into its own delta buffer (fixed
// layout: left at +0, right at +65536, tail at +131072) and records (arena_top + j * T: every member has
// the top count T of occurrences). Member walks also test every occurrence against the earlier members'
// pairs (occ_window RD: touching) and count their new pairs and top-count pairs (NeighbourHist::gadd);
// the replace decides from those which members the reference's loop would merge next (round_valid).
// RD_FREE_WGS extra workgroups bound the free Zig-map slots the members' order depends on, from the home
// summaries the naming decision saw (as pair_slack_block does for one candidate).
// ------------------------------------------------------------------------------------------
constexpr uint32_t RD_FREE_WGS = 2;
constexpr uint32_t RD_INF = 0xFFFFFFFFu;
__device__ inline uint32_t rd_delta_words() { return (uint32_t)(2 * 65536 + 64); }  // DELTA_WORDS (engine.hpp)
__device__ __attribute__((always_inline)) inline int32_t wave_carry_block(const HomeView &V, const uint32_t *cs, uint32_t b);
__device__ __attribute__((always_inline)) inline int64_t wave_homes_cover(const HomeView &V, uint32_t x, uint32_t y);
// One wave per range: range 0 = after the largest tied home's block up to C (no tied run may wrap past C-1),
// range j = after member j's home block up to the next tied home (member j stays first in slot order)
__device__ inline void round_free(const ScanArgs &A0, uint32_t K, const PairTail &PT, uint32_t w) {
    DevState *st = A0.st;
    if (w >= ROUND_MAX || (w > 0 && w >= K)) return;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t H[ROUND_MAX + 1] = {0u, PT.h2, PT.h3, PT.h4, PT.h5, PT.h6};  // member j's home: H[j]; the next tied one: H[j + 1]
    const HomeView &V = A0.hv;
    const bool ok = A0.cs && V.C >= (uint32_t)(SUMM_SLOTS * SUPER_BLOCKS);
    int64_t f = -1;
    if (ok) {
        const uint32_t x = w == 0 ? (PT.hmax / SUMM_SLOTS + 1) * SUMM_SLOTS : (H[w] / SUMM_SLOTS + 1) * SUMM_SLOTS;
        const uint32_t y = w == 0 ? V.C : H[w + 1];
        if (w > 0 && y == 0) {
            f = -1;  // no next tied home (the member is the last tied key: the replace needs no bound)
        } else if (x < y) {
            const int64_t c = wave_carry_block(V, A0.cs, x / SUMM_SLOTS);
            const int64_t h = wave_homes_cover(V, x, y);
            f = max((int64_t)0, (int64_t)y - x - h - c);
        } else {
            f = 0;
        }
    }
    if (lane == 0) st->rd.freeb[w] = (int32_t)min(f, (int64_t)0x7FFFFFFF);
}
// (P, PT, pr_full: the naming decision's words, U: the untied names, loaded by the kernel's entry with the state head)
// (PROF: the pipeline probes, st->pp_t: the member walks' phases as a list scan's, the bound workgroups' end in pp_t[13])
template <int UNROLL, bool NT, bool FILTER, bool PIPE, bool COMPACT, bool BATCH, bool PROF = false>
__device__ __attribute__((always_inline)) inline void round_scan(const ScanArgs &A0, const StateHead &H, ScanLds &S, const PairHead &P,
                                                                 const PairTail &PT, const RoundPlans &RPL, uint32_t pr_full,
                                                                 const UntiedHead &U) {
    DevState *st = A0.st;
    const unsigned long long t_in = PROF ? wall_clock64() : 0ull;
    const uint32_t X0 = H.cur_x, T = H.top_count, G = gridDim.x - RD_FREE_WGS;
    ScanArgs A = scan_args_resolve(A0, H, X0);
    // the members: merge X0 and the keys its decision named (its candidate slot names X0 + 1: a tied round), or the keys of the next
    // distinct counts the select that began X0 named (ur.x == X0: an untied round), while every one is a list walk
    // with room in the arena and below the vocabulary's end
    const bool tied = P.x == X0 + 1 && pr_full == X0 + 1, untied = !tied && U.x == X0 && U.n > 0;
    const uint32_t keys[ROUND_MAX] = {pair_key(A.a, A.b), tied ? P.key : U.key[0], tied ? PT.key2 : U.n > 1 ? U.key[1] : NO_ID,
                                      tied ? PT.key3 : U.n > 2 ? U.key[2] : NO_ID, tied ? PT.key4 : U.n > 3 ? U.key[3] : NO_ID};
    const uint32_t cnts[ROUND_MAX] = {T, tied ? T : U.cnt[0], tied ? T : U.cnt[1], tied ? T : U.cnt[2], tied ? T : U.cnt[3]};
    uint32_t K = 1;
    if (A0.round >= 2 && (tied || untied) && plan_is_list(A, H) && T) {
        const uint32_t kmax = min(min((uint32_t)A0.round, (uint32_t)ROUND_MAX), A0.x_end > X0 ? A0.x_end - X0 : 1u);
        // (a self pair's occurrences overlap in runs: the touch tests assume none do, so one ends the members)
        // (records: member j's at arena_top + j T, at most T each -- an untied member's count is below T)
        while (K < kmax && keys[K] != NO_ID && (keys[K] & 0xFFFF) != (keys[K] >> 16) && (uint64_t)(K + 1) * T <= (uint64_t)A.rec_cap) K++;
    }
    // Workgroups [0, RD_FREE_WGS) bound the free slots (one wave per range) and store the round's words; the
    // members' walks take the others in turn (member j: every K-th from RD_FREE_WGS + j), so that every member's
    // first workgroups are among the grid's first: the dispatcher starts workgroups in order, ~1000 of them
    // took several microseconds, and a member (or bound) placed after them started that much later.
    if (K == 1) {  // a round of one: the merge's own scan (any form; the stream form strides over the whole grid)
        if (blockIdx.x == 0 && threadIdx.x == 0) {  // (the replace reads the round's member keys)
            st->rd.n = 1;
            st->rd.key[0] = keys[0];
        }
        scan_dispatch<UNROLL, NT, FILTER, PIPE, COMPACT, false, BATCH>(A, S, H, blockIdx.x, gridDim.x);
        return;
    }
    if (blockIdx.x < RD_FREE_WGS) {
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            st->rd.n = K;
            st->rd.ties = tied ? P.ties : 0u;
            st->rd.live0 = st->live;
            st->rd.ties0 = st->tie_count;  // (merge X0's tied pairs, as its begin logged them: 1 in an untied round)
#pragma unroll
            for (int e = 0; e < ROUND_MAX; e++) {
                st->rd.key[e] = (uint32_t)e < K ? keys[e] : NO_ID;
                st->rd.cnt[e] = (uint32_t)e < K ? cnts[e] : 0u;
            }
        }
        if (tied) round_free(A0, K, PT, blockIdx.x * (SCAN_THREADS / 64) + (threadIdx.x >> 6));
        if (PROF) {
            __syncthreads();
            if (threadIdx.x == 0) atomicMax(&st->pp_t[13], (unsigned long long)wall_clock64());
        }
        return;
    }
    A.rd_top = &st->rd.top[0];
    A.rd_birth = &st->rd.birth[0];
    A.rd_touch = &st->rd.touch[0];
    A.rd_nmax = &st->rd.nmax[0];
    A.rd_jn = &st->rd_jn[0];
#pragma unroll
    for (int e = 0; e < ROUND_MAX; e++) A.tk[e] = (uint32_t)e < K ? keys[e] : 0u;
    A.ntk = K;
    A.tkj = 0;
    const uint32_t bi = blockIdx.x - RD_FREE_WGS, j = bi % K, vb = bi / K, vg = (G - j + K - 1) / K;
    if (j == 0) {
        scan_list_dispatch<PROF, true>(A, S, H, vb, vg);  // (a list walk: plan_is_list)
        return;
    }
    // member j: merge X0 + j of pair keys[j]; its list plan (two dependent round trips), then a list walk
    const uint32_t a = keys[j] & 0xFFFF, b = keys[j] >> 16, dw = rd_delta_words();
    A.a = a;
    A.b = b;
    A.X = X0 + j;
    A.left = A0.left + (size_t)j * dw;
    A.right = A.left + 65536;
    A.xx_out = A.left + 2 * 65536;
    A.occ_out = A.xx_out + 1;
    A.rec = A0.rec + H.arena_top + j * T;  // (rec_arena: records in the arena after the lists)
    A.rec_cap = T;
    A.rec_ctr = &st->rd.rec[j];
    A.pres = nullptr;
    // (the walk sizes its entries per thread from the pair's count)
#pragma unroll
    for (int e = 1; e < ROUND_MAX; e++)
        if ((uint32_t)e == j) A.top_count = cnts[e];
    // the plan the naming decision loaded (RoundPlans, entry words), else two dependent round trips
    uint32_t kj = 0;
#pragma unroll
    for (int e = 0; e < ROUND_MAX - 1; e++) kj = (uint32_t)e == j - 1 ? RPL.key[e] : kj;
    const bool planned = RPL.gen == A0.gen && kj == keys[j];
    if (planned) {
#pragma unroll
        for (int e = 0; e < ROUND_MAX - 1; e++)
            if ((uint32_t)e == j - 1)
#pragma unroll
                for (int k = 0; k < 6; k++) A.pl[k] = RPL.plan[e][k];
    } else {
        const uint32_t la = A.lst_len[a], lb = A.lst_len[b], oa = A.lst_off[a], ob = A.lst_off[b];
        const uint32_t ra = A.dir_row && a < H.lists_x && b < H.lists_x ? A.dir_row[a] : NO_LIST;
        uint32_t r0 = NO_LIST, r1 = NO_LIST;
        if (ra != NO_LIST) {
            const uint64_t rb = (uint64_t)ra * A.dir_w + b;
            r0 = A.dir[rb];
            r1 = A.dir[rb + 1];
        }
        A.pl[0] = la; A.pl[1] = lb; A.pl[2] = oa; A.pl[3] = ob; A.pl[4] = r0; A.pl[5] = r1;
    }
    A.plan_ok = 1;
    if (PROF && vb == 0 && threadIdx.x == 0) {  // member j's walk starts (its plan in): sel_prof[22] from the launch's start
        atomicAdd(&st->sel_prof[22], wall_clock64() - t_in);
        atomicAdd(&st->sel_prof[23], planned ? 1ull : 1ull << 32);
    }
    A.tkj = j;
    A.rd_touch = &st->rd.touch[j];
    A.rd_top = &st->rd.top[j];
    A.rd_birth = &st->rd.birth[j];
    A.rd_nmax = &st->rd.nmax[j];
    if (scan_list_dispatch<PROF, true>(A, S, H, vb, vg) && vb == 0 && threadIdx.x == 0) atomicOr(&st->rd.top[j], RT_WALKED);
}
// PROF (option sel_prof): the pipeline probes; a separate instantiation, so the production kernel's
// code and register allocation are untouched by them
// ROUND: the multi-merge round's scan (round_scan; batch mode, one GPU or replicas)
template <int UNROLL, bool NT, bool FILTER, bool PIPE = true, bool COMPACT = false, bool PROF = false, bool BATCH = false,
          bool ROUND = false>
// stp == A0.st, as the leading pointer argument: a build with kernarg preloading (Makefile KP=1) has it in
// SGPRs at entry, so the state head load needs no kernarg round trip first (aggregates are not preloaded)
__global__ void __launch_bounds__(SCAN_THREADS) __attribute__((amdgpu_waves_per_eu(4))) zbpe_scan_pairs_t(const DevState *stp, ScanArgs A0) {
    if (PROF && blockIdx.x == 0 && threadIdx.x == 0) {  // the last select's end -> this scan's start
        DevState *st = A0.st;
        const unsigned long long now = wall_clock64();
        unsigned long long *P = st->pipe_prof[pp_bucket(A0.X)];
        if (st->pp_t[7]) { P[8] += now - st->pp_t[7]; P[9]++; st->pp_t[7] = 0; }
        st->pp_t[0] = now;
    }
    // the state head and the argument words a list walk needs, fetched together (one round trip, not a
    // chain of kernarg cache misses in the order the code first uses them): one asm consumes them all
    const StateHead H = *reinterpret_cast<const StateHead *>(stp);
    // a round's scan: the naming decision's words in the same round trip
    PairHead P{};
    PairTail PT{};
    RoundPlans RPL{};
    UntiedHead U{};
    uint32_t pr_full = 0;
    if (ROUND) {
        // (both candidate slots, in the head's round trip: the round's merge picks its successor's, DevState::ph)
        const PairHead Pa = stp->ph[0], Pb = stp->ph[1];
        asm volatile("" ::"s"(Pa.x), "s"(Pa.key), "s"(Pa.ties), "s"(Pb.x), "s"(Pb.key), "s"(Pb.ties));
        P = (H.cur_x + 1) & 1 ? Pb : Pa;
        PT = *reinterpret_cast<const PairTail *>(&stp->pr_plan[0]);
        RPL = stp->rp;
        U = stp->ur;
        pr_full = stp->pr_full;
        asm volatile("" ::"s"(PT.key2), "s"(PT.key3), "s"(PT.key4), "s"(PT.h2), "s"(PT.h3),
                     "s"(PT.h4), "s"(PT.h5), "s"(PT.h6), "s"(PT.hmax), "s"(pr_full), "s"(RPL.gen), "s"(RPL.key[0]),
                     "s"(RPL.key[1]), "s"(RPL.key[2]), "s"(RPL.key[3]));
        asm volatile("" ::"s"(U.x), "s"(U.n), "s"(U.key[0]), "s"(U.key[1]), "s"(U.key[2]), "s"(U.key[3]), "s"(U.cnt[0]),
                     "s"(U.cnt[1]), "s"(U.cnt[2]), "s"(U.cnt[3]));
        // the round's argument words (a kernarg word first used deep in the walk's setup cost a cache-miss round trip)
        asm volatile("" ::"s"(A0.round), "s"(A0.x_end), "s"(A0.lst_len), "s"(A0.lst_off), "s"(A0.dir), "s"(A0.dir_w),
                     "s"(A0.log), "s"(A0.list_ratio), "s"(A0.nb), "s"(A0.tokcnt), "s"(A0.cs), "s"(A0.hv.summ), "s"(A0.hv.sup),
                     "s"(A0.hv.C), "s"(A0.hv.nb), "s"(A0.hv.nsb), "s"(A0.prof));
    }
    asm volatile("" ::"s"(A0.dyn), "s"(A0.X), "s"(A0.gen), "s"(A0.rec_arena), "s"(A0.rec_cap), "s"(A0.count_deltas),
                 "s"(A0.tok), "s"(A0.lists), "s"(A0.rec), "s"(A0.left), "s"(A0.right), "s"(A0.dir_row), "s"(A0.xx_out),
                 "s"(A0.occ_out), "s"(A0.n), "s"(H.halt), "s"(H.cur_key), "s"(H.arena_top), "s"(H.lists_valid),
                 "s"(H.lists_x), "s"(H.top_count), "s"(H.plan_x), "s"(H.plan_key), "s"(H.plan_gen), "s"(H.plan_la),
                 "s"(H.plan_lb), "s"(H.plan_oa), "s"(H.plan_ob), "s"(H.plan_r0), "s"(H.plan_r1));
    if (A0.dyn && H.halt) return;
    __shared__ ScanLds S;
    if (ROUND) {
        round_scan<UNROLL, NT, FILTER, PIPE, COMPACT, BATCH, PROF>(A0, H, S, P, PT, RPL, pr_full, U);
        return;
    }
    const ScanArgs A = scan_args_resolve(A0, H, A0.X);
    scan_dispatch<UNROLL, NT, FILTER, PIPE, COMPACT, PROF, BATCH>(A, S, H, blockIdx.x, gridDim.x);
}

// ------------------------------------------------------------------------------------------
// Batched encode (Engine::encode, basic_tokenizer.zig:71-88). A batch holds consecutive merges of
// which none uses a token that an earlier one of the batch uses or makes: their occurrences do not
// interact, so applying them together equals applying them in rank order. One launch scans every
// merge of the batch (grid row y = merge y), one applies them. Records go to a scratch region per
// merge sized by min(live count of a, live count of b) (a sound bound; the batch's tokens are
// distinct, so the regions sum to at most the live tokens), then the apply copies them to the arena,
// where they become the new tokens' occurrence lists.
// ------------------------------------------------------------------------------------------
constexpr int ENC_MAX_BATCH = 32;
struct EncBatch {
    uint32_t a[ENC_MAX_BATCH], b[ENC_MAX_BATCH], X[ENC_MAX_BATCH];
    uint32_t nb;
};
__device__ inline uint32_t enc_bound(const EncBatch &E, const int32_t *cnt, uint32_t k) {
    return (uint32_t)max(0, min(cnt[E.a[k]], cnt[E.b[k]]));
}
// scratch offset and bound of merge j (every thread computes it; nb <= 32 cached loads)
__device__ inline uint32_t enc_scratch_off(const EncBatch &E, const int32_t *cnt, uint32_t j, uint32_t *bound) {
    uint32_t off = 0;
    for (uint32_t k = 0; k < j; k++) off += enc_bound(E, cnt, k);
    *bound = enc_bound(E, cnt, j);
    return off;
}
__global__ void __launch_bounds__(SCAN_THREADS) zbpe_encode_scan_batch(ScanArgs A0, EncBatch E, const int32_t *__restrict__ cnt,
                                                                       uint32_t *ctr, uint32_t *scratch) {
    __shared__ ScanLds S;
    const uint32_t j = blockIdx.y;
    uint32_t bound;
    const uint32_t off = enc_scratch_off(E, cnt, j, &bound);
    ScanArgs A = A0;
    A.a = E.a[j];
    A.b = E.b[j];
    A.X = E.X[j];
    A.rec = scratch + off;
    A.rec_cap = bound;
    A.rec_ctr = &ctr[j];
    A.rec_arena = 0;
    A.dyn = 0;
    const StateHead H = load_head(A0.st);
    A.top_count = H.top_count;
    A.plan_ok = 0;
    scan_dispatch<4, true, true, true, true>(A, S, H, blockIdx.x, gridDim.x);
}
__global__ void __launch_bounds__(256) zbpe_encode_apply_batch(uint16_t *tok, int64_t n, EncBatch E, const uint32_t *__restrict__ scratch,
                                                               int32_t *cnt, uint32_t *ctr, uint32_t *arena, DevState *st, Tables T) {
    const uint32_t j = blockIdx.y;
    uint32_t bound, pre = 0;
    const uint32_t off = enc_scratch_off(E, cnt, j, &bound);
    for (uint32_t k = 0; k < j; k++) pre += min(ctr[k], enc_bound(E, cnt, k));
    const uint32_t m = min(ctr[j], bound), base = st->arena_top + pre, X = E.X[j];
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < m; i += gridDim.x * 256) {
        const int64_t p = scratch[off + i];
        tok[p] = (uint16_t)X;
        const int64_t q = next_live(tok, n, p);
        if (q >= 0) tok[q] = HOLE;
        arena[base + i] = (uint32_t)p;
    }
    __shared__ uint32_t s_last;
    __syncthreads();  // every thread of the block has read the counts and arena_top
    if (threadIdx.x == 0) s_last = atomicAdd(&st->ticket, 1u) == gridDim.x * gridDim.y - 1;
    __syncthreads();
    if (!s_last || threadIdx.x) return;
    uint32_t top = st->arena_top, total = 0;
    for (uint32_t k = 0; k < E.nb; k++) {
        const uint32_t mk = min(ctr[k], enc_bound(E, cnt, k));
        if (ctr[k] > mk) atomicOr(&st->error, 8u);
        T.lst_off[E.X[k]] = top;
        T.lst_len[E.X[k]] = mk;
        top += mk;
        total += mk;
        ctr[k] = 0;
    }
    for (uint32_t k = 0; k < E.nb; k++) {  // after every bound above was read
        const int32_t mk = (int32_t)T.lst_len[E.X[k]];
        cnt[E.X[k]] = mk;
        cnt[E.a[k]] -= mk;
        cnt[E.b[k]] -= mk;
    }
    st->arena_top = top;
    st->total_occ += total;
    st->ticket = 0;
}

// A walk of b's list (sharded): the occurrence leaving the shard -- its a this shard's last live token, its b the next
// shard's first (the halo), in no list here -- is this shard's; one thread checks and records it. Returns 1 if found.
__device__ inline uint32_t list_edge_occurrence(const ScanArgs &A, NeighbourHist &H, uint32_t &xx) {
    if (A.halo.nright == 0 || halo_right(A.halo, 0) != A.b) return 0;
    const int64_t p = prev_live(A.tok, A.n);
    if (p < 0 || A.tok[p] != A.a || !occ_slow(A, H, p, xx)) return 0;
    const uint32_t j = atomicAdd(A.rec_ctr, 1u);
    atomicAdd(A.occ_out, 1u);
    if (j < A.rec_cap) A.rec[j] = (uint32_t)p;
    else atomicOr(&A.st->error, 8u);
    return 1;
}

// Filtered list scan (scan_dispatch: both tokens existed at the list build). Each thread reads the
// build-time neighbours of LIST_EPT consecutive entries (two 16-B loads of the u16 neighbour array,
// coalesced); only entries whose neighbour was the pair's other token can be occurrences (about the
// pair's count of them, against the list's length). A wave compacts its matches in registers (a
// shuffle binary search over the lanes' inclusive match counts) and resolves them 64 at a time with
// the stream window loaded in one round trip. Few, fat workgroups: the per-wave record reservation
// and the per-block histogram flush are atomics on shared counters, and their number is what bounds
// a late merge's scan, not the bytes.
constexpr int LIST_EPT = 16;  // the most entries a thread filters
// (vb, vg: this workgroup's index among the vg workgroups that walk the list; NT threads each)
// all: every entry of [off, off + len) is a candidate (a successor range, zbpe_list_sort_succ: no
// neighbour words to filter), at most four per thread.
template <bool PROF, int NT, bool RD>
__device__ __attribute__((always_inline)) inline void scan_list_filtered(const ScanArgs A, bool by_b, uint32_t off, uint32_t len,
                                                                         ScanLds &S, uint32_t vb, uint32_t vg, bool all) {
    // entries per thread: about one match per two lanes (a wave resolves its matches 64 at a time, one
    // latency chain per round): the list's length over the pair's count (training; encode: 4)
    const uint32_t cnt = A.count_deltas ? A.top_count : 0u;
    const uint32_t ratio = cnt ? len / cnt : 8u;
    const uint32_t ept = all ? (ratio >= 4 ? 4u : ratio >= 2 ? 2u : 1u)
                             : ratio >= 32 ? 16u : ratio >= 16 ? 8u : ratio >= 8 ? 4u : ratio >= 4 ? 2u : 1u;
    const uint32_t per_block = NT * ept;
    const uint32_t ab = off & ~7u;                    // 16-B aligned start of the neighbour words
    const uint32_t span = off + len - ab;             // entries from ab to the list's end
    if (vb > 0 && (uint64_t)vb * per_block >= span) return;
    const uint32_t *NB = A.nb, sh = by_b ? 16u : 0u;  // the build-time neighbour on the partner's side
    const uint32_t partner = by_b ? A.a : A.b, key = by_b ? A.b : A.a;
    scan_lds_clear(S);
    if (threadIdx.x == 0) { S.any = 0; S.lrec_n = 0; S.rd[0] = S.rd[1] = S.rd[2] = 0; }
    __syncthreads();
    if (PROF && threadIdx.x == 0) atomicMax(&A.st->pp_t[1], (unsigned long long)wall_clock64());
    NeighbourHist H{S.left, S.right, A.left, A.right, S.hleft, S.hright};
    if (RD) H.rd = S.rd;
    const uint4 *tv = reinterpret_cast<const uint4 *>(A.tok);
    const int64_t nvec = (A.n + 7) / 8;
    const int lane = threadIdx.x & 63;
    uint32_t xx = 0, any = 0;
    if (by_b && vb == 0 && threadIdx.x == 0) any = list_edge_occurrence(A, H, xx);
    const uint32_t gstride = vg * per_block;
    // block-uniform trip count (every lane of a wave takes part in the shuffles and ballots)
    for (uint32_t b0 = vb * per_block; b0 < span; b0 += gstride) {
        const uint32_t e0 = ab + b0 + threadIdx.x * ept;  // this thread's first entry (absolute)
        uint32_t mk = 0;
        if (all) {
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t e = e0 + k;
                mk |= ((uint32_t)k < ept && e >= off && e < off + len) ? (1u << k) : 0u;
            }
        } else if (e0 < off + len) {
            if (ept >= 8) {  // 16-B aligned words (ab and ept are multiples of 8)
                const uint4 *q = reinterpret_cast<const uint4 *>(NB + e0);
                const uint4 none = make_uint4(~0u, ~0u, ~0u, ~0u);
                const uint4 w[4] = {q[0], q[1], ept == 16 ? q[2] : none, ept == 16 ? q[3] : none};
#pragma unroll
                for (int k = 0; k < 16; k++) {
                    const uint4 v = w[k >> 2];
                    const uint32_t word = (k & 3) == 0 ? v.x : (k & 3) == 1 ? v.y : (k & 3) == 2 ? v.z : v.w;
                    const uint32_t e = e0 + k;
                    mk |= (((word >> sh) & 0xFFFFu) == partner && e >= off && e < off + len && (uint32_t)k < ept) ? (1u << k) : 0u;
                }
            } else {
                uint32_t t[4];
#pragma unroll
                for (int k = 0; k < 4; k++) t[k] = (uint32_t)k < ept ? NB[e0 + k] : ~0u;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const uint32_t e = e0 + k;
                    mk |= (((t[k] >> sh) & 0xFFFFu) == partner && e >= off && e < off + len) ? (1u << k) : 0u;
                }
            }
        }
        // a successor range: the wave's matches are the in-range entries of its chunk, contiguous, so
        // match j is entry lo + j (no scan, no shuffle search)
        uint32_t c = 0, incl = 0, M, lo = 0;
        if (all) {
            const uint32_t cs = ab + b0 + (threadIdx.x & ~63u) * ept;
            const uint32_t hi = min(cs + 64u * ept, off + len);
            lo = max(cs, off);
            M = hi > lo ? hi - lo : 0u;
        } else {
            c = (uint32_t)__popc(mk);
            incl = wave_incl_scan_dpp(c);
            M = lane_bcast(incl, 63);
        }
        for (uint32_t r0 = 0; r0 < M; r0 += 64) {
            const uint32_t j = r0 + lane;
            int64_t p = -1;
            int owner = 0;  // the lane holding match j: the first whose inclusive count exceeds j
            if (all) {
                if (j < M) p = (int64_t)A.lists[lo + j];
            } else {
                int lo2 = 0, hi = 63;
                const uint32_t jj = j < M ? j : 0u;
#pragma unroll
                for (int s2 = 0; s2 < 6; s2++) {
                    const int mid = (lo2 + hi) >> 1;
                    const uint32_t v = (uint32_t)__shfl((int)incl, mid);
                    if (v > jj) hi = mid;
                    else lo2 = mid + 1;
                }
                owner = lo2;
                const uint32_t o_incl = (uint32_t)__shfl((int)incl, owner), o_c = (uint32_t)__shfl((int)c, owner);
                const uint32_t o_mk = (uint32_t)__shfl((int)mk, owner);
                if (j < M) {
                    uint32_t rank = j - (o_incl - o_c), m = o_mk;  // the rank-th set bit of the owner's mask
                    for (uint32_t q = 0; q < rank; q++) m &= m - 1;
                    const uint32_t e = ab + b0 + ((threadIdx.x & ~63u) + (uint32_t)owner) * ept + (uint32_t)__ffs(m) - 1;
                    p = (int64_t)A.lists[e];
                }
            }
            // the entry's stream window in one round trip (vector, the word before, the two after)
            const int64_t vi = p < 0 ? 0 : (p >> 3);
            const uint4 cv = tv[vi];
            const uint32_t pw0 = tv[vi > 0 ? vi - 1 : 0].w;
            const uint2 nv0 = *reinterpret_cast<const uint2 *>(&tv[vi + 1 < nvec ? vi + 1 : vi]);
            bool hit = false;
            uint32_t pr = 0;
            if (p >= 0) {
                const int k = (int)(p & 7);
                if (tok_at(cv, k) == key) {
                    const uint32_t pw = vi > 0 ? pw0 : 0xffffffffu;
                    const uint32_t nx = vi + 1 < nvec ? nv0.x : 0xffffffffu, ny = vi + 1 < nvec ? nv0.y : 0xffffffffu;
                    if (!by_b) {
                        pr = (uint32_t)p;
                        hit = occ_window<RD>(A, H, vi, 1u << k, xx, pw, cv, nx, ny) != 0;
                    } else {
                        int jb = k - 1;  // the live token before p inside the vector
                        while (jb >= 0 && tok_at(cv, jb) == HOLE) jb--;
                        if (jb >= 0) {
                            if (tok_at(cv, jb) == A.a && occ_window<RD>(A, H, vi, 1u << jb, xx, pw, cv, nx, ny)) {
                                pr = (uint32_t)(vi * 8 + jb);
                                hit = true;
                            }
                        } else {
                            hit = resolve_candidate<RD>(A, H, p, by_b, nvec, xx, pr);
                        }
                    }
                }
            }
            const uint64_t hm = __ballot(hit);
            if (!hm) continue;
            any = 1;
            lrec_stage(A, S, hit, pr, hm);
        }
    }
    xx = wave_sum_u32(xx);  // (every thread of the block)
    if (lane == 0 && xx) atomicAdd(A.xx_out, xx);
    if (RD && lane == 0 && xx) atomicOr(A.rd_top, RT_XX);
    if (lane == 0 && any) S.any = 1;
    __syncthreads();
    if (PROF && threadIdx.x == 0) atomicMax(&A.st->pp_t[2], (unsigned long long)wall_clock64());
    if (S.any) {
        lrec_flush(A, S);
        if (RD) scan_lds_flush_rd(A, S, H);
        else scan_lds_flush(S, A.left, A.right);
    }
    if (PROF) {
        __syncthreads();
        if (threadIdx.x == 0) atomicMax(&A.st->pp_t[3], (unsigned long long)wall_clock64());
    }
}

// List scan: every entry of the key token's list is a position that held the key when it was
// listed; entries overwritten since (merged or turned into holes) fail the token check.
template <bool PROF, int NT, bool RD>
__device__ __attribute__((always_inline)) inline void scan_list_body(const ScanArgs A, bool by_b, const uint32_t *L,
                                                                     uint32_t len, ScanLds &S, const uint16_t *NB,
                                                                     uint32_t vb, uint32_t vg) {
    // blocks past the list leave before touching LDS (the grid is sized for a stream scan)
    if (vb > 0 && (uint64_t)vb * NT >= len) return;
    uint32_t *s_left = S.left, *s_right = S.right;
    uint32_t &s_any = S.any;
    scan_lds_clear(S);
    if (threadIdx.x == 0) { s_any = 0; S.lrec_n = 0; S.rd[0] = S.rd[1] = S.rd[2] = 0; }
    __syncthreads();
    if (PROF && threadIdx.x == 0) atomicMax(&A.st->pp_t[1], (unsigned long long)wall_clock64());
    NeighbourHist H{s_left, s_right, A.left, A.right, S.hleft, S.hright};
    if (RD) H.rd = S.rd;
    const uint16_t *tok = A.tok;
    const uint32_t key = by_b ? A.b : A.a;
    uint32_t xx = 0, any = 0;
    const int lane = threadIdx.x & 63;
    if (by_b && vb == 0 && threadIdx.x == 0) any = list_edge_occurrence(A, H, xx);
    const uint32_t stride = vg * NT;
    const int64_t nvec = (A.n + 7) / 8;
    const uint32_t len64 = (len + 63) & ~63u;  // wave-uniform trip count (wave_append)
    // LU entries per thread in flight: their list words, then their 16-B vectors (one request each,
    // clamped addresses, no branches); an entry that still holds the key and whose partner slot inside
    // the vector is the other token or a hole (or lies outside the vector) loads the neighbouring
    // words too and is resolved. Most entries end after the one vector load.
    constexpr int LU = 3;
    const uint4 *tv = reinterpret_cast<const uint4 *>(tok);
    const uint32_t partner = by_b ? A.a : A.b;  // the neighbour a filtered entry must have had (NB)
    for (uint32_t i0 = vb * NT + threadIdx.x; i0 - lane < len64; i0 += LU * stride) {
        int64_t ps[LU];
#pragma unroll
        for (int u = 0; u < LU; u++) {
            const uint32_t i = i0 + u * stride, ic = i < len ? i : len - 1;
            const uint32_t e = L[ic];
            const bool keep = i < len && (!NB || NB[ic] == partner);
            ps[u] = keep ? (int64_t)e : -1;
        }
        bool anyp = false;
#pragma unroll
        for (int u = 0; u < LU; u++) anyp |= ps[u] >= 0;
        if (NB && !__ballot(anyp)) continue;  // no entry of the wave can be an occurrence
        uint4 cvs[LU];
#pragma unroll
        for (int u = 0; u < LU; u++) cvs[u] = tv[(ps[u] < 0 ? 0 : ps[u]) >> 3];
#pragma unroll 1
        for (int u = 0; u < LU; u++) {
            // this entry's values (selects, not an indexed private array)
            int64_t p = ps[0];
            uint4 cv = cvs[0];
#pragma unroll
            for (int k2 = 1; k2 < LU; k2++)
                if (u == k2) {
                    p = ps[k2];
                    cv = cvs[k2];
                }
            bool cand = false;
            if (p >= 0) {
                const int k = (int)(p & 7);
                if (tok_at(cv, k) == key) {
                    const uint32_t t = !by_b ? (k < 7 ? tok_at(cv, k + 1) : A.b) : (k > 0 ? tok_at(cv, k - 1) : A.a);
                    cand = t == HOLE || t == (by_b ? A.a : A.b);
                }
            }
            uint32_t pw = 0xffffffffu, nx = 0xffffffffu, ny = 0xffffffffu;
            if (cand) {
                const int64_t vi = p >> 3;
                if (vi > 0) pw = tv[vi - 1].w;
                if (vi + 1 < nvec) {
                    const uint2 nv = *reinterpret_cast<const uint2 *>(&tv[vi + 1]);
                    nx = nv.x;
                    ny = nv.y;
                }
            }
            bool hit = false;
            uint32_t pr = 0;
            if (cand) {
                const int64_t vi = p >> 3;
                const int k = (int)(p & 7);
                {
                    if (!by_b) {
                        pr = (uint32_t)p;
                        hit = occ_window<RD>(A, H, vi, 1u << k, xx, pw, cv, nx, ny) != 0;
                    } else {
                        int j = k - 1;  // the live token before p inside the vector
                        while (j >= 0 && tok_at(cv, j) == HOLE) j--;
                        if (j >= 0) {
                            if (tok_at(cv, j) == A.a && occ_window<RD>(A, H, vi, 1u << j, xx, pw, cv, nx, ny)) {
                                pr = (uint32_t)(vi * 8 + j);
                                hit = true;
                            }
                        } else {
                            hit = resolve_candidate<RD>(A, H, p, by_b, nvec, xx, pr);
                        }
                    }
                }
            }
            const uint64_t m = __ballot(hit);
            if (!m) continue;
            any = 1;
            lrec_stage(A, S, hit, pr, m);
        }
    }
    xx = wave_sum_u32(xx);  // (every thread of the block)
    if (lane == 0 && xx) atomicAdd(A.xx_out, xx);
    if (RD && lane == 0 && xx) atomicOr(A.rd_top, RT_XX);
    if (lane == 0 && any) s_any = 1;
    __syncthreads();
    if (PROF && threadIdx.x == 0) atomicMax(&A.st->pp_t[2], (unsigned long long)wall_clock64());
    if (s_any) {
        lrec_flush(A, S);
        if (RD) scan_lds_flush_rd(A, S, H);
        else scan_lds_flush(S, A.left, A.right);
    }
    if (PROF) {
        __syncthreads();
        if (threadIdx.x == 0) atomicMax(&A.st->pp_t[3], (unsigned long long)wall_clock64());
    }
}
// BATCH: a sparse tile's candidates are not resolved on the spot. Each is saved with its window (the
// vectors before and at it, the words after: 48 B from the lanes' registers by shuffles) in a per-wave
// LDS buffer (in the staged tile's space, 85 records at UNROLL 4), and the buffer -- candidates of many
// tiles -- is resolved one candidate per lane once it could not take another sparse tile (the next
// tile's loads already issued, so they overlap it). A tile with more than CB_DENSE candidates flushes the
// buffer and takes the compacted path on its staged tile. (At 1-4 candidates per tile, resolving in
// place spent as many wave instructions as streaming the tile: SQ_INSTS_VALU x1.9 at density 5e-4.)
constexpr uint32_t CB_DENSE = 32;
template <int UNROLL, bool NT, bool FILTER, bool PIPE, bool COMPACT, bool BATCH>
__device__ __attribute__((always_inline)) inline void scan_pairs_body(const ScanArgs A, ScanLds &S) {
    constexpr int STAGE = 2;                      // vectors per lane per record-staging step
    constexpr uint32_t WREC = 64 * STAGE * 8 / 2;  // at most one occurrence per 2 tokens
    static_assert(UNROLL % STAGE == 0 || UNROLL < STAGE, "UNROLL must be a multiple of STAGE (or < STAGE)");
    static_assert(PRES_BLK % (64 * UNROLL * 8) == 0, "presence blocks hold whole wave-tiles");
    uint32_t *s_left = S.left, *s_right = S.right;
    __shared__ uint32_t s_rec[SCAN_THREADS / 64][WREC];
    // a wave's current tile, staged in LDS when it holds candidates: phase 2 reads its windows here
    __shared__ uint4 s_tile[SCAN_THREADS / 64][64 * UNROLL];
    constexpr uint32_t CAND_CAP = COMPACT ? 128 : 1;  // compacted form: candidates resolved per round per wave
    __shared__ uint32_t s_cand[SCAN_THREADS / 64][CAND_CAP];
    uint32_t &s_any = S.any;
    unsigned long long &s_scanned = S.scanned;
    scan_lds_clear(S);
    if (threadIdx.x == 0) { s_any = 0; s_scanned = 0; }
    __syncthreads();
    NeighbourHist H{s_left, s_right, A.left, A.right, S.hleft, S.hright};
    const uint16_t *tok = A.tok;
    const int64_t nvec = (A.n + 7) / 8;
    constexpr int WT_VEC = 64 * UNROLL;  // vectors per wave-tile
    const int64_t nwt = (nvec + WT_VEC - 1) / WT_VEC;
    const int lane = threadIdx.x & 63, wib = threadIdx.x >> 6;
    const int64_t wstride = (int64_t)gridDim.x * (SCAN_THREADS / 64);
    // by_b: find occurrences from their second token (when b is the rarer one); exact with holes
    const bool by_b = A.pres && A.tokcnt && A.a != A.b && A.tokcnt[A.b] < A.tokcnt[A.a];
    const uint32_t key_tok = by_b ? A.b : A.a;
    uint32_t *wrec = s_rec[wib];
    uint32_t nbuf = 0;  // wave-uniform: records staged in wrec
    uint32_t xx = 0, any = 0, tiles = 0;
    if (by_b && blockIdx.x == 0 && threadIdx.x == 0 && A.halo.nright > 0 && halo_right(A.halo, 0) == A.b) {
        // the occurrence leaving the shard: its b is the next shard's, so no tile here holds it
        const int64_t p = prev_live(tok, A.n);
        if (p >= 0 && tok[p] == A.a && occ_slow(A, H, p, xx)) {
            const uint32_t j = atomicAdd(A.rec_ctr, 1u);
            atomicAdd(A.occ_out, 1u);
            if (j < A.rec_cap) A.rec[j] = (uint32_t)p;
            else atomicOr(&A.st->error, 8u);
            pres_set(A, p);
            any = 1;
        }
    }
    // BATCH: candidates saved with their windows (12 words each: position, the word before the previous
    // vector, the previous vector, the vector, the two words after it), ncb of them (wave-uniform)
    uint32_t ncb = 0;
    uint32_t *cbuf = reinterpret_cast<uint32_t *>(s_tile[wib]);
    bool batch_on = false;
    if constexpr (BATCH) {
        const uint64_t cnt = A.count_deltas ? A.top_count : 0u;
        batch_on = A.batch == 2 || (A.batch == 1 && (cnt == 0 || cnt * SCAN_BATCH_DENSITY < (uint64_t)A.n));
    }
    constexpr uint32_t CB_REC = 64 * UNROLL * 4 / 12;  // records the buffer holds
    auto flush_batch = [&]() {
        wave_lds_sync();
        for (uint32_t j0 = 0; j0 < ncb; j0 += 64) {
        bool hit = false;
        uint32_t pr = 0;
        if (j0 + (uint32_t)lane < ncb) {
            const uint4 *rp = reinterpret_cast<const uint4 *>(cbuf + 12 * (j0 + lane));
            const uint4 r0 = rp[0], r1 = rp[1], r2 = rp[2];
            const int64_t p = r0.x;
            const uint32_t w_pp = r0.y;
            const uint4 pv = make_uint4(r0.z, r0.w, r1.x, r1.y), cv = make_uint4(r1.z, r1.w, r2.x, r2.y);
            const uint32_t nx = r2.z, ny = r2.w;
            const int64_t vi = p >> 3;
            const int k = (int)(p & 7);
            int64_t start = p;
            bool fast = true;  // decide in a window (else occ_slow), unless known to be no occurrence
            bool none = false;
            bool in_prev = false;  // the window is the previous vector's
            int ks = k;
            if (by_b) {  // the occurrence starts at the live slot before p (window slot k + 2)
                uint32_t tl = HOLE;
                int l = -1;
#pragma unroll
                for (int i = 0; i < 10; i++) {
                    const uint32_t t = i < 2 ? (i ? pv.w >> 16 : pv.w & 0xffffu) : tok_at(cv, i - 2);
                    if (i < k + 2 && t != HOLE) { l = i; tl = t; }
                }
                if (l >= 0) {
                    none = tl != A.a;
                    start = vi * 8 + l - 2;
                    in_prev = l < 2;
                    ks = in_prev ? 6 + l : l - 2;
                } else {  // a run of holes reaches past the window (q < 0: the left shard owns it)
                    start = prev_live_h(A, p);
                    none = start < 0 || tok[start] != A.a;
                    fast = false;
                }
            }
            int r = none ? 0 : -1;
            if (!none && fast)
                r = occ_fast1(A, H, in_prev ? vi - 1 : vi, ks, xx, in_prev ? w_pp : pv.w, in_prev ? pv : cv,
                              in_prev ? cv.x : nx, in_prev ? cv.y : ny);
            if (r < 0) r = occ_slow(A, H, start, xx);
            hit = r != 0;
            pr = (uint32_t)start;
        }
        const uint64_t hm = __ballot(hit);
        if (hm) {
            any = 1;
            const uint32_t nh = (uint32_t)__popcll(hm);
            if (nbuf + nh > WREC) {
                wave_lds_sync();
                wave_flush_records(A, wrec, nbuf);
                nbuf = 0;
                wave_lds_sync();
            }
            // presence: one atomic per run of hits in one block (the records come in stream order
            // within a tile)
            const uint32_t blk = hit ? pr / PRES_BLK : 0xffffffffu;
            const uint32_t blk_up = wave_shr1(blk, 0xffffffffu);
            if (hit) {
                wrec[nbuf + (uint32_t)__popcll(hm & ((1ull << lane) - 1ull))] = pr;
                if (A.pres && (lane == 0 || blk_up != blk)) pres_set(A, pr);
            }
            nbuf += nh;
        }
        }
        ncb = 0;
        wave_lds_sync();
    };
    for (int64_t wt0 = (int64_t)blockIdx.x * (SCAN_THREADS / 64) + wib; wt0 < nwt; wt0 += 64 * wstride) {
      // block skipping: lane j looks up the presence bit of this wave's j-th next tile, so the
      // lookups of 64 tiles cost one load latency instead of one per tile
      uint64_t todo;
      {
          const int64_t mine = wt0 + (int64_t)lane * wstride;
          bool pr = mine < nwt;
          if (A.pres && pr) {
              const uint64_t blk = (uint64_t)mine * WT_VEC * 8 / PRES_BLK;
              pr = (A.pres[(blk / PRES_GROUP) * A.vp + key_tok] >> (blk % PRES_GROUP)) & 1u;
          }
          todo = __ballot(pr);
      }
      if (!todo) continue;
      // phase 1: stream UNROLL x 16 B per lane, keep only the positions holding the key token
      uint4 v[UNROLL];
      // the stream words just outside the tile (wave-uniform): the last one before it and the first
      // two after it (holes outside the stream)
      uint32_t ld_prev = 0xffffffffu, ld_nx = 0xffffffffu, ld_ny = 0xffffffffu;
      // Branch-free: addresses are clamped into the stream, and out-of-range values are replaced only
      // when the tile is used (tile_values). A select right after the load would make the compiler
      // wait for the load there -- for the prefetched next tile (PIPE) that is before this tile's
      // phase 2, which then no longer overlaps the next tile's memory latency.
      uint4 v_raw[UNROLL];
      uint32_t raw_prev = 0xffffffffu;
      uint2 raw_next = make_uint2(0xffffffffu, 0xffffffffu);
      int64_t raw_vb = 0;
      auto load_tile = [&](int64_t vb) {
          {
              const uint32_t *t32 = reinterpret_cast<const uint32_t *>(tok);
              const int64_t last = nvec * 4 - 1;  // last word of the stream
              const int64_t ip = vb > 0 ? vb * 4 - 1 : 0, in = min((vb + WT_VEC) * 4, last - 1);
              raw_prev = t32[ip];
              raw_next = *reinterpret_cast<const uint2 *>(t32 + (in & ~(int64_t)1));
          }
          raw_vb = vb;
#pragma unroll
          for (int u = 0; u < UNROLL; u++) {
              const int64_t vi = vb + u * 64 + lane;
              const uint4 *src = reinterpret_cast<const uint4 *>(tok) + min(vi, nvec - 1);
              if constexpr (NT) {
                  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
                  const u32x4 y = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(src));
                  v_raw[u] = make_uint4(y.x, y.y, y.z, y.w);
              } else {
                  v_raw[u] = *src;
              }
          }
      };
      auto tile_values = [&]() {
          const int64_t vb = raw_vb;
          const bool has_next = vb + WT_VEC < nvec;
          ld_prev = vb > 0 ? raw_prev : 0xffffffffu;
          ld_nx = has_next ? raw_next.x : 0xffffffffu;
          ld_ny = has_next ? raw_next.y : 0xffffffffu;
#pragma unroll
          for (int u = 0; u < UNROLL; u++) {
              const int64_t vi = vb + u * 64 + lane;
              v[u] = vi < nvec ? v_raw[u] : make_uint4(0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu);
          }
      };
      int64_t wt = wt0 + (int64_t)__builtin_ctzll(todo) * wstride;
      todo &= todo - 1;
      load_tile(wt * WT_VEC);
      for (;;) {
        tile_values();
        const int64_t vbase = wt * WT_VEC;
        const uint32_t e_prev = ld_prev, e_nx = ld_nx, e_ny = ld_ny;  // this tile's (ld_* may be the next's soon)
        tiles++;
        uint64_t cand = 0;  // bit 8u+k: token k of vector u is the key token
        if constexpr (FILTER) {
            // candidates: key-token positions whose partner slot holds the other token or a hole
            const uint32_t P1 = pair_key(A.a, A.b);
            // the neighbouring vector of lane 63 (by a) / lane 0 (by b) is in the next / previous
            // row of the tile, or outside it (edge_w, loaded with the tile)
            if (!by_b) {
                const uint32_t P2 = pair_key(A.a, HOLE);
#pragma unroll
                for (int u = 0; u < UNROLL; u++) {
                    const uint32_t nrow = u + 1 < UNROLL ? lane_bcast(v[u + 1 < UNROLL ? u + 1 : u].x, 0) : e_nx;
                    cand |= (uint64_t)pair_windows8<false>(v[u], wave_shl1(v[u].x, nrow), P1, P2) << (8 * u);
                }
            } else {
                const uint32_t P2 = pair_key(HOLE, A.b);
#pragma unroll
                for (int u = 0; u < UNROLL; u++) {
                    const uint32_t prow = u > 0 ? lane_bcast(v[u > 0 ? u - 1 : 0].w, 63) : e_prev;
                    cand |= (uint64_t)pair_windows8<true>(v[u], wave_shr1(v[u].w, prow), P1, P2) << (8 * u);
                }
            }
        } else {
#pragma unroll
            for (int u = 0; u < UNROLL; u++) cand |= (uint64_t)match8(v[u], key_tok) << (8 * u);
        }
        const bool tile_cand = __ballot(cand != 0) != 0;
        bool batched = false;  // (wave-uniform) this tile's candidates went to the batch buffer
        if constexpr (BATCH) {
            if (tile_cand) {
                const uint32_t cnt = (uint32_t)__popcll(cand);
                const uint32_t incl = wave_incl_scan_dpp(cnt);
                const uint32_t total = lane_bcast(incl, 63);
                batched = batch_on && total <= CB_DENSE;  // (ncb <= CB_REC - CB_DENSE here: it fits)
                if (batched) {
                    uint32_t slot = ncb + incl - cnt;  // this lane's next record
#pragma unroll
                    for (int u = 0; u < UNROLL; u++) {
                        const uint32_t cu = (uint32_t)(cand >> (8 * u)) & 0xffu;
                        if (!__ballot(cu != 0)) continue;
                        // the window of vector (u, lane) from the lanes' registers: the previous lane's vector (lane 0:
                        // the previous row's lane 63, or the word before the tile), the word two lanes back, the next
                        // lane's first two words (lane 63: the next row's lane 0, or the words after the tile)
                        const uint4 vp = u > 0 ? v[u > 0 ? u - 1 : 0] : make_uint4(0, 0, 0, 0);
                        const uint4 vn = u + 1 < UNROLL ? v[u + 1 < UNROLL ? u + 1 : u] : make_uint4(0, 0, 0, 0);
                        uint4 pv;
                        pv.x = wave_shr1(v[u].x, u > 0 ? lane_bcast(vp.x, 63) : 0xffffffffu);
                        pv.y = wave_shr1(v[u].y, u > 0 ? lane_bcast(vp.y, 63) : 0xffffffffu);
                        pv.z = wave_shr1(v[u].z, u > 0 ? lane_bcast(vp.z, 63) : 0xffffffffu);
                        pv.w = wave_shr1(v[u].w, u > 0 ? lane_bcast(vp.w, 63) : e_prev);
                        const uint32_t wpp = wave_shr1(pv.w, u > 0 ? lane_bcast(vp.w, 62) : 0xffffffffu);
                        const uint32_t nx = wave_shl1(v[u].x, u + 1 < UNROLL ? lane_bcast(vn.x, 0) : e_nx);
                        const uint32_t ny = wave_shl1(v[u].y, u + 1 < UNROLL ? lane_bcast(vn.y, 0) : e_ny);
                        uint32_t c = cu;
                        while (c) {
                            const int k = __builtin_ctz(c);
                            c &= c - 1;
                            const uint32_t pos = (uint32_t)((vbase + u * 64 + lane) * 8 + k);
                            uint4 *rp = reinterpret_cast<uint4 *>(cbuf + 12 * slot);
                            rp[0] = make_uint4(pos, wpp, pv.x, pv.y);
                            rp[1] = make_uint4(pv.z, pv.w, v[u].x, v[u].y);
                            rp[2] = make_uint4(v[u].z, v[u].w, nx, ny);
                            slot++;
                        }
                    }
                    ncb += total;
                }
            }
        }
        if (!BATCH && tile_cand) {
#pragma unroll
            for (int u = 0; u < UNROLL; u++) s_tile[wib][u * 64 + lane] = v[u];
        }
        // the tile's vectors are dead: start streaming the next present tile (its loads overlap
        // this tile's phase 2)
        const bool more = todo != 0;
        int64_t wt_next = 0;
        if (more) {
            wt_next = wt0 + (int64_t)__builtin_ctzll(todo) * wstride;
            todo &= todo - 1;
            if (PIPE) load_tile(wt_next * WT_VEC);
        }
        if constexpr (BATCH) {
            // (a dense tile: the buffer is resolved first, it is the staged tile's space)
            if (ncb > CB_REC - CB_DENSE || (ncb && tile_cand && !batched)) flush_batch();
            if (tile_cand && !batched) {
#pragma unroll
                for (int u = 0; u < UNROLL; u++) s_tile[wib][u * 64 + lane] = v[u];
            }
        }
        // window of vector vi of this tile: tok[8 vi - 2 .. 8 vi + 11] from the LDS tile and the edge words
        auto tile_window = [&](int64_t vi, uint32_t &pw, uint4 &cv, uint32_t &nx, uint32_t &ny) {
            const int j = (int)(vi - vbase);
            const uint4 *T = s_tile[wib];
            cv = T[j];
            pw = j > 0 ? T[j - 1].w : e_prev;
            nx = e_nx;
            ny = e_ny;
            if (j + 1 < WT_VEC) {
                const uint2 q = *reinterpret_cast<const uint2 *>(&T[j + 1]);
                nx = q.x;
                ny = q.y;
            }
        };
        // candidate p (holding the key token) of this tile: is it part of an occurrence? *pr = its start.
        // One window test and one slow-path call site (register pressure of the inlined code)
        auto resolve = [&](int64_t p, uint32_t &pr) -> bool {
            int64_t vi = p >> 3;
            const int k = (int)(p & 7);
            uint32_t pw, nx, ny;
            uint4 cv;
            tile_window(vi, pw, cv, nx, ny);
            int64_t start = p;
            bool in_win = true;
            if (by_b) {  // the occurrence starts at the live slot before p (window slot k + 2)
                uint32_t tl = HOLE;
                int l = -1;
#pragma unroll
                for (int i = 0; i < 10; i++) {
                    const uint32_t t = i < 2 ? (i ? pw >> 16 : pw & 0xffffu) : tok_at(cv, i - 2);
                    if (i < k + 2 && t != HOLE) { l = i; tl = t; }
                }
                if (l >= 0) {
                    if (tl != A.a) return false;
                    start = vi * 8 + l - 2;
                    if (l < 2) {
                        if (vi > vbase) {  // the start is in the previous vector of the tile
                            vi -= 1;
                            tile_window(vi, pw, cv, nx, ny);
                        } else {
                            in_win = false;
                        }
                    }
                } else {  // a run of holes reaches past the window (q < 0: the left shard owns it)
                    start = prev_live_h(A, p);
                    if (start < 0 || tok[start] != A.a) return false;
                    in_win = false;
                }
            }
            pr = (uint32_t)start;
            int r = in_win ? occ_fast1(A, H, vi, (int)(start - vi * 8), xx, pw, cv, nx, ny) : -1;
            if (r < 0) r = occ_slow(A, H, start, xx);
            return r != 0;
        };
        if (tile_cand && !batched) {
        wave_lds_sync();  // the staged tile is visible to every lane of the wave
        if constexpr (COMPACT) {
            // phase 2, dense form: the tile's candidates are compacted into a per-wave LDS list and
            // resolved one per lane (a lane-per-vector loop would iterate as often as the busiest lane)
            const uint32_t cnt = (uint32_t)__popcll(cand);
            const uint32_t incl = wave_incl_scan_dpp(cnt);
            const uint32_t total = lane_bcast(incl, 63);
            const uint64_t tile_blk = (uint64_t)vbase * 8 / PRES_BLK;
            bool tile_hit = false;
            uint32_t *wc = s_cand[wib];
            for (uint32_t r0 = 0; r0 < total; r0 += CAND_CAP) {
                uint32_t idx = incl - cnt;
                uint64_t cc = cand;
                while (cc) {
                    const int bit = __builtin_ctzll(cc);
                    cc &= cc - 1;
                    if (idx >= r0 && idx < r0 + CAND_CAP)
                        wc[idx - r0] = (uint32_t)((vbase + (bit >> 3) * 64 + lane) * 8 + (bit & 7));
                    idx++;
                }
                wave_lds_sync();
                const uint32_t nr = min(total - r0, (uint32_t)CAND_CAP);
                for (uint32_t j = lane; j - lane < nr; j += 64) {
                    bool hit = false;
                    uint32_t pr = 0;
                    if (j < nr) hit = resolve(wc[j], pr);
                    const uint64_t hm = __ballot(hit);
                    if (!hm) continue;
                    any = 1;
                    const uint32_t nh = (uint32_t)__popcll(hm);
                    if (nbuf + nh > WREC) {
                        wave_lds_sync();
                        wave_flush_records(A, wrec, nbuf);
                        nbuf = 0;
                        wave_lds_sync();
                    }
                    if (hit) {
                        wrec[nbuf + (uint32_t)__popcll(hm & ((1ull << lane) - 1ull))] = pr;
                        if (A.pres && pr / PRES_BLK != tile_blk) pres_set(A, pr);
                    }
                    nbuf += nh;
                    tile_hit = true;
                }
                wave_lds_sync();
            }
            if (A.pres && tile_hit && lane == 0) pres_set(A, vbase * 8);
        } else {
        // phase 2 (lanes with candidates): resolve occurrences on the LDS tile, stage their starts per
        // STAGE vectors; occ holds 16 bits per vector, bit s = start 8 vi - 2 + s
        const uint64_t tile_blk = (uint64_t)vbase * 8 / PRES_BLK;
#pragma unroll 1
        for (int ug = 0; ug < UNROLL; ug += STAGE) {
            constexpr int SG = STAGE < UNROLL ? STAGE : UNROLL;
            uint64_t occ = 0;
            uint64_t c = (cand >> (8 * ug)) & ((SG * 8 >= 64) ? ~0ull : ((1ull << (SG * 8)) - 1));
#pragma unroll 1
            while (c) {
                const int k8 = __ffsll((unsigned long long)c) - 1;
                c &= c - 1;
                const int u = k8 >> 3;
                const int64_t vi = vbase + (ug + u) * 64 + lane;
                uint32_t pr;
                if (!resolve(vi * 8 + (k8 & 7), pr)) continue;
                const int64_t sft = (int64_t)pr - (vi * 8 - 2);
                if (sft >= 0 && sft < 16) {
                    occ |= 1ull << (16 * u + sft);
                } else {  // a start beyond the window (hole run): record it directly
                    const uint32_t j = atomicAdd(A.rec_ctr, 1u);
                    atomicAdd(A.occ_out, 1u);
                    if (j < A.rec_cap) A.rec[j] = pr;
                    else atomicOr(&A.st->error, 8u);
                    if (A.pres) pres_set(A, pr);
                    any = 1;
                }
            }
            const uint32_t cnt = (uint32_t)__popcll(occ);
            const uint32_t incl = wave_incl_scan(cnt);
            const uint32_t total = (uint32_t)__shfl((int)incl, 63);
            if (total == 0) continue;
            any = 1;
            if (nbuf + total > WREC) {
                wave_lds_sync();
                wave_flush_records(A, wrec, nbuf);
                nbuf = 0;
                wave_lds_sync();
            }
            uint32_t o = nbuf + incl - cnt;
            while (occ) {
                const int bit = __ffsll((unsigned long long)occ) - 1;
                occ &= occ - 1;
                const int64_t p = (vbase + (ug + (bit >> 4)) * 64 + lane) * 8 + (bit & 15) - 2;
                if (A.pres && (uint64_t)p / PRES_BLK != tile_blk) pres_set(A, p);
                wrec[o++] = (uint32_t)p;
            }
            nbuf += total;
            if (A.pres && lane == 0) pres_set(A, vbase * 8);
        }
        }  // per-vector phase 2
        }  // tile has candidates
        if (!more) break;
        wt = wt_next;
        if (!PIPE) load_tile(wt * WT_VEC);
      }
    }
    if constexpr (BATCH) {
        if (ncb) flush_batch();
    }
    if (nbuf) {
        wave_lds_sync();
        wave_flush_records(A, wrec, nbuf);
    }
    // flush LDS neighbour histograms, the xx count and the streamed-slot count
    xx = wave_sum_u32(xx);  // (every thread of the block)
    if (lane == 0 && xx) atomicAdd(A.xx_out, xx);
    const bool wave_any = __ballot(any != 0) != 0;  // (a directly recorded occurrence sets it in one lane)
    if (lane == 0 && wave_any) s_any = 1;
    if (lane == 0 && tiles) atomicAdd(&s_scanned, (unsigned long long)tiles * WT_VEC * 8);
    __syncthreads();
    if (threadIdx.x == 0 && s_scanned) atomicAdd(&A.st->scanned_slots, s_scanned);
    if (s_any) scan_lds_flush(S, A.left, A.right);
}

// Presence bitmap from the stream: one workgroup per PRES_GROUP blocks, a bitset per block in LDS
// (tokens < vp <= 32768), then one coalesced row of words pres[g * vp + t].
constexpr int PRES_THREADS = 1024;
__global__ void __launch_bounds__(PRES_THREADS) zbpe_pres_build(const uint16_t *__restrict__ tok, int64_t n, uint32_t vp,
                                                                 uint32_t *__restrict__ pres) {
    extern __shared__ __attribute__((aligned(16))) uint32_t bits[];  // PRES_GROUP x (vp / 32) words
    const uint32_t W = vp / 32;
    for (uint32_t i = threadIdx.x; i < PRES_GROUP * W; i += PRES_THREADS) bits[i] = 0;
    __syncthreads();
    const int64_t g = blockIdx.x;
    const int64_t beg = g * (int64_t)PRES_GROUP * PRES_BLK, end = min(n, beg + (int64_t)PRES_GROUP * PRES_BLK);
    for (int64_t p = beg + 8 * threadIdx.x; p < end; p += 8 * PRES_THREADS) {
        const uint4 v = *reinterpret_cast<const uint4 *>(tok + p);
        const uint32_t j = (uint32_t)((p - beg) / PRES_BLK);
        // (a bit already set is not set again: the frequent tokens' bits are set early, and an LDS read of one address
        // broadcasts, while atomics on one address serialise -- 2.8 ms per C4 build with an atomic per slot)
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const uint32_t t = tok_at(v, k);
            if (t < vp && p + k < end) {
                uint32_t *w = &bits[j * W + (t >> 5)];
                if (!((*w >> (t & 31)) & 1u)) atomicOr(w, 1u << (t & 31));
            }
        }
    }
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < vp; t += PRES_THREADS) {
        uint32_t w = 0;
#pragma unroll 8
        for (int j = 0; j < PRES_GROUP; j++) w |= ((bits[j * W + (t >> 5)] >> (t & 31)) & 1u) << j;
        pres[g * vp + t] = w;
    }
}

// ------------------------------------------------------------------------------------------
// Token occurrence lists (counting sort of the compacted stream by token): per chunk histograms,
// per-token exclusive scan over chunks, offsets over tokens (tokens too frequent to ever key a
// list scan get none), scatter of positions. Rebuilt after every compaction while lists are on.
// ------------------------------------------------------------------------------------------
constexpr int LIST_CHUNK = 1 << 20;
constexpr int LIST_THREADS = 1024;
__global__ void __launch_bounds__(LIST_THREADS) zbpe_list_hist(const uint16_t *__restrict__ tok, int64_t n, uint32_t vp,
                                                               uint32_t *__restrict__ cnt) {
    extern __shared__ __attribute__((aligned(16))) uint32_t h[];
    for (uint32_t i = threadIdx.x; i < vp; i += LIST_THREADS) h[i] = 0;
    __syncthreads();
    const int64_t beg = (int64_t)blockIdx.x * LIST_CHUNK, end = min(n, beg + (int64_t)LIST_CHUNK);
    for (int64_t p = beg + 8 * threadIdx.x; p < end; p += 8 * LIST_THREADS) {
        const uint4 v = *reinterpret_cast<const uint4 *>(tok + p);
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const uint32_t t = tok_at(v, k);
            if (t < vp && p + k < end) atomicAdd(&h[t], 1u);
        }
    }
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < vp; t += LIST_THREADS) cnt[(uint64_t)blockIdx.x * vp + t] = h[t];
}
// in place: cnt[c][t] -> sum of cnt[c'][t] for c' < c; total[t] = column sum
__global__ void __launch_bounds__(256) zbpe_list_colscan(uint32_t *__restrict__ cnt, uint32_t nchunks, uint32_t vp,
                                                         uint32_t *__restrict__ total) {
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    if (t >= vp) return;
    uint32_t run = 0;
#pragma unroll 8
    for (uint32_t c = 0; c < nchunks; c++) {
        const uint32_t v = cnt[(uint64_t)c * vp + t];
        cnt[(uint64_t)c * vp + t] = run;
        run += v;
    }
    total[t] = run;
}
// one block: list offsets over tokens; tokens with total > max_len get NO_LIST
__global__ void __launch_bounds__(1024) zbpe_list_offsets(const uint32_t *__restrict__ total, uint32_t vp, uint32_t max_len,
                                                          uint32_t *__restrict__ lst_off, uint32_t *__restrict__ lst_len,
                                                          DevState *st, uint32_t lists_x) {
    __shared__ uint32_t s_part[1024];
    const uint32_t per = (vp + 1023) / 1024, t0 = threadIdx.x * per, t1 = min(vp, t0 + per);
    uint32_t sum = 0;
    for (uint32_t t = t0; t < t1; t++) sum += total[t] <= max_len ? total[t] : 0;
    s_part[threadIdx.x] = sum;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {  // inclusive scan (Hillis-Steele)
        const uint32_t v = threadIdx.x >= (uint32_t)off ? s_part[threadIdx.x - off] : 0;
        __syncthreads();
        s_part[threadIdx.x] += v;
        __syncthreads();
    }
    uint32_t run = s_part[threadIdx.x] - sum;
    for (uint32_t t = t0; t < t1; t++) {
        const uint32_t c = total[t];
        if (c <= max_len) {
            lst_off[t] = run;
            lst_len[t] = c;
            run += c;
        } else {
            lst_off[t] = 0;
            lst_len[t] = NO_LIST;
        }
    }
    if (threadIdx.x == 1023) {
        st->arena_top = s_part[1023];
        st->lists_valid = 1;
        st->lists_x = lists_x;
    }
}
__global__ void __launch_bounds__(LIST_THREADS) zbpe_list_scatter(const uint16_t *__restrict__ tok, int64_t n, uint32_t vp,
                                                                  const uint32_t *__restrict__ colpre,
                                                                  const uint32_t *__restrict__ lst_off,
                                                                  const uint32_t *__restrict__ lst_len,
                                                                  uint32_t *__restrict__ lists, uint32_t *__restrict__ nb,
                                                                  uint32_t tail_succ) {
    extern __shared__ __attribute__((aligned(16))) uint32_t cur[];
    for (uint32_t t = threadIdx.x; t < vp; t += LIST_THREADS)
        cur[t] = lst_len[t] == NO_LIST ? NO_LIST : lst_off[t] + colpre[(uint64_t)blockIdx.x * vp + t];
    __syncthreads();
    const int64_t beg = (int64_t)blockIdx.x * LIST_CHUNK, end = min(n, beg + (int64_t)LIST_CHUNK);
    for (int64_t p = beg + 8 * threadIdx.x; p < end; p += 8 * LIST_THREADS) {
        const uint4 v = *reinterpret_cast<const uint4 *>(tok + p);
        // the neighbours of the compacted stream (the padding past n reads as HOLE: no token)
        const uint32_t before = p > 0 ? tok[p - 1] : HOLE, after = tok[p + 8];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const uint32_t t = tok_at(v, k);
            if (t < vp && p + k < end && cur[t] != NO_LIST) {
                const uint32_t j = atomicAdd(&cur[t], 1u);
                lists[j] = (uint32_t)(p + k);
                if (nb) {
                    // (the last position's successor: tail_succ, the next shard's first live token, or HOLE)
                    const uint32_t sc = k < 7 ? (p + k + 1 < n ? tok_at(v, k + 1) : tail_succ) : (p + 8 < n ? after : tail_succ);
                    const uint32_t pd = k > 0 ? tok_at(v, k - 1) : before;
                    nb[j] = pd << 16 | sc;
                }
            }
        }
    }
}

// Successor ranges (round 3). A long list (at least min_len entries) gets a directory row, and its
// entries (positions and neighbour words together) are reordered by build-time successor: a chunked
// counting sort over the lists_x + 1 successor bins (lists_x: the stream's end) -- per chunk of
// SORT_CHUNK entries an LDS histogram and a copy to tmp; per (row, bin) the chunks' exclusive offsets;
// per row the bins' offsets (the row); per chunk the scatter back from tmp. A scan of (a, b) with both
// tokens older than the build then walks only the entries of a's list whose successor was b
// (scan_dispatch), about the pair's count instead of the list's length.
constexpr uint32_t DIR_MAX_TOK = 36 * 1024;  // successor bins of one sorting workgroup (144 KiB of LDS)
constexpr int DIR_THREADS = 1024;
constexpr uint32_t SORT_CHUNK = 1u << 18;  // list entries per sorting workgroup
// one block: rows in token order for lists of min_len..max_len entries (at most max_rows); every other
// token NO_LIST. rows[0] = rows, rows[1] = chunks, row_tok[r], row_ch0[r] = the row's first chunk
__global__ void __launch_bounds__(1024) zbpe_dir_rows(const uint32_t *__restrict__ lst_len, uint32_t ntok, uint32_t min_len,
                                                      uint32_t max_len, uint32_t max_rows, uint32_t *__restrict__ dir_row,
                                                      uint32_t *__restrict__ row_tok, uint32_t *__restrict__ row_ch0,
                                                      uint32_t *__restrict__ rows) {
    __shared__ uint32_t s_part[1024], s_ch[1024];
    constexpr uint32_t PER = 65536 / 1024;
    const uint32_t t0 = threadIdx.x * PER;
    auto want = [&](uint32_t t) { return t < ntok && lst_len[t] != NO_LIST && lst_len[t] >= min_len && lst_len[t] <= max_len; };
    uint32_t c = 0;
    for (uint32_t t = t0; t < t0 + PER; t++) c += want(t) ? 1u : 0u;
    s_part[threadIdx.x] = c;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {  // inclusive scan (Hillis-Steele)
        const uint32_t v = threadIdx.x >= (uint32_t)off ? s_part[threadIdx.x - off] : 0;
        __syncthreads();
        s_part[threadIdx.x] += v;
        __syncthreads();
    }
    // this thread's rows (below max_rows) and their chunks
    uint32_t r = s_part[threadIdx.x] - c, ch = 0;
    for (uint32_t t = t0, q = r; t < t0 + PER; t++)
        if (want(t)) { if (q < max_rows) ch += (lst_len[t] + SORT_CHUNK - 1) / SORT_CHUNK; q++; }
    s_ch[threadIdx.x] = ch;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
        const uint32_t v = threadIdx.x >= (uint32_t)off ? s_ch[threadIdx.x - off] : 0;
        __syncthreads();
        s_ch[threadIdx.x] += v;
        __syncthreads();
    }
    uint32_t c0 = s_ch[threadIdx.x] - ch;
    for (uint32_t t = t0; t < t0 + PER; t++) {
        uint32_t row = NO_LIST;
        if (want(t)) {
            if (r < max_rows) {
                row = r;
                row_tok[r] = t;
                row_ch0[r] = c0;
                c0 += (lst_len[t] + SORT_CHUNK - 1) / SORT_CHUNK;
            }
            r++;
        }
        dir_row[t] = row;
    }
    if (threadIdx.x == 1023) {
        const uint32_t nr = min(s_part[1023], max_rows);
        rows[0] = nr;
        rows[1] = s_ch[1023];
        row_ch0[nr] = s_ch[1023];
    }
}
// the chunk's row (binary search over the rows' first chunks) and its entries [b0, b1) of the list
struct SortChunk {
    uint32_t r, t, off, b0, b1;
};
__device__ inline bool sort_chunk(uint32_t c, const uint32_t *rows, const uint32_t *row_tok, const uint32_t *row_ch0,
                                  const uint32_t *lst_off, const uint32_t *lst_len, SortChunk &k) {
    const uint32_t nr = rows[0];
    if (c >= rows[1]) return false;
    uint32_t lo = 0, hi = nr;  // row_ch0[lo] <= c < row_ch0[lo + 1]
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (row_ch0[mid] <= c) lo = mid; else hi = mid;
    }
    k.r = lo;
    k.t = row_tok[lo];
    k.off = lst_off[k.t];
    const uint32_t len = lst_len[k.t];
    k.b0 = (c - row_ch0[lo]) * SORT_CHUNK;
    k.b1 = min(len, k.b0 + SORT_CHUNK);
    return true;
}
__device__ inline uint32_t succ_bin(uint32_t w, uint32_t ntok) {
    const uint32_t s = w & 0xFFFFu;
    return s < ntok ? s : ntok;
}
// per chunk: LDS histogram of the successor bins -> chunk_hist[c][bin]; the entries copied to tmp
__global__ void __launch_bounds__(DIR_THREADS) zbpe_list_sort_hist(const uint32_t *__restrict__ lists, const uint32_t *__restrict__ nb,
                                                                   uint2 *__restrict__ tmp, const uint32_t *__restrict__ lst_off,
                                                                   const uint32_t *__restrict__ lst_len, const uint32_t *__restrict__ rows,
                                                                   const uint32_t *__restrict__ row_tok, const uint32_t *__restrict__ row_ch0,
                                                                   uint32_t ntok, uint32_t *__restrict__ chunk_hist) {
    __shared__ uint32_t h[DIR_MAX_TOK + 1];
    SortChunk k;
    if (!sort_chunk(blockIdx.x, rows, row_tok, row_ch0, lst_off, lst_len, k)) return;
    const uint32_t nbin = ntok + 1, tid = threadIdx.x;
    for (uint32_t i = tid; i < nbin; i += DIR_THREADS) h[i] = 0;
    __syncthreads();
    for (uint32_t i0 = k.b0 + tid; i0 < k.b1; i0 += 4 * DIR_THREADS) {  // four entries per thread per step
        uint32_t w[4], q[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t i = i0 + u * DIR_THREADS;
            w[u] = i < k.b1 ? nb[k.off + i] : 0u;
            q[u] = i < k.b1 ? lists[k.off + i] : 0u;
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t i = i0 + u * DIR_THREADS;
            if (i < k.b1) {
                atomicAdd(&h[succ_bin(w[u], ntok)], 1u);
                tmp[k.off + i] = make_uint2(q[u], w[u]);
            }
        }
    }
    __syncthreads();
    for (uint32_t i = tid; i < nbin; i += DIR_THREADS) chunk_hist[(uint64_t)blockIdx.x * nbin + i] = h[i];
}
// per (row, bin): the row's chunks' exclusive offsets within the bin (in place); the bin's size -> dir
__global__ void __launch_bounds__(256) zbpe_list_sort_cols(uint32_t *__restrict__ chunk_hist, const uint32_t *__restrict__ rows,
                                                           const uint32_t *__restrict__ row_ch0, uint32_t ntok,
                                                           uint32_t *__restrict__ dir, uint32_t dir_w) {
    const uint32_t nbin = ntok + 1, b = blockIdx.x * 256 + threadIdx.x, nr = rows[0];
    if (b >= nbin) return;
    for (uint32_t r = blockIdx.y; r < nr; r += gridDim.y) {
        uint32_t run = 0;
        for (uint32_t c = row_ch0[r]; c < row_ch0[r + 1]; c++) {
            const uint64_t i = (uint64_t)c * nbin + b;
            const uint32_t v = chunk_hist[i];
            chunk_hist[i] = run;
            run += v;
        }
        dir[(uint64_t)r * dir_w + b] = run;
    }
}
// per row: the bins' exclusive offsets -> the row (absolute arena indices; the entry past the last bin
// is the list's end)
__global__ void __launch_bounds__(DIR_THREADS) zbpe_list_sort_row(const uint32_t *__restrict__ lst_off, const uint32_t *__restrict__ lst_len,
                                                                  const uint32_t *__restrict__ rows, const uint32_t *__restrict__ row_tok,
                                                                  uint32_t ntok, uint32_t *__restrict__ dir, uint32_t dir_w) {
    __shared__ uint32_t s_w[DIR_THREADS / 64];
    const uint32_t nr = rows[0];
    for (uint32_t r = blockIdx.x; r < nr; r += gridDim.x) {  // (block-uniform)
    const uint32_t t = row_tok[r], off = lst_off[t], len = lst_len[t], nbin = ntok + 1, tid = threadIdx.x;
    uint32_t *D = dir + (uint64_t)r * dir_w;
    const uint32_t per = (nbin + DIR_THREADS - 1) / DIR_THREADS, b0 = min(nbin, tid * per), b1 = min(nbin, b0 + per);
    uint32_t sum = 0;
    for (uint32_t b = b0; b < b1; b++) sum += D[b];
    const uint32_t incl = wave_incl_scan(sum);
    if ((tid & 63) == 63) s_w[tid >> 6] = incl;
    __syncthreads();
    uint32_t base = incl - sum;
    for (uint32_t w = 0; w < (tid >> 6); w++) base += s_w[w];
    for (uint32_t b = b0; b < b1; b++) {
        const uint32_t c = D[b];
        D[b] = off + base;
        base += c;
    }
    if (tid == 0) D[nbin] = off + len;
    __syncthreads();  // s_w reused by the next row
    }
}
// per chunk: cursors = bin start + the chunk's offset within the bin; the chunk's entries scattered
// from tmp back into the list
__global__ void __launch_bounds__(DIR_THREADS) zbpe_list_sort_scatter(uint32_t *__restrict__ lists, uint32_t *__restrict__ nb,
                                                                      const uint2 *__restrict__ tmp, const uint32_t *__restrict__ lst_off,
                                                                      const uint32_t *__restrict__ lst_len, const uint32_t *__restrict__ rows,
                                                                      const uint32_t *__restrict__ row_tok, const uint32_t *__restrict__ row_ch0,
                                                                      uint32_t ntok, const uint32_t *__restrict__ chunk_hist,
                                                                      const uint32_t *__restrict__ dir, uint32_t dir_w) {
    __shared__ uint32_t h[DIR_MAX_TOK + 1];
    SortChunk k;
    if (!sort_chunk(blockIdx.x, rows, row_tok, row_ch0, lst_off, lst_len, k)) return;
    const uint32_t nbin = ntok + 1, tid = threadIdx.x;
    const uint32_t *D = dir + (uint64_t)k.r * dir_w;
    for (uint32_t i = tid; i < nbin; i += DIR_THREADS) h[i] = D[i] + chunk_hist[(uint64_t)blockIdx.x * nbin + i];
    __syncthreads();
    for (uint32_t i0 = k.b0 + tid; i0 < k.b1; i0 += 4 * DIR_THREADS) {
        uint2 e[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t i = i0 + u * DIR_THREADS;
            e[u] = i < k.b1 ? tmp[k.off + i] : make_uint2(0, 0);
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            if (i0 + u * DIR_THREADS < k.b1) {
                const uint32_t j = atomicAdd(&h[succ_bin(e[u].y, ntok)], 1u);  // absolute arena index
                lists[j] = e[u].x;
                nb[j] = e[u].y;
            }
        }
    }
}

// default variant and the alternatives selectable for A/B runs (option "scan_variant")
#define zbpe_scan_pairs zbpe_scan_pairs_t<SCAN_UNROLL, true, true>

// apply: tok[p] = X, next live slot after p (the `b`) becomes a hole. Occurrences are disjoint.
__global__ void __launch_bounds__(256) zbpe_apply(uint16_t *tok, int64_t n, const uint32_t *__restrict__ rec,
                                                  uint32_t rec_cap, const DevState *st, uint32_t X) {
    const uint32_t cnt = min(st->rec_count, rec_cap);
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < cnt; i += gridDim.x * 256) {
        int64_t p = rec[i];
        tok[p] = (uint16_t)X;
        int64_t q = next_live(tok, n, p);
        if (q >= 0) tok[q] = HOLE;
    }
}

// Count update after merge X = (a, b), per neighbour token t < X: group 0 decrements (t, a) by
// left[t], group 1 creates (t, X) = left[t], group 2 decrements (b, t) by right[t], group 3 creates
// (X, t) = right[t]; the last block handles (b, a) -> (X, X) and the merged pair itself. A block
// owns UPD_THREADS * per consecutive t of one group: it gathers the nonzero deltas into LDS, then
// every shared counter (ids, live pairs, hot list, dirty home blocks) takes one atomic per block.
constexpr int UPD_THREADS = 256;
constexpr int UPD_MAX_PER = 8;
// A multi-merge round's update blocks (zbpe_replace, round mode): member j of the round's members applied
// (keys, their delta buffers at base + i * DELTA_WORDS). A pair tied at the round's start counts for the tie
// count of the first member that decrements it (the reference's loop sees it tied only there): the one
// decrement that finds the top count -- the first to land -- looks up which members decrement the pair (their
// deltas) and credits the smallest (RoundHead::dec).
struct RoundCtx {
    const uint32_t *base;
    uint32_t j;
    const uint32_t *keys;  // RoundHead::key
    uint32_t *dec;         // RoundHead::dec
    uint32_t mask;         // the members merged (round_valid)
    const uint32_t *jn;    // the junction counts (DevState::rd_jn)
    uint32_t n;            // members
};
__device__ inline void round_credit(const RoundCtx &rc, uint32_t key) {
    const uint32_t x = key & 0xFFFF, y = key >> 16;
    uint32_t m = rc.j;
    for (uint32_t i = 0; i < rc.j; i++) {
        if (!(rc.mask >> i & 1u)) continue;  // (a skipped member's deltas are not applied)
        // member i's junction decrements (round_junction_adjust): (b_i, a_e) and (b_e, a_i), unless e merged first
        bool jd = false;
        for (uint32_t e = 0; e < rc.n; e++) {
            if (e == i || ((rc.mask >> e & 1u) && e < i)) continue;
            const uint32_t ke = rc.keys[e];
            jd |= (rc.jn[i * RJ + e] && x == (rc.keys[i] >> 16) && y == (ke & 0xFFFF)) ||
                  (rc.jn[RJ_R + e * RJ + i] && x == (ke >> 16) && y == (rc.keys[i] & 0xFFFF));
        }
        if (jd) { m = i; break; }
        const uint32_t *l = rc.base + (size_t)i * (2 * 65536 + 64);
        const uint32_t ki = rc.keys[i], ai = ki & 0xFFFF, bi = ki >> 16;
        if ((y == ai && l[x]) || (x == bi && l[65536 + y]) || (x == bi && y == ai && l[2 * 65536])) { m = i; break; }
    }
    atomicAdd(&rc.dec[m], 1u);
}
__host__ __device__ inline uint32_t update_chunks(uint32_t X, uint32_t per) { return (X + UPD_THREADS * per - 1) / (UPD_THREADS * per); }
__host__ __device__ inline uint32_t update_blocks(uint32_t X, uint32_t per) { return 4 * update_chunks(X, per) + 1; }
// t per thread: about 16 blocks per group (fewer, fatter blocks cut the shared atomics)
__host__ __device__ inline uint32_t update_per(uint32_t X) {
    const uint32_t p = X / (16 * UPD_THREADS);
    return p < 1 ? 1 : (p > UPD_MAX_PER ? UPD_MAX_PER : p);
}
__device__ inline void update_block(const Tables &T, DevState *st, const uint32_t *__restrict__ left,
                                    const uint32_t *__restrict__ right, const uint32_t *__restrict__ tail, uint32_t a,
                                    uint32_t b, uint32_t X, uint32_t top_key, uint32_t ublk, uint32_t per,
                                    const uint32_t (&dv)[UPD_MAX_PER], uint32_t theta, int prof = 0,
                                    uint32_t top_count = 0, uint32_t pr_key = NO_ID, uint32_t pr_key2 = NO_ID,
                                    uint32_t pr_key3 = NO_ID, uint32_t pr_key4 = NO_ID, const RoundCtx *rc = nullptr,
                                    uint32_t Xc = 0, PairHead *ph = nullptr) {
    // Xc: the bound the blocks' groups and ranges were laid out for (update_preload's X; 0: X itself -- a round's
    // replace lays them out for the batch's bound on every member's X)
    // pr_key != NO_ID: merge X+1 has a pair-select candidate (ph: its slot DevState::ph[(X + 1) & 1]): count the new
    // pairs, the tied pairs decremented (old count == top_count) and flag what rules the candidate out
    // option sel_prof: the latest stamp of each phase over the update blocks (st->pp_t[8..11])
    const auto stamp = [&](int k) {
        if (prof && threadIdx.x == 0) atomicMax(&st->pp_t[k], (unsigned long long)wall_clock64());
    };
    __shared__ uint32_t s_t[UPD_THREADS * UPD_MAX_PER], s_c[UPD_THREADS * UPD_MAX_PER];
    __shared__ uint32_t s_hot[UPD_THREADS * UPD_MAX_PER];
    __shared__ uint32_t s_n, s_nhot, s_base, s_hbase;
    __shared__ int s_live;
    const uint32_t nch = update_chunks(Xc ? Xc : X, per);
    const uint32_t tid = threadIdx.x;
    if (ublk >= 4 * nch) {  // specials: three independent chains
        if (tid >= 3) return;
        int live_delta = 0;
        const uint32_t xx = tail[0];
        if (tid == 0 && xx) {
            const uint32_t old = pair_dec(T, st, pair_key(b, a), xx);
            if (rc && old == top_count) round_credit(*rc, pair_key(b, a));
        }
        if (tid == 0 && xx && pr_key != NO_ID) atomicOr(&ph->dt, 1u << 18);
        if (tid == 1 && xx) pair_new(T, st, pair_key(X, X), xx);
        if (tid == 2) {
            const uint32_t occ = tail[1];
            const uint32_t top_id = ht_find(T, top_key);
            if (top_id == NO_ID) key_missing(st, top_key, 2);
            else {
                hot_sub(T, top_id, occ);
                const uint32_t old = atomicSub(&T.id_cnt[top_id], occ);
                if (old < occ) atomicOr(&st->error, 2u);
                if (old == occ) { live_delta--; home_add(T, st, top_key, false); }
            }
            if (T.tok_cnt && rc) {  // (a round's members may share tokens)
                atomicAdd(&T.tok_cnt[X], (int32_t)occ);
                atomicSub(&T.tok_cnt[a], (int32_t)occ);
                atomicSub(&T.tok_cnt[b], (int32_t)occ);
            } else if (T.tok_cnt) {
                T.tok_cnt[X] += (int32_t)occ;
                T.tok_cnt[a] -= (int32_t)occ;
                T.tok_cnt[b] -= (int32_t)occ;
            }
        }
        if (live_delta) atomicAdd(&st->live, live_delta);
        return;
    }
    const uint32_t g = ublk / nch, beg = (ublk - g * nch) * UPD_THREADS * per;
    if (tid == 0) { s_n = 0; s_nhot = 0; s_live = 0; }
    __syncthreads();
    if (prof) {  // the deltas arrived (every thread's loads)
        uint32_t any = 0;
#pragma unroll
        for (uint32_t k = 0; k < UPD_MAX_PER; k++) any |= dv[k];
        if (any == 0xFFFFFFFFu) atomicOr(&st->error, 0u);  // (keeps the loads ahead of the stamp)
        __syncthreads();
        stamp(8);
    }
#pragma unroll
    for (uint32_t k = 0; k < UPD_MAX_PER; k++) {
        const uint32_t t = beg + k * UPD_THREADS + tid;
        const uint32_t c = k < per ? dv[k] : 0u;  // (update_preload: delta[t], 0 past X)
        if (c) {
            const uint32_t j = atomicAdd(&s_n, 1u);
            s_t[j] = t;
            s_c[j] = c;
        }
    }
    __syncthreads();
    stamp(9);
    const uint32_t n = s_n;
    if (n == 0) return;
    const bool create = g == 1 || g == 3;
    // a creating thread's first new key: its home bucket is read while the ids are reserved (the
    // insert's CAS then follows the reservation directly instead of a second memory round trip)
    unsigned long long pre[HT_BUCKET];
    const uint32_t key0 = create && tid < n ? (g == 1 ? pair_key(s_t[tid], X) : pair_key(X, s_t[tid])) : 0u;
    if (create && tid < n) ht_load_bucket(T, ht_home(T, key0), pre);
    if (create) {
        // the new ids that reach theta join the hot list: their slots are reserved by the same
        // thread and at the same time as the ids (two returning atomics in flight, not in series)
        for (uint32_t i = tid; i < n; i += UPD_THREADS)
            if (s_c[i] >= theta) s_hot[atomicAdd(&s_nhot, 1u)] = i;
        __syncthreads();
        if (tid == 0) {
            const uint32_t nh = s_nhot;
            uint32_t hb = 0;
            if (nh) hb = atomicAdd(&st->hot_len, nh);
            s_base = atomicAdd(&st->num_ids, n);
            atomicAdd(&st->live, (int)n);
            if (pr_key != NO_ID) atomicAdd(&ph->births, n);
            s_hbase = hb;
        }
        __syncthreads();
        stamp(10);
        const uint32_t base = s_base, hbase = s_hbase;
        for (uint32_t j = tid; j < s_nhot; j += UPD_THREADS)
            if (base + s_hot[j] < T.id_cap) {
                const uint32_t i = s_hot[j];
                hot_put(T, hbase + j, base + i, g == 1 ? pair_key(s_t[i], X) : pair_key(X, s_t[i]), s_c[i]);
            }
    }
    int live_delta = 0;
    for (uint32_t i = tid; i < n; i += UPD_THREADS) {
        const uint32_t t = s_t[i], c = s_c[i];
        if (!create) {
            const uint32_t key = g == 0 ? pair_key(t, a) : pair_key(b, t);
            const uint32_t id = ht_find(T, key);
            if (id == NO_ID) key_missing(st, key, 3);
            else {
                hot_sub(T, id, c);
                const uint32_t old = atomicSub(&T.id_cnt[id], c);
                if (old < c) atomicOr(&st->error, 2u);
                if (old == c) { live_delta--; home_add(T, st, key, false); }
                // (a pair's first decrement sees its count before the merge: each tied pair counts once; a self
                // pair's lone trailing a decrements the merged pair itself, which is no other tied pair)
                if (rc && old == top_count && key != top_key) round_credit(*rc, key);
                if (pr_key != NO_ID && old == top_count && key != top_key)
                    atomicAdd(&ph->dt, key == pr_key    ? 0x10001u
                                          : key == pr_key2 ? 0x80001u
                                          : key == pr_key3 ? 0x100001u
                                          : key == pr_key4 ? 0x200001u
                                                           : 1u);
            }
        } else {
            const uint32_t id = s_base + i;
            const uint32_t key = g == 1 ? pair_key(t, X) : pair_key(X, t);
            if (pr_key != NO_ID && c >= top_count) atomicOr(&ph->dt, 1u << 17);
            if (id >= T.id_cap) atomicOr(&st->error, 1u);
            else {
                T.id_key[id] = key;
                T.id_cnt[id] = c;
                if (c < theta) T.hpos[id] = NO_ID;  // (a listed one's slot was set by hot_put above)
                home_add(T, st, key, true);
                if (i == tid) ht_insert_loaded(T, key, id, pre);
                else ht_insert_new(T, key, id);
            }
        }
    }
    if (prof) {
        __syncthreads();
        stamp(11);
    }
    if (create) return;  // creating blocks kill no pair
    if (live_delta) atomicAdd(&s_live, live_delta);
    __syncthreads();
    if (tid == 0 && s_live) atomicAdd(&st->live, s_live);
}

// replaceTopPairWithNewToken in one launch: blocks [0, apply_blocks) rewrite the stream at the
// recorded occurrences (X at the start, a hole at the consumed b), the rest update the counts
// (identical on every rank: the deltas were summed), and one thread checks whether this shard's
// first live token is the b of an occurrence owned by the left rank (then it becomes a hole).
// error 64 (the occurrences a merge found != its pair's count): the first one's merge and numbers, for the message
__device__ inline void occ_check_failed(DevState *st, uint32_t X, uint32_t occ, uint32_t cnt, uint32_t key) {
    if (atomicCAS(&st->err_x, 0u, X) == 0u) {
        st->err_occ = occ;
        st->err_cnt = cnt;
        st->err_key = key;
        st->err_mode = st->scan_mode;
        st->err_light = st->last_light == X ? 1u : 0u;
    }
    atomicOr(&st->error, 64u);
}
struct ReplaceArgs {
    uint16_t *tok;
    int64_t n;
    const uint32_t *rec;
    uint32_t rec_cap;
    const uint32_t *left, *right, *tail;  // summed deltas; tail = {xx, occurrences}
    uint32_t a, b, X, top_key;
    uint32_t apply_blocks;
    Halo halo;
    const uint8_t *x0;  // self pairs: parity of the run of a's entering the shard (nullptr: none)
    int dyn;            // batch mode (see ScanArgs::dyn)
    const Halo *dhalo;
    int rec_arena;      // records at rec + st->arena_top (ScanArgs::rec_arena)
    int prof;           // option sel_prof: probe stamps (st->pp_t)
    // pair selects: the last workgroup of the grid computes merge X+1's candidate bound (pair_slack_block)
    int pair_blk;
    const Summ *summ, *sup;  // the home view of the decision (HomeView: summ, sup, C, nb, nsb)
    uint32_t C, nb, nsb;
    const uint32_t *cs;
    const uint32_t *dir_row, *dir;  // the candidate's scan plan (ScanArgs::dir_row, dir, dir_w)
    uint32_t dir_w, gen;
    int plan;
    // multi-merge rounds (batch mode, one GPU or replicas): `round` member slots of per_member workgroups each
    // (apply_blocks of them apply, the rest update), member j's deltas at left + j * DELTA_WORDS (fixed layout:
    // right at +65536, tail at +131072); no member at or past token x_end (round_valid; C: the Zig capacity)
    int round;
    uint32_t per_member, x_end;
};
__device__ inline uint64_t dev_zig_cap_for(uint64_t D);
__device__ inline bool dev_zig_at_max_load(uint64_t cap, uint64_t D);
// Which members of a multi-merge round the reference's loop merges next, one after the other (every workgroup
// of the round's replace evaluates it on the same words: the scan's RoundHead, final at this launch).
// Tied rounds: the named keys are the decision's tied pairs in home order; member j >= 1 is
//   - skipped when an occurrence of it shares a token with one of a merged member's (RT_SHARED): merging that
//     member decrements its pair, which leaves the tied set, so the loop never takes it (tied pairs only fall);
//   - else merged next (merge X0 + the members merged before it) when it was walked (a list form) with exactly
//     T occurrences, none next to a merged member's (RT_NEIGHBOUR; so its occurrences, its neighbours and its
//     count are what they would be when its turn comes), no merged member made a pair with the top count or
//     adjacent occurrences (the tied set is the decision's less the merged and the decremented: member j is its
//     smallest home), the merged members' new pairs are fewer than the free Zig-map slots after member j's home
//     block before the next tied home and after the largest tied home's block (each new key fills at most one:
//     member j's run still ends before the next tied home and no tied run wraps, so it is first in slot order
//     -- the pair-select argument of zbpe_select_next, per member), and the Zig capacity is C and not at a max
//     load for every live-pair count the merged members can leave (each kills its own pair and at most one pair
//     per new pair: D in [D0 - k, D0 + births - k] after k merges);
//   - else the round ends.
// Untied rounds (ties0 == 1): member j holds the j-th distinct count T_j below T (the only pair with it; every
// pair outside the round is below the last member's count). It is merged next when no merged member shares a
// token with it (else its count fell: the round ends), it was walked with exactly T_j occurrences, its
// junctions agree, and no pair a merged member made -- its neighbours' new pairs, (X, X), junction pairs --
// reaches T_j: then T_j is the unique top count, whatever the Zig map's order; else the round ends.
enum RoundWhy : uint32_t { RW_ALL, RW_FLAGS, RW_WALK, RW_TOUCH, RW_REC, RW_END, RW_ARENA, RW_SLACK, RW_CAP, RW_JUNC, RW_N };
// DevState::rd_why: [0, RW_N) tied rounds' ends, [RW_N, RW_N + 6) tied-round details (sel_prof), untied rounds' ends
// from RW_U, then untied rounds named (RW_U + RW_N) and their merged members (RW_U + RW_N + 1)
constexpr uint32_t RW_U = 16;
struct RoundVerdict {
    uint32_t mask;   // members merged (bit j: member j; bit 0 always)
    uint32_t k;      // how many
    uint32_t why;    // what ended the round (RoundWhy), at member jend
    uint32_t jend;
    uint32_t flags;  // (RW_FLAGS: 1 a new pair at the top count, 2 adjacent occurrences at it, 4 a junction's pair
                     // with a non-member at it, 8 two merged members' junction pair at it)
};
// (dbase: the members' delta buffers, DELTA_WORDS apart. A member's adjacent occurrences (xx, its tail word) make
// (X, X), one more new pair, with count xx; the (b, a) they decrement is a tied pair leaving the set, or a later
// member that shares their tokens (skipped, or the untied round's end). jn: the junction counts: a merged member's
// junction side makes one more new pair -- (X_e, a_o) or (b_o, X_e), with its count in e's deltas plus the
// junctions --, and two merged members' junctions one more, (X_L, X_R), counted alike by both walks.)
__device__ inline RoundVerdict round_valid(const RoundHead &R, const uint32_t *dbase, const uint32_t *jn, uint32_t T, uint32_t X0,
                                           uint32_t x_end, uint32_t C, uint32_t arena_top, uint32_t rec_cap) {
    constexpr uint32_t DW = 2 * 65536 + 64;
    RoundVerdict v{1u, 1u, RW_ALL, 0u, 0u};
    const uint32_t n = min(R.n, (uint32_t)ROUND_MAX);
    const bool untied = R.ties0 == 1;
    uint32_t anyj = 0;
#pragma unroll
    for (uint32_t e = 0; e < (uint32_t)ROUND_MAX; e++)
        if (e < n) anyj |= R.top[e] & RT_JUNCTION;
    uint64_t births = 0;
    uint32_t flags = 0;
    uint32_t M = 0;  // the largest count of a pair the merged members made
    const auto bring = [&](uint32_t e) {  // what merging member e adds to the map
        const uint32_t *de = dbase + (size_t)e * DW;
        const uint32_t xxe = de[2 * 65536];
        births += R.birth[e] + (xxe ? 1u : 0u);
        M = max(M, max(R.nmax[e], xxe));
        flags |= (R.nmax[e] >= T ? 1u : 0u) | (xxe >= T ? 2u : 0u);
        if (anyj) {
#pragma unroll
            for (uint32_t o = 0; o < (uint32_t)ROUND_MAX; o++) {
                if (o >= n || o == e) continue;
                const uint32_t ko = R.key[o], cl = jn[e * RJ + o], cr = jn[RJ_R + o * RJ + e];
                if (cl) { births++; const uint32_t c = de[65536 + (ko & 0xFFFF)] + cl; M = max(M, c); if (c >= T) flags |= 4u; }  // (X_e, a_o)
                if (cr) { births++; const uint32_t c = de[ko >> 16] + cr; M = max(M, c); if (c >= T) flags |= 4u; }            // (b_o, X_e)
            }
        }
    };
    bring(0);
#pragma unroll
    for (uint32_t j = 1; j < (uint32_t)ROUND_MAX; j++) {
        if (j >= n) break;
        v.jend = j;
        const uint32_t Tj = untied ? R.cnt[j] : T;
        if (untied ? M >= Tj : flags != 0) { v.why = RW_FLAGS; v.flags = flags; break; }
        const uint32_t tch = R.touch[j];
        if (tch & v.mask * RT_SHARED) {  // decremented: no longer tied (skipped), or no longer T_j (the end)
            if (untied) { v.why = RW_TOUCH; break; }
            continue;
        }
        uint64_t jb = 0;
        uint32_t jf = 0, jm = 0;
        bool jbad = false;
        if (anyj) {
#pragma unroll
            for (uint32_t i = 0; i < (uint32_t)ROUND_MAX; i++) {
                if (i >= j || !(v.mask >> i & 1u)) continue;
                const uint32_t a1 = jn[i * RJ + j], a2 = jn[RJ_R + i * RJ + j], b1 = jn[j * RJ + i], b2 = jn[RJ_R + j * RJ + i];
                jbad |= a1 != a2 || b1 != b2;
                if (a1) { jb++; jm = max(jm, a1); if (a1 >= T) jf |= 8u; }  // (X_i, X_j)
                if (b1) { jb++; jm = max(jm, b1); if (b1 >= T) jf |= 8u; }  // (X_j, X_i)
            }
        }
        v.why = !(R.top[j] & RT_WALKED)                                   ? RW_WALK
                : jbad                                                    ? RW_JUNC
                : R.rec[j] != Tj                                          ? RW_REC
                : X0 + v.k >= x_end                                       ? RW_END
                : (uint64_t)arena_top + (uint64_t)(j + 1) * T > rec_cap   ? RW_ARENA
                                                                          : RW_ALL;
        if (v.why != RW_ALL) break;
        if (!untied) {  // the Zig order among the tied keys
            const uint64_t slack = R.ties == j + 1 ? ~0ull
                                   : (R.freeb[j] < 0 || R.freeb[0] < 0) ? 0ull
                                                                        : (uint64_t)min(R.freeb[j], R.freeb[0]);
            if (births >= slack) { v.why = RW_SLACK; break; }
            const int64_t lo = (int64_t)R.live0 - (int64_t)v.k, hi = (int64_t)R.live0 + (int64_t)births - (int64_t)v.k;
            if (lo < 1 || dev_zig_cap_for((uint64_t)lo) != C || dev_zig_cap_for((uint64_t)hi) != C ||
                dev_zig_at_max_load(C, (uint64_t)hi)) {
                v.why = RW_CAP;
                break;
            }
        }
        v.mask |= 1u << j;
        v.k++;
        bring(j);
        births += jb;
        flags |= jf;
        M = max(M, jm);
    }
    if (v.why == RW_ALL) v.jend = n;
    return v;
}
// Member j's junction sides in its update blocks' deltas (group g of the count update, its threads' t from beg):
// with the partner merged, the first of the two decrements (b_L, a_R) and the second makes (X_L, X_R); a partner
// not merged leaves member j's side a plain neighbour (decrement and new pair with the original token).
__device__ inline void round_junction_adjust(uint32_t (&dv)[UPD_MAX_PER], uint32_t g, uint32_t beg, uint32_t per, uint32_t j,
                                             uint32_t mask, uint32_t n, const uint32_t *keys, const uint32_t *jn, uint32_t X0) {
    const auto add = [&](uint32_t t, uint32_t c) {
#pragma unroll
        for (uint32_t k = 0; k < UPD_MAX_PER; k++)
            if (k < per && beg + k * UPD_THREADS + threadIdx.x == t) dv[k] += c;
    };
#pragma unroll
    for (uint32_t e = 0; e < (uint32_t)ROUND_MAX; e++) {
        if (e >= n || e == j) continue;
        const uint32_t ke = keys[e], ae = ke & 0xFFFF, be = ke >> 16;
        const bool me = mask >> e & 1u;
        const uint32_t Xe = X0 + (uint32_t)__popc(mask & ((1u << e) - 1u));
        const uint32_t cl = jn[j * RJ + e], cr = jn[RJ_R + e * RJ + j];  // j -> e (j's right side), e -> j (its left side)
        if (cl) {
            if (!me) { if (g == 2 || g == 3) add(ae, cl); }
            else if (j < e) { if (g == 2) add(ae, cl); }  // decrement (b_j, a_e)
            else if (g == 3) add(Xe, cl);                 // make (X_j, X_e)
        }
        if (cr) {
            if (!me) { if (g == 0 || g == 1) add(be, cr); }
            else if (j < e) { if (g == 0) add(be, cr); }  // decrement (b_e, a_j)
            else if (g == 1) add(Xe, cr);                 // make (X_e, X_j)
        }
    }
}
// pair selects: merge X+1's candidate bound, by the replace's extra workgroup (defined with the home views below)
__device__ inline void pair_slack_block(DevState *st, const Summ *summ, const Summ *sup, uint32_t C, uint32_t nb,
                                        uint32_t nsb, const uint32_t *cs, uint32_t X, const uint32_t *lst_off,
                                        const uint32_t *lst_len, const uint32_t *dir_row, const uint32_t *dir,
                                        uint32_t dir_w, uint32_t lists_x, bool plan_on, uint32_t gen);
// this thread's deltas of an update block, loaded before anything that waits on the state (they do
// not depend on the merged pair: group and range follow from the block index)
__device__ inline void update_preload(const uint32_t *left, const uint32_t *right, uint32_t X, uint32_t ublk, uint32_t per,
                                      uint32_t (&dv)[UPD_MAX_PER]) {
    const uint32_t nch = update_chunks(X, per);
    const uint32_t g = ublk < 4 * nch ? ublk / nch : 0u, beg = (ublk - g * nch) * UPD_THREADS * per;
    const uint32_t *delta = (g < 2) ? left : right;
    const bool real = ublk < 4 * nch;
#pragma unroll
    for (uint32_t k = 0; k < UPD_MAX_PER; k++) {
        const uint32_t t = beg + k * UPD_THREADS + threadIdx.x;
        dv[k] = real && k < per && t < X ? delta[t] : 0u;
    }
}
// The leading scalar arguments (kernarg-preloaded) are what the delta loads need (== R.left, R.X,
// R.apply_blocks; right = left + X), so they issue at entry beside the state head.
__global__ void __launch_bounds__(256) zbpe_replace(DevState *st, const uint32_t *__restrict__ left, uint32_t Xp, uint32_t apply_blocks,
                                                    ReplaceArgs R, Tables T) {
    uint32_t dv[UPD_MAX_PER];
    const uint32_t per = update_per(Xp);
    if (blockIdx.x >= apply_blocks) update_preload(left, left + Xp, Xp, blockIdx.x - apply_blocks, per, dv);
    const StateHead H = load_head(st);  // (with the deltas: one round trip)
    PairHead *ph = &st->ph[(R.X + 1) & 1];  // (merge X+1's candidate slot)
    const uint32_t pr_x = ph->x, pr_key0 = ph->key, pr_key2 = st->pr_key2, pr_key3 = st->pr_key3, pr_key4 = st->pr_key4;
    const uint32_t theta = H.theta;
    if (R.prof && blockIdx.x == 0 && threadIdx.x == 0) {  // fold the list scan's stamps
        const unsigned long long now = wall_clock64();
        if (st->pp_t[4]) {
            unsigned long long *P = st->pipe_prof[pp_bucket(R.X)];
            const unsigned long long t0 = st->pp_t[0];
            P[0] += st->pp_t[1] - t0;
            P[1] += st->pp_t[2] - t0;
            P[2] += st->pp_t[3] - t0;
            P[3] += now - t0;
            P[4]++;
        }
        st->pp_t[1] = st->pp_t[2] = st->pp_t[3] = st->pp_t[4] = 0;
        st->pp_t[5] = now;
    }
    if (R.dyn) {
        if (H.halt) return;
        if (R.pair_blk && blockIdx.x == gridDim.x - 1) {
            pair_slack_block(st, R.summ, R.sup, R.C, R.nb, R.nsb, R.cs, R.X, T.lst_off, T.lst_len, R.dir_row, R.dir, R.dir_w,
                             H.lists_x, R.plan && T.lst_off && H.lists_valid, R.gen);
            return;
        }
        R.top_key = H.cur_key;
        R.a = R.top_key & 0xFFFF;
        R.b = R.top_key >> 16;
    }
    if (blockIdx.x < apply_blocks) {
        if (R.rec_arena) {
            const uint32_t top = H.arena_top;
            R.rec += top;
            R.rec_cap = R.rec_cap > top ? R.rec_cap - top : 0;
        }
        const uint32_t cnt = min(H.rec_count, R.rec_cap);
        uint32_t made = 0;  // an occurrence whose b lies in the next shard makes no hole here
        for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < cnt; i += apply_blocks * 256) {
            const int64_t p = R.rec[i];
            R.tok[p] = (uint16_t)R.X;
            const int64_t q = next_live(R.tok, R.n, p);
            if (q >= 0) {
                R.tok[q] = HOLE;
                made++;
            }
        }
        made = wave_sum(made);
        if ((threadIdx.x & 63) == 0 && made) atomicAdd(&st->holes_made, made);
        if (R.prof) {
            __syncthreads();
            if (threadIdx.x == 0) atomicMax(&st->pp_t[12], (unsigned long long)wall_clock64());
            if (threadIdx.x == 0) atomicMax(&st->pp_t[6], (unsigned long long)wall_clock64());
        }
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            st->consumed = 0;
            if (R.dhalo) R.halo = *R.dhalo;
            const Halo &Hl = R.halo;
            if (Hl.nleft > 0 || R.x0) {
                const int64_t f = next_live(R.tok, R.n, -1);
                if (f >= 0) {
                    const uint32_t tf = R.tok[f];
                    const bool c = R.a != R.b ? (Hl.nleft > 0 && halo_left(Hl, 0) == R.a && tf == R.b)
                                              : (tf == R.a && R.x0 && (*R.x0 & 1));
                    if (c) {
                        R.tok[f] = HOLE;
                        st->consumed = 1;
                        atomicAdd(&st->holes_made, 1u);
                    }
                }
            }
        }
        return;
    }
    const uint32_t ublk = blockIdx.x - apply_blocks;
    // (a self pair: runs of a hold fewer occurrences than (a, a) pairs)
    if (R.dyn && ublk == 0 && threadIdx.x == 0 && R.tail[1] != H.top_count && R.a != R.b)
        occ_check_failed(st, R.X, R.tail[1], H.top_count, R.top_key);
    update_block(T, st, R.left, R.right, R.tail, R.a, R.b, R.X, R.top_key, ublk, per, dv, theta, R.prof, H.top_count,
                 R.dyn && pr_x == R.X + 1 ? pr_key0 : NO_ID, pr_key2, pr_key3, pr_key4, nullptr, 0, ph);
    if (R.prof) {
        __syncthreads();
        if (threadIdx.x == 0) atomicMax(&st->pp_t[6], (unsigned long long)wall_clock64());
    }
}

// The replace of a multi-merge round (batch mode, one GPU or replicas): R.round member slots of R.per_member
// workgroups, the first apply_blocks of each rewrite the stream at the member's records, the rest update the
// counts from its deltas (update_block); every workgroup evaluates round_valid on the scan's RoundHead and the
// slots of members past the valid prefix return at once. Members' occurrences touch none of each other's, so
// their rewrites and count updates commute: applying them together is applying them in order.
__global__ void __launch_bounds__(256) zbpe_replace_round(DevState *st, const uint32_t *__restrict__ left, uint32_t Xp,
                                                          uint32_t apply_blocks, ReplaceArgs R, Tables T) {
    constexpr uint32_t DW = 2 * 65536 + 64;  // DELTA_WORDS
    const uint32_t j = blockIdx.x / R.per_member, lb = blockIdx.x - j * R.per_member, per = update_per(Xp);
    const uint32_t *lj = left + (size_t)j * DW;
    uint32_t dv[UPD_MAX_PER];
    if (lb >= apply_blocks) update_preload(lj, lj + 65536, Xp, lb - apply_blocks, per, dv);
    const StateHead H = load_head(st);
    const RoundHead &RH = st->rd;  // (read in place: a register copy indexed by the member went to scratch)
    if (R.prof && blockIdx.x == 0 && threadIdx.x == 0) {  // fold the round scan's stamps (as zbpe_replace)
        const unsigned long long now = wall_clock64();
        if (st->pp_t[4]) {
            unsigned long long *P = st->pipe_prof[pp_bucket(H.cur_x)];
            const unsigned long long t0 = st->pp_t[0];
            P[0] += st->pp_t[1] - t0;
            P[1] += st->pp_t[2] - t0;
            P[2] += st->pp_t[3] - t0;
            P[3] += now - t0;
            P[4]++;
            if (st->pp_t[13] > t0) P[15] += st->pp_t[13] - t0;
        }
        st->pp_t[1] = st->pp_t[2] = st->pp_t[3] = st->pp_t[4] = st->pp_t[13] = 0;
        st->pp_t[5] = now;
    }
    if (H.halt) return;
    const uint32_t Tc = H.top_count;
    const RoundVerdict v = round_valid(RH, left, st->rd_jn, Tc, H.cur_x, R.x_end, R.C, H.arena_top, R.rec_cap);
    const bool untied = RH.ties0 == 1;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        st->rd_v = v.k;
        st->rd_mask = v.mask;
        if (RH.n > 1 && untied) {  // (untied rounds: what ended them, how many, their members merged)
            atomicAdd(&st->rd_why[RW_U + v.why], 1u);
            atomicAdd(&st->rd_why[RW_U + RW_N], 1u);
            atomicAdd(&st->rd_why[RW_U + RW_N + 1], v.k - 1);
        } else if (RH.n > 1) {  // (rounds with named keys: what ended them, the ending touch's kinds, the members skipped)
            atomicAdd(&st->rd_why[v.why], 1u);
            uint32_t jm = 0;  // members merged with a junction to an earlier merged member
#pragma unroll
            for (uint32_t e = 1; e < (uint32_t)ROUND_MAX; e++)
                if ((v.mask >> e & 1u) && (RH.touch[e] & (v.mask & ((1u << e) - 1u)) * RT_NEIGHBOUR)) jm++;
            if (jm) atomicAdd(&st->rd_why[RW_N], jm);
            if (v.why == RW_FLAGS) atomicAdd(&st->rd_why[RW_N + 4 + (v.flags & 13u ? 0 : 1)], 1u);
            const uint32_t skipped = ((1u << v.jend) - 1u) & ~v.mask;
            if (skipped) atomicAdd(&st->rd_why[RW_N + 3], (uint32_t)__popc(skipped));
        }
    }
    if (!(v.mask >> j & 1u)) return;
    // member j is merge X0 + (the members merged before it)
    const uint32_t X = H.cur_x + (uint32_t)__popc(v.mask & ((1u << j) - 1u)), key = RH.key[j], a = key & 0xFFFF, b = key >> 16;
    const uint32_t Tj = j ? RH.cnt[j] : Tc;  // member j's count (below Tc in an untied round)
    if (lb < apply_blocks) {
        // X at each occurrence start, a hole at its b (one GPU: the b is always in the stream)
        const uint32_t *rec = R.rec + H.arena_top + (size_t)j * Tc;
        const uint32_t cnt = min(j ? RH.rec[j] : H.rec_count, Tj);
        uint32_t made = 0;
        for (uint32_t i = lb * 256 + threadIdx.x; i < cnt; i += apply_blocks * 256) {
            const int64_t p = rec[i];
            R.tok[p] = (uint16_t)X;
            const int64_t q = next_live(R.tok, R.n, p);
            if (q >= 0) {
                R.tok[q] = HOLE;
                made++;
            }
        }
        made = wave_sum(made);
        if ((threadIdx.x & 63) == 0 && made) atomicAdd(&st->holes_made, made);
        return;
    }
    const uint32_t ublk = lb - apply_blocks;
    const uint32_t *tj = lj + 2 * 65536;
    if (ublk == 0 && threadIdx.x == 0 && tj[1] != Tj && a != b) occ_check_failed(st, X, tj[1], Tj, key);
    const uint32_t nch = update_chunks(Xp, per);
    if (ublk < 4 * nch && (RH.top[j] & RT_JUNCTION)) {  // (member j's walk counted junctions)
        const uint32_t g = ublk / nch;
        round_junction_adjust(dv, g, (ublk - g * nch) * UPD_THREADS * per, per, j, v.mask, min(RH.n, (uint32_t)ROUND_MAX),
                              &RH.key[0], st->rd_jn, H.cur_x);
    }
    const RoundCtx rc{left, j, &st->rd.key[0], &st->rd.dec[0], v.mask, st->rd_jn, min(RH.n, (uint32_t)ROUND_MAX)};
    // (the tie counts' credit: pairs tied at the round's start, the top count -- none besides member 0 in an untied round)
    update_block(T, st, lj, lj + 65536, tj, a, b, X, key, ublk, per, dv, H.theta, 0, untied ? 0xFFFFFFFFu : Tc, NO_ID, NO_ID, NO_ID,
                 NO_ID, &rc, Xp);
}

// this shard's boundary record: first 3 / last 2 live tokens (holes skipped) and its live count
__global__ void zbpe_boundary(const uint16_t *__restrict__ tok, int64_t n, int64_t nlive, Boundary *out, const DevState *st) {
    if (threadIdx.x || blockIdx.x || (st && st->halt)) return;
    Boundary B{};
    for (int k = 0; k < 3; k++) B.first[k] = HOLE;
    B.last[0] = B.last[1] = HOLE;
    for (int64_t p = 0; p < n && B.nfirst < 3; p++)
        if (tok[p] != HOLE) B.first[B.nfirst++] = tok[p];
    for (int64_t p = n - 1; p >= 0 && B.nlast < 2; p--)
        if (tok[p] != HOLE) B.last[B.nlast++] = tok[p];
    B.nlive = (uint32_t)nlive;
    *out = B;
}
// batch mode: this rank's halo from the gathered boundary records (Engine::halo_from_boundaries)
__global__ void zbpe_halo_build(const Boundary *__restrict__ bnd, int rank, int world, Halo *out, const DevState *st) {
    if (threadIdx.x || blockIdx.x || st->halt) return;
    Halo H = halo_empty();
    for (int r = rank - 1; r >= 0 && H.nleft < 2; r--)
        for (int k = 0; k < bnd[r].nlast && H.nleft < 2; k++) halo_push_left(H, bnd[r].last[k]);
    for (int r = rank + 1; r < world && H.nright < 3; r++)
        for (int k = 0; k < bnd[r].nfirst && H.nright < 3; k++) halo_push_right(H, bnd[r].first[k]);
    *out = H;
}
// encode: apply one merge at the recorded occurrences, then (last block to finish) roll the
// counters; with occurrence lists the records, kept in the arena, become X's list
__global__ void __launch_bounds__(256) zbpe_encode_apply(uint16_t *tok, int64_t n, uint32_t *rec, uint32_t rec_cap, int rec_arena,
                                                         uint32_t X, DevState *st, Tables T, uint32_t *scratch,
                                                         int32_t *tcnt = nullptr, uint32_t a = 0, uint32_t b = 0) {
    const uint32_t top = rec_arena ? st->arena_top : 0;
    const uint32_t cap = rec_cap > top ? rec_cap - top : 0;
    const uint32_t cnt = min(st->rec_count, cap);
    const uint32_t *r = rec + top;
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < cnt; i += gridDim.x * 256) {
        const int64_t p = r[i];
        tok[p] = (uint16_t)X;
        const int64_t q = next_live(tok, n, p);
        if (q >= 0) tok[q] = HOLE;
    }
    __shared__ uint32_t s_last;
    __syncthreads();  // every thread of the block has read rec_count / arena_top
    if (threadIdx.x == 0) s_last = atomicAdd(&st->ticket, 1u) == gridDim.x - 1;
    __syncthreads();
    if (!s_last || threadIdx.x) return;
    st->total_occ += cnt;
    if (rec_arena && T.lst_off) {
        T.lst_off[X] = top;
        T.lst_len[X] = cnt;
        st->arena_top = top + cnt;
    }
    if (tcnt) {  // live token counts of the batched path (a self pair consumes 2 a's per occurrence)
        tcnt[X] = (int32_t)cnt;
        tcnt[a] -= (int32_t)cnt;
        tcnt[b] -= (int32_t)cnt;
    }
    st->rec_count = 0;
    st->ticket = 0;
    scratch[0] = scratch[1] = 0;  // the scan's xx / occurrence tallies (encode keeps no counts)
}
// end of merge: clear the neighbour histograms [0, X) and roll the per-merge counters
__global__ void __launch_bounds__(256) zbpe_reset_merge(DevState *st, uint32_t *left, uint32_t *right, uint32_t X) {
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    if (t < X) { left[t] = 0; right[t] = 0; }
    if (t == 0) {
        st->last_occ = st->rec_count;
        st->total_occ += st->rec_count;
        st->rec_count = 0;
        st->xx = 0;
    }
}

// ------------------------------------------------------------------------------------------
// Self pair (a, a): left-greedy over runs needs each position's offset parity inside its run
// of a's (basic_tokenizer.zig:217-226 consumes a run of L a's as floor(L/2) merges). Runs are runs
// of LIVE tokens: holes are transparent, so the stream needs no compaction first. A segment of the
// stream acts on the parity x of the run entering it as x -> has_non_a ? p : x ^ p (p = parity of
// the live a's after its last live non-a); tiles and threads compose these functions in order.
// ------------------------------------------------------------------------------------------
constexpr int SELF_THREADS = 256;
constexpr int SELF_PER_THREAD = 32;
constexpr int SELF_TILE = SELF_THREADS * SELF_PER_THREAD;  // 8192
constexpr int64_t SELF_GRID = 768;                          // persistent zbpe_scan_self workgroups (3 per CU)
static_assert(SELF_TILE == PRES_BLK, "a self-pair tile is one presence block");
// run-parity function of a segment: bit0 = no live non-a (x -> x ^ p), bit1 = p
__device__ inline uint8_t self_apply(uint8_t f, uint8_t x) { return (f & 1) ? (uint8_t)(x ^ ((f >> 1) & 1)) : (uint8_t)((f >> 1) & 1); }
// g after f
__device__ inline uint8_t self_compose(uint8_t f, uint8_t g) { return (g & 1) ? (uint8_t)((f & 1) | ((f ^ g) & 2)) : g; }
// a thread's SELF_PER_THREAD slots [p0, p0 + 32) in registers, two tokens a word (HOLE past end):
// four 16-B loads, not 32 two-byte ones
__device__ inline void self_load(const uint16_t *tok, int64_t p0, int64_t end, uint32_t (&w)[16]) {
    if (p0 + SELF_PER_THREAD <= end) {
        const uint4 *q = reinterpret_cast<const uint4 *>(tok + p0);
#pragma unroll
        for (int v = 0; v < 4; v++) {
            const uint4 x = q[v];
            w[4 * v] = x.x; w[4 * v + 1] = x.y; w[4 * v + 2] = x.z; w[4 * v + 3] = x.w;
        }
    } else {
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const uint32_t lo = p0 + 2 * k < end ? tok[p0 + 2 * k] : HOLE;
            const uint32_t hi = p0 + 2 * k + 1 < end ? tok[p0 + 2 * k + 1] : HOLE;
            w[k] = lo | (hi << 16);
        }
    }
}
// the run-parity function of the 32 slots, and (when x_in >= 0) the mask of the slots holding an a
// at an even offset of its live run given the parity x_in of the run entering them
__device__ inline uint8_t self_walk(const uint32_t (&w)[16], uint32_t a, int x_in, uint32_t *even_a) {
    uint8_t all = 1, par = 0, x = (uint8_t)(x_in & 1);
    uint32_t m = 0;
#pragma unroll
    for (int i = 0; i < SELF_PER_THREAD; i++) {
        const uint32_t t = (w[i >> 1] >> (16 * (i & 1))) & 0xFFFFu;
        if (t == HOLE) continue;
        if (t != a) { all = 0; par = 0; x = 0; continue; }
        par ^= 1;
        if (!x) m |= 1u << i;
        x ^= 1;
    }
    if (even_a) *even_a = m;
    return (uint8_t)(all | (par << 1));
}
// exclusive composition of the threads' functions in thread order (wave shuffles, then the waves
// through LDS); *total: the whole block's function
// (every thread of the block; the wave scan by DPP: row_shr:1,2,4,8, then row_bcast:15 / :31, a lane with no source
// composing the identity 1 -- x -> x)
template <int CTRL, int ROWS>
__device__ __attribute__((always_inline)) inline uint8_t self_dpp(uint8_t f) {
    return (uint8_t)__builtin_amdgcn_update_dpp(1, (int)f, CTRL, ROWS, 0xF, false);
}
__device__ inline uint8_t self_block_scan(uint8_t f, uint8_t *s_wave, uint8_t *total) {
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint8_t inc = f;
    inc = self_compose(self_dpp<0x111, 0xF>(inc), inc);
    inc = self_compose(self_dpp<0x112, 0xF>(inc), inc);
    inc = self_compose(self_dpp<0x114, 0xF>(inc), inc);
    inc = self_compose(self_dpp<0x118, 0xF>(inc), inc);
    inc = self_compose(self_dpp<0x142, 0xA>(inc), inc);
    inc = self_compose(self_dpp<0x143, 0xC>(inc), inc);
    const uint8_t ex = (uint8_t)wave_shr1(inc, 1u);  // (lane 0: the identity)
    if (lane == 63) s_wave[wv] = inc;
    __syncthreads();
    uint8_t pre = 1;
    for (uint32_t j = 0; j < wv; j++) pre = self_compose(pre, s_wave[j]);
    if (total) {
        uint8_t t = 1;
        for (uint32_t j = 0; j < SELF_THREADS / 64; j++) t = self_compose(t, s_wave[j]);
        *total = t;
    }
    return self_compose(pre, ex);
}
__global__ void __launch_bounds__(SELF_THREADS) zbpe_self_tiles(const uint16_t *__restrict__ tok, int64_t n, uint32_t a,
                                                                uint8_t *__restrict__ tile_fn) {
    // tile_fn bit0: the tile holds no live non-a; bit1: parity of its trailing live a-run
    const int64_t beg = blockIdx.x * (int64_t)SELF_TILE;
    const int64_t end = min(n, beg + SELF_TILE);
    __shared__ uint8_t s_wave[SELF_THREADS / 64];
    uint32_t w[16];
    self_load(tok, beg + threadIdx.x * SELF_PER_THREAD, end, w);
    uint8_t total;
    (void)self_block_scan(self_walk(w, a, -1, nullptr), s_wave, &total);
    if (threadIdx.x == 0) tile_fn[blockIdx.x] = total;
}
// carry_in[t] = parity of the a-run entering tile t. One block; each thread composes a segment.
// carry_in[t] = parity of the a-run entering tile t, starting from *x0 (the run entering the shard
// from the ranks to the left; nullptr = 0). shard_fn (optional) = the whole shard as one function.
__global__ void __launch_bounds__(1024) zbpe_self_carry(const uint8_t *__restrict__ tile_fn, int64_t ntiles,
                                                        uint8_t *__restrict__ carry_in, const uint8_t *x0,
                                                        uint32_t *shard_fn) {
    // function of a tile: x -> all_a ? x ^ p : p   (x, p parities)
    // (a thread's segment is a whole number of 16-tile words, read and written as 16-B vectors: one byte at a time,
    // each a dependent miss, the launch took 0.1-0.25 ms at C4)
    __shared__ uint8_t s_all[1024], s_par[1024];
    const int64_t per = ((ntiles + 1023) / 1024 + 15) & ~(int64_t)15;
    const int64_t b0 = threadIdx.x * per, b1 = min(ntiles, b0 + per);
    const auto word = [&](int64_t t, uint8_t (&f)[16]) {  // tile functions [t, t + 16) (past ntiles: identity)
        if (t + 16 <= ntiles) {
            const uint4 v = *reinterpret_cast<const uint4 *>(tile_fn + t);
            const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int k = 0; k < 16; k++) f[k] = (uint8_t)(u[k >> 2] >> (8 * (k & 3)));
        } else {
#pragma unroll
            for (int k = 0; k < 16; k++) f[k] = t + k < ntiles ? tile_fn[t + k] : (uint8_t)1;
        }
    };
    uint8_t all = 1, par = 0;  // identity
    for (int64_t t = b0; t < b1; t += 16) {
        uint8_t f[16];
        word(t, f);
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const uint8_t fa = f[k] & 1, fp = (f[k] >> 1) & 1;
            if (fa) par ^= fp;  // compose: g(x) = f(cur(x))
            else { all = 0; par = fp; }
        }
    }
    s_all[threadIdx.x] = all;
    s_par[threadIdx.x] = par;
    __syncthreads();
    if (threadIdx.x == 0) {  // sequential exclusive composition over 1024 segments
        uint8_t x = x0 ? (*x0 & 1) : 0, A = 1, P = 0;
        for (int t = 0; t < 1024; t++) {
            if (s_all[t]) P ^= s_par[t];
            else { A = 0; P = s_par[t]; }
            uint8_t nx = s_all[t] ? (x ^ s_par[t]) : s_par[t];
            s_par[t] = x;  // carry into segment t
            x = nx;
        }
        if (shard_fn) *shard_fn = (uint32_t)A | ((uint32_t)P << 1);
    }
    __syncthreads();
    uint8_t x = s_par[threadIdx.x];
    for (int64_t t = b0; t < b1; t += 16) {
        uint8_t f[16], c[16];
        word(t, f);
#pragma unroll
        for (int k = 0; k < 16; k++) {
            c[k] = x;
            const uint8_t fa = f[k] & 1, fp = (f[k] >> 1) & 1;
            x = fa ? (x ^ fp) : fp;
        }
        if (t + 16 <= ntiles) {
            uint32_t u[4] = {0, 0, 0, 0};
#pragma unroll
            for (int k = 0; k < 16; k++) u[k >> 2] |= (uint32_t)c[k] << (8 * (k & 3));
            *reinterpret_cast<uint4 *>(carry_in + t) = make_uint4(u[0], u[1], u[2], u[3]);
        } else {
            for (int k = 0; k < 16 && t + k < ntiles; k++) carry_in[t + k] = c[k];
        }
    }
}
// parity of the a-run entering shard `rank` from the gathered whole-shard functions of ranks < rank
__global__ void zbpe_self_x0(const uint32_t *__restrict__ fns, int rank, uint8_t *x0) {
    if (threadIdx.x || blockIdx.x) return;
    uint8_t x = 0;
    for (int r = 0; r < rank; r++) {
        const uint32_t f = fns[r];
        x = (f & 1) ? (x ^ ((f >> 1) & 1)) : ((f >> 1) & 1);
    }
    *x0 = x;
}
// (persistent: a workgroup takes tiles blockIdx.x, blockIdx.x + gridDim.x, ...; its LDS neighbour bins are
// cleared once and flushed once, and its records are staged over several tiles: a flush (one global atomic on the
// shared record counter) only once another tile might not fit. One workgroup per tile with a flush each made
// ~2.6e5 same-address atomics per launch at C4 -- ~12 ns each at the counter, most of the launch's 1-2 ms.)
constexpr uint32_t SELF_REC = 2 * (SELF_TILE / 2);  // staged records: two tiles' worth (a tile holds <= SELF_TILE / 2)
__global__ void __launch_bounds__(SELF_THREADS) zbpe_scan_self(ScanArgs A0, const uint8_t *__restrict__ carry_in) {
    const ScanArgs A = scan_args_resolve(A0, load_head(A0.st), A0.X);
    __shared__ uint32_t s_left[LDS_BINS], s_right[LDS_BINS];
    __shared__ uint32_t s_rec[SELF_REC];
    __shared__ uint8_t s_wave[SELF_THREADS / 64];
    __shared__ uint32_t s_nrec, s_base;
    for (int i = threadIdx.x; i < LDS_BINS; i += SELF_THREADS) { s_left[i] = 0; s_right[i] = 0; }
    if (threadIdx.x == 0) s_nrec = 0;
    NeighbourHist H{s_left, s_right, A.left, A.right};
    const uint16_t *tok = A.tok;
    const uint32_t a = A.a, lane = threadIdx.x & 63;
    const int64_t ntiles = (A.n + SELF_TILE - 1) / SELF_TILE;
    uint32_t xx = 0, staged = 0, occ = 0;  // (staged, occ: workgroup-uniform)
    const auto flush = [&]() {  // every thread; after a barrier that published s_nrec == staged
        if (threadIdx.x == 0) s_base = atomicAdd(A.rec_ctr, staged);
        __syncthreads();
        const uint32_t base = s_base;
        for (uint32_t i = threadIdx.x; i < staged; i += SELF_THREADS)
            if (base + i < A.rec_cap) A.rec[base + i] = s_rec[i];
        if (threadIdx.x == 0 && base + staged > A.rec_cap) atomicOr(&A.st->error, 8u);
        occ += staged;
        staged = 0;
        __syncthreads();  // (every thread has read s_base and s_rec)
        if (threadIdx.x == 0) s_nrec = 0;
    };
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t beg = tile * (int64_t)SELF_TILE;
        const int64_t end = min(A.n, beg + SELF_TILE);
        const int64_t t0 = beg + threadIdx.x * SELF_PER_THREAD;
        uint32_t w[16];
        self_load(tok, t0, end, w);
        // parity of the live a-run entering my slots: the tile's carry through the threads before mine
        // (self_block_scan's barrier also orders a flush's s_nrec reset before this tile's records)
        const uint8_t pre = self_block_scan(self_walk(w, a, -1, nullptr), s_wave, nullptr);
        uint32_t cand;
        (void)self_walk(w, a, self_apply(pre, carry_in[tile] & 1), &cand);
        // a's at even offsets of their runs: occurrences when the next live token is an a (wave-uniform steps:
        // one LDS atomic per wave and step reserves the records)
        while (__ballot(cand != 0)) {
            bool hit = false;
            int64_t p = 0;
            if (cand) {
                const int i = __builtin_ctz(cand);
                cand &= cand - 1;
                p = t0 + i;
                const int64_t q = next_live_h(A, p);
                hit = q != NONE_POS && tok_h(A, q) == a;
                if (hit && A.count_deltas) {  // occurrence (p, q)
                    // the left neighbour, unless it is the end of a previous occurrence
                    const int64_t l = prev_live_h(A, p);
                    if (l != NONE_POS) {
                        const uint32_t tl = tok_h(A, l);
                        if (tl != a) H.left((uint16_t)tl);
                    }
                    const int64_t r = next_live_h(A, q);
                    if (r != NONE_POS) {
                        const uint32_t tr = tok_h(A, r);
                        bool r_occ = false;
                        if (tr == a) {
                            const int64_t r2 = next_live_h(A, r);
                            r_occ = r2 != NONE_POS && tok_h(A, r2) == a;
                        }
                        if (r_occ) xx++;
                        else H.right((uint16_t)tr);
                    }
                }
            }
            const uint64_t hm = __ballot(hit);
            if (hm) {
                uint32_t base = 0;
                if (lane == 0) base = atomicAdd(&s_nrec, (uint32_t)__popcll(hm));
                base = lane_bcast(base, 0);
                if (hit) s_rec[base + (uint32_t)__popcll(hm & ((1ull << lane) - 1ull))] = (uint32_t)p;
            }
        }
        __syncthreads();
        const uint32_t nrec = s_nrec;
        if (nrec != staged && threadIdx.x == 0 && A.pres) pres_set(A, beg);  // (SELF_TILE == PRES_BLK: one block)
        staged = nrec;
        if (staged > SELF_REC - SELF_TILE / 2) flush();  // the next tile might not fit
    }
    if (staged) flush();
    if (threadIdx.x == 0 && occ) atomicAdd(A.occ_out, occ);
    xx = wave_sum_u32(xx);  // (every thread of the block)
    if ((threadIdx.x & 63) == 0 && xx) atomicAdd(A.xx_out, xx);
    __syncthreads();
    if (occ) {
        for (int i = threadIdx.x; i < LDS_BINS; i += SELF_THREADS) {
            uint32_t l = s_left[i], r = s_right[i];
            if (l) atomicAdd(&A.left[i], l);
            if (r) atomicAdd(&A.right[i], r);
        }
    }
}

// Self pair (a, a) from the occurrence list of a on the host path (self_list_walk)
__global__ void __launch_bounds__(SCAN_THREADS) zbpe_scan_self_list(ScanArgs A0) {
    const ScanArgs A = scan_args_resolve(A0, load_head(A0.st), A0.X);
    __shared__ ScanLds S;
    self_list_walk(A, S, blockIdx.x, gridDim.x);
}

// ------------------------------------------------------------------------------------------
// Compaction (squeeze holes): tile counts -> exclusive scan -> scatter
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) zbpe_compact_count(const uint16_t *__restrict__ tok, int64_t n,
                                                          uint32_t *__restrict__ tile_cnt) {
    const int64_t beg = blockIdx.x * (int64_t)COMPACT_TILE;
    uint32_t c = 0;
    for (int i = threadIdx.x; i < COMPACT_TILE / 8; i += 256) {
        int64_t p = beg + 8 * i;
        if (p >= n) break;
        uint4 v = *reinterpret_cast<const uint4 *>(tok + p);
#pragma unroll
        for (int k = 0; k < 8; k++) c += (tok_at(v, k) != HOLE) && (p + k < n);
    }
    c = wave_sum(c);
    __shared__ uint32_t s[4];
    if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) tile_cnt[blockIdx.x] = s[0] + s[1] + s[2] + s[3];
}
// exclusive scan of tile counts (one block, 1024 threads, sequential segments)
__global__ void __launch_bounds__(1024) zbpe_scan_u32(const uint32_t *__restrict__ in, int64_t m,
                                                      uint64_t *__restrict__ out, uint64_t *total) {
    __shared__ uint64_t s[1024];
    const int64_t per = (m + 1023) / 1024;
    const int64_t b0 = threadIdx.x * per, b1 = min(m, b0 + per);
    uint64_t sum = 0;
    for (int64_t i = b0; i < b1; i++) sum += in[i];
    s[threadIdx.x] = sum;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
        uint64_t v = threadIdx.x >= off ? s[threadIdx.x - off] : 0;
        __syncthreads();
        s[threadIdx.x] += v;
        __syncthreads();
    }
    uint64_t run = s[threadIdx.x] - sum;
    for (int64_t i = b0; i < b1; i++) { out[i] = run; run += in[i]; }
    if (threadIdx.x == 1023) *total = s[1023];
}
// The tile's live tokens are packed in LDS first and then written out contiguously (a wave's store covers 64
// consecutive u16): each thread storing its own run of up to 32 tokens put every store instruction of a wave on 64
// different cache lines, ~2 ms per 1 GiB compaction.
__global__ void __launch_bounds__(256) zbpe_compact_scatter(const uint16_t *__restrict__ tok, int64_t n,
                                                            const uint64_t *__restrict__ tile_off, uint16_t *__restrict__ out) {
    __shared__ uint16_t s_out[COMPACT_TILE];
    __shared__ uint32_t s_w[4];
    // each thread owns 32 consecutive tokens of the tile
    const int64_t beg = blockIdx.x * (int64_t)COMPACT_TILE + threadIdx.x * 32;
    uint16_t t[32];
    uint32_t c = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        int64_t p = beg + 8 * q;
        uint4 v = p < n ? *reinterpret_cast<const uint4 *>(tok + p) : make_uint4(0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu);
#pragma unroll
        for (int k = 0; k < 8; k++) {
            uint32_t x = (p + k < n) ? tok_at(v, k) : HOLE;
            t[8 * q + k] = (uint16_t)x;
            c += x != HOLE;
        }
    }
    // block exclusive scan of c (wave scans, then the four wave totals)
    const uint32_t incl = wave_incl_scan(c);
    if ((threadIdx.x & 63) == 63) s_w[threadIdx.x >> 6] = incl;
    __syncthreads();
    uint32_t o = incl - c;
    for (uint32_t w = 0; w < (threadIdx.x >> 6); w++) o += s_w[w];
    const uint32_t total = s_w[0] + s_w[1] + s_w[2] + s_w[3];
#pragma unroll
    for (int k = 0; k < 32; k++)
        if (t[k] != HOLE) s_out[o++] = t[k];
    __syncthreads();
    uint16_t *dst = out + tile_off[blockIdx.x];
    for (uint32_t i = threadIdx.x; i < total; i += 256) dst[i] = s_out[i];
}
__global__ void zbpe_fill_u16(uint16_t *p, int64_t beg, int64_t end, uint16_t v) {
    for (int64_t i = beg + blockIdx.x * 256 + threadIdx.x; i < end; i += (int64_t)gridDim.x * 256) p[i] = v;
}

// ------------------------------------------------------------------------------------------
// Zig-order tie-break. The Zig map of iteration t has capacity C_f; its set
// of occupied slots depends only on the multiset of home slots hash & (C_f-1), so a parallel
// linear-probing insert of every live key reproduces it exactly. Tied keys sit in the run that
// holds their home; the tied key with the smallest home wins unless the second-smallest home is
// in the same run or a tied key could have wrapped past slot C_f-1 (then: exact emulation).
// ------------------------------------------------------------------------------------------
// ------------------------------------------------------------------------------------------
// Hot list: argmax over the ids whose count was >= theta when they entered the list. Counts of
// existing pairs only fall and a new pair's count never exceeds the current top, so every id with
// count >= theta is in the list; if none of them still has count >= theta the host rebuilds the
// list with a lower theta (zbpe_count_hist -> choose theta -> zbpe_hot_build).
// ------------------------------------------------------------------------------------------
__device__ inline uint32_t count_bin(uint32_t c) {
    if (c < 64) return c;
    const uint32_t e = 31 - __clz(c);
    return 64 + (e - 6) * 32 + ((c >> (e - 5)) & 31);
}
__global__ void __launch_bounds__(256) zbpe_count_hist(Tables T, const DevState *st, uint32_t *__restrict__ hist) {
    __shared__ uint32_t h[COUNT_BINS];
    for (int i = threadIdx.x; i < COUNT_BINS; i += 256) h[i] = 0;
    __syncthreads();
    const uint32_t n = min(st->num_ids, T.id_cap);
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        const uint32_t c = T.id_cnt[i];
        if (c) atomicAdd(&h[count_bin(c)], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < COUNT_BINS; i += 256)
        if (h[i]) atomicAdd(&hist[i], h[i]);
}
// before a rebuild: the ids of the current list unlisted (their hpos back to NO_ID)
__global__ void __launch_bounds__(256) zbpe_hot_clear(Tables T, const DevState *st) {
    const uint32_t n = min(st->hot_len, T.hot_cap);
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        const uint32_t id = (uint32_t)T.hot[i];
        if (id < T.id_cap) T.hpos[id] = NO_ID;
    }
}
__global__ void __launch_bounds__(256) zbpe_hot_build(Tables T, DevState *st) {
    const uint32_t n = min(st->num_ids, T.id_cap), theta = st->theta;
    const uint32_t stride = gridDim.x * 256;
    for (uint32_t i0 = blockIdx.x * 256 + (threadIdx.x & ~63u); i0 < n; i0 += stride) {  // wave-uniform trip count
        const uint32_t i = i0 + (threadIdx.x & 63);
        const uint32_t c = i < n ? T.id_cnt[i] : 0u;
        const bool take = i < n && c >= theta;
        const uint32_t j = wave_append(&st->hot_len, take);
        if (take) hot_put(T, j, i, T.id_key[i], c);
    }
}
// Fused select: argmax over the hot list, the final reduction by the last block to finish
// (agent-scope release/acquire around the ticket, cdna_hip_programming.md Guideline 16), the
// stream's last-pair count, and the end-of-merge resets (neighbour histograms, counters) when
// roll != 0. One launch per merge instead of three.
// the state words merge_begin_eval / merge_begin_commit read, as select_finish left them (the fused
// select passes them on in registers instead of reloading what the same thread just stored)
struct FinishOut {
    int32_t live;
    uint32_t hot_len, top_count, tie_count, arena_top, arena_rep, lastpair, key;
    long long live_tokens;
};
// the state words the roll reads (select_finish), in the order of RollIn's slots
enum RollIn : int { RI_REC, RI_TOTAL_OCC, RI_HOLES, RI_ARENA_TOP, RI_ARENA_REP, RI_GOCC, RI_LIVE_TOK_LO, RI_LIVE_TOK_HI,
                    RI_LIVE, RI_HOT_LEN, RI_LASTPAIR, RI_WORDS };
// The fused select's roll words, loaded at kernel start straight into LDS by lanes [0, RI_WORDS) of
// wave 0 (global_load_lds: no registers held across the kernel); they are stable until the last
// block rolls, and block_ticket_last's vmcnt(0) + barrier publishes them to the block.
// (rd: a multi-merge round's select -- lanes [RI_WORDS, RI_WORDS + RD_WORDS) load the RoundHead words too)
constexpr uint32_t RD_WORDS = sizeof(RoundHead) / 4;
static_assert(RI_WORDS + RD_WORDS <= 64, "one wave loads the roll words");
__device__ inline void roll_preload(const DevState *st, const uint32_t *delta, uint32_t X, uint32_t *s_pre, bool rd = false) {
    const uint32_t lane = threadIdx.x;
    if (rd && lane >= RI_WORDS && lane < RI_WORDS + RD_WORDS) {
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const uint32_t *>(&st->rd) + (lane - RI_WORDS),
                                         (__attribute__((address_space(3))) void *)s_pre, 4, 0, 0);
        return;
    }
    if (lane >= RI_WORDS) return;
    const uint32_t *w = lane == RI_REC ? &st->rec_count : lane == RI_TOTAL_OCC ? &st->total_occ
                        : lane == RI_HOLES ? &st->holes_made : lane == RI_ARENA_TOP ? &st->arena_top
                        : lane == RI_ARENA_REP ? &st->arena_rep : lane == RI_GOCC ? delta + 2 * X + 1
                        : lane == RI_LIVE_TOK_LO ? reinterpret_cast<const uint32_t *>(&st->live_tokens)
                        : lane == RI_LIVE_TOK_HI ? reinterpret_cast<const uint32_t *>(&st->live_tokens) + 1
                        : lane == RI_LIVE ? reinterpret_cast<const uint32_t *>(&st->live)
                        : lane == RI_HOT_LEN ? &st->hot_len : &st->lastpair_count;
    __builtin_amdgcn_global_load_lds(w, (__attribute__((address_space(3))) void *)s_pre, 4, 0, 0);
}
__device__ inline uint64_t dev_zig_cap_for(uint64_t D);
__device__ inline bool dev_zig_at_max_load(uint64_t cap, uint64_t D);
__device__ inline void select_finish(const Tables &T, DevState *st, MaxRec q, const uint16_t *tok, int64_t n,
                                     uint32_t *delta, uint32_t X, int roll, const Boundary *bnd, int world,
                                     uint32_t key_hint = NO_ID, uint32_t lastpair_hint = NO_ID, FinishOut *fo = nullptr,
                                     const uint32_t *pre = nullptr, bool defer_key = false, bool lazy_lp = false);
__global__ void __launch_bounds__(ARGMAX_THREADS) zbpe_select(Tables T, DevState *st, MaxRec *__restrict__ partial,
                                                              const uint16_t *__restrict__ tok, int64_t n, uint32_t *delta,
                                                              uint32_t X, int roll, const Boundary *__restrict__ bnd, int world) {
    if (st->halt) return;
    for (uint32_t t = blockIdx.x * ARGMAX_THREADS + threadIdx.x; t < 2 * X; t += gridDim.x * ARGMAX_THREADS) delta[t] = 0;
    const uint32_t nh = min(st->hot_len, T.hot_cap), theta = st->theta;
    MaxRec r{0, 0, NO_ID};
    for (uint32_t i = blockIdx.x * ARGMAX_THREADS + threadIdx.x; i < nh; i += gridDim.x * ARGMAX_THREADS) {
        const uint32_t id = (uint32_t)T.hot[i], c = T.id_cnt[id];
        if (c >= theta && c) r = max_combine(r, MaxRec{c, 1u, id});
    }
    r = wave_max(r);
    __shared__ MaxRec sm[ARGMAX_THREADS / WAVE];
    __shared__ uint32_t s_last;
    if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = r;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < ARGMAX_THREADS / WAVE; w++) r = max_combine(r, sm[w]);
        // write-through (sc1) partial, drained before the ticket; the last block reads the partials
        // with sc1 loads (no release / acquire fences: cdna_hip_programming.md section 6 G16, R1)
        __hip_atomic_store(&partial[blockIdx.x].cnt, r.cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&partial[blockIdx.x].ties, r.ties, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&partial[blockIdx.x].id, r.id, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        s_last = atomicAdd(&st->ticket, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (!s_last) return;
    MaxRec q{0, 0, NO_ID};
    for (uint32_t i = threadIdx.x; i < gridDim.x; i += ARGMAX_THREADS)
        q = max_combine(q, MaxRec{__hip_atomic_load(&partial[i].cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                                  __hip_atomic_load(&partial[i].ties, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                                  __hip_atomic_load(&partial[i].id, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)});
    q = wave_max(q);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = q;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < ARGMAX_THREADS / WAVE; w++) q = max_combine(q, sm[w]);
        select_finish(T, st, q, tok, n, delta, X, roll, bnd, world);
    }
}
// the selection's state update (one thread): top pair, tie count, the stream's last pair (ties),
// and at roll the end-of-merge bookkeeping (occurrence list of X, counters, deltas' tail)
__device__ inline void select_finish(const Tables &T, DevState *st, MaxRec q, const uint16_t *tok, int64_t n,
                                     uint32_t *delta, uint32_t X, int roll, const Boundary *bnd, int world,
                                     uint32_t key_hint, uint32_t lastpair_hint, FinishOut *fo, const uint32_t *pre,
                                     bool defer_key, bool lazy_lp) {
    {
        // every state word the roll reads, loaded together before the first store (the stores
        // below may alias them as far as the compiler knows, which would serialise each load), or
        // preloaded (pre: roll_preload's LDS words)
        uint32_t *tail = delta + 2 * X;
        uint32_t rec_count, total_occ, holes_made, arena_top, arena_rep, gocc, hot_len, lastpair_old;
        long long live_tokens;
        int32_t live;
        if (pre) {
            rec_count = pre[RI_REC]; total_occ = pre[RI_TOTAL_OCC]; holes_made = pre[RI_HOLES];
            arena_top = pre[RI_ARENA_TOP]; arena_rep = pre[RI_ARENA_REP]; gocc = roll ? pre[RI_GOCC] : 0u;
            live_tokens = (long long)(((uint64_t)pre[RI_LIVE_TOK_HI] << 32) | pre[RI_LIVE_TOK_LO]);
            live = (int32_t)pre[RI_LIVE]; hot_len = pre[RI_HOT_LEN]; lastpair_old = pre[RI_LASTPAIR];
        } else {
            rec_count = st->rec_count; total_occ = st->total_occ; holes_made = st->holes_made;
            arena_top = st->arena_top; arena_rep = st->arena_rep; gocc = roll ? tail[1] : 0u;
            live_tokens = st->live_tokens;
            live = st->live; hot_len = st->hot_len; lastpair_old = st->lastpair_count;
        }
        // defer_key: the caller stores top_key itself later (its load is off the critical path; the
        // key matters to merge_begin only without a tie, when key_hint has it)
        const uint32_t top_key = q.id == NO_ID ? EMPTY_KEY : key_hint != NO_ID ? key_hint : defer_key ? NO_ID : T.id_key[q.id];
        uint32_t lastpair = lastpair_old;
        st->top_count = q.cnt;
        st->tie_count = q.cnt ? q.ties : 0;
        st->top_id = q.id;
        if (top_key != NO_ID) st->top_key = top_key;
        if (q.ties > 1 && lastpair_hint != NO_ID) {
            st->lastpair_count = lastpair = lastpair_hint;
        } else if (q.ties > 1 && !(lazy_lp && !dev_zig_at_max_load(dev_zig_cap_for((uint64_t)max(live, 0)), (uint64_t)max(live, 0)))) {
            // (lazy_lp: only when the capacity depends on it -- D exactly at a max load; else the stale
            // count gives the same capacity, here and in the host's resolve_tie, which reads the same D)
            uint32_t lt[2];  // last live token of the whole stream, then the one before
            int got = 0;
            if (world > 1) {
                for (int r = world - 1; r >= 0 && got < 2; r--)
                    for (int k = 0; k < bnd[r].nlast && got < 2; k++) lt[got++] = bnd[r].last[k];
            } else {
                for (int64_t p = n - 1; p >= 0 && got < 2; p--)
                    if (tok[p] != HOLE) lt[got++] = tok[p];
            }
            st->lastpair_count = lastpair = got == 2 ? ht_find_count(T, pair_key(lt[1], lt[0])) : 0;
        }
        if (fo) {
            fo->live = live;
            fo->hot_len = hot_len;
            fo->top_count = q.cnt;
            fo->tie_count = q.cnt ? q.ties : 0;
            fo->arena_top = roll && T.lst_off ? arena_top + rec_count : arena_top;
            fo->arena_rep = roll ? arena_rep + gocc : arena_rep;
            fo->lastpair = lastpair;
            fo->key = top_key;
            fo->live_tokens = roll ? live_tokens - holes_made : live_tokens;
        }
        if (roll) {
            st->last_occ = rec_count;
            st->total_occ = total_occ + rec_count;
            st->last_gocc = gocc;
            st->arena_rep = arena_rep + gocc;
            st->last_holes = holes_made;
            st->live_tokens = live_tokens - holes_made;
            st->tie_len = 0;
            if (T.lst_off) {  // this merge's records (positions of X) are X's occurrence list
                T.lst_off[X] = arena_top;
                T.lst_len[X] = rec_count;
                st->arena_top = arena_top + rec_count;
            }
            st->holes_made = 0;
            st->rec_count = 0;
            tail[0] = tail[1] = 0;
        }
        st->ticket = 0;
    }
}

// ------------------------------------------------------------------------------------------
// Zig-order tie-break. The Zig map of this merge has capacity C; its set of
// occupied slots depends only on the multiset of home slots hash & (C-1) of the live pairs, kept
// in T.home_cnt. Scanning slots in order, the carry c (keys displaced past slot s) obeys
// c(s+1) = max(0, c(s) + cnt[s] - 1), and slot s is occupied iff c(s) + cnt[s] >= 1. A run of
// slots acts on the carry as c -> max(m, c + q); runs compose associatively, so the carry into any
// slot is one ordered reduction over the other C-1 slots. The tied pair with the smallest home
// wins unless the second-smallest home lies in the same occupied run, or a tied pair sits in a
// run that wraps past slot C-1 (both rare): then the exact first-occurrence emulation decides.
// ------------------------------------------------------------------------------------------
__device__ inline Summ summ_cat(Summ a, Summ b) { return Summ{a.q + b.q, max(b.m, a.m + b.q)}; }
__device__ inline Summ summ_slot(uint32_t k) {
    const int32_t q = (int32_t)k - 1;
    return Summ{q, q > 0 ? q : 0};
}
// summ_cat(x, summ_slot(k)) for x.m >= 0, which every summary has (summ_slot and summ_cat keep m >= 0):
// max(max(k - 1, 0), x.m + k - 1) = max(0, x.m + k - 1)
__device__ inline Summ slot_fold(Summ x, uint32_t k) {
    const int32_t d = (int32_t)k - 1;
    return Summ{x.q + d, max(0, x.m + d)};
}
// Ordered scans of carry summaries by DPP (every lane of the wave active). Summ{0, 0} is the identity of
// summ_cat: every summary has m >= max(q, 0) (summ_slot, slot_fold and summ_cat keep it), so
// summ_cat({0, 0}, b) = {b.q, max(b.m, b.q)} = b and summ_cat(a, {0, 0}) = {a.q, max(0, a.m)} = a; a DPP lane
// with no source keeps the 0 it starts from. Inclusive: row_shr:1,2,4,8 inside each 16-lane row, then row 0's
// total into row 1 and row 2's into row 3 (row_bcast:15), rows 0-1's into rows 2 and 3 (row_bcast:31), each
// composed on the left. (One VALU op per move; the __shfl forms were six dependent ds_bpermute steps on the tie
// decision's and the home refresh's paths.)
template <int CTRL, int ROWS>
__device__ __attribute__((always_inline)) inline Summ summ_dpp(Summ x) {
    return Summ{__builtin_amdgcn_update_dpp(0, x.q, CTRL, ROWS, 0xF, false), __builtin_amdgcn_update_dpp(0, x.m, CTRL, ROWS, 0xF, false)};
}
__device__ __attribute__((always_inline)) inline Summ summ_scan_dpp(Summ x) {  // lane i: x_0 . x_1 . ... . x_i
    x = summ_cat(summ_dpp<0x111, 0xF>(x), x);
    x = summ_cat(summ_dpp<0x112, 0xF>(x), x);
    x = summ_cat(summ_dpp<0x114, 0xF>(x), x);
    x = summ_cat(summ_dpp<0x118, 0xF>(x), x);
    x = summ_cat(summ_dpp<0x142, 0xA>(x), x);
    x = summ_cat(summ_dpp<0x143, 0xC>(x), x);
    return x;
}
// the exclusive scan from the inclusive one (lane 0: the identity)
__device__ __attribute__((always_inline)) inline Summ summ_excl_dpp(Summ inc) {
    return Summ{(int32_t)wave_shr1((uint32_t)inc.q, 0u), (int32_t)wave_shr1((uint32_t)inc.m, 0u)};
}
__device__ __attribute__((always_inline)) inline Summ summ_lane(Summ x, int l) {
    return Summ{(int32_t)lane_bcast((uint32_t)x.q, l), (int32_t)lane_bcast((uint32_t)x.m, l)};
}
// ordered reduction over the lanes of one wave (x_0 . x_1 . ... . x_63), wave-uniform (every lane active)
__device__ inline Summ wave_reduce_summ(Summ x) { return summ_lane(summ_scan_dpp(x), 63); }
// the summary of 64 consecutive slots (16 words of 4 one-byte home counts): q from byte sums
// (v_sad_u8, one per word), m by the slot_fold recurrence
__device__ inline Summ fold64(const uint32_t (&w)[16]) {
    uint32_t ks = 0;
    int32_t m = 0;
#pragma unroll
    for (int j = 0; j < 16; j++) {
        ks = __builtin_amdgcn_sad_u8(w[j], 0u, ks);
#pragma unroll
        for (int b = 0; b < 4; b++) m = max(0, m + (int32_t)((w[j] >> (8 * b)) & 0xffu) - 1);
    }
    return Summ{(int32_t)ks - 64, m};
}
__device__ inline uint32_t home_at(const uint32_t *hc, uint32_t s) { return (hc[s >> 2] >> (8 * (s & 3))) & 0xffu; }

__device__ inline bool tie_skip(const DevState *st, int dyn) { return dyn && (st->halt || !st->tie_on); }
// Zig map final capacity for D live pairs (zig_order.hpp zig_final_capacity, on the device)
// Closed form, no loop and no division (a 64-bit division by 100 per doubling was ~1 us of one thread on
// a tied merge's critical path): floor(cap * 80 / 100) >= D  <=>  4 cap >= 5 D, so cap is the smallest power
// of two >= max(8, ceil(5 D / 4)); the max load equals D exactly iff 4 cap - 5 D < 5.
__device__ inline uint64_t dev_zig_cap_for(uint64_t D) {
    const uint64_t m = (5 * D + 3) / 4;
    return m <= 8 ? 8ull : 1ull << (64 - __builtin_clzll(m - 1));
}
__device__ inline bool dev_zig_at_max_load(uint64_t cap, uint64_t D) { return 4 * cap - 5 * D < 5; }
__device__ inline uint64_t dev_zig_final_capacity(uint64_t D, bool call_after) {
    const uint64_t cap = dev_zig_cap_for(D);
    return call_after && dev_zig_at_max_load(cap, D) ? 2 * cap : cap;
}
// Batch mode, start of merge X: can the device run this merge by itself? Every block of the first
// kernel of the merge evaluates the same predicate on the (read-only here) selection state; block 0
// records the outcome: the halt, or tie_on / cur_key and the merge log.
struct BeginArgs {
    uint32_t X;
    uint64_t home_cap;  // Zig capacity the home histogram is kept for
    uint32_t rec_cap;   // arena entries the halt test allows (records go at st->arena_top)
    MergeLog *log;
    int rep;            // sharded: test the replicated bound st->arena_rep (every rank halts alike)
    // a self pair (a, a) runs in the batch when a's list is shorter than self_lim (the host path's self_list_ok:
    // one GPU or replicas, valid lists); self_len: the list lengths, nullptr: every self pair halts
    const uint32_t *self_len;
    uint32_t self_lim;
};
__device__ inline uint32_t self_verdict(const BeginArgs &B, uint32_t key) {
    return B.self_len && B.self_len[key & 0xFFFF] < B.self_lim ? HALT_NONE : HALT_SELF;
}
__device__ inline uint32_t merge_begin_eval_v(const Tables &T, const FinishOut &f, const BeginArgs &B, bool *tie) {
    *tie = false;
    const int32_t live = f.live;
    const uint32_t hot_len = f.hot_len, top_count = f.top_count, tie_count = f.tie_count;
    const uint32_t arena_top = B.rep ? f.arena_rep : f.arena_top;
    const uint32_t lastpair = f.lastpair, key = f.key;
    if (live <= 0) return HALT_DONE;
    if (hot_len > T.hot_cap || top_count == 0) return HALT_SELECT;
    if ((uint64_t)arena_top + top_count > B.rec_cap) return HALT_RECORDS;
    if (tie_count > 1) {
        if (dev_zig_final_capacity((uint64_t)live, lastpair >= 2) != B.home_cap) return HALT_HOME;
        *tie = true;
        return HALT_NONE;
    }
    return (key & 0xFFFF) == (key >> 16) ? self_verdict(B, key) : HALT_NONE;
}
// the state words read, loaded together
__device__ inline FinishOut finish_state(const DevState *st) {
    FinishOut f;
    f.live = st->live;
    f.hot_len = st->hot_len;
    f.top_count = st->top_count;
    f.tie_count = st->tie_count;
    f.arena_top = st->arena_top;
    f.arena_rep = st->arena_rep;
    f.lastpair = st->lastpair_count;
    f.key = st->top_key;
    f.live_tokens = st->live_tokens;
    return f;
}
__device__ inline uint32_t merge_begin_eval(const Tables &T, const DevState *st, const BeginArgs &B, bool *tie) {
    return merge_begin_eval_v(T, finish_state(st), B, tie);
}
__device__ inline void merge_begin_commit_v(DevState *st, const BeginArgs &B, uint32_t h, bool tie, const FinishOut &f) {
    const uint32_t key = f.key, top_count = f.top_count, tie_count = f.tie_count;
    const long long live_tokens = f.live_tokens;
    st->cur_x = B.X;
    st->tie_on = tie ? 1u : 0u;
    if (h) {
        st->halt = h;
        st->halt_at = B.X;
    } else if (!tie) {
        st->cur_key = key;
        B.log[B.X - 256] = MergeLog{key, top_count, (uint32_t)live_tokens, tie_count};
    }
}
__device__ inline void merge_begin_commit(DevState *st, const BeginArgs &B, uint32_t h, bool tie) {
    merge_begin_commit_v(st, B, h, tie, finish_state(st));
}
__global__ void __launch_bounds__(256) zbpe_tie_collect(Tables T, DevState *st, uint32_t top, uint32_t cap_mask,
                                                        uint64_t *__restrict__ tie_list, uint32_t tie_cap, int dyn,
                                                        BeginArgs B) {
    if (dyn) {
        if (st->halt) return;
        bool tie;
        const uint32_t h = merge_begin_eval(T, st, B, &tie);
        __syncthreads();  // every thread has read the state before block 0 updates it
        if (blockIdx.x == 0 && threadIdx.x == 0) merge_begin_commit(st, B, h, tie);
        if (h || !tie) return;
        top = st->top_count;
    }
    const uint32_t n = min(st->hot_len, T.hot_cap);
    const uint32_t stride = gridDim.x * 256;
    for (uint32_t i0 = blockIdx.x * 256 + (threadIdx.x & ~63u); i0 < n; i0 += stride) {
        const uint32_t i = i0 + (threadIdx.x & 63);
        uint32_t id = NO_ID;
        bool tied = false;
        if (i < n) {
            id = (uint32_t)T.hot[i];
            tied = T.id_cnt[id] == top;
        }
        const uint32_t j = wave_append(&st->tie_len, tied);
        if (tied && j < tie_cap) {
            const uint32_t key = T.id_key[id];
            tie_list[j] = ((uint64_t)(zig_pair_hash(key) & cap_mask) << 32) | key;
        }
    }
}
// block summaries of the home histogram (block b covers slots [b*SUMM_SLOTS, ...)), every block
// (after a rebuild for a new capacity)
__global__ void __launch_bounds__(256) zbpe_home_summary(Tables T, DevState *st, uint32_t nslots, uint32_t nb,
                                                         Summ *__restrict__ out) {
    constexpr int PER = SUMM_SLOTS / 256;  // 16 slots = 4 words per thread
    __shared__ Summ sm[256];
    for (uint32_t blk = blockIdx.x; blk < nb; blk += gridDim.x) {
        const uint32_t beg = blk * SUMM_SLOTS + threadIdx.x * PER;
        Summ acc{0, 0};
        if (beg < nslots) {
            const uint32_t end = min(nslots, beg + PER);
            for (uint32_t s = beg; s < end; s += 4) {
                const uint32_t word = T.home_cnt[s >> 2];
                for (int k = 0; k < 4 && s + k < end; k++) acc = slot_fold(acc, ((word >> (8 * k)) & 0xffu));
            }
        }
        sm[threadIdx.x] = acc;
        __syncthreads();
        for (int sp = 1; sp < 256; sp <<= 1) {
            if ((threadIdx.x & (2 * sp - 1)) == 0) sm[threadIdx.x] = summ_cat(sm[threadIdx.x], sm[threadIdx.x + sp]);
            __syncthreads();
        }
        if (threadIdx.x == 0) out[blk] = sm[0];
        __syncthreads();
    }
}
// Refresh after merges: one workgroup per super-block (SUPER_BLOCKS = 64 blocks = two dirty-bitmap
// words). Each wave recomputes dirty blocks (a lane composes 64 slots read as four 16-B vectors,
// then an ordered wave reduction); wave 0 then recomposes the super-block. No cross-workgroup data.
constexpr int REFRESH_THREADS = 1024;
// one super-block (all threads of the block call it). wt: write-through (sc1) stores, for a reader
// in another workgroup of the same launch
__device__ inline uint64_t home_dirty_bits(const Tables &T, uint32_t sb) {
    static_assert(SUPER_BLOCKS == 64, "two dirty-bitmap words per super-block");
    const uint2 w = *reinterpret_cast<const uint2 *>(T.home_dirty + 2 * sb);
    return (uint64_t)w.x | ((uint64_t)w.y << 32);
}
__device__ inline void refresh_super(const Tables &T, uint32_t sb, uint32_t nslots, uint32_t nb, Summ *__restrict__ summ,
                                     Summ *__restrict__ sup, bool wt, uint64_t bits) {
    if (!bits) return;
    __shared__ Summ s_new[SUPER_BLOCKS];
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63, nwaves = blockDim.x >> 6;
    // wave 0: the clean blocks' summaries, loaded while the dirty ones are composed
    Summ old{0, 0};
    if (wave == 0 && sb * SUPER_BLOCKS + lane < nb && !((bits >> lane) & 1)) old = summ[sb * SUPER_BLOCKS + lane];
    const int ndirty = __popcll(bits);
    // two dirty blocks per wave per round, both blocks' slots loaded before either is folded (one
    // memory latency per round, not two)
    auto kth = [&](int k) -> uint32_t {  // index of the k-th set bit of `bits`
        uint64_t m = bits;
        for (int j = 0; j < k; j++) m &= m - 1;
        return (uint32_t)__builtin_ctzll(m);
    };
    auto load = [&](uint32_t blk, uint32_t (&w)[16]) {
        const uint32_t s0 = blk * SUMM_SLOTS + 64 * lane;
        if (s0 < nslots) {
            const uint4 *p = reinterpret_cast<const uint4 *>(T.home_cnt + s0 / 4);
#pragma unroll
            for (int v = 0; v < 4; v++) {
                const uint4 q = p[v];
                w[4 * v] = q.x; w[4 * v + 1] = q.y; w[4 * v + 2] = q.z; w[4 * v + 3] = q.w;
            }
        }
    };
    auto fold = [&](uint32_t blk, const uint32_t (&w)[16]) -> Summ {
        const uint32_t s0 = blk * SUMM_SLOTS + 64 * lane;
        Summ x{0, 0};
        if (s0 + 64 <= nslots) {
            x = fold64(w);
        } else if (s0 < nslots) {
#pragma unroll
            for (int kk = 0; kk < 64; kk++)
                if (s0 + kk < nslots) x = slot_fold(x, ((w[kk >> 2] >> (8 * (kk & 3))) & 0xffu));
        }
        return wave_reduce_summ(x);  // (the wave's loop is uniform: every lane active)
    };
    auto put = [&](uint32_t bi, Summ x) {
        const uint32_t blk = sb * SUPER_BLOCKS + bi;
        if (wt) {
            __hip_atomic_store(&summ[blk].q, x.q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&summ[blk].m, x.m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            summ[blk] = x;
        }
        s_new[bi] = x;
    };
    for (int k = wave; k < ndirty; k += 2 * nwaves) {
        const bool two = k + nwaves < ndirty;
        const uint32_t bi0 = kth(k), bi1 = two ? kth(k + nwaves) : bi0;
        uint32_t w0[16], w1[16];
        load(sb * SUPER_BLOCKS + bi0, w0);
        if (two) load(sb * SUPER_BLOCKS + bi1, w1);
        const Summ x0 = fold(sb * SUPER_BLOCKS + bi0, w0);
        if (lane == 0) put(bi0, x0);
        if (two) {
            const Summ x1 = fold(sb * SUPER_BLOCKS + bi1, w1);
            if (lane == 0) put(bi1, x1);
        }
    }
    __syncthreads();
    if (wave == 0) {
        const uint32_t bi = lane, blk = sb * SUPER_BLOCKS + bi;
        Summ x{0, 0};
        if (blk < nb) x = ((bits >> bi) & 1) ? s_new[bi] : old;
        x = wave_reduce_summ(x);
        if (lane == 0) {
            if (wt) {
                __hip_atomic_store(&sup[sb].q, x.q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&sup[sb].m, x.m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                sup[sb] = x;
            }
            T.home_dirty[2 * sb] = 0;
            T.home_dirty[2 * sb + 1] = 0;
        }
    }
    __syncthreads();
}
// Refresh after merges: one workgroup per super-block (SUPER_BLOCKS = 64 blocks = two dirty-bitmap
// words). Each wave recomputes dirty blocks (a lane composes 64 slots read as four 16-B vectors,
// then an ordered wave reduction); wave 0 then recomposes the super-block. No cross-workgroup data.
__global__ void __launch_bounds__(REFRESH_THREADS) zbpe_home_refresh(Tables T, DevState *st, uint32_t nslots, uint32_t nb,
                                                                     Summ *__restrict__ summ, Summ *__restrict__ sup,
                                                                     int dyn) {
    if (tie_skip(st, dyn)) return;
    refresh_super(T, blockIdx.x, nslots, nb, summ, sup, false, home_dirty_bits(T, blockIdx.x));
}
// super-block summaries: one wave composes SUPER_BLOCKS block summaries
__global__ void __launch_bounds__(256) zbpe_super_summary(const Summ *__restrict__ summ, uint32_t nb, Summ *__restrict__ sup,
                                                          const DevState *st, int dyn) {
    if (tie_skip(st, dyn)) return;
    const uint32_t nsb = (nb + SUPER_BLOCKS - 1) / SUPER_BLOCKS;
    const uint32_t w = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (w >= nsb) return;
    const uint32_t bi = w * SUPER_BLOCKS + lane;
    Summ x = bi < nb ? summ[bi] : Summ{0, 0};
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {  // ordered tree: lane i absorbs lane i+off
        Summ y;
        y.q = __shfl_down(x.q, off);
        y.m = __shfl_down(x.m, off);
        if ((lane & (2 * off - 1)) == 0) x = summ_cat(x, y);
    }
    if (lane == 0) sup[w] = x;
}
// ordered composition by one wave of f(i), i in [lo, hi) (each lane a contiguous chunk)
template <typename F>
__device__ inline Summ wave_compose(uint32_t lo, uint32_t hi, F f) {
    const uint32_t lane = threadIdx.x & 63;
    Summ x{0, 0};
    if (hi > lo) {
        const uint32_t per = (hi - lo + 63) / 64, b = lo + min(hi - lo, lane * per), e = min(hi, b + per);
        for (uint32_t i = b; i < e; i++) x = summ_cat(x, f(i));
    }
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        Summ y;
        y.q = __shfl_down(x.q, off);
        y.m = __shfl_down(x.m, off);
        if ((lane & (2 * off - 1)) == 0) x = summ_cat(x, y);
    }
    Summ r;
    r.q = __shfl(x.q, 0);
    r.m = __shfl(x.m, 0);
    return r;
}
// write-through (sc1) loads of bytes another workgroup of the same launch stored write-through and
// handed over through block_ticket_last: they bypass this CU's L1, so no acquire is needed
// (MI355X_MICROARCH.md, valid hand-off forms, first table row)
__device__ inline uint32_t ld_wt(const uint32_t *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ inline Summ ld_wt(const Summ *p) {
    const unsigned long long v = __hip_atomic_load(reinterpret_cast<const unsigned long long *>(p), __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
    return Summ{(int32_t)(uint32_t)v, (int32_t)(uint32_t)(v >> 32)};
}
// ordered composition by one wave of the slots [lo, hi) inside the summary block starting at
// `base`: lane L owns slots base + 64L .. +63 and reads them as four 16-B vectors (the histogram
// is allocated in whole 4096-slot blocks)
__device__ __attribute__((always_inline)) inline Summ wave_compose_slots(const uint32_t *hc, uint32_t base, uint32_t lo, uint32_t hi) {
    const uint32_t lane = threadIdx.x & 63, s0 = base + 64 * lane;
    Summ x{0, 0};
    if (hi > lo && s0 < hi && s0 + 64 > lo) {
        const uint4 *p = reinterpret_cast<const uint4 *>(hc + s0 / 4);
#pragma unroll
        for (int v = 0; v < 4; v++) {
            const uint4 w4 = p[v];
            const uint32_t w[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
            for (int k = 0; k < 16; k++) {
                const uint32_t s = s0 + 16 * v + k;
                if (s >= lo && s < hi) x = slot_fold(x, ((w[k >> 2] >> (8 * (k & 3))) & 0xffu));
            }
        }
    }
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        Summ y;
        y.q = __shfl_down(x.q, off);
        y.m = __shfl_down(x.m, off);
        if ((lane & (2 * off - 1)) == 0) x = summ_cat(x, y);
    }
    Summ r;
    r.q = __shfl(x.q, 0);
    r.m = __shfl(x.m, 0);
    return r;
}
// carry into slot s = m of the composition over slots s+1 .. s-1 (circular), by one wave: the
// slots after s in its block, the blocks after it in its super-block, the other super-blocks, the
// blocks before it in its super-block, the slots before s. Every load is issued before the first
// reduction (one memory latency, not five).
// w: on return, this lane's 64 slots of s's block (zeros past the map), for the caller's own use
// this lane's 64 slots (16 words of 4 one-byte home counts) folded in two parts around relative
// slot r: slots [0, r) into lo, slots (r, 64) into hi (r < 0: all in hi; r >= 64: all in lo).
// 32-bit and branch-free: q from byte sums of masked words (v_sad_u8), m by one slot_fold chain in
// slot order that hands its value to lo and restarts at r (no array of extracted bytes, which the
// compiler would spill)
__device__ __attribute__((always_inline)) inline void fold64_split(const uint32_t (&w)[16], int r, Summ &lo, Summ &hi) {
    uint32_t klo = 0, khi = 0;
    int32_t m = 0, mlo = 0;
#pragma unroll
    for (int j = 0; j < 16; j++) {
        const int nlo = min(max(r - 4 * j, 0), 4);          // bytes of word j before r
        const int nhi = min(max(4 * j + 3 - r, 0), 4);      // bytes of word j after r
        const uint32_t mask_lo = (uint32_t)((1ull << (8 * nlo)) - 1ull);
        const uint32_t mask_hi = (uint32_t)(0xFFFFFFFF00000000ull >> (8 * nhi));
        klo = __builtin_amdgcn_sad_u8(w[j] & mask_lo, 0u, klo);
        khi = __builtin_amdgcn_sad_u8(w[j] & mask_hi, 0u, khi);
#pragma unroll
        for (int bb = 0; bb < 4; bb++) {
            const int k = 4 * j + bb;
            const int32_t t = max(0, m + (int32_t)((w[j] >> (8 * bb)) & 0xffu) - 1);
            const bool at = k == r;
            mlo = at ? m : mlo;
            m = at ? 0 : t;
        }
    }
    const int32_t clo = min(max(r, 0), 64), chi = min(max(63 - r, 0), 64);
    if (r >= 64) mlo = m;
    lo = Summ{(int32_t)klo - clo, mlo};
    hi = Summ{(int32_t)khi - chi, r >= 64 ? 0 : m};
}
// carry into slot s = m of the composition over slots s+1 .. s-1 (circular), by one wave: the
// slots after s in its block, the blocks after it in its super-block, the other super-blocks, the
// blocks before it in its super-block, the slots before s. Every load is issued before the first
// reduction (one memory latency, not five).
// w: on return, this lane's 64 slots of s's block (zeros past the map), for the caller's own use
__device__ __attribute__((always_inline)) inline int32_t wave_carry_into(const HomeView &V, uint32_t s, uint32_t (&w)[16]) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t b = s / SUMM_SLOTS, sb = b / SUPER_BLOCKS, bbase = b * SUMM_SLOTS;
    const uint32_t s0 = bbase + 64 * lane, bend = min(V.C, bbase + SUMM_SLOTS);
    if (s0 < bend) {
        const uint4 *p = reinterpret_cast<const uint4 *>(V.hc + s0 / 4);
#pragma unroll
        for (int v = 0; v < 4; v++) {
            const uint4 q = p[v];
            w[4 * v] = q.x; w[4 * v + 1] = q.y; w[4 * v + 2] = q.z; w[4 * v + 3] = q.w;
        }
    } else {
#pragma unroll
        for (int k = 0; k < 16; k++) w[k] = 0;
    }
    const uint32_t bi = sb * SUPER_BLOCKS + lane;
    const Summ bs = bi < V.nb ? ld_wt(V.summ + bi) : Summ{0, 0};
    const uint32_t nsup = V.nsb - 1, per = (nsup + 63) / 64, i0 = min(nsup, lane * per), i1 = min(nsup, i0 + per);
    Summ x3{0, 0};
    if (per <= 8) {  // up to 512 super-blocks (C <= 2^27): every load issued at once
        Summ sv[8];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const uint32_t i = i0 + k;
            uint32_t j = sb + 1 + i;
            j = j >= V.nsb ? j - V.nsb : j;
            sv[k] = i < i1 ? ld_wt(V.sup + j) : Summ{0, 0};
        }
#pragma unroll
        for (int k = 0; k < 8; k++) x3 = summ_cat(x3, sv[k]);
    } else {
        for (uint32_t i = i0; i < i1; i++) x3 = summ_cat(x3, ld_wt(V.sup + (sb + 1 + i) % V.nsb));
    }
    Summ x1{0, 0}, x5{0, 0};
    if (bend - bbase == SUMM_SLOTS) {  // a whole block (every map of >= 4096 slots)
        fold64_split(w, (int)s - (int)s0, x5, x1);
    } else {  // a map of fewer than 4096 slots: slots past it are not folded
#pragma unroll
        for (int k = 0; k < 64; k++) {
            const uint32_t t = s0 + k;
            const uint32_t e = (w[k >> 2] >> (8 * (k & 3))) & 0xffu;
            if (t > s && t < bend) x1 = slot_fold(x1, e);
            if (t < s) x5 = slot_fold(x5, e);
        }
    }
    const Summ x2 = (bi > b && bi < V.nb) ? bs : Summ{0, 0};
    const Summ x4 = bi < b ? bs : Summ{0, 0};
    Summ x = wave_reduce_summ(x1);
    x = summ_cat(x, wave_reduce_summ(x2));
    x = summ_cat(x, wave_reduce_summ(x3));
    x = summ_cat(x, wave_reduce_summ(x4));
    x = summ_cat(x, wave_reduce_summ(x5));
    return x.m;
}
__device__ __attribute__((always_inline)) inline int32_t wave_carry_into(const HomeView &V, uint32_t s) {
    uint32_t w[16];
    return wave_carry_into(V, s, w);
}
// first free slot at or after h given the carry into h, by one wave, 64 slots per step; -1 when
// the run reaches slot C-1 (wraps) or is absurdly long
__device__ __attribute__((always_inline)) inline int64_t wave_first_free(const HomeView &V, uint32_t h, int32_t carry_in) {
    const uint32_t lane = threadIdx.x & 63;
    int32_t c = carry_in;
    for (uint32_t base = h; base < V.C && base - h <= (1u << 20); base += 64) {
        const uint32_t s = base + lane;
        const bool valid = s < V.C;
        const uint32_t k = valid ? home_at(V.hc, s) : 0u;
        // carry into slot s: composition of the slots [base, s) applied to c (exclusive scan)
        const Summ inc = summ_scan_dpp(summ_slot(k)), ex = summ_excl_dpp(inc);
        const int32_t cin = max(ex.m, c + ex.q);
        const uint64_t fr = __ballot(valid && cin + (int32_t)k == 0);
        if (fr) return (int64_t)base + __builtin_ctzll(fr);
        if (base + 64 >= V.C) return -1;
        const Summ t = summ_lane(inc, 63);
        c = max(t.m, c + t.q);
    }
    return -1;
}
// first free slot at or after h (-1 as wave_first_free), by one wave: wave_first_free re-reads the
// slots wave_carry_into has just read (L1 hits, not a second memory round trip)
__device__ __attribute__((always_inline)) inline int64_t wave_free_from(const HomeView &V, uint32_t h) {
    return wave_first_free(V, h, wave_carry_into(V, h));
}
// last free slot in [lo, hi) given the carry into lo, by one wave (-1 if none); lo is a multiple
// of 64 and hi - lo <= 4096: lane L owns slots lo + 64L .. +63, read once as four 16-B vectors
// this lane's 64 slots lo + 64L .. +63 of [lo, hi) as 16 words (zeros past hi's lane)
__device__ __attribute__((always_inline)) inline void wave_load_slots(const HomeView &V, uint32_t lo, uint32_t hi, uint32_t (&w)[16]) {
    const uint32_t lane = threadIdx.x & 63, s0 = lo + 64 * lane;
    if (s0 < hi) {
        const uint4 *p = reinterpret_cast<const uint4 *>(V.hc + s0 / 4);
#pragma unroll
        for (int v = 0; v < 4; v++) {
            const uint4 q = p[v];
            w[4 * v] = q.x; w[4 * v + 1] = q.y; w[4 * v + 2] = q.z; w[4 * v + 3] = q.w;
        }
    } else {
#pragma unroll
        for (int k = 0; k < 16; k++) w[k] = 0;
    }
}
__device__ __attribute__((always_inline)) inline int64_t wave_last_free_w(const uint32_t (&w)[16], uint32_t lo, uint32_t hi, int32_t carry_in);
__device__ __attribute__((always_inline)) inline int64_t wave_last_free(const HomeView &V, uint32_t lo, uint32_t hi, int32_t carry_in) {
    uint32_t w[16];
    wave_load_slots(V, lo, hi, w);
    return wave_last_free_w(w, lo, hi, carry_in);
}
// wave_last_free on slots already loaded (wave_load_slots)
__device__ __attribute__((always_inline)) inline int64_t wave_last_free_w(const uint32_t (&w)[16], uint32_t lo, uint32_t hi, int32_t carry_in) {
    const uint32_t lane = threadIdx.x & 63, s0 = lo + 64 * lane;
    // slots of this lane inside [lo, hi): all 64, none, or (a map of < 64 slots) a prefix
    const int nin = (int)min(64u, hi > s0 ? hi - s0 : 0u);
    Summ x{0, 0}, unused;
    if (nin == 64) x = fold64(w);
    else if (nin > 0) fold64_split(w, nin, x, unused);
    // exclusive ordered scan over lanes
    const Summ ex = summ_excl_dpp(summ_scan_dpp(x));
    int32_t c = max(ex.m, carry_in + ex.q);
    int32_t last = -1;
#pragma unroll
    for (int j = 0; j < 16; j++) {
#pragma unroll
        for (int bb = 0; bb < 4; bb++) {
            const int k = 4 * j + bb;
            const int32_t t = c + (int32_t)((w[j] >> (8 * bb)) & 0xffu);
            const bool ok = k < nin;
            last = ok && t == 0 ? (int32_t)(s0 + k) : last;
            c = ok ? max(0, t - 1) : c;
        }
    }
    return (int32_t)wave_max_u32((uint32_t)(last + 1)) - 1;  // (-1 or a slot below 2^31)
}
// sel_prof: add the ticks since *t to st->sel_prof[k] (one thread; fire-and-forget atomic)
__device__ inline void sel_tick(DevState *st, int k, unsigned long long *t) {
    const unsigned long long now = wall_clock64();
    atomicAdd(&st->sel_prof[k], now - *t);
    *t = now;
}
// carry into slot s from the carry into its super-block, cs[s / 2^18] (refresh_prefix): the
// blocks before s's block in its super-block, then the slots before s in its block; one load round
// trip, two wave reductions. The lanes also load the 64 slots after s (wave_first_free re-reads
// them from L1).
__device__ __attribute__((always_inline)) inline int32_t wave_carry_from_super(const HomeView &V, const uint32_t *cs, uint32_t s) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t b = s / SUMM_SLOTS, sb = b / SUPER_BLOCKS, s0 = b * SUMM_SLOTS + 64 * lane;
    uint32_t w[16];
    if (s0 < s + 64) {
        const uint4 *p = reinterpret_cast<const uint4 *>(V.hc + s0 / 4);
#pragma unroll
        for (int v = 0; v < 4; v++) {
            const uint4 q = p[v];
            w[4 * v] = q.x; w[4 * v + 1] = q.y; w[4 * v + 2] = q.z; w[4 * v + 3] = q.w;
        }
    } else {
#pragma unroll
        for (int k = 0; k < 16; k++) w[k] = 0;
    }
    const uint32_t bi = sb * SUPER_BLOCKS + lane;
    const Summ bs = bi < b ? ld_wt(V.summ + bi) : Summ{0, 0};
    const int32_t c_in = (int32_t)ld_wt(cs + sb);
    // slots [s0, s) of this lane: all 64 below s, a prefix in s's lane, none above (identity)
    const int r = (int)min((int64_t)s - (int64_t)s0, (int64_t)64);
    Summ xs, unused;
    fold64_split(w, r, xs, unused);
    const Summ x = summ_cat(wave_reduce_summ(bs), wave_reduce_summ(xs));
    return max(x.m, c_in + x.q);
}
__device__ inline void st_wt(uint32_t *p, uint32_t v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
// by the last home-refresh workgroup of a zbpe_select_next launch (every summary fresh), for the
// launch's tie decision: cs[k] = the carry into super-block k's first slot (cs[0] = the carry into
// slot 0), cs[nsb] = the last free slot of the map's last 4096 slots given the carry into them, or
// -2 when no run wraps past slot C-1 (cs[0] == 0). Needs nsb <= blockDim.x. Write-through stores.
__device__ inline void refresh_prefix(const HomeView &V, uint32_t *cs) {
    constexpr int MAXW = 16;
    __shared__ Summ s_tot[MAXW];
    __shared__ int32_t s_c0, s_clast;
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    // every load up front: the super summaries (all threads); the carry into slot 0 (wave 0); the
    // wrap test's last block and the block summaries before it in the last super-block (wave 1)
    const Summ S = tid < V.nsb ? ld_wt(V.sup + tid) : Summ{0, 0};
    const uint32_t kl = V.nsb - 1, ws = V.nb > 1 ? V.C - SUMM_SLOTS : 0u;
    uint32_t hw[16];
    Summ xl{0, 0};
    if (w == 1) {
        const uint32_t bi = kl * SUPER_BLOCKS + lane;
        const Summ bl = V.nb > 1 && bi < V.nb - 1 ? ld_wt(V.summ + bi) : Summ{0, 0};
        wave_load_slots(V, ws, V.C, hw);
        xl = wave_reduce_summ(bl);
    } else if (w == 0) {
        const int32_t c = wave_carry_into(V, 0u);
        if (lane == 0) s_c0 = c;
    }
    const Summ inc = summ_scan_dpp(S);  // inclusive ordered scan over the wave's super-blocks
    if (lane == 63) s_tot[w] = inc;
    __syncthreads();
    Summ pre{0, 0};
    for (uint32_t k = 0; k < w; k++) pre = summ_cat(pre, s_tot[k]);
    const Summ E = summ_cat(pre, summ_excl_dpp(inc));  // super-blocks [0, tid)
    const int32_t c0 = s_c0;
    const int32_t cin = max(E.m, c0 + E.q);
    if (tid < V.nsb) st_wt(cs + tid, (uint32_t)cin);
    if (tid == kl) s_clast = cin;
    __syncthreads();
    if (w == 1) {  // the carry into ws = C - 4096 (the last block), then the last free slot of [ws, C)
        const int32_t cw = V.nb > 1 ? max(xl.m, s_clast + xl.q) : c0;
        const int32_t lf = c0 > 0 ? (int32_t)wave_last_free_w(hw, ws, V.C, cw) : -2;
        if (lane == 0) st_wt(cs + V.nsb, (uint32_t)lf);
    }
}
constexpr int DECIDE_THREADS = 256;
// two smallest of two (smallest, second smallest) pairs
// Scan plan of the next merge (zbpe_select_next): what scan_dispatch would load first -- both tokens'
// list lengths and offsets, and the successor range of (a, b) in a's sorted list -- loaded by one lane
// of the select while its other waves work (the decision's carries), so the scan starts walking after
// one state round trip instead of three. Token xn (made by the merge this launch rolled) has its
// records as its list: offset xoff, length xlen (select_finish stores them in this launch).
// (a multi-merge round made xnum tokens xn, xn + 1, ..: token xn + i's list is at xoff + i * xlen, xlen long)
struct PlanCtx {
    const uint32_t *lst_off, *lst_len, *dir_row, *dir;
    uint32_t dir_w, lists_x, xn, xoff, xlen, xnum = 1;
    uint32_t xmask = 0;  // (a round that skipped members: token xn + i is member m_i, the i-th set bit; list at xoff + m_i * xlen)
    // (a round: member m >= 1's list is xcnt[m] long -- RoundHead::cnt, in LDS -- its count, below xlen in an untied round)
    const uint32_t *xcnt = nullptr;
};
// the member of a round's i-th merge (the i-th set bit of the mask; the identity without one)
__device__ inline uint32_t round_member(uint32_t mask, uint32_t i) {
    if (!mask) return i;
    uint32_t m = 0;
#pragma unroll
    for (uint32_t e = 0; e < (uint32_t)ROUND_MAX; e++) {
        if (mask >> e & 1u) {
            if (i == 0) m = e;
            i--;
        }
    }
    return m;
}
__device__ inline void plan_compute(const PlanCtx &P, uint32_t key, uint32_t *out) {
    const uint32_t a = key & 0xFFFF, b = key >> 16;
    uint32_t la = P.lst_len[a], lb = P.lst_len[b], oa = P.lst_off[a], ob = P.lst_off[b];
    const uint32_t ra = P.dir_row && a < P.lists_x && b < P.lists_x && b + 1 < P.dir_w ? P.dir_row[a] : NO_LIST;
    uint32_t r0 = NO_LIST, r1 = NO_LIST;
    if (ra != NO_LIST) {
        const uint64_t rb = (uint64_t)ra * P.dir_w + b;
        r0 = P.dir[rb];
        r1 = P.dir[rb + 1];
    }
    if (a - P.xn < P.xnum) {
        const uint32_t m = round_member(P.xmask, a - P.xn);
        la = P.xcnt && m ? P.xcnt[m] : P.xlen;
        oa = P.xoff + m * P.xlen;
    }
    if (b - P.xn < P.xnum) {
        const uint32_t m = round_member(P.xmask, b - P.xn);
        lb = P.xcnt && m ? P.xcnt[m] : P.xlen;
        ob = P.xoff + m * P.xlen;
    }
    out[0] = la; out[1] = lb; out[2] = oa; out[3] = ob; out[4] = r0; out[5] = r1;
}
// the plan of merge x1 = key (after the state's cur_key for it is stored; the next kernel boundary orders both)
__device__ inline void plan_store(DevState *st, uint32_t x1, uint32_t key, uint32_t gen, const uint32_t *pl) {
    st->plan_la = pl[0]; st->plan_lb = pl[1]; st->plan_oa = pl[2]; st->plan_ob = pl[3]; st->plan_r0 = pl[4]; st->plan_r1 = pl[5];
    st->plan_gen = gen;
    st->plan_key = key;
    st->plan_x = x1;
}
// Pair selects (DevState::pr_*): the three smallest entries of the tied-key list (home << 32 | key, unique)
// and the largest home, by one wave. Branch-free: the three smallest of two sorted triples a, b are
// min(a1, b1), min(max(a1, b1), a2, b2) and min(a3, b3, max(a2, b1), max(a1, b2)) (an if-chain per insert
// diverged across the lanes and cost ~3 us on the decision's critical path)
__device__ inline void min3_merge(uint64_t &a1, uint64_t &a2, uint64_t &a3, uint64_t b1, uint64_t b2, uint64_t b3) {
    const uint64_t r1 = min(a1, b1), r2 = min(max(a1, b1), min(a2, b2));
    const uint64_t r3 = min(min(a3, b3), min(max(a2, b1), max(a1, b2)));
    a1 = r1; a2 = r2; a3 = r3;
}
// the K smallest of two sorted K-tuples: r_k = min over i of max(a_i, b_{k-i}) (a_0 = b_0 = -inf)
template <int K>
__device__ inline void minK_merge(uint64_t (&a)[K], const uint64_t (&b)[K]) {
    uint64_t r[K];
#pragma unroll
    for (int k = 0; k < K; k++) {
        uint64_t v = min(a[k], b[k]);
#pragma unroll
        for (int i = 0; i < k; i++) v = min(v, max(a[i], b[k - 1 - i]));
        r[k] = v;
    }
#pragma unroll
    for (int k = 0; k < K; k++) a[k] = r[k];
}
// The K smallest of the wave (and the largest home) by DPP, every lane active: a butterfly inside each 16-lane row
// (quad_perm [1,0,3,2], [2,3,0,1], half-row mirror, row mirror -- each joins two disjoint halves, so no entry is
// merged twice), then the four rows' lists from v_readlane (wave-uniform results)
template <int CTRL>
__device__ __attribute__((always_inline)) inline uint64_t dpp_mov64(uint64_t x) {
    return (uint64_t)dpp_mov<CTRL>((uint32_t)x) | ((uint64_t)dpp_mov<CTRL>((uint32_t)(x >> 32)) << 32);
}
__device__ __attribute__((always_inline)) inline uint64_t lane_bcast64(uint64_t x, int l) {
    return (uint64_t)lane_bcast((uint32_t)x, l) | ((uint64_t)lane_bcast((uint32_t)(x >> 32), l) << 32);
}
template <int K, int CTRL>
__device__ __attribute__((always_inline)) inline void minK_dpp_step(uint64_t (&m)[K], uint32_t &hmax) {
    uint64_t b[K];
#pragma unroll
    for (int k = 0; k < K; k++) b[k] = dpp_mov64<CTRL>(m[k]);
    minK_merge<K>(m, b);
    hmax = max(hmax, dpp_mov<CTRL>(hmax));
}
template <int K>
__device__ __attribute__((always_inline)) inline void wave_minK_reduce_dpp(uint64_t (&m)[K], uint32_t &hmax) {
    minK_dpp_step<K, 0xB1>(m, hmax);
    minK_dpp_step<K, 0x4E>(m, hmax);
    minK_dpp_step<K, 0x141>(m, hmax);
    minK_dpp_step<K, 0x140>(m, hmax);
    uint64_t r[K];
    uint32_t h = lane_bcast(hmax, 0);
#pragma unroll
    for (int k = 0; k < K; k++) r[k] = lane_bcast64(m[k], 0);
#pragma unroll
    for (int l = 16; l < 64; l += 16) {
        uint64_t b[K];
#pragma unroll
        for (int k = 0; k < K; k++) b[k] = lane_bcast64(m[k], l);
        minK_merge<K>(r, b);
        h = max(h, lane_bcast(hmax, l));
    }
#pragma unroll
    for (int k = 0; k < K; k++) m[k] = r[k];
    hmax = h;
}
template <int K>
__device__ inline void wave_minK(const uint64_t *list, uint32_t len, uint64_t (&m)[K], uint32_t &hmax) {
    const uint32_t lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < K; k++) m[k] = ~0ull;
    hmax = 0;
    for (uint32_t i = lane; i < len; i += 64) {
        const uint64_t e = list[i];
        uint64_t b[K];
#pragma unroll
        for (int k = 0; k < K; k++) b[k] = k ? ~0ull : e;
        minK_merge<K>(m, b);
        hmax = max(hmax, (uint32_t)(e >> 32));
    }
    wave_minK_reduce_dpp<K>(m, hmax);  // (the caller's whole wave)
}
__device__ inline void wave_min3(const uint64_t *list, uint32_t len, uint64_t &m1, uint64_t &m2, uint64_t &m3, uint32_t &hmax) {
    const uint32_t lane = threadIdx.x & 63;
    m1 = m2 = m3 = ~0ull;
    hmax = 0;
    for (uint32_t i = lane; i < len; i += 64) {
        const uint64_t e = list[i];
        min3_merge(m1, m2, m3, e, ~0ull, ~0ull);
        hmax = max(hmax, (uint32_t)(e >> 32));
    }
    uint64_t q[3] = {m1, m2, m3};  // (minK_merge<3> is min3_merge's rule; the caller's whole wave)
    wave_minK_reduce_dpp<3>(q, hmax);
    m1 = q[0]; m2 = q[1]; m3 = q[2];
}
// keys whose home lies in the 4096-slot blocks covering [x, y) (0 <= x < y <= C, C >= one super-block):
// block summaries for the partial super-blocks at the two ends, super-block summaries between (one wave,
// one round trip; write-through loads). A summary's q is homes - slots.
__device__ __attribute__((always_inline)) inline int64_t wave_homes_cover(const HomeView &V, uint32_t x, uint32_t y) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t bx = x / SUMM_SLOTS, by = (y - 1) / SUMM_SLOTS, sx = bx / SUPER_BLOCKS, sy = by / SUPER_BLOCKS;
    int64_t h = 0;
    if (sx == sy) {
        const uint32_t b = bx + lane;
        if (b <= by) h += (int64_t)ld_wt(V.summ + b).q + SUMM_SLOTS;
    } else {
        const uint32_t b1 = bx + lane, b2 = sy * SUPER_BLOCKS + lane;
        if (b1 < (sx + 1) * SUPER_BLOCKS) h += (int64_t)ld_wt(V.summ + b1).q + SUMM_SLOTS;
        if (b2 <= by) h += (int64_t)ld_wt(V.summ + b2).q + SUMM_SLOTS;
        // the super-blocks between: up to 8 per lane with every load issued before the first use (a loop
        // with a run-time trip count waited for each load in turn); past 512 of them (C > 2^27) a loop
        constexpr int SB_U = 8;
        Summ sv[SB_U];
#pragma unroll
        for (int j = 0; j < SB_U; j++) {
            const uint32_t k = sx + 1 + lane + 64u * j;
            sv[j] = k < sy ? ld_wt(V.sup + k) : Summ{-(SUMM_SLOTS * SUPER_BLOCKS), 0};
        }
#pragma unroll
        for (int j = 0; j < SB_U; j++) h += (int64_t)sv[j].q + (int64_t)SUMM_SLOTS * SUPER_BLOCKS;
        for (uint32_t k = sx + 1 + lane + 64u * SB_U; k < sy; k += 64) h += (int64_t)ld_wt(V.sup + k).q + (int64_t)SUMM_SLOTS * SUPER_BLOCKS;
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) h += __shfl_xor(h, off);
    return h;
}
// Pair selects: the bound on the free Zig-map slots that keep merge X+1's candidate first, by one extra
// workgroup of merge X's replace, from the home summaries the decision saw (only the selects refresh them;
// the home counts this replace changes are not read). A range [x, y) has at least (y - x) - homes - carry(x)
// free slots (its keys came from homes in it or were carried in). The ranges start at the block after the
// candidate's home (free slots there end its run before the third-smallest home h3) and after the largest
// tied home's block (a free slot there: no tied key's run wraps past slot C-1). Four waves: the carry into
// each range (the super-block carry cs composed with the block summaries before it) and its homes.
// Mixed states: a refresh workgroup of a light launch may refresh some summaries after merge X
// changed the key set (S -> S - R + B) while cs is the decision's. The bound stays a lower bound for the set
// merge X+1 sees: carries and occupied slots are monotone in the key set, so cs (from S) >= the carries of
// S - R, and the mixed homes (S with some of R gone and some of B in) >= the homes of S - R; the bound is then
// <= the free slots of S - R. Every birth of merge X is compared against it (pr_births counts all of B, also
// those a refreshed summary already holds), and S - R + B has at least free(S - R) - |B| free slots.
__device__ __attribute__((always_inline)) inline int32_t wave_carry_block(const HomeView &V, const uint32_t *cs, uint32_t b) {
    const uint32_t lane = threadIdx.x & 63, sb = b / SUPER_BLOCKS, bi = sb * SUPER_BLOCKS + lane;
    const Summ bs = bi < b ? ld_wt(V.summ + bi) : Summ{0, 0};
    const int32_t c_in = (int32_t)ld_wt(cs + sb);
    const Summ x = wave_reduce_summ(bs);
    return max(x.m, c_in + x.q);
}
__device__ inline void pair_slack_block(DevState *st, const Summ *summ, const Summ *sup, uint32_t C, uint32_t nb,
                                        uint32_t nsb, const uint32_t *cs, uint32_t X, const uint32_t *lst_off,
                                        const uint32_t *lst_len, const uint32_t *dir_row, const uint32_t *dir,
                                        uint32_t dir_w, uint32_t lists_x, bool plan_on, uint32_t gen) {
    const HomeView V{nullptr, summ, sup, C, nb, nsb};
    __shared__ int64_t s_r[4];
    PairHead &ph = st->ph[(X + 1) & 1];  // merge X+1's candidate
    const uint32_t px = ph.x, slack = ph.slack, h2 = st->pr_h2, h3 = st->pr_h3, hmax = st->pr_hmax, key = ph.key;
    if (px != X + 1) return;
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    // the candidate's scan plan (its tokens existed before merge X: their lists are the ones the scan of
    // merge X+1 finds, unless the layout generation changes), by one lane beside the bound
    if (plan_on && threadIdx.x == 64) {
        const PlanCtx plan{lst_off, lst_len, dir_row, dir, dir_w, lists_x, NO_ID, 0u, 0u};
        uint32_t pl[6];
        plan_compute(plan, key, pl);
        for (int k = 0; k < 6; k++) st->pr_plan[k] = pl[k];
        ph.plan_gen = gen;
    }
    if (slack != 0 || !cs || V.C < (uint32_t)(SUMM_SLOTS * SUPER_BLOCKS)) return;
    const uint32_t x23 = (h2 / SUMM_SLOTS + 1) * SUMM_SLOTS, xe = (hmax / SUMM_SLOTS + 1) * SUMM_SLOTS;
    int64_t r = 0;
    if (w == 0) r = x23 < h3 ? wave_carry_block(V, cs, x23 / SUMM_SLOTS) : 0;
    else if (w == 1) r = x23 < h3 ? wave_homes_cover(V, x23, h3) : 0;
    else if (w == 2) r = xe < V.C ? wave_carry_block(V, cs, xe / SUMM_SLOTS) : 0;
    else if (w == 3) r = xe < V.C ? wave_homes_cover(V, xe, V.C) : 0;
    if (lane == 0 && w < 4) s_r[w] = r;
    __syncthreads();
    if (threadIdx.x) return;
    const int64_t f23 = x23 < h3 ? (int64_t)h3 - x23 - s_r[1] - s_r[0] : 0;
    const int64_t fe = xe < V.C ? (int64_t)V.C - xe - s_r[3] - s_r[2] : 0;
    const int64_t f = min(f23, fe);
    ph.slack = f <= 0 ? 0u : (uint32_t)min(f, (int64_t)0xFFFFFFFEll);
}
__device__ inline void min2_combine(uint64_t &m1, uint64_t &m2, uint64_t b1, uint64_t b2) {
    const uint64_t a1 = m1, a2 = m2;
    m1 = min(a1, b1);
    m2 = min(max(a1, b1), min(a2, b2));
}
// Zig-order decision over the tied keys `list` (home << 32 | key; `len` of `total` collected: a
// shortfall decides nothing). NT threads (>= 192: three waves compute carries). dyn: batch mode
// (halt / commit).
template <int NT = DECIDE_THREADS>
__device__ __attribute__((always_inline)) inline void decide_body(DevState *st, const uint64_t *list, uint32_t len, uint32_t total, const HomeView &V,
                                   MergeLog *log, int dyn, unsigned long long *prof_t = nullptr,
                                   const uint32_t *cs = nullptr, bool plan_on = false, const PlanCtx &plan = PlanCtx{},
                                   uint32_t plan_gen = 0, uint32_t pair_x = 0, bool m3_w4 = false,
                                   bool chain = false, bool chain2 = false, bool chain3 = false, bool rplan = false,
                                   const BeginArgs *self_b = nullptr) {
    static_assert(NT >= 192 && NT % 64 == 0, "three waves");
    // plan (NT >= 256): wave 3 finds the smallest home's key itself and loads its scan plan during the
    // carries; the commit below stores it with cur_key
    __shared__ uint32_t s_plan[6];
    // three waves at once, one barrier: wave 0 reduces the tied keys (the two smallest home << 32 |
    // key, the largest home) and finds the end of the smallest home's run; wave 1 the carry into
    // slot 0; wave 2 the last free slot of the map's last 4096 slots (where a run wrapping past
    // slot C-1 would start)
    __shared__ long long s_c0, s_last, s_free;
    __shared__ uint64_t s_m1, s_m2;
    __shared__ uint32_t s_hmax;
    const int w = threadIdx.x >> 6;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t ws = V.C > 4096 ? V.C - 4096 : 0;
    __shared__ uint64_t s_m3, s_m4, s_m5, s_m6;
    if (w == 0) {
        uint64_t m1 = ~0ull, m2 = ~0ull, m3 = ~0ull;
        uint32_t hmax = 0;
        if (NT >= 512 && pair_x && !m3_w4) {
            wave_min3(list, len, m1, m2, m3, hmax);
        } else {
            for (uint32_t i = lane; i < len; i += 64) {
                const uint64_t e = list[i];
                if (e < m1) { m2 = m1; m1 = e; } else if (e < m2) m2 = e;
                hmax = max(hmax, (uint32_t)(e >> 32));
            }
            uint64_t q[2] = {m1, m2};  // (minK_merge<2> is min2_combine's rule; wave 0 whole)
            wave_minK_reduce_dpp<2>(q, hmax);
            m1 = q[0];
            m2 = q[1];
        }
        if (lane == 0 && !(NT >= 512 && pair_x && m3_w4)) { s_m3 = m3; s_m4 = ~0ull; s_m5 = ~0ull; s_m6 = ~0ull; }
        const uint32_t h1 = (uint32_t)(m1 >> 32);
        const int64_t f = !len ? -1 : cs ? wave_first_free(V, h1, wave_carry_from_super(V, cs, h1)) : wave_free_from(V, h1);
        if (lane == 0) { s_free = f; s_m1 = m1; s_m2 = m2; s_hmax = hmax; }
    } else if (cs) {  // carry into slot 0 and the wrap test's last free slot: precomputed (refresh_prefix)
        if (w == 1 && lane == 0) {
            s_c0 = (int32_t)ld_wt(cs);
            s_last = (int32_t)ld_wt(cs + V.nsb);
        }
    } else if (w == 1) {
        const int64_t c = wave_carry_into(V, 0);
        if (lane == 0) s_c0 = c;
    } else if (w == 2 && ws) {
        const int64_t lf = wave_last_free(V, ws, V.C, wave_carry_into(V, ws));
        if (lane == 0) s_last = lf;
    }
    // pair_x (merge X+1 = pair_x, NT >= 512, precomputed carries): the second-smallest home's key is merge
    // X+1's candidate; wave 0 also finds the third-smallest home (merge X's replace bounds the free slots
    // between them and loads the candidate's scan plan: pair_slack_block)
    const bool pair_on = NT >= 512 && pair_x && cs && len >= 2;
    if (NT >= 512 && pair_x && m3_w4 && w == 4) {  // (option pair_m3w: the third- and fourth-smallest by a wave of its own)
        uint64_t q[6];
        uint32_t hmx;
        wave_minK<6>(list, len, q, hmx);
        if (lane == 0) { s_m3 = q[2]; s_m4 = q[3]; s_m5 = q[4]; s_m6 = q[5]; }
    }
    if (NT >= 256 && plan_on && w == 3 && len) {
        uint64_t m1 = ~0ull;
        for (uint32_t i = lane; i < len; i += 64) m1 = min(m1, list[i]);
        uint64_t q[1] = {m1};
        uint32_t hx = 0;
        wave_minK_reduce_dpp<1>(q, hx);  // (wave 3 whole)
        m1 = q[0];
        if (lane == 0) plan_compute(plan, (uint32_t)m1, s_plan);
    }
    // rplan (a multi-merge round's select): wave 5 finds the next tied keys by home itself and loads their scan
    // plans, one lane each, beside the carries (the round's scan then walks them without a plan round trip)
    if (NT >= 512 && rplan && plan_on && w == 5 && len >= 2) {
        uint64_t q[ROUND_MAX];
        uint32_t hmx;
        wave_minK<ROUND_MAX>(list, len, q, hmx);
        if (lane >= 1 && lane < (uint32_t)ROUND_MAX && q[lane] != ~0ull) {
            const uint32_t key = (uint32_t)q[lane];
            uint32_t pl[6];
            plan_compute(plan, key, pl);
#pragma unroll
            for (int k = 0; k < 6; k++) st->rp.plan[lane - 1][k] = pl[k];
            st->rp.key[lane - 1] = key;
        }
        if (lane == 0) st->rp.gen = plan_gen;
    }
    __syncthreads();
    if (!ws && !cs) {  // a map of at most 4096 slots: the last free slot needs the carry into slot 0
        if (w == 2) {
            const int64_t lf = s_c0 > 0 ? wave_last_free(V, 0, V.C, s_c0) : -2;
            if (lane == 0) s_last = lf;
        }
        __syncthreads();
    }
    const uint64_t m1 = s_m1, m2 = s_m2;
    const uint32_t hmax = s_hmax;
    if (threadIdx.x) return;
    if (prof_t) sel_tick(st, 9, prof_t);  // the three waves' carries
    uint32_t verdict = total > len ? 1u : 0u;
    const int64_t s = s_free;  // first free slot at or after h1
    if (s < 0) verdict = 1;     // the run of h1 wraps (or is absurdly long)
    if (m2 != ~0ull && s > (int64_t)(m2 >> 32)) verdict = 1;  // second tied pair in the same run
    const long long lf = s_c0 > 0 ? s_last : -2;  // -2: no run wraps past slot C-1
    if (lf != -2 && (lf < 0 || (long long)hmax >= lf + 1)) verdict = 1;  // a tied pair may have wrapped
    st->tie_verdict = verdict;
    st->tie_winner = (uint32_t)m1;
    if (dyn) {
        if (total != st->tie_count) atomicOr(&st->error, 128u);
        const uint32_t key = (uint32_t)m1;
        if (verdict) {
            st->halt = HALT_TIE;
            st->halt_at = st->cur_x;
        } else if ((key & 0xFFFF) == (key >> 16) && (!self_b || self_verdict(*self_b, key) != HALT_NONE)) {
            st->halt = HALT_SELF;
            st->halt_at = st->cur_x;
        } else {
            st->cur_key = key;
            log[st->cur_x - 256] = MergeLog{key, st->top_count, (uint32_t)st->live_tokens, st->tie_count};
            if (NT >= 256 && plan_on && len) plan_store(st, st->cur_x, key, plan_gen, s_plan);
            // merge X+1's pair-select candidate: the second-smallest home's key (not a self pair)
            const uint32_t k2 = (uint32_t)m2;
            if (pair_on && m2 != ~0ull && (k2 & 0xFFFF) != (k2 >> 16) && total == len &&
                (len == 2 || V.C >= (uint32_t)(SUMM_SLOTS * SUPER_BLOCKS))) {
                // two tied pairs: the candidate is the only one left (no bound needed); else 0 until merge
                // X's replace has bounded the free slots (pair_slack_block)
                PairHead &ph = st->ph[pair_x & 1];  // (merge pair_x's slot: not the one this launch's light test read)
                ph.slack = len == 2 ? 0xFFFFFFFFu : 0u;
                st->pr_h2 = (uint32_t)(m2 >> 32);
                st->pr_h3 = len >= 3 ? (uint32_t)(s_m3 >> 32) : 0u;
                st->pr_h4 = len >= 4 && s_m4 != ~0ull ? (uint32_t)(s_m4 >> 32) : 0u;
                st->pr_h5 = len >= 5 && s_m5 != ~0ull ? (uint32_t)(s_m5 >> 32) : 0u;
                st->pr_h6 = len >= 6 && s_m6 != ~0ull ? (uint32_t)(s_m6 >> 32) : 0u;
                st->pr_hmax = hmax;
                // chain: the third-smallest home's key for merge X+2 (found with the fourth, wave 4)
                const uint32_t k3 = (uint32_t)s_m3;
                const bool c2 = chain && m3_w4 && len >= 3 && s_m3 != ~0ull && (k3 & 0xFFFF) != (k3 >> 16) &&
                                (len == 3 || s_m4 != ~0ull);
                st->pr_key2 = c2 ? k3 : NO_ID;
                // chain depth 2 (option pair_chain 2): the fourth key, merge X+3's candidate
                const uint32_t k4 = (uint32_t)s_m4;
                const bool c3 = c2 && chain2 && len >= 4 && s_m4 != ~0ull && (k4 & 0xFFFF) != (k4 >> 16) && (len == 4 || s_m5 != ~0ull);
                st->pr_key3 = c3 ? k4 : NO_ID;
                // depth 3 (option pair_chain 3): the fifth key, merge X+4's
                const uint32_t k5 = (uint32_t)s_m5;
                st->pr_key4 = c3 && chain3 && len >= 5 && s_m5 != ~0ull && (k5 & 0xFFFF) != (k5 >> 16) && (len == 5 || s_m6 != ~0ull)
                                  ? k5 : NO_ID;
                ph.plan_gen = 0xFFFFFFFFu;  // (the replace's extra workgroup loads the plan)
                ph.births = 0;
                ph.dt = 0;
                ph.key = k2;
                ph.ties = total;
                ph.x = pair_x;
                st->pr_full = pair_x;
            }
        }
    }
}
__global__ void __launch_bounds__(DECIDE_THREADS) zbpe_tie_decide(DevState *st, const uint64_t *__restrict__ tie_list,
                                                                  uint32_t tie_cap, HomeView V, MergeLog *log, int dyn) {
    if (tie_skip(st, dyn)) return;
    const uint32_t total = st->tie_len;
    decide_body<DECIDE_THREADS>(st, tie_list, min(total, tie_cap), total, V, log, dyn);
}

// ------------------------------------------------------------------------------------------
// Fused end of merge X + start of merge X+1 (batch mode): one launch instead of select, collect,
// refresh and decide. Two roles, each with its own arrival count:
//   - blocks [0, nref) (nref = home super-blocks, 0 without a home histogram) refresh one dirty home
//     super-block each and clear merge X's deltas for merge X + 2; they arrive on eight per-XCD
//     counters (N.rtk, parity X & 1; block_ticket_last_x). When merge X was tied (log[X].ties > 1: ties
//     come in streaks) the arrivals are returning and elect the last refresh workgroup, which
//     precomputes the tie decision's carries (refresh_prefix into N.cs) unless the argmax side has
//     already stored st->ref_noprefix = X (merge X + 1 needs no decision), then arrives once more on the
//     top counter.
//   - blocks [nref, nref + sel_blocks) run the hot-list argmax and keep the keys at their block's max;
//     the last of them through the launch parity's ticket (N.rtk counter 9; block_ticket_last: write-through
//     partials, no fences)
//     reduces, rolls merge X, evaluates the start of merge X + 1 and, on a tie, gathers the tied keys
//     and takes the Zig-order decision in this launch (decide_body). Before deciding it spin-waits for
//     the refresh arrivals (and, with precomputed carries, for the prefix's final arrival).
// The wait only makes progress because the refresh workgroups -- lower workgroup ids -- are
// dispatched before the argmax workgroups and never wait on them: the GPU dispatches a grid's
// workgroups in id order, so every refresh workgroup is resident or finished by the time the last
// argmax workgroup spins. The grid is sized (launch bounds: 4 waves per SIMD) so that every workgroup
// fits one dispatch round.
// ------------------------------------------------------------------------------------------
// The roll of a multi-merge round (the last argmax workgroup's thread 0, after select_finish without its roll):
// every member's records become its new token's list (member j's at arena_top + j T, cnt[j] of them), the stream
// and arena counters advance by all of them, the members' merge-log rows get their pairs, counts, live tokens
// and tie counts (tied: member j's tied set is member j-1's less member j-1 and the tied pairs member j-1
// decremented first, RoundHead::dec; untied: 1), and the round's words are cleared for the next round's scan.
__device__ inline void round_roll(const Tables &T, DevState *st, const StateHead &H0, MergeLog *log, const uint32_t *pre,
                                  FinishOut *fo, uint32_t *rlog) {
    const uint32_t k = H0.rd_v, X0 = H0.cur_x, Tc = H0.top_count, mask = H0.rd_mask;
    RoundHead &R = st->rd;
    // the RoundHead words, preloaded into LDS at the kernel's entry (roll_preload rd)
    const RoundHead &RP = *reinterpret_cast<const RoundHead *>(pre + RI_WORDS);
    uint32_t rec[ROUND_MAX], key[ROUND_MAX], dec[ROUND_MAX], cnt[ROUND_MAX];
#pragma unroll
    for (int j = 0; j < ROUND_MAX; j++) {
        rec[j] = RP.rec[j];
        key[j] = RP.key[j];
        dec[j] = RP.dec[j];
        cnt[j] = RP.cnt[j];
    }
    rec[0] = pre[RI_REC];
    cnt[0] = Tc;
    const bool untied = RP.ties0 == 1;
    const uint32_t holes = pre[RI_HOLES], arena_top = pre[RI_ARENA_TOP], arena_rep = pre[RI_ARENA_REP], total_occ = pre[RI_TOTAL_OCC];
    const long long live_tokens = (long long)(((uint64_t)pre[RI_LIVE_TOK_HI] << 32) | pre[RI_LIVE_TOK_LO]);
    // merge X0 + x is member m (the x-th set bit of mask); member m's records are at arena_top + m Tc
    uint32_t ties = RP.ties0, sum = 0, x = 0, prev = 0, last = 0;
    long long gone = 0;  // tokens the merged members before this one removed (one per occurrence)
#pragma unroll
    for (uint32_t m = 0; m < (uint32_t)ROUND_MAX; m++) {
        if (!(mask >> m & 1u)) continue;
        if (T.lst_off) {
            T.lst_off[X0 + x] = arena_top + m * Tc;
            T.lst_len[X0 + x] = rec[m];
        }
        if (x) {  // (the whole row: d_log is not cleared between trains)
            ties = untied ? 1u : ties - 1u - dec[prev];
            log[X0 + x - 256] = MergeLog{key[m], cnt[m], (uint32_t)(live_tokens - gone), ties, 1u, rec[m], 0u, 0u};
        }
        gone += cnt[m];
        sum += rec[m];
        prev = last = m;
        x++;
    }
    (void)k;
    const uint32_t top = arena_top + last * Tc + rec[last];
    if (T.lst_off) st->arena_top = top;
    st->last_occ = sum;
    st->total_occ = total_occ + sum;
    st->last_gocc = sum;
    st->arena_rep = arena_rep + sum;
    st->last_holes = holes;
    st->live_tokens = live_tokens - holes;
    st->tie_len = 0;
    st->holes_made = 0;
    st->rec_count = 0;
#pragma unroll
    for (int j = 0; j < ROUND_MAX; j++) {
        R.touch[j] = 0; R.top[j] = 0; R.birth[j] = 0; R.rec[j] = 0; R.dec[j] = 0; R.nmax[j] = 0;
    }
    uint32_t anyj = 0;
#pragma unroll
    for (int j = 0; j < ROUND_MAX; j++) anyj |= RP.top[j] & RT_JUNCTION;
    if (anyj) {
        uint4 *jw = reinterpret_cast<uint4 *>(&st->rd_jn[0]);
#pragma unroll
        for (int w = 0; w < 16; w++) jw[w] = make_uint4(0, 0, 0, 0);
    }
    st->rd_v = 0;
    st->rd_merges += k - 1;
    fo->arena_top = T.lst_off ? top : arena_top;
    fo->arena_rep = arena_rep + sum;
    fo->live_tokens = live_tokens - holes;
    *rlog = X0 | (k << 16);
}
constexpr int NEXT_THREADS = 512;  // launch bounds: 4 waves per SIMD (two workgroups per CU; the decision spills a little)
constexpr int NEXT_CAND = 64;          // keys kept per argmax block at the block's max
constexpr int NEXT_MAX_SEL = 1024;     // argmax blocks (the reducer keeps one LDS entry per block)
constexpr int SEL_U = 8;               // hot entries per argmax thread per step (loads issued together)
constexpr int NEXT_TIE_LDS = 512;      // tied keys the decision reads from LDS (more: from N.tie_list)
// bounded spin-waits: 1 s of wall_clock64 (100 MHz). Only a guard against a broken dispatch-order assumption, not a
// performance limit: a queue time-sliced away (several processes on one GPU) can stall a wait for many ms
constexpr unsigned long long SPIN_LIMIT_TICKS = 100000000ull;
struct NextArgs {
    BeginArgs B;          // merge X + 1 (B.X < x_end)
    uint32_t x_end;       // vocab size: no merge starts at x_end
    HomeView V;           // V.C == 0: no home histogram, no refresh blocks
    uint64_t *tie_list;
    uint32_t tie_cap;
    uint32_t sel_blocks;
    uint32_t *cand;       // [sel_blocks][NEXT_CAND]
    uint32_t *pkey;       // [sel_blocks] key of the block's max when it is unique
    uint32_t *lastpair;   // [1] count of the stream's last pair (one GPU)
    const Boundary *bnd;  // multi-GPU: boundary records (the stream's last pair on ties)
    int world;
    int prof;             // option sel_prof: accumulate phase times into st->sel_prof
    uint32_t *cs;         // [nsb + 1] refresh_prefix's carries (nullptr: the decision computes them; nsb > NEXT_THREADS)
    uint32_t *rtk;        // [RTK_WORDS] refresh arrival counters
    // the next merge's scan plan (DevState::plan_*): the scan's successor directory (ScanArgs::dir_row,
    // dir, dir_w; dir_row nullptr: no ranges) and the host's layout generation; plan 0: none
    const uint32_t *dir_row, *dir;
    uint32_t dir_w, gen;
    int plan;
    // option lp_lazy: the stream's last pair count (the Zig map's final grow) is looked up by the last block
    // only for a tie whose capacity depends on it, not by argmax wave 1 at every merge (its dependent loads
    // held the argmax block's max behind them)
    int lp_lazy;
    int pair;             // option pair_select (DevState::pr_*)
    int skip_refresh;     // option pair_refresh 0: a pair select's refresh workgroups leave the dirty blocks to the next launch
    int m3_w4;            // option pair_m3w: the decision's third-smallest home by wave 4 (else wave 0)
    int chain;            // option pair_chain: a pair select names merge X+2's candidate (needs skip_refresh, m3_w4); 2: and X+3's; 3: X+4's
    // multi-merge rounds (option round_k; batch mode, one GPU or replicas): `round` member slots. The merges this
    // launch rolls are the state's (cur_x .. cur_x + rd_v - 1; the kernel's X is the host's bound on them, for the
    // clearing of the members' delta buffers `delta`, fixed layout); no pair selects (every select is a full
    // one). par: the refresh counters' parity (launch order); seq: a launch id (ref_noprefix); rlog[rlog_i] =
    // the round's first merge | its members << 16.
    int round;
    uint32_t par, seq, rlog_i;
    uint32_t *rlog;
    int untied;           // option round_untied: a round's select that begins an untied merge names the next distinct counts' pairs
};
// every thread of the block calls it after its last global store of the phase; true in the last block.
// Every byte the last block reads from another workgroup was stored write-through (sc1: agent-scope
// relaxed atomic stores) and is drained here, so no release fence (an L2 writeback, 1.7-6.5 us on
// the critical path) is needed; the last block reads those bytes with sc1 loads (ld_wt), which
// bypass its CU's L1, so no acquire either (MI355X_MICROARCH.md, valid hand-off forms: one lane of
// each storing workgroup adds to one counter after the workgroup's vmcnt(0) and barrier; the
// workgroup whose add came last loads after its add has returned, its other waves after a barrier)
// pair selects: does this launch start merge X+1 with the candidate (the conditions at the light path in
// zbpe_select_next)? Both roles evaluate it on the same words: the refresh workgroups then leave the dirty
// home blocks to the next launch, whose decision reads them.
// Invariant (single-sourced verdict): every workgroup of the launch evaluates it on merge X+1's PairHead slot
// (DevState::ph[x1 & 1]) and DevState::live, and no kernel writes either while the launch runs -- the committing
// block writes the chain and a decision's candidate into merge X+2's slot, and the select writes no pair count --
// so a workgroup that starts after the committing block has moved on to merge X+2 still gets the launch's verdict.
// (scalar arguments: a reference to the kernel's NextArgs made the compiler copy all of it to scratch at entry)
__device__ inline bool pair_light(int pair, uint32_t x1, uint32_t x_end, uint32_t C, const PairHead &P0, int32_t live0) {
    if (!pair || P0.x != x1 || x1 >= x_end) return false;
    const uint32_t dT = P0.dt & 0xFFFFu, kc = P0.key;
    const uint64_t D1 = (uint64_t)max(live0, 0);
    return ((P0.dt >> 16) & 7u) == 0 && P0.births < P0.slack && dT + 1 < P0.ties && C && dev_zig_cap_for(D1) == C &&
           !dev_zig_at_max_load(C, D1) && (kc & 0xFFFF) != (kc >> 16);
}
__device__ inline bool block_ticket_last(uint32_t *ticket, uint32_t nblocks, uint32_t *s_flag) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *s_flag = t == nblocks - 1 ? 1u : 0u;
    }
    __syncthreads();
    return *s_flag != 0;
}
// block_ticket_last for many arrivals: workgroups [0, nblocks) count on eight per-XCD counters
// (workgroup i in i % 8: the dispatcher's XCD round robin), the last of each group on the top one
// (ctr: RTK_SET words; a single counter saturates at ~11-13 ns per arrival, MI355X_MICROARCH.md fanin)
__device__ inline bool block_ticket_last_x(uint32_t *ctr, uint32_t nblocks, uint32_t *s_flag) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t g = blockIdx.x & 7, gsize = (nblocks - g + 7) / 8, ngroups = min(nblocks, 8u);
        uint32_t last = 0;
        if (__hip_atomic_fetch_add(ctr + g * RTK_STRIDE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gsize - 1)
            last = __hip_atomic_fetch_add(ctr + 8 * RTK_STRIDE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ngroups - 1;
        *s_flag = last;
    }
    __syncthreads();
    return *s_flag != 0;
}
__device__ __attribute__((always_inline)) inline MaxRec block_max(MaxRec r, MaxRec *sm) {  // (every thread of the block)
    r = wave_max_dpp(r);
    if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = r;
    __syncthreads();
    MaxRec q = sm[0];
    for (uint32_t w = 1; w < blockDim.x / 64; w++) q = max_combine(q, sm[w]);
    __syncthreads();
    return q;
}
// The leading scalar arguments (kernarg-preloaded: in SGPRs at entry) are what the first loads need -- the
// state, the hot list and its capacity, the role split (nref = the refresh workgroups), the argmax grid
// and the stream's tail -- so those loads issue at entry, before any kernarg round trip.
__global__ void __launch_bounds__(NEXT_THREADS, 4) zbpe_select_next(DevState *st, const unsigned long long *__restrict__ hot,
                                                                 const uint32_t *__restrict__ hcnt,
                                                                 uint32_t hot_cap, uint32_t nref_arg, uint32_t sel_blocks,
                                                                 const uint16_t *__restrict__ tok, int64_t n, Tables T,
                                                                 MaxRec *__restrict__ partial, uint32_t *delta, uint32_t X,
                                                                 NextArgs N) {
    // blocks [0, nref) refresh the home super-blocks (the longest role: dispatched first, one
    // workgroup per CU at this kernel's VGPR count), blocks [nref, nref + sel_blocks) run the argmax
    const uint32_t nref = nref_arg;  // N.V.C ? min(N.V.nsb, refresh_wgs) : 0
    const uint32_t tid = threadIdx.x;
    if (blockIdx.x < nref) {
        const unsigned long long t_ref0 = N.prof ? wall_clock64() : 0ull;
        // refresh role, off the argmax's ticket: the last argmax block reduces, rolls and starts
        // merge X+1 while these blocks work, and waits for their arrivals only before a tie
        // decision. They run even after a halt (a halted batch dirties no blocks; a refresh is
        // always valid), so that every launch's arrivals reach nref.
        // pfx: the decision's carries are precomputed when merge X was tied (ties come in streaks: the
        // last quarter of C4 is 94 % tied), a predicate the decision reads alike (merge X's log entry,
        // written by the launch before); then the last workgroup to arrive is elected (returning
        // atomics, per-XCD counters, then the top one) and arrives once more when done. Else a
        // workgroup's arrival is one non-returning add to its XCD's counter.
        // (rounds: always, see below)
        // (rounds: always -- a round's merges are mostly tied, and the carries are what lets the next decision
        // name a round's keys; a round of one with an untied merge skipping them ended the naming, measured)
        const bool pfx = N.cs && (N.round ? true : N.B.log[X - 256].ties > 1);
        // merge X's neighbour deltas, cleared for merge X + 2 by these workgroups (off the argmax's
        // critical path: the argmax grid is sized by the hot list alone; nothing in this launch reads
        // [0, 2X) -- the roll reads the tail words past it)
        if (N.round) {  // every member buffer: left [0, X), right [65536, 65536 + X), the tail's two words
            const uint32_t per = 2 * X + 2;
            for (uint32_t t = blockIdx.x * NEXT_THREADS + tid; t < (uint32_t)N.round * per; t += nref * NEXT_THREADS) {
                const uint32_t m = t / per, o = t - m * per;
                delta[(size_t)m * (2 * 65536 + 64) + (o < X ? o : o < 2 * X ? 65536 + (o - X) : 2 * 65536 + (o - 2 * X))] = 0;
            }
        } else {
            for (uint32_t t = blockIdx.x * NEXT_THREADS + tid; t < 2 * X; t += nref * NEXT_THREADS) delta[t] = 0;
        }
        if (N.pair && N.skip_refresh && !N.round) {  // a pair select: no decision in this launch reads the summaries
            const PairHead P0 = st->ph[N.B.X & 1];  // (merge X+1's slot: no workgroup of this launch writes it)
            if (pair_light(N.pair, N.B.X, N.x_end, N.V.C, P0, st->live)) return;
        }
        // nref may be below the super-block count (option refresh_wgs): a smaller grid ends sooner -- a kernel
        // boundary after 256 workgroups costs ~3.7 us, after 64 ~1.6 (tools/launch_lat.hip, boundary rows)
        for (uint32_t sb = blockIdx.x; sb < N.V.nsb; sb += nref) {
            refresh_super(T, sb, N.V.C, N.V.nb, const_cast<Summ *>(N.V.summ), const_cast<Summ *>(N.V.sup), true,
                          home_dirty_bits(T, sb));
            if (nref < N.V.nsb) __syncthreads();  // (refresh_super's LDS summaries are reused by the next one)
        }
        if (N.prof && tid == 0) {
            const unsigned long long t_ref1 = wall_clock64();
            atomicMax(&st->sel_tr, t_ref1);
            atomicAdd(&st->sel_prof[15], t_ref1 - t_ref0);
            atomicAdd(&st->sel_prof[16], 1ull);
        }
        __shared__ uint32_t s_rlast;
        uint32_t *rtk = N.rtk + (N.round ? N.par : X & 1) * RTK_SET;
        if (!pfx) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the write-through summaries drained
            __syncthreads();
            if (tid == 0) __hip_atomic_fetch_add(rtk + (blockIdx.x & 7) * RTK_STRIDE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
        if (block_ticket_last_x(rtk, nref, &s_rlast) && ld_wt(&st->ref_noprefix) != (N.round ? N.seq : X)) {
            if (N.prof && tid == 0)
                __hip_atomic_store(&st->sel_prof_pq, (unsigned long long)wall_clock64(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            refresh_prefix(N.V, N.cs);
            if (N.prof && tid == 0)
                __hip_atomic_store(&st->sel_prof_pp, (unsigned long long)wall_clock64(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0) __hip_atomic_fetch_add(rtk + 8 * RTK_STRIDE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return;
    }
    // Issued before the state head (they do not depend on it), so that head, hot entries and tail tokens
    // take one round trip together: the first step of hot entries (bounded by the capacity, filtered by
    // the list length once the head is in) and wave 1's last 64 stream slots (the stream's last pair)
    const uint32_t bx = blockIdx.x - nref;  // argmax block index
    const uint32_t G = sel_blocks * NEXT_THREADS, i00 = bx * NEXT_THREADS + tid;
    unsigned long long e0[SEL_U];
#pragma unroll
    for (int u = 0; u < SEL_U; u++) e0[u] = i00 + u * G < hot_cap ? hot[i00 + u * G] : (unsigned long long)NO_ID;
    uint32_t c0[SEL_U];  // their counts (Tables::hcnt), in the same round trip
#pragma unroll
    for (int u = 0; u < SEL_U; u++) c0[u] = i00 + u * G < hot_cap ? hcnt[i00 + u * G] : 0u;  // (a leading argument: preloaded)
    const bool lp_wave = bx == 0 && tid >= 64 && tid < 128 && N.world == 1 && !N.lp_lazy;
    const uint32_t t_tail = lp_wave && n - 1 - (int64_t)(tid - 64) >= 0 ? tok[n - 1 - (int64_t)(tid - 64)] : HOLE;
    const StateHead H0 = load_head(st);
    // multi-merge rounds: this launch rolls the round's members, merges cur_x .. Xr, and begins merge Xr + 1
    const uint32_t Xr = N.round && H0.rd_v ? H0.cur_x + H0.rd_v - 1 : X;
    BeginArgs NB = N.B;
    if (N.round) NB.X = Xr + 1;
    // pair select: merge X+1's candidate from merge X's tie decision and what merge X's replace counted (in
    // the head's round trip)
    PairHead P0{};
    int32_t live0 = 0;
    if (N.pair) {
        P0 = st->ph[N.B.X & 1];  // (merge X+1's slot: no workgroup of this launch writes it, DevState::ph)
        live0 = st->live;
    }
    if (H0.halt) return;
    __shared__ MaxRec sm[NEXT_THREADS / WAVE];
    __shared__ uint32_t s_flag, s_nc, s_h, s_tie, s_len, s_ntb, s_ovf;
    __shared__ uint32_t s_key[NEXT_CAND];
    __shared__ uint32_t s_pc[NEXT_MAX_SEL], s_pt[NEXT_MAX_SEL], s_pk[NEXT_MAX_SEL];
    __shared__ uint32_t s_pre[64];
    roll_preload(st, delta, X, s_pre, N.round != 0);
    if (N.prof && blockIdx.x == nref && tid == 0) {  // the first argmax block
        const unsigned long long now = wall_clock64();
        st->sel_t0 = now;
        if (st->pp_t[5]) {  // the replace launch: its work span, its start -> this select's start, its phases
            unsigned long long *P = st->pipe_prof[pp_bucket(X)];
            const unsigned long long t5 = st->pp_t[5];
            // (pp_t[6]: the replace's latest block end, 0 when no probed replace block stamped it since pp_t[5])
            if (st->pp_t[6] >= t5) P[5] += st->pp_t[6] - t5;
            P[6] += now - t5;
            P[7]++;
            for (int k = 8; k <= 12; k++) {
                if (st->pp_t[k]) P[k + 2] += st->pp_t[k] - t5;
                st->pp_t[k] = 0;
            }
            st->pp_t[5] = st->pp_t[6] = 0;
        }
    }
    // ---- pair select: merge X+1 is the candidate that merge X's decision named, with no argmax and no
    // decision, when (a) merge X's replace decremented neither it nor made adjacent occurrences (it still
    // has the top count T; every other count only fell), (b) no new pair reached T (the tied set is the old
    // one minus merge X, minus the tied pairs merge X decremented), (c) the new pairs are fewer than the
    // free slots the decision counted (the candidate's run still ends before the next tied home, and no
    // tied run wraps: it is the first tied key in slot order) and (d) the Zig capacity is the same and not
    // at a max load (the stream's last pair is not needed). Then the Zig order is the one the decision saw.
    // (one roll and begin below serve both: a second inlined copy of them pushed the kernel into spills)
    const bool light = !N.round && pair_light(N.pair, N.B.X, N.x_end, N.V.C, P0, live0);
    if (light && bx != 0) return;
    // the candidate's words wait in LDS (kept in registers across the argmax and decision code, they pushed
    // the kernel's scalar registers into spills)
    __shared__ uint32_t s_p0[5];
    enum { P0_KEY, P0_TIES, P0_DT, P0_BIRTHS, P0_PGEN };
    if (light && tid == 0) {
        s_p0[P0_KEY] = P0.key; s_p0[P0_TIES] = P0.ties; s_p0[P0_DT] = P0.dt; s_p0[P0_BIRTHS] = P0.births; s_p0[P0_PGEN] = P0.plan_gen;
    }
    // one argmax workgroup (a short hot list): it is the last one by construction -- no ticket, no
    // partials through global memory
    const bool single = sel_blocks == 1 || light;
    __shared__ uint32_t s_lastpair;
    MaxRec R{0, 0, NO_ID};
    if (!light) {
        if (!nref)  // (no refresh workgroups: the argmax ones clear the deltas)
            for (uint32_t t = bx * NEXT_THREADS + tid; t < 2 * X; t += G) delta[t] = 0;
        const uint32_t nh = min(H0.hot_len, T.hot_cap), theta = H0.theta;
        // SEL_U hot entries per thread per step, every load of a step issued together (the first step's
        // entries were loaded at entry); their counts are gathered here, beside wave 1's cached last-pair
        // words, so both wait together
        MaxRec r{0, 0, NO_ID};
        uint32_t ids[SEL_U], cs[SEL_U], ks[SEL_U];
#pragma unroll
        for (int u = 0; u < SEL_U; u++) {
            const unsigned long long e = i00 + u * G < nh ? e0[u] : (unsigned long long)NO_ID;
            ids[u] = (uint32_t)e;
            ks[u] = (uint32_t)(e >> 32);  // the key rides along: the block's keys at its max come from registers
        }
#pragma unroll
        for (int u = 0; u < SEL_U; u++) cs[u] = ids[u] != NO_ID ? c0[u] : 0u;
        if (lp_wave) {
            // wave 1 of block 0: the count of the stream's last pair (a tie needs it: Zig map capacity).
            // The pair id of the last lookup (state head) is checked and its count loaded with the hot
            // counts (the tail tokens came with the head); a changed tail looks the key up.
            const uint32_t lane = tid - 64;
            const uint32_t cid = H0.lp_id < T.id_cap ? H0.lp_id : 0u;
            const uint32_t c_key = T.id_key[cid], c_cnt = T.id_cnt[cid], c_nid = st->num_ids;
            uint32_t lt[2] = {HOLE, HOLE};
            int got = 0;
            for (int64_t e = n; e > 0 && got < 2; e -= 64) {
                const int64_t p = e - 1 - lane;
                const uint32_t t = e == n ? t_tail : p >= 0 ? tok[p] : HOLE;
                uint64_t live = __ballot(t != HOLE);
                while (live && got < 2) {  // lowest lane = highest position
                    const int l = __builtin_ctzll(live);
                    live &= live - 1;
                    lt[got++] = (uint32_t)__shfl((int)t, l);
                }
            }
            if (lane == 0) {
                uint32_t lp = 0;
                if (got == 2) {
                    const uint32_t key = pair_key(lt[1], lt[0]);
                    if (key == H0.lp_key && c_key == key && H0.lp_id < c_nid && H0.lp_id < T.id_cap) {
                        lp = c_cnt;
                    } else {
                        const uint32_t id = ht_find(T, key);
                        lp = id == NO_ID ? 0u : T.id_cnt[id];
                        if (id != NO_ID) { st->lp_key = key; st->lp_id = id; }
                    }
                }
                __hip_atomic_store(N.lastpair, lp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                s_lastpair = lp;
            }
        }
#pragma unroll
        for (int u = 0; u < SEL_U; u++)
            if (cs[u] >= theta && cs[u]) r = max_combine(r, MaxRec{cs[u], 1u, ids[u]});
        if (N.prof && bx == 0 && tid == 0) {
            atomicAdd(&st->sel_prof[17], wall_clock64() - st->sel_t0);  // thread 0's counts in
            atomicAdd(&st->sel_prof[19], (unsigned long long)nh);        // the hot list's length
        }
        const bool one_step = SEL_U * G >= nh;  // (every entry was in the first step)
        for (uint32_t i0 = i00 + SEL_U * G; i0 < nh; i0 += SEL_U * G) {
#pragma unroll
            for (int u = 0; u < SEL_U; u++) {
                const unsigned long long e = i0 + u * G < nh ? T.hot[i0 + u * G] : (unsigned long long)NO_ID;
                ids[u] = (uint32_t)e;
                ks[u] = (uint32_t)(e >> 32);  // the key rides along: the block's keys at its max come from registers
            }
#pragma unroll
            for (int u = 0; u < SEL_U; u++) cs[u] = ids[u] != NO_ID ? T.hcnt[i0 + u * G] : 0u;
#pragma unroll
            for (int u = 0; u < SEL_U; u++)
                if (cs[u] >= theta && cs[u]) r = max_combine(r, MaxRec{cs[u], 1u, ids[u]});
        }
        if (tid == 0) s_nc = 0;
        R = block_max(r, sm);
        if (N.prof && bx == 0 && tid == 0) atomicAdd(&st->sel_prof[18], wall_clock64() - st->sel_t0);
        // the block's keys at its max (from the registers when the thread's entries fit one step)
        if (R.cnt && r.cnt == R.cnt) {
            if (one_step && SEL_U * G >= nh) {
#pragma unroll
                for (int u = 0; u < SEL_U; u++) {
                    if (ids[u] != NO_ID && cs[u] == R.cnt) {
                        const uint32_t j = atomicAdd(&s_nc, 1u);
                        if (j < NEXT_CAND) s_key[j] = ks[u];
                    }
                }
            } else {
                for (uint32_t i = bx * NEXT_THREADS + tid; i < nh; i += G) {
                    const unsigned long long e = T.hot[i];
                    if (T.hcnt[i] == R.cnt) {
                        const uint32_t j = atomicAdd(&s_nc, 1u);
                        if (j < NEXT_CAND) s_key[j] = (uint32_t)(e >> 32);
                    }
                }
            }
        }
        __syncthreads();
        // write-through stores: the last block reads them (block_ticket_last)
        if (!single && tid < min(s_nc, (uint32_t)NEXT_CAND))
            __hip_atomic_store(&N.cand[bx * NEXT_CAND + tid], s_key[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!single && tid == 0) {
            __hip_atomic_store(&partial[bx].cnt, R.cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&partial[bx].ties, R.cnt ? s_nc : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&partial[bx].id, R.id, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            // the key of a block's unique max
            __hip_atomic_store(&N.pkey[bx], s_nc == 1 ? s_key[0] : NO_ID, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    if (N.prof && tid == 0) atomicMax(&st->sel_ta, (unsigned long long)wall_clock64());
    // (the ticket is the launch parity's, zeroed by the launch before. Round 5 found argmax workgroups of a pair
    // select that started late, saw the candidate words block 0 had already rewritten for the next merge, took the
    // full path and arrived on a shared ticket, which then elected a later launch's last block early; the verdict's
    // words now live in a slot this launch never writes (pair_light), and the per-launch ticket stays as a second
    // guard: arrivals of a launch never count for another)
    if (!single && !block_ticket_last(N.rtk + (N.round ? N.par : X & 1) * RTK_SET + 9 * RTK_STRIDE, sel_blocks, &s_flag)) return;
    if (N.round) {  // roll_preload's LDS words (wave 0) landed (a single argmax block took no ticket)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    // the refresh precomputes the carries (its predicate; a round's RoundHead words are in s_pre: roll_preload)
    const bool pfx = nref && N.cs && (N.round ? true : N.B.log[X - 256].ties > 1);
    // the next launch's refresh count (the launch before this one used it and has ended)
    if (tid < 10) st_wt(N.rtk + (N.round ? N.par ^ 1u : (X + 1) & 1) * RTK_SET + tid * RTK_STRIDE, 0u);
    unsigned long long pt = 0;
    if (N.prof && tid == 0 && !light) {
        pt = st->sel_t0;
        const unsigned long long ta = __hip_atomic_load(&st->sel_ta, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long tr = __hip_atomic_load(&st->sel_tr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        atomicAdd(&st->sel_prof[5], ta - pt);
        // refresh blocks that finished before this point (the rest run on; stale stamps are < pt)
        (void)tr;
        st->sel_ta = 0;
        sel_tick(st, 0, &pt);
        atomicAdd(&st->sel_prof[7], 1ull);
    }
    // ---- the last block: argmax, roll of merge X -------------------------------------------------
    // the stream's last pair count (block 0 stored it write-through): in flight with the partials
    const uint32_t lastpair_wt = tid == 0 && N.world == 1 && !N.lp_lazy && !light ? (single ? s_lastpair : ld_wt(N.lastpair)) : NO_ID;
    MaxRec Q = R;
    if (light) {  // the candidate: the top count, the tied set less merge X and the tied pairs merge X decremented
        if (tid == 0) s_key[0] = s_p0[P0_KEY];
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // roll_preload's LDS words (wave 0) landed
        __syncthreads();
        Q = MaxRec{H0.top_count, s_p0[P0_TIES] - 1u - (s_p0[P0_DT] & 0xFFFFu), 0u};
    } else if (single) {  // (s_nc, s_key from the argmax above; the barrier after it published them)
        if (tid == 0) {
            s_pc[0] = R.cnt;
            s_pt[0] = R.cnt ? s_nc : 0u;
            s_pk[0] = s_nc == 1 ? s_key[0] : NO_ID;
        }
        Q.ties = R.cnt ? s_nc : 0u;
        __syncthreads();
    } else {
        MaxRec q{0, 0, NO_ID};
        for (uint32_t b = tid; b < sel_blocks; b += NEXT_THREADS) {
            const MaxRec p{ld_wt(&partial[b].cnt), ld_wt(&partial[b].ties), ld_wt(&partial[b].id)};
            s_pc[b] = p.cnt;
            s_pt[b] = p.ties;
            s_pk[b] = ld_wt(N.pkey + b);  // (with the partial: no second round trip once the max is known)
            q = max_combine(q, p);
        }
        Q = block_max(q, sm);  // (its barriers also publish s_pc / s_pt)
    }
    if (!light && Q.ties == 1 && Q.cnt) {  // the unique max: its block kept its key
        for (uint32_t b = tid; b < sel_blocks; b += NEXT_THREADS)
            if (s_pc[b] == Q.cnt) s_key[0] = s_pk[b];
    }
    // a tied top pair's key (select_finish defers it; only the host reads it, after a halt): loaded now
    // straight into LDS by the last wave, which has nothing else to do (an LDS-DMA load makes its wave's
    // next LDS read wait for it), and stored by it at the launch's end
    constexpr uint32_t KEY_TID = NEXT_THREADS - 64;
    __shared__ uint32_t s_qkey;
    if (tid == KEY_TID && Q.cnt && Q.ties > 1 && !light)
        __builtin_amdgcn_global_load_lds(&T.id_key[Q.id], (__attribute__((address_space(3))) void *)&s_qkey, 4, 0, 0);
    __syncthreads();
    // the next merge's scan plan: its list loads (one lane of wave 1) overlap the roll and begin below;
    // for an untied next merge the key is known now, a tied one's comes from the decision (decide_body)
    __shared__ uint32_t s_plan[6];
    // (X's list: the roll's lst_off / lst_len, from the same words; a round's members: T records each)
    const PlanCtx plan = N.round && H0.rd_v ? PlanCtx{T.lst_off, T.lst_len, N.dir_row, N.dir, N.dir_w, H0.lists_x, H0.cur_x, H0.arena_top,
                                                      H0.top_count, H0.rd_v, H0.rd_mask,
                                                      s_pre + RI_WORDS + offsetof(RoundHead, cnt) / 4}
                                            : PlanCtx{T.lst_off, T.lst_len, N.dir_row, N.dir, N.dir_w, H0.lists_x, X, H0.arena_top,
                                                      H0.rec_count, 1u};
    const bool plan_on = N.plan && T.lst_off && H0.lists_valid;
    if (plan_on && tid == 64) {
        if (light) {  // the candidate's plan, by merge X's replace (pair_slack_block), unless the layout changed since
            const PairTail &PT = *reinterpret_cast<const PairTail *>(&st->pr_plan[0]);
            if (s_p0[P0_PGEN] == N.gen)
                for (int k = 0; k < 6; k++) s_plan[k] = PT.plan[k];
            else
                plan_compute(plan, s_key[0], s_plan);
        } else if (Q.ties == 1 && Q.cnt) {
            plan_compute(plan, s_key[0], s_plan);
        }
    }
    if (N.prof && tid == 0 && !light) sel_tick(st, 1, &pt);
    // ---- untied rounds (N.untied): merge X+1 has the unique top count T_0. Waves 2..7, beside thread 0's roll and
    // begin, find the next ROUND_MAX - 1 distinct counts below it among the hot entries (every pair with a count
    // >= theta is listed), each with how many entries hold it and one of their keys: per wave, then (below) merged
    // by wave 2. A distinct count held by one pair names it as the next round member (UntiedHead).
    constexpr uint32_t UR_U = 16;  // hot entries per thread (the pass covers hot lists of up to 384 * UR_U ids)
    constexpr uint32_t UR_L = ROUND_MAX - 1;
    __shared__ uint32_t s_uw[6 * UR_L * 3];
    const bool ur_on = N.round && N.untied && !light && Q.ties == 1 && Q.cnt && NB.X + 1 < N.x_end &&
                       min(H0.hot_len, T.hot_cap) <= 384u * UR_U;
    if (ur_on && tid >= 128) {
        const uint32_t w = (tid >> 6) - 2, t = tid - 128, lane = tid & 63;
        const uint32_t nh = min(H0.hot_len, T.hot_cap), theta = H0.theta;
        const uint32_t *hk = reinterpret_cast<const uint32_t *>(hot);  // (a hot entry's upper word: its key)
        uint32_t c[UR_U], k[UR_U];
#pragma unroll
        for (uint32_t u = 0; u < UR_U; u++) {
            const uint32_t i = t + u * 384u;
            c[u] = i < nh ? hcnt[i] : 0u;
            k[u] = i < nh ? hk[2 * i + 1] : NO_ID;
        }
        uint32_t Lp = Q.cnt;
#pragma unroll
        for (uint32_t l = 0; l < UR_L; l++) {
            uint32_t L = 0;
#pragma unroll
            for (uint32_t u = 0; u < UR_U; u++) L = c[u] < Lp && c[u] >= theta && c[u] > L ? c[u] : L;
            L = wave_max_u32(L);  // (waves 2..7 whole: DPP all-reduces)
            uint32_t m = 0, kk = NO_ID;
#pragma unroll
            for (uint32_t u = 0; u < UR_U; u++) {
                const bool eq = L && c[u] == L;
                m += eq ? 1u : 0u;
                kk = eq ? k[u] : kk;
            }
            const uint64_t has = __ballot(m != 0);
            kk = has ? (uint32_t)__builtin_amdgcn_readlane((int)kk, __ffsll((unsigned long long)has) - 1) : NO_ID;
            m = wave_sum_u32(m);
            if (lane == 0) {
                s_uw[(w * UR_L + l) * 3 + 0] = L;
                s_uw[(w * UR_L + l) * 3 + 1] = m;
                s_uw[(w * UR_L + l) * 3 + 2] = kk;
            }
            Lp = L;
        }
    }
    if (tid == 0) {
        FinishOut fo;
        const bool rnd = N.round && H0.rd_v;
        select_finish(T, st, Q, tok, n, delta, X, rnd ? 0 : 1, N.bnd, N.world, light || (Q.ties == 1 && Q.cnt) ? s_key[0] : NO_ID,
                      lastpair_wt, &fo, s_pre, Q.ties > 1 && !light, N.lp_lazy != 0 || light);
        if (rnd) round_roll(T, st, H0, N.B.log, s_pre, &fo, N.rlog + N.rlog_i);
        s_h = HALT_DONE;
        s_tie = 0;
        if (NB.X < N.x_end) {
            bool tie;
            const uint32_t h = merge_begin_eval_v(T, fo, NB, &tie);
            if (light && !h && tie) {  // a pair select: the decision's commit, with its winner
                st->last_light = N.B.X;
                st->cur_x = N.B.X;
                st->tie_on = 0;
                st->cur_key = s_key[0];
                N.B.log[N.B.X - 256] = MergeLog{s_key[0], fo.top_count, (uint32_t)fo.live_tokens, fo.tie_count};
                tie = false;
            } else {
                merge_begin_commit_v(st, NB, h, tie, fo);
            }
            if (light) {
                // chain: merge X+2's candidate is the next tied key by home, once this pair select is committed;
                // its bound (the free slots between its home and the next, and after the largest, against the
                // new pairs of both merges) and plan come from merge X+1's replace, whose home summaries are
                // still the decision's (this launch refreshed none)
                const PairTail &PT = *reinterpret_cast<const PairTail *>(&st->pr_plan[0]);
                const uint32_t key2 = PT.key2, key3 = PT.key3, key4 = PT.key4, h3 = PT.h3, h4 = PT.h4, h5 = PT.h5, h6 = PT.h6;
                // (merge X+2's slot: the other one than this launch's workgroups read at entry, DevState::ph)
                PairHead &pn = st->ph[(N.B.X + 1) & 1];
                if (!h && N.skip_refresh && key2 != NO_ID && N.B.X + 1 < N.x_end) {
                    pn.key = key2;  // the chain moves up one: key2 -> key, key3 -> key2, their flags with them
                    st->pr_key2 = key3;
                    st->pr_key3 = key4;
                    st->pr_key4 = NO_ID;
                    const uint32_t ties0 = s_p0[P0_TIES], dt0 = s_p0[P0_DT];
                    pn.ties = ties0 - 1u;
                    pn.dt = (dt0 & 0xFFFFu) | (((dt0 >> 19) & 1u) << 16) | (((dt0 >> 20) & 1u) << 19) | (((dt0 >> 21) & 1u) << 20);
                    pn.births = s_p0[P0_BIRTHS];  // (the next bound is against the new pairs of both merges)
                    st->pr_h2 = h3;
                    st->pr_h3 = h4;
                    st->pr_h4 = h5;
                    st->pr_h5 = h6;
                    pn.slack = ties0 == 3u ? 0xFFFFFFFFu : 0u;  // (the third was the last tied key)
                    pn.plan_gen = 0xFFFFFFFFu;
                    pn.x = N.B.X + 1;
                } else {
                    pn.x = 0;
                }
                atomicAdd(&st->pr_hits, 1u);
            }
            s_h = h;
            s_tie = tie ? 1u : 0u;
        } else if (N.round) {  // the round reached the vocabulary's end: the launches after it have nothing to do
            st->halt = HALT_DONE;
            st->halt_at = NB.X;
        }
        s_len = 0;
        s_ovf = 0;
    }
    __syncthreads();
    // merge X+1 needs no tie decision: the last refresh workgroup may skip its carries
    if (tid == 0 && (s_h || !s_tie)) st_wt(&st->ref_noprefix, N.round ? N.seq : X);
    if (N.prof && tid == 0 && !light) sel_tick(st, 2, &pt);
    // the tied top pair's key, deferred by select_finish (stored on every way out below)
    auto put_key = [&]() {
        if (tid == KEY_TID && Q.cnt && Q.ties > 1 && !light) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            st->top_key = s_qkey;
        }
    };
    if (s_h || !s_tie) {
        if (plan_on && tid == 64 && !s_h && (light || (Q.ties == 1 && Q.cnt))) plan_store(st, NB.X, s_key[0], N.gen, s_plan);
        if (ur_on && !s_h && tid >= 128 && tid < 192) {  // wave 2: the waves' counts merged, the round's names stored
            const uint32_t lane = tid - 128;
            const bool rec = lane < 6 * UR_L;
            const uint32_t L = rec ? s_uw[lane * 3] : 0u, M = rec ? s_uw[lane * 3 + 1] : 0u, K = rec ? s_uw[lane * 3 + 2] : NO_ID;
            uint32_t Lp = Q.cnt, nu = 0, uk[UR_L], uc[UR_L];
            bool go = true;
#pragma unroll
            for (uint32_t l = 0; l < UR_L; l++) {
                uk[l] = NO_ID;
                uc[l] = 0;
                if (!go) continue;
                const uint32_t Lk = wave_max_u32(L < Lp ? L : 0u);  // (wave 2 whole: DPP all-reduces)
                const uint32_t msum = wave_sum_u32(Lk && L == Lk ? M : 0u);
                const uint64_t has = __ballot(Lk && L == Lk);
                const uint32_t key = has ? (uint32_t)__builtin_amdgcn_readlane((int)K, __ffsll((unsigned long long)has) - 1) : NO_ID;
                // (a count held by several pairs is a tie: the Zig order decides it, so the names end; so does a self pair)
                go = Lk && msum == 1 && key != NO_ID && (key & 0xFFFF) != (key >> 16);
                if (go) { uk[l] = key; uc[l] = Lk; nu++; }
                Lp = Lk;
            }
            if (lane == 0) {
                UntiedHead u;
                u.x = NB.X;
                u.n = nu;
#pragma unroll
                for (uint32_t l = 0; l < UR_L; l++) { u.key[l] = uk[l]; u.cnt[l] = uc[l]; }
                st->ur = u;
            }
        }
        if (N.prof && tid == 0) {
            const unsigned long long now = wall_clock64();
            st->pp_t[7] = now;
            if (light) {
                atomicAdd(&st->sel_prof[20], 1ull);
                atomicAdd(&st->sel_prof[21], now - st->sel_t0);
            }
        }
        put_key();
        return;
    }
    // ---- merge X+1 ties: gather the keys of the blocks whose max is the top count ----------------
    const uint32_t top = Q.cnt, total = Q.ties;
    for (uint32_t b = tid; b < sel_blocks; b += NEXT_THREADS) {
        if (s_pc[b] == top) {
            if (s_pt[b] > NEXT_CAND) atomicOr(&s_ovf, 1u);
            atomicAdd(&s_len, s_pt[b]);
        }
    }
    __syncthreads();
    if (total > N.tie_cap) {  // the host path decides (replicated state: every rank takes it)
        if (tid == 0) { st->halt = HALT_TIE; st->halt_at = NB.X; }
        put_key();
        return;
    }
    const uint32_t cap_mask = N.V.C - 1;
    // the tied keys go to LDS when they fit (the decision reads them there: no global store and
    // reload between the gather and the decision), else to N.tie_list
    __shared__ uint64_t s_tl[NEXT_TIE_LDS];
    const uint64_t *tie_list = N.tie_list;
    if (s_ovf || s_len != total) {
        // a block held more tied keys than it kept (how the hot list spreads them depends on the
        // rank's id numbering): collect them from the whole hot list here, so every rank agrees
        const uint32_t nh = min(st->hot_len, T.hot_cap);
        if (tid == 0) s_len = 0;
        __syncthreads();
        for (uint32_t i0 = tid & ~63u; i0 < nh; i0 += NEXT_THREADS) {  // wave-uniform trip count
            const uint32_t i = i0 + (tid & 63);
            uint32_t id = NO_ID;
            unsigned long long e = NO_ID;
            if (i < nh) e = T.hot[i];
            id = (uint32_t)e;
            const bool tied = id != NO_ID && T.id_cnt[id] == top;
            const uint32_t j = wave_append(&s_len, tied);
            if (tied && j < total) {
                const uint32_t key = (uint32_t)(e >> 32);
                N.tie_list[j] = ((uint64_t)(zig_pair_hash(key) & cap_mask) << 32) | key;
            }
        }
        __syncthreads();
        if (tid == 0) {
            if (s_len != total) atomicOr(&st->error, 128u);
            st->tie_len = total;
        }
    } else {
    // tied blocks in block order and the exclusive offsets of their keys (wave 0, 64 blocks per step)
    __shared__ uint32_t s_tb[NEXT_MAX_SEL], s_to[NEXT_MAX_SEL + 1];
    if (tid < 64) {
        uint32_t k = 0, o = 0;
        for (uint32_t b0 = 0; b0 < sel_blocks; b0 += 64) {
            const uint32_t b = b0 + tid;
            const bool t = b < sel_blocks && s_pc[b] == top;
            const uint32_t c = t ? s_pt[b] : 0u;
            const uint64_t m = __ballot(t);
            const uint32_t below = (uint32_t)__popcll(m & ((1ull << tid) - 1ull));
            const uint32_t inc = wave_incl_scan_dpp(c);  // (wave 0 whole, a uniform trip count)
            if (t) { s_tb[k + below] = b; s_to[k + below] = o + inc - c; }
            k += (uint32_t)__popcll(m);
            o += lane_bcast(inc, 63);
        }
        if (tid == 0) { s_ntb = k; s_to[k] = o; }
    }
    __syncthreads();
    const uint32_t ntb = s_ntb;
    for (uint32_t e = tid; e < total; e += NEXT_THREADS) {
        uint32_t lo = 0, hi = ntb;  // the tied block holding key e: s_to[lo] <= e < s_to[lo + 1]
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (s_to[mid] <= e) lo = mid; else hi = mid;
        }
        const uint32_t key = single ? s_key[e] : ld_wt(N.cand + s_tb[lo] * NEXT_CAND + (e - s_to[lo]));
        const uint64_t ent = ((uint64_t)(zig_pair_hash(key) & cap_mask) << 32) | key;
        if (total <= NEXT_TIE_LDS) s_tl[e] = ent;
        else N.tie_list[e] = ent;
    }
    if (total <= NEXT_TIE_LDS) tie_list = s_tl;
    if (tid == 0) st->tie_len = total;
    }
    // ---- merge X+1 ties: the Zig-order decision, by this block (the list is this block's writes;
    // the refreshed home summaries were stored write-through and drained before each refresh
    // block's count: wait for all nref, then read them with sc1 loads) --------------------------------
    if (N.prof && tid == 0) sel_tick(st, 3, &pt);
    if (nref && tid < 64) {
        // every refresh block is resident or done (they never wait), so this ends. It relies on the GPU
        // dispatching a grid's workgroups in id order: the refresh workgroups (ids [0, nref)) were
        // dispatched before this argmax workgroup, so none of them waits for a slot this one holds.
        // pfx: the top counter reaches the groups + the prefix's arrival; else the XCD counters sum to nref
        // Bounded: a wait past SPIN_LIMIT_TICKS (a broken dispatch-order assumption) reads the counters once
        // more and, still short, sets error bit 1024 (sync_state fails the train); the decision goes on with
        // whatever summaries it reads.
        const uint32_t *rtk = N.rtk + (N.round ? N.par : X & 1) * RTK_SET;
        const unsigned long long t_spin = wall_clock64();
        if (pfx) {
            const uint32_t want = min(nref, 8u) + 1u;
            while (ld_wt(rtk + 8 * RTK_STRIDE) < want) {
                __builtin_amdgcn_s_sleep(1);
                if (wall_clock64() - t_spin > SPIN_LIMIT_TICKS) {
                    if (tid == 0 && ld_wt(rtk + 8 * RTK_STRIDE) < want) atomicOr(&st->error, 1024u);
                    break;
                }
            }
        } else {
            for (bool last = false;;) {
                uint32_t c = tid < 8 ? ld_wt(rtk + tid * RTK_STRIDE) : 0u;
#pragma unroll
                for (int off = 4; off >= 1; off >>= 1) c += (uint32_t)__shfl_xor((int)c, off);
                const bool done = (uint32_t)__shfl((int)c, 0) >= nref;
                if (done) break;
                if (last) {  // timed out, and the counters read once more are still short
                    if (tid == 0) atomicOr(&st->error, 1024u);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
                last = wall_clock64() - t_spin > SPIN_LIMIT_TICKS;
            }
        }
    }
    __syncthreads();
    if (N.prof && tid == 0) {
        sel_tick(st, 10, &pt);
        const unsigned long long t0 = st->sel_t0;
        // every refresh workgroup has arrived: the latest one's finish (from this launch's t0)
        const unsigned long long tr = __hip_atomic_load(&st->sel_tr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (tr >= t0) { atomicAdd(&st->sel_prof[12], tr - t0); atomicAdd(&st->sel_prof[13], 1ull); }
        if (N.cs && pfx) {  // the last refresh workgroup's prefix of this launch: start, end (from t0)
            const unsigned long long pq = __hip_atomic_load(&st->sel_prof_pq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned long long pp = __hip_atomic_load(&st->sel_prof_pp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (pq >= t0 && pp >= pq) {  // (stamps of an earlier launch are older than t0)
                atomicAdd(&st->sel_prof[6], pq - t0);
                atomicAdd(&st->sel_prof[11], pp - t0);
                atomicAdd(&st->sel_prof[14], 1ull);
            }
        }
    }
    decide_body<NEXT_THREADS>(st, tie_list, total, total, N.V, N.B.log, 1, N.prof ? &pt : nullptr, pfx ? N.cs : nullptr,
                              plan_on, plan, N.gen, N.pair && NB.X + 1 < N.x_end ? NB.X + 1 : 0u, N.m3_w4 != 0,
                              N.skip_refresh != 0 && N.chain != 0, N.chain >= 2, N.chain >= 3, N.round != 0, &NB);
    if (N.prof && tid == 0) { sel_tick(st, 4, &pt); atomicAdd(&st->sel_prof[8], 1ull); st->pp_t[7] = wall_clock64(); }
    put_key();
}

// rebuild the home histogram for a new Zig capacity: counts only (the caller recomputes every summary;
// home_add's dirty-bit OR would put ~5e7 atomics on the few hundred dirty-bitmap words)
__global__ void __launch_bounds__(256) zbpe_home_build(Tables T, DevState *st) {
    const uint32_t n = min(st->num_ids, T.id_cap);
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        if (!T.id_cnt[i]) continue;
        const uint32_t s = (uint32_t)(zig_pair_hash(T.id_key[i]) & T.home_mask);
        atomicAdd(&T.home_cnt[s >> 2], 1u << (8 * (s & 3)));
    }
}

// exact fallback: first occurrence position of every live pair in the current stream
// first-occurrence position (shard-local) of every live pair: the exact tie fallback's insertion order
__global__ void __launch_bounds__(256) zbpe_first_occ(ScanArgs A, Tables T, uint32_t *first, DevState *st) {
    for (int64_t p = blockIdx.x * 256 + threadIdx.x; p < A.n; p += (int64_t)gridDim.x * 256) {
        const uint16_t x = A.tok[p];
        if (x == HOLE) continue;
        const int64_t q = next_live_h(A, p);  // the pair leaving the shard is owned here
        if (q == NONE_POS) continue;
        const uint32_t id = ht_find(T, pair_key(x, tok_h(A, q)));
        if (id == NO_ID) { key_missing(st, pair_key(x, tok_h(A, q)), 4); continue; }
        atomicMin(&first[id], (uint32_t)p);
    }
}
__global__ void __launch_bounds__(256) zbpe_gather_live(Tables T, const uint32_t *__restrict__ first, DevState *st,
                                                        LiveRec *__restrict__ out, uint32_t out_cap) {
    const uint32_t n = min(st->num_ids, T.id_cap);
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        uint32_t c = T.id_cnt[i];
        if (!c) continue;
        uint32_t j = atomicAdd(&st->gather_len, 1u);
        if (j < out_cap) out[j] = LiveRec{first[i], T.id_key[i], c, 0};
    }
}

// The exact tie emulation's input on one GPU: every live pair as a (first occurrence, entry) pair for a
// device radix sort by position; entry = zig_emu_entry (zig_order.hpp): low 31 bits of the Zig hash,
// the tied bit (count == top), the key. One wave-aggregated append per wave.
__global__ void __launch_bounds__(256) zbpe_gather_order(Tables T, const uint32_t *__restrict__ first, DevState *st, uint32_t top,
                                                         uint32_t *__restrict__ pos_out, unsigned long long *__restrict__ ent_out,
                                                         uint32_t out_cap) {
    const uint32_t n = min(st->num_ids, T.id_cap);
    const uint32_t n_round = (n + 63) & ~63u;  // whole waves reach the ballot
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n_round; i += gridDim.x * 256) {
        const uint32_t c = i < n ? T.id_cnt[i] : 0;
        const uint32_t j = wave_append(&st->gather_len, c != 0);
        if (c && j < out_cap) {
            const uint32_t key = T.id_key[i];
            const uint32_t h = ((uint32_t)zig_pair_hash(key) & 0x7FFFFFFFu) | (c == top ? 0x80000000u : 0u);
            pos_out[j] = first[i];
            ent_out[j] = ((unsigned long long)h << 32) | key;
        }
    }
}

// verification: recount every live pair of the stream and compare with the maintained counts
// recount every pair this shard owns (the pair leaving the shard included, through the halo)
__global__ void __launch_bounds__(256) zbpe_recount(ScanArgs A, Tables T, uint32_t *recount, DevState *st) {
    for (int64_t p = blockIdx.x * 256 + threadIdx.x; p < A.n; p += (int64_t)gridDim.x * 256) {
        const uint16_t x = A.tok[p];
        if (x == HOLE) continue;
        const int64_t q = next_live_h(A, p);
        if (q == NONE_POS) continue;
        const uint32_t id = ht_find(T, pair_key(x, tok_h(A, q)));
        if (id == NO_ID) { atomicAdd(&st->mismatches, 1u); continue; }
        atomicAdd(&recount[id], 1u);
    }
}
// Full pair histogram of a hole-free stream (countCodePointPairs over the whole stream,
// basic_tokenizer.zig:257-278, against the table's ids): the verification recount and the north-star
// histogram kernel. One 1024-thread workgroup per CU streams 16-B vectors (non-temporal, a lane's
// successor token from its neighbour lane by a shuffle) and counts pairs in an LDS open-addressed table
// of PH_SLOTS keys (128 KiB): hot pairs take one LDS atomic each, and only a pair that finds no slot
// within PH_PROBES probes pays the global hash lookup + atomic. The LDS table is flushed once at the
// end (one lookup + one atomic per distinct pair per workgroup). `next_tok` is the token after the
// stream (the next shard's first, or -1).
constexpr int PH_THREADS = 1024;
constexpr uint32_t PH_SLOTS = 16384;
constexpr int PH_PROBES = 8;
constexpr int PH_U = 4;  // 16-B vectors per lane in flight
constexpr uint32_t PH_EMPTY = 0xFFFFFFFFu;  // (65535, 65535): two holes, never a pair
// home pair of slots of a key: the even slot its hash picks and the next one (one 8-B LDS read; a
// 4-slot group by 16-B reads was measured slower: 1.10 vs 0.92 ms at C4 t = 0)
__device__ inline uint32_t ph_home(uint32_t key) { return ((key * 0x9E3779B1u) >> (32 - 14)) & ~1u; }
// a key missing from its home pair: linear probing from the home pair (insert at the first empty slot),
// else the global table's id and a global atomic
__device__ inline void ph_count(uint32_t *s_key, uint32_t *s_cnt, const Tables &T, uint32_t *recount, DevState *st,
                                uint32_t key) {
    uint32_t h = ph_home(key);
#pragma unroll 1
    for (int q = 0; q < PH_PROBES; q++) {
        const uint32_t k = __hip_atomic_load(&s_key[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (k == key) { atomicAdd(&s_cnt[h], 1u); return; }
        if (k == PH_EMPTY) {
            const uint32_t old = atomicCAS(&s_key[h], PH_EMPTY, key);
            if (old == PH_EMPTY || old == key) { atomicAdd(&s_cnt[h], 1u); return; }
        }
        h = (h + 1) & (PH_SLOTS - 1);
    }
    const uint32_t id = ht_find(T, key);
    if (id == NO_ID) { atomicAdd(&st->mismatches, 1u); return; }
    atomicAdd(&recount[id], 1u);
}
__global__ void __launch_bounds__(PH_THREADS) zbpe_pair_hist(const uint16_t *__restrict__ tok, int64_t n, int32_t next_tok,
                                                              Tables T, uint32_t *__restrict__ recount, DevState *st) {
    extern __shared__ __attribute__((aligned(16))) uint32_t ph_lds[];
    uint32_t *s_key = ph_lds, *s_cnt = ph_lds + PH_SLOTS;
    for (uint32_t i = threadIdx.x; i < PH_SLOTS; i += PH_THREADS) { s_key[i] = PH_EMPTY; s_cnt[i] = 0; }
    __syncthreads();
    const uint4 *tv = reinterpret_cast<const uint4 *>(tok);
    const int64_t nvec = (n + 7) / 8;
    const int lane = threadIdx.x & 63;
    // a wave takes tiles of PH_U x 64 vectors: all PH_U loads are in flight before any counting
    const int64_t wave = (int64_t)blockIdx.x * (PH_THREADS / 64) + (threadIdx.x >> 6);
    const int64_t waves = (int64_t)gridDim.x * (PH_THREADS / 64);
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    for (int64_t tile = wave * PH_U * 64; tile < nvec; tile += waves * PH_U * 64) {
        uint4 v[PH_U];
#pragma unroll
        for (int u = 0; u < PH_U; u++) {
            const int64_t vi = tile + u * 64 + lane;
            const u32x4 y = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(tv + (vi < nvec ? vi : 0)));
            v[u] = vi < nvec ? make_uint4(y.x, y.y, y.z, y.w) : make_uint4(0, 0, 0, 0);
        }
        const int64_t p_last = (tile + PH_U * 64) * 8;  // the token after the tile
        const uint32_t after_tile = lane == 63 && p_last < n ? (uint32_t)tok[p_last] : PH_EMPTY;
#pragma unroll
        for (int u = 0; u < PH_U; u++) {
            const int64_t vi = tile + u * 64 + lane;
            // the next vector's first token: the next lane's, or (lane 63) the next row's lane 0 / the tile's end
            // (DPP: the next lane's first token; lane 63 the next row's lane 0, or the token after the tile)
            uint32_t nx = wave_shl1(v[u].x & 0xFFFFu, u + 1 < PH_U ? lane_bcast(v[u + 1 < PH_U ? u + 1 : u].x & 0xFFFFu, 0) : after_tile);
            const int64_t p8 = vi * 8 + 8;
            if (p8 >= n) nx = p8 == n && next_tok >= 0 ? (uint32_t)next_tok : PH_EMPTY;
            if (vi >= nvec) continue;
            // the 8 pairs' first probes are issued together (one LDS round trip for the common hit), then
            // hits take a non-returning LDS add; the misses of the vector's 8 pairs are taken together
            // after them (one divergent slow path per vector, not one per pair: at 64 lanes some lane
            // nearly always misses)
            uint32_t key[8], h[8];
            uint2 k0[8];
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const int64_t p = vi * 8 + k;
                const uint32_t b = k < 7 ? (p + 1 < n ? tok_at(v[u], k + 1) : (p + 1 == n && next_tok >= 0 ? (uint32_t)next_tok : PH_EMPTY)) : nx;
                key[k] = p < n && b != PH_EMPTY ? pair_key(tok_at(v[u], k), b) : PH_EMPTY;
                h[k] = ph_home(key[k]);
            }
            // (a plain LDS read: a slot's key only ever goes from empty to its final value, and a stale
            // empty read just sends the pair to the probing path, which re-reads with atomics)
#pragma unroll
            for (int k = 0; k < 8; k++) k0[k] = *reinterpret_cast<const uint2 *>(&s_key[h[k]]);
            uint32_t miss = 0;
#pragma unroll
            for (int k = 0; k < 8; k++) {
                if (key[k] == PH_EMPTY) continue;
                const uint32_t j = k0[k].x == key[k] ? 0u : k0[k].y == key[k] ? 1u : 2u;
                if (j < 2) atomicAdd(&s_cnt[h[k] + j], 1u);
                else miss |= 1u << k;
            }
            while (miss) {
                const int k = __builtin_ctz(miss);
                miss &= miss - 1;
                uint32_t kk = key[0];
#pragma unroll
                for (int j = 1; j < 8; j++)
                    if (k == j) kk = key[j];
                ph_count(s_key, s_cnt, T, recount, st, kk);
            }
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < PH_SLOTS; i += PH_THREADS) {
        const uint32_t k = s_key[i];
        if (k == PH_EMPTY) continue;
        const uint32_t id = ht_find(T, k);
        if (id == NO_ID) { atomicAdd(&st->mismatches, s_cnt[i]); continue; }
        atomicAdd(&recount[id], s_cnt[i]);
    }
}

// The full pair histogram of a stream of BYTES (t = 0: every token < 256): all 65,536 byte
// pairs in 16-bit LDS bins, two to a word (128 KiB), so a pair is a fixed bin -- no key, no hash, no
// probe, no compare. The hashed form above spends most of its ~2,500-instruction tile on exactly those
// (2.2 TB/s at C4 t = 0, instruction-bound); here a pair is a byte permute, three bit operations and one
// LDS add.
//   Bin of (a, b): word (a << 7) | ((b >> 1) ^ (a & 127)) -- the row rotated by a so that text's
//   successors (letters, space) spread over the LDS banks -- half b & 1 (low: +1, high: +0x10000).
// A bin can pass 65,535 within a workgroup (C4's hottest pair: ~71 K per workgroup), so overflow is
// accounted exactly, race-free, from the value each add returns (adds on one word are linearisable):
//   - a low-half add that returns low == 0xFFFF wrapped the low bin: +65,536 to that pair's global count,
//     and the carry it put into the high half is taken back by an LDS subtract;
//   - an add (or the carry of a low add) that carries out of bit 31 wrapped the high bin: +65,536 to the
//     high pair; a take-back subtract that borrows out of bit 31 undoes one such carry: -65,536.
// Then a word's final halves are each pair's count mod 65,536 and the events add the multiples (a bin with
// events always has real adds, so the pairs they name exist). Events are rare (one per 65,536 adds of a
// bin) and taken in a divergent branch behind one test per vector. (Spilling every half past 32,768 after
// each 32,768-pair pass instead -- non-returning adds, no event test -- was slower: 892 vs 642 us at C4
// t = 0, the pass barriers keep the waves from hiding each other's load latency.)
constexpr uint32_t PHB_WORDS = 32768;
__device__ inline uint32_t phb_word(uint32_t ab) { return (ab >> 1) ^ ((ab >> 8) & 127u); }  // ab = a << 8 | b
__device__ inline uint32_t phb_pair(uint32_t w, uint32_t half) {  // (a, b) of word w, half -> pair key
    const uint32_t a = w >> 7, b = (((w & 127u) ^ (a & 127u)) << 1) | half;
    return pair_key(a, b);
}
__device__ inline void phb_global(const Tables &T, uint32_t *recount, DevState *st, uint32_t key, uint32_t add) {
    const uint32_t id = ht_find(T, key);
    if (id == NO_ID) { atomicAdd(&st->mismatches, 1u); return; }
    atomicAdd(&recount[id], add);
}
// an add to pair ab returned `old`: its overflow events (divergent, rare)
__device__ inline void phb_events(uint32_t *bins, const Tables &T, uint32_t *recount, DevState *st, uint32_t ab, uint32_t old) {
    const uint32_t w = phb_word(ab), half = ab & 1u, inc = half ? 0x10000u : 1u;
    if (!half && (old & 0xFFFFu) == 0xFFFFu) {  // the low bin wrapped: count it, take its carry back
        phb_global(T, recount, st, phb_pair(w, 0), 0x10000u);
        const uint32_t o2 = atomicSub(&bins[w], 0x10000u);
        if (o2 < 0x10000u) phb_global(T, recount, st, phb_pair(w, 1), 0u - 0x10000u);  // the take-back borrowed
    }
    if (old + inc < old) phb_global(T, recount, st, phb_pair(w, 1), 0x10000u);  // carry out of bit 31: high wrapped
}
__device__ inline uint32_t phb_add(uint32_t *bins, uint32_t ab) {  // the pair's add; returns the word's old value
    return atomicAdd(&bins[phb_word(ab)], (ab & 1u) ? 0x10000u : 1u);
}
__device__ inline bool phb_event(uint32_t ab, uint32_t old) {  // did this add wrap a half?
    const uint32_t inc = (ab & 1u) ? 0x10000u : 1u, nw = old + inc;
    return nw < old || (inc == 1u && (nw & 0xFFFFu) == 0u);
}
__global__ void __launch_bounds__(PH_THREADS) zbpe_pair_hist_bytes(const uint16_t *__restrict__ tok, int64_t n, int32_t next_tok,
                                                                    Tables T, uint32_t *__restrict__ recount, DevState *st) {
    extern __shared__ __attribute__((aligned(16))) uint32_t bins[];  // PHB_WORDS words: 65,536 16-bit bins
    for (uint32_t i = threadIdx.x; i < PHB_WORDS; i += PH_THREADS) bins[i] = 0;
    __syncthreads();
    // vectors whose eight pairs all have their successor inside the stream (the loop below, no edge tests);
    // the pairs of the stream's last vector or two (successor next_tok or none) are counted at the end
    const int64_t nfull = n >= 1 ? (n - 1) / 8 : 0, nvec = (n + 7) / 8;
    const uint4 *tv = reinterpret_cast<const uint4 *>(tok);
    const int lane = threadIdx.x & 63;
    const int64_t wave = (int64_t)blockIdx.x * (PH_THREADS / 64) + (threadIdx.x >> 6);
    const int64_t waves = (int64_t)gridDim.x * (PH_THREADS / 64);
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    for (int64_t tile = wave * PH_U * 64; tile < nfull; tile += waves * PH_U * 64) {
        uint4 v[PH_U];
#pragma unroll
        for (int u = 0; u < PH_U; u++) {
            // (loaded up to the stream's end: the last full vector's successor is the next one's first token)
            const int64_t vi = tile + u * 64 + lane;
            const u32x4 y = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(tv + (vi < nvec ? vi : 0)));
            v[u] = make_uint4(y.x, y.y, y.z, y.w);
        }
        const int64_t p_last = (tile + PH_U * 64) * 8;  // the token after the tile
        const uint32_t after_tile = lane == 63 && p_last < n ? (uint32_t)tok[p_last] : 0u;
#pragma unroll
        for (int u = 0; u < PH_U; u++) {
            const int64_t vi = tile + u * 64 + lane;
            // (DPP: the next lane's first word; lane 63 the next row's lane 0, or the word after the tile)
            const uint32_t nx = wave_shl1(v[u].x, u + 1 < PH_U ? lane_bcast(v[u + 1 < PH_U ? u + 1 : u].x, 0) : after_tile);
            if (vi >= nfull) continue;
            // ab = a << 8 | b by one byte permute per pair: a pair inside a word (t0, t1) takes bytes {2, 0}
            // of it, a pair across words (t1 of w, t0 of the next) bytes {4, 2} of (next : w)
            const uint32_t w[5] = {v[u].x, v[u].y, v[u].z, v[u].w, nx};
            uint32_t ab[8], old[8];
#pragma unroll
            for (int k = 0; k < 8; k++)
                ab[k] = (k & 1) ? __builtin_amdgcn_perm(w[k / 2 + 1], w[k / 2], 0x0C0C0204u)
                                : __builtin_amdgcn_perm(w[k / 2], w[k / 2], 0x0C0C0002u);
#pragma unroll
            for (int k = 0; k < 8; k++) old[k] = phb_add(bins, ab[k]);
            bool ev = false;
#pragma unroll
            for (int k = 0; k < 8; k++) ev |= phb_event(ab[k], old[k]);
            if (__builtin_expect(ev, 0)) {
#pragma unroll
                for (int k = 0; k < 8; k++)
                    if (phb_event(ab[k], old[k])) phb_events(bins, T, recount, st, ab[k], old[k]);
            }
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // pairs starting in vectors [nfull, ...): successor next_tok or none
        for (int64_t p = nfull * 8; p < n; p++) {
            const int32_t b = p + 1 < n ? (int32_t)tok[p + 1] : next_tok;
            if (b < 0) continue;
            const uint32_t ab = ((uint32_t)tok[p] << 8) | (uint32_t)b;
            const uint32_t old = phb_add(bins, ab);
            if (phb_event(ab, old)) phb_events(bins, T, recount, st, ab, old);
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < PHB_WORDS; i += PH_THREADS) {
        const uint32_t x = bins[i];
        if (x & 0xFFFFu) phb_global(T, recount, st, phb_pair(i, 0), x & 0xFFFFu);
        if (x >> 16) phb_global(T, recount, st, phb_pair(i, 1), x >> 16);
    }
}

// (key, table count, this shard's recount) of every id, for the cross-rank comparison
__global__ void __launch_bounds__(256) zbpe_recount_dump(Tables T, const uint32_t *recount, const DevState *st, uint32_t *out) {
    const uint32_t n = min(st->num_ids, T.id_cap);
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        out[3 * i] = T.id_key[i];
        out[3 * i + 1] = T.id_cnt[i];
        out[3 * i + 2] = recount[i];
    }
}
__global__ void __launch_bounds__(256) zbpe_recount_compare(Tables T, const uint32_t *recount, DevState *st) {
    const uint32_t n = min(st->num_ids, T.id_cap);
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256)
        if (recount[i] != T.id_cnt[i]) atomicAdd(&st->mismatches, 1u);
}

// rebuild: keep live ids only (drops dead pairs so the argmax pass stays short)
__global__ void __launch_bounds__(256) zbpe_rebuild(const uint32_t *__restrict__ old_key, const uint32_t *__restrict__ old_cnt,
                                                    uint32_t old_n, Tables T, DevState *st) {
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < old_n; i += gridDim.x * 256) {
        uint32_t c = old_cnt[i];
        if (!c) continue;
        uint32_t id = atomicAdd(&st->num_ids, 1u);
        if (id >= T.id_cap) { atomicOr(&st->error, 1u); continue; }
        T.id_key[id] = old_key[i];
        T.id_cnt[id] = c;
        ht_insert_new(T, old_key[i], id);
    }
}

}  // namespace zbpe

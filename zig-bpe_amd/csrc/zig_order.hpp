// Host-side emulation of the Zig 0.13 std.HashMapUnmanaged(CharPair, usize) iteration order,
// used by the engine only when the GPU cluster test (kernels.hpp zbpe_tie_resolve) cannot decide
// a tie (two tied pairs in one probe run, or a run that wraps). The input is what the GPU computed:
// every live pair of the current stream with its first-occurrence position and count.
//
// Semantics restated from Zig 0.13 lib/std/hash_map.zig (the reference's call sites are
// basic_tokenizer.zig:265 AutoHashMap.init, :269 getOrPut, :291 iterator, :299 std.mem.sort):
//   - getOrPut calls growIfNeeded(1) before every lookup: a full table grows even when the key
//     exists, so only (a) the order of first insertions and (b) whether any getOrPut follows the
//     last insertion matter;
//   - capacity doubles from 8 (capacityForSize(max_load+1)), max_load = cap*80/100;
//   - grow re-inserts the old keys in old-slot order with linear probing;
//   - iteration is ascending slot order; the stable sort keeps that order among equal counts.
#pragma once
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>
#include <thread>
#include <vector>

namespace zbpe {

inline uint64_t host_mulhi(uint64_t a, uint64_t b) { return (uint64_t)(((unsigned __int128)a * b) >> 64); }
inline uint64_t host_mix(uint64_t a, uint64_t b) { return (a * b) ^ host_mulhi(a, b); }
inline uint64_t host_zig_pair_hash(uint32_t w) {
    const uint64_t s0 = 0xa0761d6478bd642fULL, s1 = 0xe7037ed1a0b428dbULL;
    const uint64_t seed = host_mix(s0, s1);
    uint64_t a = ((uint64_t)w << 32) | w, b = a;
    a ^= s1;
    b ^= seed;
    uint64_t lo = a * b, hi = host_mulhi(a, b);
    return host_mix(lo ^ s0 ^ 4ull, hi ^ s1);
}
inline uint64_t zig_max_load(uint64_t cap) { return cap * 80 / 100; }

// Final capacity of the Zig pair map for D distinct pairs.
inline uint64_t zig_final_capacity(uint64_t D, bool call_after_last_insert) {
    uint64_t cap = 8;
    while (zig_max_load(cap) < D) cap *= 2;
    if (zig_max_load(cap) == D && call_after_last_insert) cap *= 2;
    return cap;
}

struct ZigOrderInput {
    uint64_t first_pos;  // first-occurrence order key (multi-GPU: shard index << 32 | shard-local position)
    uint32_t key, count;
};

// One live pair for the emulation: the low 31 bits of its Zig hash (homes of every capacity up to
// 2^31), whether it is tied at the top count, and its key.
inline uint64_t zig_emu_entry(uint32_t key, bool tied) {
    return ((uint64_t)(((uint32_t)host_zig_pair_hash(key) & 0x7FFFFFFFu) | (tied ? 0x80000000u : 0u)) << 32) | key;
}

// Emulates the Zig map's life -- insertions in first-occurrence order, a grow to twice the capacity
// whenever a getOrPut finds the table full (re-inserting in old-slot order), the trailing grow when
// a getOrPut follows the last insertion -- and returns the key of the first slot (ascending) whose
// pair is tied (bit 63 of zig_emu_entry). `ins` lists the live pairs in insertion order.
//
// Level by level: the table of capacity c is built from its insertion sequence, the table of c/2 in
// slot order followed by the keys inserted after that grow. Tables hold the entries themselves (key
// 0xFFFFFFFF -- two hole tokens -- never occurs, so ~0 marks an empty slot).
//
// Large levels are built in parallel, exactly: the occupied slots of a linear-probing table do not
// depend on the insertion order (a max-plus carry over the home histogram gives them), and no probe
// ever passes a slot that is empty in the final table. Cutting the table at T such empty slots splits
// it into independent segments: each keeps exactly the keys whose homes lie in it, in their sequence
// order (a stable partition), and one thread replays first-come-first-served probing inside each.
struct ZigEmuWork {
    struct Buf {
        uint64_t *p = nullptr;
        size_t cap = 0;
        ~Buf() { delete[] p; }
        uint64_t *get(size_t n) {
            if (n > cap) {
                delete[] p;
                p = new uint64_t[n];  // uninitialised: the builders fill what they use
                cap = n;
            }
            return p;
        }
    };
    Buf tab, nxt, seq, part, cnt;  // cnt: the home histogram, two u32 per u64
};

template <typename F>
inline void zig_par_for(int T, F f) {
    std::vector<std::thread> th;
    th.reserve(T > 1 ? T - 1 : 0);
    for (int t = 1; t < T; t++) th.emplace_back(f, t);
    f(0);
    for (auto &x : th) x.join();
}

inline int zig_emu_threads() {
    if (const char *v = getenv("ZBPE_EMU_THREADS")) return std::max(1, std::min(64, atoi(v)));
    const unsigned h = std::thread::hardware_concurrency();
    int t = 1;
    while (t * 2 <= (int)std::min(16u, h ? h : 1u)) t *= 2;  // the GPU box's CPU share is 16
    return t;
}
inline size_t zig_emu_par_min() {  // levels with fewer keys are built on one thread
    if (const char *v = getenv("ZBPE_EMU_PAR_MIN")) return (size_t)strtoull(v, nullptr, 10);
    return (size_t)1 << 20;
}

constexpr uint64_t ZIG_EMPTY = ~0ull;
inline uint64_t zig_emu_home(uint64_t e, uint64_t m) { return (e >> 32) & 0x7FFFFFFFu & m; }

// FCFS linear probing of seq[0, n) into an empty table of `cap` slots, one thread
inline void zig_level_seq(const uint64_t *seq, size_t n, uint64_t *tab, uint64_t cap) {
    constexpr size_t PF = 16;
    const uint64_t m = cap - 1;
    std::fill(tab, tab + cap, ZIG_EMPTY);
    for (size_t i = 0; i < n; i++) {
        if (i + PF < n) __builtin_prefetch(&tab[zig_emu_home(seq[i + PF], m)], 1);
        uint64_t s = zig_emu_home(seq[i], m);
        while (tab[s] != ZIG_EMPTY) s = (s + 1) & m;
        tab[s] = seq[i];
    }
}

// The same in parallel (see above). Returns false (nothing done) if some chunk holds no empty slot.
inline bool zig_level_par(const uint64_t *seq, size_t n, uint64_t *tab, uint64_t cap, ZigEmuWork &w, int T) {
    const uint64_t m = cap - 1;
    auto lo_of = [&](int t) { return cap * (uint64_t)t / (uint64_t)T; };  // chunk t = slots [lo_of(t), lo_of(t + 1))
    uint32_t *cnt = reinterpret_cast<uint32_t *>(w.cnt.get(cap / 2 + 1));
    zig_par_for(T, [&](int t) { std::fill(cnt + lo_of(t), cnt + lo_of(t + 1), 0u); });
    // homes histogram
    zig_par_for(T, [&](int t) {
        const size_t a = n * t / T, b = n * (t + 1) / T;
        for (size_t i = a; i < b; i++) __atomic_fetch_add(&cnt[zig_emu_home(seq[i], m)], 1u, __ATOMIC_RELAXED);
    });
    // carry c(s+1) = max(0, c(s) + cnt[s] - 1) over each chunk as max(M, x + Q)
    std::vector<int64_t> Q(T), M(T), cin(T), cut(T);
    zig_par_for(T, [&](int t) {
        int64_t q = 0, mx = 0;  // composition of x -> max(0, x + cnt - 1)
        bool first = true;
        for (uint64_t s = lo_of(t); s < lo_of(t + 1); s++) {
            const int64_t d = (int64_t)cnt[s] - 1;
            if (first) { q = d; mx = 0; first = false; }
            else { mx = std::max<int64_t>(0, mx + d); q += d; }
        }
        Q[t] = q;
        M[t] = mx;
    });
    // the ring's carry into slot 0 is the fixed point of the whole composition (its Q < 0): its M
    int64_t Mt = M[0], Qt = Q[0];
    for (int t = 1; t < T; t++) { Mt = std::max(M[t], Mt + Q[t]); Qt += Q[t]; }
    if (Qt >= 0) return false;  // (a full table: impossible at the 80 % max load)
    int64_t x = Mt;
    for (int t = 0; t < T; t++) { cin[t] = x; x = std::max(M[t], x + Q[t]); }
    // cut t: the first slot of chunk t that is empty in the final table
    zig_par_for(T, [&](int t) {
        int64_t c = cin[t];
        cut[t] = -1;
        for (uint64_t s = lo_of(t); s < lo_of(t + 1); s++) {
            if (c + (int64_t)cnt[s] == 0) { cut[t] = (int64_t)s; break; }
            c = std::max<int64_t>(0, c + (int64_t)cnt[s] - 1);
        }
    });
    for (int t = 0; t < T; t++)
        if (cut[t] < 0) return false;
    // segment t = homes in [cut[t], cut[t+1]); the last one wraps to [cut[T-1], cap) + [0, cut[0])
    auto seg_of = [&](uint64_t h) -> int {
        int t = (int)(h * (uint64_t)T / cap);  // h in chunk t, whose cut is at or after lo_of(t)
        if ((int64_t)h < cut[t]) t = t > 0 ? t - 1 : T - 1;
        return t;
    };
    // stable partition of seq by segment: per (thread slice, segment) counts, offsets, scatter
    std::vector<size_t> pc((size_t)T * T, 0);
    zig_par_for(T, [&](int t) {
        const size_t a = n * t / T, b = n * (t + 1) / T;
        size_t *c = &pc[(size_t)t * T];
        for (size_t i = a; i < b; i++) c[seg_of(zig_emu_home(seq[i], m))]++;
    });
    std::vector<size_t> off((size_t)T * T), seg_beg(T + 1);
    size_t run = 0;
    for (int g = 0; g < T; g++) {
        seg_beg[g] = run;
        for (int t = 0; t < T; t++) { off[(size_t)t * T + g] = run; run += pc[(size_t)t * T + g]; }
    }
    seg_beg[T] = run;
    uint64_t *part = w.part.get(n + 1);
    zig_par_for(T, [&](int t) {
        const size_t a = n * t / T, b = n * (t + 1) / T;
        size_t *o = &off[(size_t)t * T];
        for (size_t i = a; i < b; i++) part[o[seg_of(zig_emu_home(seq[i], m))]++] = seq[i];
    });
    // each segment: its slots cleared, then FCFS probing of its keys (the last one wraps past cap - 1)
    zig_par_for(T, [&](int t) {
        const uint64_t lo = (uint64_t)cut[t], hi = t + 1 < T ? (uint64_t)cut[t + 1] : cap + (uint64_t)cut[0];
        for (uint64_t s = lo; s < hi; s++) tab[s & m] = ZIG_EMPTY;
        for (size_t i = seg_beg[t]; i < seg_beg[t + 1]; i++) {
            const uint64_t e = part[i];
            uint64_t s = zig_emu_home(e, m);
            while (tab[s] != ZIG_EMPTY) s = (s + 1) & m;
            tab[s] = e;
        }
    });
    return true;
}

// the non-empty slots of tab[0, cap) in slot order into out; returns their number
inline size_t zig_compact(const uint64_t *tab, uint64_t cap, uint64_t *out, int T) {
    if (T <= 1 || cap < ((uint64_t)1 << 20)) {
        size_t k = 0;
        for (uint64_t s = 0; s < cap; s++)
            if (tab[s] != ZIG_EMPTY) out[k++] = tab[s];
        return k;
    }
    auto lo_of = [&](int t) { return cap * (uint64_t)t / (uint64_t)T; };
    std::vector<size_t> c(T + 1, 0);
    zig_par_for(T, [&](int t) {
        size_t k = 0;
        for (uint64_t s = lo_of(t); s < lo_of(t + 1); s++) k += tab[s] != ZIG_EMPTY;
        c[t + 1] = k;
    });
    for (int t = 0; t < T; t++) c[t + 1] += c[t];
    zig_par_for(T, [&](int t) {
        size_t k = c[t];
        for (uint64_t s = lo_of(t); s < lo_of(t + 1); s++)
            if (tab[s] != ZIG_EMPTY) out[k++] = tab[s];
    });
    return c[T];
}

inline bool zig_emulate_first_tied(const uint64_t *ins, size_t n, bool call_after_last_insert, uint32_t *winner,
                                   ZigEmuWork &work) {
    if (n == 0) return false;
    const int T = zig_emu_threads();
    const size_t par_min = zig_emu_par_min();
    const uint64_t final_cap = zig_final_capacity(n, call_after_last_insert);
    uint64_t *seq = work.seq.get(n + 1);
    uint64_t *tab = nullptr, cap = 0;
    size_t K = 0;  // keys in the current table
    while (cap < final_cap) {
        const uint64_t c = cap ? cap * 2 : 8;
        const size_t N = std::min<size_t>(n, zig_max_load(c));
        // the insertion sequence of capacity c: the old table in slot order, then the keys inserted since
        const size_t k_old = tab ? zig_compact(tab, cap, seq, N >= par_min ? T : 1) : 0;
        if (k_old != K) return false;
        std::copy(ins + K, ins + N, seq + K);
        uint64_t *nt = (tab == work.tab.p ? work.nxt : work.tab).get(c);
        if (!(N >= par_min && T > 1 && c >= (uint64_t)T * 64 && zig_level_par(seq, N, nt, c, work, T)))
            zig_level_seq(seq, N, nt, c);
        tab = nt;
        cap = c;
        K = N;
    }
    for (uint64_t s = 0; s < cap; s++)
        if (tab[s] != ZIG_EMPTY && (tab[s] >> 63)) {
            *winner = (uint32_t)tab[s];
            return true;
        }
    return false;
}

// Returns the key of the first slot (ascending) holding a pair with count == top.
inline bool zig_order_winner(std::vector<ZigOrderInput> live, uint32_t top, bool call_after_last_insert,
                             uint32_t *winner) {
    std::sort(live.begin(), live.end(),
              [](const ZigOrderInput &x, const ZigOrderInput &y) { return x.first_pos < y.first_pos; });
    std::vector<uint64_t> ins(live.size());
    for (size_t i = 0; i < live.size(); i++) ins[i] = zig_emu_entry(live[i].key, live[i].count == top);
    static thread_local ZigEmuWork work;  // reused across calls, like the engine's (the host tests call this many times)
    return zig_emulate_first_tied(ins.data(), ins.size(), call_after_last_insert, winner, work);
}

}  // namespace zbpe

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
#include <algorithm>
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
// The table holds the entries themselves, so a grow re-inserts from the old table in slot order: the
// new homes of consecutive old slots are two sequential streams (h, h + cap), and only the new
// insertions hit random slots, which are prefetched a few keys ahead. Key 0xFFFFFFFF (two hole
// tokens) never occurs, so ~0 marks an empty slot.
inline bool zig_emulate_first_tied(const uint64_t *ins, size_t n, bool call_after_last_insert, uint32_t *winner) {
    constexpr uint64_t EMPTY = ~0ull;
    constexpr size_t PF = 16;
    std::vector<uint64_t> tab, old;
    uint64_t cap = 0, avail = 0, size = 0;
    auto place = [&](uint64_t e) {
        const uint64_t m = cap - 1;
        uint64_t s = (e >> 32) & 0x7FFFFFFFu & m;
        while (tab[s] != EMPTY) s = (s + 1) & m;
        tab[s] = e;
    };
    auto grow = [&](uint64_t nc) {
        old.swap(tab);
        tab.assign(nc, EMPTY);
        cap = nc;
        for (uint64_t e : old)
            if (e != EMPTY) place(e);
        avail = zig_max_load(cap) - size;
    };
    for (size_t i = 0; i < n; i++) {
        if (avail == 0) grow(cap ? cap * 2 : 8);
        if (i + PF < n) __builtin_prefetch(&tab[(ins[i + PF] >> 32) & 0x7FFFFFFFu & (cap - 1)], 1);
        place(ins[i]);
        avail--;
        size++;
    }
    if (avail == 0 && call_after_last_insert) grow(cap * 2);
    for (uint64_t e : tab)
        if (e != EMPTY && (e >> 63)) {
            *winner = (uint32_t)e;
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
    return zig_emulate_first_tied(ins.data(), ins.size(), call_after_last_insert, winner);
}

}  // namespace zbpe

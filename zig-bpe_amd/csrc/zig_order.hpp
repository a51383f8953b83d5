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

// Returns the key of the first slot (ascending) holding a pair with count == top.
inline bool zig_order_winner(std::vector<ZigOrderInput> live, uint32_t top, bool call_after_last_insert,
                             uint32_t *winner) {
    std::sort(live.begin(), live.end(),
              [](const ZigOrderInput &x, const ZigOrderInput &y) { return x.first_pos < y.first_pos; });
    uint64_t cap = 0, avail = 0;
    std::vector<uint32_t> key, idx;  // idx: index into live, or UINT32_MAX when empty
    auto place = [&](uint32_t i) {
        uint64_t m = cap - 1, s = host_zig_pair_hash(live[i].key) & m;
        while (idx[s] != UINT32_MAX) s = (s + 1) & m;
        idx[s] = i;
        avail--;
    };
    auto grow = [&](uint64_t nc) {
        std::vector<uint32_t> old = std::move(idx);
        cap = nc;
        idx.assign(cap, UINT32_MAX);
        avail = zig_max_load(cap);
        for (uint32_t i : old)
            if (i != UINT32_MAX) place(i);
    };
    for (uint32_t i = 0; i < live.size(); i++) {
        if (avail == 0) grow(cap ? cap * 2 : 8);
        place(i);
    }
    if (avail == 0 && call_after_last_insert) grow(cap * 2);
    for (uint64_t s = 0; s < cap; s++)
        if (idx[s] != UINT32_MAX && live[idx[s]].count == top) {
            *winner = live[idx[s]].key;
            return true;
        }
    return false;
}

}  // namespace zbpe

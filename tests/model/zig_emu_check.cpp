// Test infrastructure: the parallel level builder of the exact Zig-order emulation
// (zig-bpe_amd/csrc/zig_order.hpp, zig_level_par) must build the same table, slot for slot, as the
// one-thread first-come-first-served replay (zig_level_seq), for random insertion sequences at the
// map's real loads (up to 80 %) and for several thread counts.
//   build: g++ -O2 -std=c++17 -pthread -o zig_emu_check zig_emu_check.cpp
#include <cstdio>
#include <random>

#include "../../zig-bpe_amd/csrc/zig_order.hpp"

int main() {
    using namespace zbpe;
    std::mt19937_64 rng(12345);
    int bad = 0, runs = 0, par_runs = 0;
    for (uint64_t cap : {1ull << 12, 1ull << 16, 1ull << 20}) {
        for (double load : {0.30, 0.55, 0.80}) {
            for (int T : {2, 4, 8, 16}) {
                const size_t n = (size_t)(zig_max_load(cap) * load / 0.80);
                std::vector<uint64_t> seq(n);
                for (auto &e : seq) e = zig_emu_entry((uint32_t)rng(), (rng() & 7) == 0);
                std::vector<uint64_t> a(cap), b(cap);
                ZigEmuWork w;
                zig_level_seq(seq.data(), n, a.data(), cap);
                const bool par = zig_level_par(seq.data(), n, b.data(), cap, w, T);
                runs++;
                if (!par) continue;  // (a chunk without an empty slot: the engine falls back to the replay)
                par_runs++;
                if (a != b) {
                    bad++;
                    fprintf(stderr, "mismatch: cap %llu load %.2f threads %d\n", (unsigned long long)cap, load, T);
                }
            }
        }
    }
    printf("%d runs, %d parallel, %d mismatches\n", runs, par_runs, bad);
    return bad || par_runs < runs / 2 ? 1 : 0;
}

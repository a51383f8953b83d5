// Design-validation model (test infrastructure, never shipped): the incremental pair-count
// algorithm used by the HIP engine, run on the CPU so its delta rules and the Zig-order tie
// fast path can be checked against the oracle before they are written as kernels.
//   build: g++ -O2 -std=c++17 -o inc_model inc_model.cpp
//   run:   ./inc_model <corpus file> <vocab> [check_fast 0/1] [max_merges]  -> merges on stdout, stats on stderr
// Also the algorithm-matched CPU baseline of bench.py (one core, -O3): the same incremental counting as
// the device, with a pass over the stream per merge to find the occurrences, timed on C4's first merges.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <unordered_map>
#include <vector>
#include <algorithm>
#include <chrono>

static const uint16_t HOLE = 0xFFFF;
static inline void mum(uint64_t &a, uint64_t &b) { __uint128_t x = (__uint128_t)a * b; a = (uint64_t)x; b = (uint64_t)(x >> 64); }
static inline uint64_t mix(uint64_t a, uint64_t b) { mum(a, b); return a ^ b; }
static uint64_t pair_hash(uint32_t w) {  // Wyhash(0, 4 bytes)
    const uint64_t s0 = 0xa0761d6478bd642fULL, s1 = 0xe7037ed1a0b428dbULL;
    uint64_t seed = 0 ^ mix(0 ^ s0, s1);
    uint64_t a = ((uint64_t)w << 32) | w, b = a;
    a ^= s1; b ^= seed; mum(a, b);
    return mix(a ^ s0 ^ 4ULL, b ^ s1);
}
static uint32_t max_load(uint64_t cap) { return (uint32_t)(cap * 80 / 100); }

struct Model {
    std::vector<uint16_t> tok;
    std::unordered_map<uint32_t, int64_t> cnt;  // key -> count (0 = dead)
    int64_t D = 0;
    uint64_t fallbacks = 0, ties = 0, max_ids = 0, new_keys_total = 0, compactions = 0, holes = 0;

    long prev_live(long i) { for (long k = i - 1; k >= 0; k--) if (tok[k] != HOLE) return k; return -1; }
    long next_live(long i) { for (long k = i + 1; k < (long)tok.size(); k++) if (tok[k] != HOLE) return k; return -1; }
    void add(uint32_t key, int64_t d) {
        int64_t &c = cnt[key];
        int64_t o = c; c += d;
        if (o == 0 && c > 0) D++;
        if (o > 0 && c == 0) D--;
        if (c < 0) { fprintf(stderr, "negative count\n"); exit(3); }
    }
    void compact() {
        size_t j = 0;
        for (size_t i = 0; i < tok.size(); i++) if (tok[i] != HOLE) tok[j++] = tok[i];
        tok.resize(j); holes = 0; compactions++;
    }
    // Exact Zig order: emulate insertion of live keys in first-occurrence order.
    uint32_t exact_winner(uint64_t top) {
        std::vector<uint32_t> order; std::unordered_map<uint32_t, char> seen;
        long i = next_live(-1);
        long last_pos = -1; uint32_t last_key = 0;
        while (i >= 0) { long j = next_live(i); if (j < 0) break;
            uint32_t k = tok[i] | ((uint32_t)tok[j] << 16);
            if (!seen.count(k)) { seen[k] = 1; order.push_back(k); }
            last_key = k; last_pos = i; i = j; }
        (void)last_pos;
        // emulate grow history
        uint64_t cap = 0; uint32_t avail = 0; std::vector<uint32_t> slots; std::vector<char> used;
        auto insert = [&](uint32_t k) {
            uint64_t m = cap - 1, s = pair_hash(k) & m;
            while (used[s]) s = (s + 1) & m;
            used[s] = 1; slots[s] = k; avail--;
        };
        for (size_t q = 0; q < order.size(); q++) {
            if (avail == 0) {
                uint64_t nc = cap ? cap * 2 : 8;
                std::vector<uint32_t> os = slots; std::vector<char> ou = used; uint64_t oc = cap;
                cap = nc; slots.assign(cap, 0); used.assign(cap, 0); avail = max_load(cap);
                for (uint64_t s = 0; s < oc; s++) if (ou[s]) insert(os[s]);
            }
            insert(order[q]);
        }
        // trailing grow: last call found an existing key while avail == 0
        if (avail == 0 && cnt[last_key] >= 2) {
            std::vector<uint32_t> os = slots; std::vector<char> ou = used; uint64_t oc = cap;
            cap *= 2; slots.assign(cap, 0); used.assign(cap, 0); avail = max_load(cap);
            for (uint64_t s = 0; s < oc; s++) if (ou[s]) insert(os[s]);
        }
        for (uint64_t s = 0; s < cap; s++) if (used[s] && (uint64_t)cnt[slots[s]] == top) return slots[s];
        fprintf(stderr, "exact_winner failed\n"); exit(4);
    }
    // Fast path: occupancy of the final Zig table is order independent.
    bool fast_winner(uint64_t top, uint32_t &win) {
        long a0 = -1, a1 = -1;  // last two live positions
        for (long k = (long)tok.size() - 1; k >= 0 && a0 < 0; k--) if (tok[k] != HOLE) { if (a1 < 0) a1 = k; else a0 = k; }
        uint32_t lastkey = tok[a0] | ((uint32_t)tok[a1] << 16);
        uint64_t cap = 8; while (max_load(cap) < (uint64_t)D) cap *= 2;
        if (max_load(cap) == (uint64_t)D && cnt[lastkey] >= 2) cap *= 2;
        std::vector<char> occ(cap, 0); uint64_t m = cap - 1;
        uint64_t h1 = UINT64_MAX, h2 = UINT64_MAX, hmax = 0; uint32_t k1 = 0;
        for (auto &kv : cnt) if (kv.second > 0) {
            uint64_t h = pair_hash(kv.first) & m, s = h;
            while (occ[s]) s = (s + 1) & m;
            occ[s] = 1;
            if ((uint64_t)kv.second == top) {
                if (h < h1) { h2 = h1; h1 = h; k1 = kv.first; } else if (h < h2) h2 = h;
                hmax = std::max(hmax, h);
            }
        }
        // same cluster?  no free slot in [h1, h2]
        uint64_t f = h1; while (f < cap && occ[f]) f++;
        if (f == cap) return false;            // cluster of h1 runs into the wrap
        if (h2 != UINT64_MAX && f > h2) return false;
        if (occ[cap - 1] && occ[0]) {           // wrap cluster: its tail may wrap below h1
            uint64_t sw = cap - 1; while (sw > 0 && occ[sw - 1]) sw--;
            if (hmax >= sw) return false;
        }
        win = k1; return true;
    }
};

int main(int argc, char **argv) {
    if (argc < 3) return 1;
    FILE *f = fopen(argv[1], "rb"); if (!f) return 1;
    std::vector<uint8_t> text;
    { uint8_t buf[1 << 16]; size_t k; while ((k = fread(buf, 1, sizeof buf, f)) > 0) text.insert(text.end(), buf, buf + k); }
    fclose(f);
    auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    const double t_start = now();
    int V = atoi(argv[2]); int check_fast = argc > 3 ? atoi(argv[3]) : 1;
    long max_merges = argc > 4 ? atol(argv[4]) : 0;
    if (max_merges > 0 && 256 + max_merges < V) V = (int)(256 + max_merges);
    Model M; M.tok.assign(text.begin(), text.end());
    {  // initial counts: byte pairs in a dense histogram, then into the map
        std::vector<int64_t> h(65536, 0);
        for (size_t i = 0; i + 1 < text.size(); i++) h[text[i] | (text[i + 1] << 8)]++;
        for (uint32_t p = 0; p < 65536; p++) if (h[p]) M.add((p & 0xFF) | ((p >> 8) << 16), h[p]);
    }
    const double t_init = now();
    std::vector<int64_t> left(65536), right(65536);
    for (int X = 256; X < V; X++) {
        if (M.D == 0) { fprintf(stderr, "No more pairs to merge. Stopping early.\n"); break; }
        uint64_t top = 0, nt = 0; uint32_t win = 0;
        for (auto &kv : M.cnt) if (kv.second > 0) { if ((uint64_t)kv.second > top) { top = kv.second; nt = 1; win = kv.first; } else if ((uint64_t)kv.second == top) nt++; }
        if (nt > 1) {
            M.ties++;
            uint32_t ex = M.exact_winner(top), fw;
            if (check_fast) { if (M.fast_winner(top, fw)) { if (fw != ex) { fprintf(stderr, "FAST PATH WRONG at %d\n", X); return 5; } } else M.fallbacks++; }
            win = ex;
        }
        uint16_t a = win & 0xFFFF, b = win >> 16;
        printf("%u,%u,%d\n", a, b, X);
        if (a == b && M.holes) M.compact();
        int64_t xx = 0, occs = 0;
        std::vector<std::pair<long, long>> rec;
        long n = (long)M.tok.size();
        if (a != b) {
            for (long i = 0; i < n; i++) {
                if (M.tok[i] != a) continue;
                long j = M.next_live(i); if (j < 0 || M.tok[j] != b) continue;
                occs++;
                long l = M.prev_live(i);
                if (l >= 0) { bool me = false; if (M.tok[l] == b) { long pl = M.prev_live(l); me = pl >= 0 && M.tok[pl] == a; }
                              if (!me) left[M.tok[l]]++; }
                long r = M.next_live(j);
                if (r >= 0) { bool ro = false; if (M.tok[r] == a) { long rn = M.next_live(r); ro = rn >= 0 && M.tok[rn] == b; }
                              if (ro) xx++; else right[M.tok[r]]++; }
                rec.push_back({i, j});
            }
        } else {
            long rs = -1;
            for (long i = 0; i < n; i++) {
                if (M.tok[i] != a) { rs = -1; continue; }
                if (rs < 0) rs = i;
                if (((i - rs) & 1) || i + 1 >= n || M.tok[i + 1] != a) continue;
                occs++;
                if (i == rs && i > 0) left[M.tok[i - 1]]++;
                if (i + 2 < n) { bool ro = M.tok[i + 2] == a && i + 3 < n && M.tok[i + 3] == a; if (ro) xx++; else right[M.tok[i + 2]]++; }
                rec.push_back({i, i + 1});
            }
        }
        for (auto &p : rec) { M.tok[p.first] = (uint16_t)X; M.tok[p.second] = HOLE; }
        M.holes += rec.size();
        M.add(win, -occs);
        uint64_t newk = 0;
        for (int t = 0; t < X; t++) {
            if (left[t]) { M.add(t | ((uint32_t)a << 16), -left[t]); M.add(t | ((uint32_t)X << 16), left[t]); left[t] = 0; newk++; }
            if (right[t]) { M.add(b | ((uint32_t)t << 16), -right[t]); M.add(X | ((uint32_t)t << 16), right[t]); right[t] = 0; newk++; }
        }
        if (xx) { M.add(b | ((uint32_t)a << 16), -xx); M.add(X | ((uint32_t)X << 16), xx); newk++; }
        M.new_keys_total += newk;
        if (M.cnt[win] != 0) { fprintf(stderr, "top pair not zero after merge\n"); return 6; }
        M.max_ids = std::max<uint64_t>(M.max_ids, M.cnt.size());
        if (M.holes * 8 > M.tok.size()) M.compact();
        if ((X & 1023) == 0) fprintf(stderr, "X=%d D=%lld ids=%zu top=%llu n=%zu\n", X, (long long)M.D, M.cnt.size(), (unsigned long long)top, M.tok.size() - M.holes);
    }
    fprintf(stderr, "timing: init_s=%.3f merges_s=%.3f\n", t_init - t_start, now() - t_init);
    fprintf(stderr, "ties=%llu fallbacks=%llu D=%lld ids=%zu new_keys=%llu compactions=%llu\n", (unsigned long long)M.ties,
            (unsigned long long)M.fallbacks, (long long)M.D, M.cnt.size(), (unsigned long long)M.new_keys_total, (unsigned long long)M.compactions);
    return 0;
}

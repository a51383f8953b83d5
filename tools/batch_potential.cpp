// How many merges could share one scan -> replace -> select round? (design study for multi-merge rounds)
//
// Runs the fast CPU oracle (oracle/zig_fast.cpp, included) and, before every merge, records its footprint
// (the positions of every left-greedy occurrence and of its left and right neighbours), the neighbour-token
// histograms the device's scan produces (left[L], right[R]), the largest count a new pair of the merge gets,
// and the Zig map capacity / home slot of the tied pairs. Then it greedily groups consecutive merges into
// rounds of at most K merges, under two rules:
//   exact:        merge j joins the round when it had the leader's top count and was tied with it at the
//                 leader (so the leader's select could name it), its occurrences touch no earlier member's
//                 footprint, no earlier member made a pair with the top count, and the map capacity is the
//                 same at every member;
//   conservative: the same, with "touches" replaced by what the device can check from the earlier members'
//                 delta histograms alone: right_i[first_j] == 0 and left_i[second_j] == 0 (no occurrence of
//                 member i is followed by first_j or preceded by second_j), and member j's key is the next
//                 home slot among the leader's tied pairs.
// Build: g++ -O3 -std=c++17 -pthread -o /tmp/batch_potential tools/batch_potential.cpp
// Run:   /tmp/batch_potential corpus.bin vocab [K] [from_merge] [tied_winners.txt]
#include "../oracle/zig_fast.cpp"

#include <map>
#include <set>
#include <unordered_set>

namespace {
struct MergeInfo {
    uint32_t key = 0, T = 0, ties = 0, cap = 0, max_new = 0;
    bool self = false, ok = true;
    std::vector<uint32_t> tied_keys_by_home;  // the tied pairs' keys in home-slot order (then first occurrence)
    std::unordered_set<uint32_t> foot;        // L, p, q, R of every occurrence (pre-merge positions)
    std::vector<uint32_t> occ_p, occ_q;       // occurrence positions
    std::map<uint32_t, uint32_t> left, right; // neighbour token histograms
};
std::vector<MergeInfo> g_info;
uint32_t g_from = 0;  // merges before it are not recorded (their footprints would not fit in memory at C4)
bool g_stream = false;  // pair rule only: keep just the previous merge (no footprint history)

// Pair rounds as the device can decide them (streaming, greedy): merge k-1 leads, merge k joins when k-1 was
// tied and not self, k's key is the tied pair with the 2nd-smallest home (strictly between the 1st and 3rd),
// k-1's new pairs stay below the top count, capacity is unchanged and no occurrence of k touches k-1's
// footprint (the scan can test that exactly from two neighbours on each side).
struct PairStats {
    uint64_t leaders = 0, paired = 0, not_tied = 0, self = 0, not_second = 0, same_home = 0, new_top = 0, cap = 0,
             touch = 0, wrong = 0, merges = 0;
    std::map<uint32_t, uint64_t> by_band;  // merges paired per 4096-merge band
} g_pair;
MergeInfo g_prev;
bool g_prev_valid = false, g_prev_member2 = false;

void pair_rule(uint32_t k, const MergeInfo &m);

void hook(Trainer &t, uint32_t k, uint32_t win, uint32_t T, const std::vector<uint32_t> &tied) {
    if (g_info.size() <= k) g_info.resize(k + 1);
    if (k < g_from) return;
    MergeInfo m;
    m.key = t.pkey[win];
    m.T = T;
    m.ties = (uint32_t)tied.size();
    const uint16_t a = (uint16_t)m.key, b = (uint16_t)(m.key >> 16);
    m.self = a == b;
    m.cap = zig_final_capacity(t.n_live, t.extra_lookup());
    std::vector<std::pair<uint64_t, uint32_t>> hk;
    for (uint32_t id : tied) hk.push_back({(zig_hash(t.pkey[id]) & (m.cap - 1)) << 32 | t.pfo[id], t.pkey[id]});
    std::sort(hk.begin(), hk.end());
    for (auto &x : hk) m.tied_keys_by_home.push_back(x.second);
    // occurrences, left-greedy (a consumed position is skipped), read-only
    const uint32_t *L0 = t.arena + t.poff[win];
    uint32_t last_q = NONE;
    std::map<uint32_t, uint32_t> lcnt, rcnt;
    for (uint32_t e = t.pcur[win]; e < t.plen[win]; e++) {
        uint32_t p = L0[e];
        if (!t.entry_live(m.key, p) || p == last_q) continue;
        uint32_t q = t.nxt[p], L = t.prv[p], R = t.nxt[q];
        m.occ_p.push_back(p);
        m.occ_q.push_back(q);
        m.foot.insert(p);
        m.foot.insert(q);
        if (L != NONE) { m.foot.insert(L); m.left[t.tok[L]]++; }
        if (R != NONE) { m.foot.insert(R); m.right[t.tok[R]]++; }
        last_q = q;
    }
    for (auto &x : m.left) m.max_new = std::max(m.max_new, x.second);
    for (auto &x : m.right) m.max_new = std::max(m.max_new, x.second);
    if (g_stream) { pair_rule(k, m); g_prev = std::move(m); g_prev_valid = true; return; }
    if (g_info.size() <= k) g_info.resize(k + 1);
    g_info[k] = std::move(m);
}

bool touches(const MergeInfo &i, const MergeInfo &j) {
    for (size_t o = 0; o < j.occ_p.size(); o++)
        if (i.foot.count(j.occ_p[o]) || i.foot.count(j.occ_q[o])) return true;
    return false;
}
bool token_clash(const MergeInfo &i, const MergeInfo &j) {
    const uint32_t c = j.key & 0xFFFF, d = j.key >> 16;
    auto has = [](const std::map<uint32_t, uint32_t> &h, uint32_t t) { auto it = h.find(t); return it != h.end() && it->second; };
    return has(i.right, c) || has(i.left, d);
}
void pair_rule(uint32_t k, const MergeInfo &m) {
    g_pair.merges++;
    if (!g_prev_valid || g_prev_member2) { g_prev_member2 = false; g_pair.leaders++; return; }
    const MergeInfo &l = g_prev;
    auto fail = [&](uint64_t &c) { c++; g_pair.leaders++; g_prev_member2 = false; };
    if (l.ties < 2) return fail(g_pair.not_tied);
    if (l.self || m.self) return fail(g_pair.self);
    if (l.tied_keys_by_home.size() < 2 || l.tied_keys_by_home[1] != m.key) {
        // the device would predict tied_keys_by_home[1]; it is only wrong if the checks below pass
        return fail(g_pair.not_second);
    }
    auto home = [&](uint32_t key) { return zig_hash(key) & (l.cap - 1); };
    const auto &tk = l.tied_keys_by_home;
    if (home(tk[0]) == home(tk[1]) || (tk.size() > 2 && home(tk[1]) == home(tk[2]))) return fail(g_pair.same_home);
    if (l.max_new >= l.T || m.T != l.T) return fail(g_pair.new_top);
    if (m.cap != l.cap) return fail(g_pair.cap);
    if (touches(l, m)) return fail(g_pair.touch);
    g_pair.paired++;
    g_pair.by_band[k / 4096]++;
    g_prev_member2 = true;
}
}  // namespace

int main(int argc, char **argv) {
    if (argc < 3) { fprintf(stderr, "usage: %s corpus.bin vocab [K] [from]\n", argv[0]); return 1; }
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 1;
    fseek(f, 0, SEEK_END);
    size_t n = ftell(f);
    fseek(f, 0, SEEK_SET);
    std::vector<uint8_t> text(n);
    if (fread(text.data(), 1, n, f) != n) return 1;
    fclose(f);
    const uint32_t vocab = atoi(argv[2]);
    const int K = argc > 3 ? atoi(argv[3]) : 4;
    const uint32_t from = argc > 4 ? atoi(argv[4]) : 0;
    g_from = from;
    g_stream = K == 2 && getenv("PAIR_STREAM");
    Log log;
    std::vector<Override> ov;
    // optional: the tied merges' winners from a verified golden ("k key" lines), taken without a replay
    if (argc > 5) {
        FILE *o = fopen(argv[5], "r");
        unsigned k, key;
        while (o && fscanf(o, "%u %u", &k, &key) == 2) ov.push_back(Override{k, key});
        if (o) fclose(o);
    }
    Trainer t;
    t.text = text.data();
    t.n = n;
    t.vocab = vocab;
    t.threads = 8;
    t.fnv_every = 0;
    t.sync_limit = ~0ULL;
    t.log = &log;
    t.overrides = &ov;
    const size_t M = vocab - 256;
    std::vector<uint16_t> tri(3 * M);
    std::vector<uint64_t> cnt(M), lens(M);
    std::vector<uint32_t> ties(M), dist(M);
    t.out_triples = tri.data();
    t.out_counts = cnt.data();
    t.out_ties = ties.data();
    t.out_distinct = dist.data();
    t.out_len_after = lens.data();
    t.pre_apply = hook;
    t.no_replay = !ov.empty();
    if (t.run(nullptr) != 0) { fprintf(stderr, "oracle run failed\n"); return 2; }
    const uint32_t m = t.merges_done;
    if (g_stream) {
        const PairStats &P = g_pair;
        printf("device pair rule, merges %u..%u: %llu merges in %llu rounds = %.3f merges/round\n", from, m,
               (unsigned long long)(P.merges), (unsigned long long)P.leaders, (double)P.merges / P.leaders);
        printf("  leader not paired because: not tied %llu, self %llu, next merge not the 2nd home %llu, equal homes %llu, "
               "new pair at the top count %llu, capacity %llu, footprints touch %llu\n",
               (unsigned long long)P.not_tied, (unsigned long long)P.self, (unsigned long long)P.not_second,
               (unsigned long long)P.same_home, (unsigned long long)P.new_top, (unsigned long long)P.cap, (unsigned long long)P.touch);
        printf("  paired merges per 4096-merge band:");
        for (auto &x : P.by_band) printf(" %u:%llu", x.first * 4096, (unsigned long long)x.second);
        printf("\n");
        return 0;
    }
    for (int rule = 0; rule < 3; rule++) {  // 2: exact, but only rounds whose leader's tie set has exactly two pairs
        uint64_t rounds = 0, merges = 0;
        std::map<int, uint64_t> sizes;
        uint32_t k = from;
        while (k < m) {
            const MergeInfo &lead = g_info[k];
            std::vector<uint32_t> members{k};
            uint32_t j = k + 1;
            size_t next_home = 1;  // conservative: the leader's tied pairs in home order
            while ((int)members.size() < (rule == 2 ? 2 : K) && j < m && !lead.self && lead.ties > 1 && (rule != 2 || lead.ties == 2)) {
                const MergeInfo &c = g_info[j];
                if (c.self || c.T != lead.T || c.cap != lead.cap) break;
                bool was_tied = std::find(lead.tied_keys_by_home.begin(), lead.tied_keys_by_home.end(), c.key) != lead.tied_keys_by_home.end();
                if (!was_tied) break;
                bool ok = true;
                for (uint32_t i : members) {
                    const MergeInfo &mi = g_info[i];
                    if (mi.max_new >= lead.T) ok = false;
                    if (rule != 1 && touches(mi, c)) ok = false;
                    if (rule == 1 && token_clash(mi, c)) ok = false;
                }
                if (rule == 1) {
                    while (next_home < lead.tied_keys_by_home.size() && lead.tied_keys_by_home[next_home] != c.key) next_home++;
                    if (next_home != members.size()) ok = false;  // not the next home in order: a pair in between left
                    next_home = members.size() + 1;
                }
                if (!ok) break;
                members.push_back(j++);
            }
            rounds++;
            merges += members.size();
            sizes[(int)members.size()]++;
            k += (uint32_t)members.size();
        }
        printf("%s rule, K=%d, merges %u..%u: %llu merges in %llu rounds = %.3f merges/round; sizes:", rule == 2 ? "exact-two-tied" : rule ? "conservative" : "exact", rule == 2 ? 2 : K,
               from, m, (unsigned long long)merges, (unsigned long long)rounds, (double)merges / rounds);
        for (auto &x : sizes) printf(" %d:%llu", x.first, (unsigned long long)x.second);
        printf("\n");
    }
    return 0;
}

/*
 * oracle/zig_fast.cpp -- TEST INFRASTRUCTURE ONLY (a parity checker, never the product).
 *
 * A second CPU restatement of BasicTokenizer.train (/root/reference/src/basic_tokenizer.zig:140-306),
 * fast enough to run C4 (1 GiB, vocab 32000) to the end in the 8-core build container, so the
 * headline workload gets an unconditional full-sequence golden.  It shares no code with the product
 * (zig-bpe_amd/) and none with its tie shortcut; it shares the Zig 0.13 hash arithmetic with
 * oracle/zig_ref.c (restated below, cross-checked by zfast_selftest against zref_pair_hash).
 *
 * What it computes is what the literal loop computes, by other means:
 *
 *  - counts (countCodePointPairs, :257-278): a pair table updated exactly per merge.  Every pair's
 *    occurrences come into existence at one merge (a merge only makes pairs with its new token), so a
 *    pair's occurrence list is written once, in position order, and only ever loses entries; an
 *    entry is live while tok[p] == first && tok[next(p)] == second (once false it stays false).
 *    The stream is a doubly linked list over the original positions (no compaction), so positions
 *    keep their order and each pair's first occurrence is the first live entry of its list.
 *  - the winner (sortCodePointPairs + [0], :280-306, :193): the largest count; among equal counts
 *    the first in std.AutoHashMap slot order.  At EVERY tied merge the map is rebuilt literally: the
 *    live pairs are inserted in first-occurrence order (the order countCodePointPairs inserts them)
 *    into a restated HashMapUnmanaged -- growIfNeeded(1) before every insert, grow() re-inserting in
 *    old slot order, linear probing, and the one extra grow when a getOrPut of an existing key
 *    follows the last insertion -- and the tied key in the lowest slot wins.  No cluster or
 *    home-slot shortcut decides anything.
 *  - replaceTopPairWithNewToken (:207-232): the top pair's live entries in position order are exactly
 *    the left-greedy matches (a consumed position is a hole, so its entry is dead).
 *
 * Speed: with small maps (D <= sync_limit) the replay runs before the merge is applied.  With large
 * maps the loop goes on with a predicted winner (smallest Zig home slot) while worker threads replay
 * the map from a snapshot; a replay that disagrees stops the run, and the run restarts from the raw
 * bytes with that merge's winner fixed (an "override"), so every decision in the final output was
 * made or confirmed by a literal replay.
 *
 * Progress log (zfast_train): one line per merge "k first second new count ties distinct len_after"
 * (the same fields as zref_train_log), "fnv k len hex" every fnv_every merges, "tie k ok|MISMATCH ..."
 * per verified tie, "restart k key" when an override is added, "done m len hex" at the end.
 */
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include <sys/mman.h>

#ifndef ZFAST_PF
#define ZFAST_PF 32
#endif

namespace {

constexpr uint16_t HOLE = 0xFFFF;
constexpr uint32_t NONE = 0xFFFFFFFFu;
constexpr uint32_t EMPTY_KEY = 0xFFFFFFFFu;

/* ---------------------------------------------------------------------------------------------- */
/* Zig 0.13: Wyhash.hash(0, bytes of CharPair{first, second}) and HashMapUnmanaged sizing          */
/* (the arithmetic of oracle/zig_ref.c key_hash / capacity_for_size / zmap_max_load)              */
/* ---------------------------------------------------------------------------------------------- */
inline void mum(uint64_t &a, uint64_t &b) {
    __uint128_t x = (__uint128_t)a * b;
    a = (uint64_t)x;
    b = (uint64_t)(x >> 64);
}
inline uint64_t mix(uint64_t a, uint64_t b) { mum(a, b); return a ^ b; }
constexpr uint64_t S0 = 0xa0761d6478bd642fULL, S1 = 0xe7037ed1a0b428dbULL;

inline uint64_t zig_hash(uint32_t key) { /* key = first | second << 16: the 4 little-endian bytes */
    static const uint64_t seed_state = mix(S0, S1);
    uint64_t w = (uint64_t)key << 32 | key;
    uint64_t a = w ^ S1, b = w ^ seed_state;
    mum(a, b);
    return mix(a ^ S0 ^ 4u, b ^ S1);
}
inline uint32_t zig_max_load(uint32_t cap) { return (uint32_t)((uint64_t)cap * 80 / 100); }
inline uint32_t zig_cap_for_size(uint32_t size) {
    uint64_t want = (uint64_t)size * 100 / 80 + 1, p = 1;
    while (p < want) p <<= 1;
    return (uint32_t)p;
}

/* Capacity after inserting d distinct keys (plus the extra grow), without building the table. */
uint32_t zig_final_capacity(uint64_t d, bool extra_lookup) {
    uint32_t cap = 0, avail = 0;
    uint64_t size = 0;
    while (size < d) {
        if (avail < 1) {
            uint32_t nc = zig_cap_for_size((uint32_t)size + 1);
            if (nc < 8) nc = 8;
            avail = zig_max_load(nc) - (uint32_t)size;
            cap = nc;
        }
        uint64_t take = std::min<uint64_t>(avail, d - size);
        size += take;
        avail -= (uint32_t)take;
    }
    if (extra_lookup && avail < 1) cap = std::max<uint32_t>(zig_cap_for_size((uint32_t)size + 1), 8);
    return cap;
}

/* Buffers on 2 MiB pages: the replay table and the stream arrays are accessed at random, and with
 * 4 KiB pages nearly every access is also a TLB miss. */
template <class T>
struct HBuf {
    T *p = nullptr;
    size_t n = 0, bytes = 0;
    HBuf() = default;
    explicit HBuf(size_t cnt) { alloc(cnt); }
    HBuf(const HBuf &) = delete;
    HBuf &operator=(const HBuf &) = delete;
    HBuf(HBuf &&o) noexcept { *this = std::move(o); }
    HBuf &operator=(HBuf &&o) noexcept {
        release();
        p = o.p; n = o.n; bytes = o.bytes; mapped = o.mapped;
        o.p = nullptr; o.n = o.bytes = 0;
        return *this;
    }
    ~HBuf() { release(); }
    bool mapped = false;
    void alloc(size_t cnt) {
        release();
        n = cnt;
        size_t want = cnt * sizeof(T);
        if (want < (8u << 20)) { /* small: the heap (a fresh mapping per snapshot costs more) */
            bytes = want ? want : sizeof(T);
            p = (T *)malloc(bytes);
            if (!p) { fprintf(stderr, "zig_fast: malloc %zu bytes failed\n", bytes); abort(); }
            mapped = false;
            return;
        }
        const size_t H = 2u << 20;
        bytes = (want + H - 1) & ~(H - 1);
        /* map one extra huge page and trim, so the buffer starts on a 2 MiB boundary */
        char *m = (char *)mmap(nullptr, bytes + H, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
        if (m == MAP_FAILED) { fprintf(stderr, "zig_fast: mmap %zu bytes failed\n", bytes); abort(); }
        char *a = (char *)(((uintptr_t)m + H - 1) & ~(uintptr_t)(H - 1));
        if (a > m) munmap(m, a - m);
        if (a + bytes < m + bytes + H) munmap(a + bytes, (m + bytes + H) - (a + bytes));
        madvise(a, bytes, MADV_HUGEPAGE);
        p = (T *)a;
        mapped = true;
    }
    void release() {
        if (p) {
            if (mapped) munmap(p, bytes);
            else free(p);
        }
        p = nullptr;
        n = bytes = 0;
    }
    T &operator[](size_t i) { return p[i]; }
    const T &operator[](size_t i) const { return p[i]; }
    T *data() { return p; }
    const T *data() const { return p; }
    size_t size() const { return n; }
};

/* ---------------------------------------------------------------------------------------------- */
/* literal map replay                                                                              */
/* ---------------------------------------------------------------------------------------------- */
struct ReplayResult {
    uint32_t winner;     /* tied key in the lowest slot */
    uint32_t slot;       /* its slot */
    uint32_t cap;        /* final capacity */
};

/* The keys (low 32 bits of vals[0..d)) in insertion order, i.e. first-occurrence order: the inserts of
 * countCodePointPairs' getOrPut sequence, plus one trailing getOrPut of an existing key when
 * `extra_lookup`.  Lookups of existing keys between inserts change nothing: growIfNeeded(1) of such a
 * lookup grows the same key set the next insert's growIfNeeded would. */
ReplayResult zig_replay(const uint64_t *vals, size_t d, bool extra_lookup, const uint32_t *tied, size_t nt) {
    HBuf<uint32_t> tbl;
    std::vector<uint64_t> seq;
    uint32_t cap = 0, avail = 0, size = 0;
    constexpr int PF = ZFAST_PF;
    auto insert_all = [&](const uint64_t *ks, size_t m) {
        const uint32_t mask = cap - 1;
        uint32_t *t = tbl.data();
        uint32_t homes[PF];
        size_t pre = std::min<size_t>(m, PF);
        for (size_t i = 0; i < pre; i++) {
            homes[i] = (uint32_t)(zig_hash((uint32_t)ks[i]) & mask);
            __builtin_prefetch(t + homes[i], 1);
        }
        for (size_t i = 0; i < m; i++) {
            uint32_t idx = homes[i % PF];
            if (i + PF < m) {
                uint32_t h = (uint32_t)(zig_hash((uint32_t)ks[i + PF]) & mask);
                homes[i % PF] = h;
                __builtin_prefetch(t + h, 1);
            }
            while (t[idx] != EMPTY_KEY) idx = (idx + 1) & mask;
            t[idx] = (uint32_t)ks[i];
        }
    };
    auto grow = [&](uint32_t new_capacity) {
        uint32_t nc = new_capacity < 8 ? 8 : new_capacity;
        seq.clear();
        for (uint32_t s = 0; s < cap; s++)
            if (tbl[s] != EMPTY_KEY) seq.push_back(tbl[s]); /* old slot order */
        HBuf<uint32_t> nt(nc);
        memset(nt.data(), 0xFF, (size_t)nc * sizeof(uint32_t));
        tbl = std::move(nt);
        cap = nc;
        avail = zig_max_load(nc) - size;
        insert_all(seq.data(), seq.size());
    };
    size_t i = 0;
    while (i < d) {
        if (avail < 1) grow(zig_cap_for_size(size + 1)); /* growIfNeeded(1), load == size */
        size_t m = std::min<size_t>(avail, d - i);
        insert_all(vals + i, m);
        i += m;
        size += (uint32_t)m;
        avail -= (uint32_t)m;
    }
    if (extra_lookup && avail < 1) grow(zig_cap_for_size(size + 1));
    ReplayResult r{NONE, NONE, cap};
    const uint32_t mask = cap - 1;
    for (size_t j = 0; j < nt; j++) {
        uint32_t idx = (uint32_t)(zig_hash(tied[j]) & mask);
        uint32_t guard = cap;
        while (tbl[idx] != tied[j] && guard--) idx = (idx + 1) & mask;
        if (tbl[idx] != tied[j]) return ReplayResult{NONE, NONE, cap}; /* not in the map: a bug */
        if (idx < r.slot) { r.slot = idx; r.winner = tied[j]; }
    }
    return r;
}

uint64_t fnv64_u16(const uint16_t *t, size_t len) {
    uint64_t h = 0xcbf29ce484222325ULL;
    const uint8_t *p = (const uint8_t *)t;
    for (size_t i = 0; i < 2 * len; i++) h = (h ^ p[i]) * 0x100000001b3ULL;
    return h;
}

template <class F>
void parallel_for(size_t n, int threads, F f) { /* f(begin, end, thread_index) over contiguous chunks */
    std::vector<std::thread> th;
    size_t chunk = (n + threads - 1) / threads;
    for (int t = 0; t < threads; t++) {
        size_t b = std::min(n, t * chunk), e = std::min(n, b + chunk);
        th.emplace_back(f, b, e, t);
    }
    for (auto &x : th) x.join();
}

/* ---------------------------------------------------------------------------------------------- */
/* worker pool: tie replays and stream checksums                                                   */
/* ---------------------------------------------------------------------------------------------- */
/* (first occurrence << 32 | key) of every live pair, sorted: the insertion order of the pair map.
 * Immutable once published; the trainer derives the next one from it and the changes since. */
struct Snap {
    HBuf<uint64_t> v;
    size_t n = 0;
};

struct Job {
    int kind = 0; /* 0: tie replay, 1: fnv */
    uint32_t k = 0;
    std::shared_ptr<const Snap> snap;
    std::vector<uint32_t> tied;   /* keys at the top count */
    uint32_t used = 0;            /* the key the run merged */
    bool extra = false;
    std::vector<uint16_t> stream; /* fnv: the compacted stream */
};

struct Log {
    FILE *f = nullptr;
    std::mutex mu;
    void line(const char *fmt, ...) __attribute__((format(printf, 2, 3)));
};
void Log::line(const char *fmt, ...) {
    if (!f) return;
    std::lock_guard<std::mutex> g(mu);
    va_list ap;
    va_start(ap, fmt);
    vfprintf(f, fmt, ap);
    va_end(ap);
    fflush(f);
}

struct Pool {
    std::mutex mu;
    std::condition_variable cv_job, cv_space, cv_idle;
    std::deque<Job> q;
    size_t max_pending;
    int busy = 0;
    bool stop = false;
    std::vector<std::thread> th;
    Log *log;
    std::atomic<uint32_t> mismatch_k{NONE};
    std::atomic<uint32_t> mismatch_key{NONE};
    std::atomic<uint64_t> verified{0};
    std::atomic<uint64_t> verify_failures{0};

    Pool(int workers, size_t pending, Log *lg) : max_pending(pending), log(lg) {
        for (int i = 0; i < workers; i++) th.emplace_back([this] { run(); });
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> g(mu);
            stop = true;
        }
        cv_job.notify_all();
        for (auto &t : th) t.join();
    }
    void submit(Job &&j) {
        std::unique_lock<std::mutex> g(mu);
        cv_space.wait(g, [&] { return q.size() < max_pending; });
        q.push_back(std::move(j));
        cv_job.notify_one();
    }
    void drain() {
        std::unique_lock<std::mutex> g(mu);
        cv_idle.wait(g, [&] { return q.empty() && busy == 0; });
    }
    void run() {
        for (;;) {
            Job j;
            {
                std::unique_lock<std::mutex> g(mu);
                cv_job.wait(g, [&] { return stop || !q.empty(); });
                if (q.empty()) return;
                j = std::move(q.front());
                q.pop_front();
                busy++;
                cv_space.notify_one();
            }
            if (j.kind == 0) replay(j);
            else log->line("fnv %u %zu %016llx\n", j.k, j.stream.size(),
                           (unsigned long long)fnv64_u16(j.stream.data(), j.stream.size()));
            {
                std::lock_guard<std::mutex> g(mu);
                busy--;
                if (q.empty() && busy == 0) cv_idle.notify_all();
            }
        }
    }
    void replay(Job &j) {
        ReplayResult r = zig_replay(j.snap->v.data(), j.snap->n, j.extra, j.tied.data(), j.tied.size());
        j.snap.reset();
        if (r.winner == j.used) {
            verified++;
            log->line("tie %u ok %u %u %u %zu\n", j.k, r.winner, r.slot, r.cap, j.tied.size());
        } else {
            verify_failures++;
            log->line("tie %u MISMATCH used %u replay %u slot %u cap %u\n", j.k, j.used, r.winner, r.slot, r.cap);
            /* keep the earliest mismatch */
            while (true) {
                uint32_t cur = mismatch_k.load();
                if (cur != NONE && cur <= j.k) break;
                if (mismatch_k.compare_exchange_weak(cur, j.k)) {
                    mismatch_key.store(r.winner);
                    break;
                }
            }
        }
    }
};

/* ---------------------------------------------------------------------------------------------- */
/* the trainer                                                                                      */
/* ---------------------------------------------------------------------------------------------- */
struct KeyMap { /* pair key -> id, open addressing (not the Zig map: only the counting side) */
    std::vector<uint64_t> slot; /* key << 32 | id */
    uint64_t mask = 0, used = 0;
    static inline uint64_t h(uint32_t k) { return (uint64_t)k * 0x9E3779B97F4A7C15ULL; }
    void init(uint64_t cap) { slot.assign(cap, ~0ULL); mask = cap - 1; used = 0; }
    uint32_t find(uint32_t k) const {
        int bits = __builtin_ctzll(mask + 1);
        uint64_t i = h(k) >> (64 - bits);
        for (;;) {
            uint64_t s = slot[i];
            if (s == ~0ULL) return NONE;
            if ((uint32_t)(s >> 32) == k) return (uint32_t)s;
            i = (i + 1) & mask;
        }
    }
    void insert(uint32_t k, uint32_t id) {
        if ((used + 1) * 2 > mask + 1) {
            std::vector<uint64_t> old;
            old.swap(slot);
            init((mask + 1) * 2);
            for (uint64_t s : old)
                if (s != ~0ULL) put(s);
        }
        put((uint64_t)k << 32 | id);
    }
    void put(uint64_t s) {
        int bits = __builtin_ctzll(mask + 1);
        uint64_t i = h((uint32_t)(s >> 32)) >> (64 - bits);
        while (slot[i] != ~0ULL) i = (i + 1) & mask;
        slot[i] = s;
        used++;
    }
};

struct Override { uint32_t k, key; };

struct Trainer {
    /* inputs */
    const uint8_t *text;
    size_t n;
    uint32_t vocab;
    int threads;
    uint32_t fnv_every;
    uint64_t sync_limit;
    Log *log;
    const std::vector<Override> *overrides;
    /* outputs */
    uint16_t *out_triples;
    uint64_t *out_counts;
    uint32_t *out_ties, *out_distinct;
    uint64_t *out_len_after;
    uint32_t merges_done = 0;
    uint32_t mismatch_k = NONE, mismatch_key = NONE;
    uint64_t ties_sync = 0, ties_async = 0;
    double t_apply = 0, t_snap = 0, t_sync = 0, t_copy = 0, t_init = 0, t_wait = 0;
    static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

    /* stream: doubly linked list over original positions */
    std::vector<uint16_t> tok;
    std::vector<uint32_t> nxt, prv;
    uint32_t tail = NONE;
    uint64_t live_tokens = 0;

    /* pairs */
    std::vector<uint32_t> pkey, pcnt, plen, pcur, pfo, plive, pstamp, padv, ptie;
    uint32_t tie_round = 0;
    std::vector<uint64_t> poff;
    KeyMap km;
    uint32_t *arena = nullptr;
    size_t arena_cap = 0, arena_top = 0;
    uint64_t n_live = 0;
    /* the insertion order: S as of the last snapshot, plus the pairs changed since (born, dead, or a
     * new first occurrence), with the value each had in S */
    std::shared_ptr<const Snap> S;
    std::vector<uint64_t> sval;
    std::vector<uint8_t> pdirty;
    std::vector<uint32_t> dirty;
    std::vector<uint64_t> heap;   /* (count << 32 | id), max-heap, lazily invalidated */
    bool no_replay = false; /* analysis tools: a forced winner (override) is taken without a replay */
    /* analysis hook (tools/batch_potential.cpp): called with the winner before each merge is applied */
    void (*pre_apply)(Trainer &, uint32_t k, uint32_t win_id, uint32_t T, const std::vector<uint32_t> &tied) = nullptr;

    ~Trainer() {
        if (arena) munmap(arena, arena_cap * sizeof(uint32_t));
    }

    static uint32_t key_of(uint16_t a, uint16_t b) { return (uint32_t)a | (uint32_t)b << 16; }

    bool entry_live(uint32_t key, uint32_t p) const {
        if (tok[p] != (uint16_t)key) return false;
        uint32_t q = nxt[p];
        return q != NONE && tok[q] == (uint16_t)(key >> 16);
    }

    uint32_t new_pair(uint32_t key, uint32_t cnt, uint64_t off, uint32_t len) {
        uint32_t id = (uint32_t)pkey.size();
        pkey.push_back(key);
        pcnt.push_back(cnt);
        poff.push_back(off);
        plen.push_back(len);
        pcur.push_back(0);
        pfo.push_back(arena[off]);
        plive.push_back(1);
        sval.push_back(~0ULL);
        pdirty.push_back(0);
        pstamp.push_back(NONE);
        padv.push_back(NONE);
        ptie.push_back(NONE);
        n_live++;
        mark(id);
        km.insert(key, id);
        heap.push_back((uint64_t)cnt << 32 | id);
        std::push_heap(heap.begin(), heap.end());
        return id;
    }

    void mark(uint32_t id) {
        if (!pdirty[id]) { pdirty[id] = 1; dirty.push_back(id); }
    }

    void kill(uint32_t id) {
        plive[id] = NONE;
        n_live--;
        mark(id);
    }

    /* the live pairs in first-occurrence order: S minus the changed pairs' old values, merged with
     * their new ones (an O(D) pass instead of a sort) */
    std::shared_ptr<const Snap> snapshot() {
        if (S && dirty.empty()) return S;
        std::vector<uint64_t> rem, ins;
        for (uint32_t id : dirty) {
            if (sval[id] != ~0ULL) rem.push_back(sval[id]);
            uint64_t nv = plive[id] != NONE ? (uint64_t)pfo[id] << 32 | pkey[id] : ~0ULL;
            if (nv != ~0ULL) ins.push_back(nv);
            sval[id] = nv;
            pdirty[id] = 0;
        }
        dirty.clear();
        std::sort(rem.begin(), rem.end());
        std::sort(ins.begin(), ins.end());
        auto nsnap = std::make_shared<Snap>();
        nsnap->v.alloc(n_live);
        uint64_t *out = nsnap->v.data();
        const uint64_t *a = S ? S->v.data() : nullptr;
        size_t na = S ? S->n : 0, i = 0, r = 0, j = 0, o = 0;
        while (i < na || j < ins.size()) {
            if (i < na && r < rem.size() && a[i] == rem[r]) { i++; r++; continue; }
            if (j == ins.size() || (i < na && a[i] < ins[j])) out[o++] = a[i++];
            else out[o++] = ins[j++];
        }
        if (o != n_live || r != rem.size()) {
            fprintf(stderr, "zig_fast: snapshot has %zu entries for %llu live pairs (%zu/%zu removed)\n", o,
                    (unsigned long long)n_live, r, rem.size());
            abort();
        }
        nsnap->n = o;
        S = nsnap;
        return S;
    }

    bool init() {
        tok.resize(n);
        nxt.resize(n);
        prv.resize(n);
        parallel_for(n, threads, [&](size_t b, size_t e, int) {
            for (size_t i = b; i < e; i++) {
                tok[i] = text[i];
                nxt[i] = i + 1 < n ? (uint32_t)(i + 1) : NONE;
                prv[i] = i ? (uint32_t)(i - 1) : NONE;
            }
        });
        tail = n ? (uint32_t)(n - 1) : NONE;
        live_tokens = n;
        /* births over the whole run are at most 2 per removed token: reserve 3n entries (untouched
         * pages cost nothing) */
        arena_cap = 3 * n + 1024;
        void *m = mmap(nullptr, arena_cap * sizeof(uint32_t), PROT_READ | PROT_WRITE,
                       MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
        if (m == MAP_FAILED) return false;
        arena = (uint32_t *)m;
        km.init(1 << 20);
        size_t np = n >= 1 ? n - 1 : 0;
        /* initial pairs are byte pairs: dense 65536 bins, per-thread counts, then a stable scatter */
        std::vector<std::vector<uint64_t>> cnt(threads, std::vector<uint64_t>(65536, 0));
        parallel_for(np, threads, [&](size_t b, size_t e, int t) {
            uint64_t *c = cnt[t].data();
            for (size_t i = b; i < e; i++) c[text[i] | text[i + 1] << 8]++;
        });
        std::vector<uint64_t> total(65536, 0), base(65536, 0);
        uint64_t acc = 0;
        for (int k = 0; k < 65536; k++) {
            base[k] = acc;
            for (int t = 0; t < threads; t++) {
                uint64_t c = cnt[t][k];
                cnt[t][k] = acc; /* becomes thread t's write offset */
                acc += c;
                total[k] += c;
            }
        }
        parallel_for(np, threads, [&](size_t b, size_t e, int t) {
            uint64_t *o = cnt[t].data();
            for (size_t i = b; i < e; i++) arena[o[text[i] | text[i + 1] << 8]++] = (uint32_t)i;
        });
        arena_top = acc;
        for (int k = 0; k < 65536; k++) {
            if (!total[k]) continue;
            if (total[k] >= (1ULL << 32)) return false;
            new_pair(key_of((uint16_t)(k & 255), (uint16_t)(k >> 8)), (uint32_t)total[k], base[k], (uint32_t)total[k]);
        }
        return true;
    }

    /* pop the top count and every pair sharing it */
    uint32_t top(std::vector<uint32_t> &tied) {
        tied.clear();
        tie_round++;
        uint32_t T = 0;
        while (!heap.empty()) {
            uint64_t e = heap.front();
            uint32_t id = (uint32_t)e, c = (uint32_t)(e >> 32);
            if (plive[id] == NONE || pcnt[id] != c || c == 0) {
                std::pop_heap(heap.begin(), heap.end());
                heap.pop_back();
                continue;
            }
            if (tied.empty()) T = c;
            else if (c != T) break;
            std::pop_heap(heap.begin(), heap.end());
            heap.pop_back();
            if (ptie[id] != tie_round) { ptie[id] = tie_round; tied.push_back(id); }
        }
        return T;
    }

    /* does a getOrPut of an existing key follow the last insertion?  (the stream's last pair is not
     * the first occurrence of its key) */
    bool extra_lookup() const {
        if (tail == NONE || prv[tail] == NONE) return false;
        uint32_t p = prv[tail];
        uint32_t id = km.find(key_of(tok[p], tok[tail]));
        return pfo[id] != p;
    }

    uint32_t predict(const std::vector<uint32_t> &tied, bool extra) const {
        uint32_t cap = zig_final_capacity(n_live, extra), best = NONE;
        uint64_t best_rank = ~0ULL;
        for (uint32_t id : tied) {
            uint64_t rank = (zig_hash(pkey[id]) & (cap - 1)) << 32 | pfo[id];
            if (rank < best_rank) { best_rank = rank; best = pkey[id]; }
        }
        return best;
    }

    void stream_copy(std::vector<uint16_t> &out) const { /* the compacted stream, in parallel chunks */
        out.resize(live_tokens);
        const int T = 8;
        std::vector<size_t> cnt(T + 1, 0);
        const uint16_t *t = tok.data();
        parallel_for(n, T, [&](size_t b, size_t e, int i) {
            size_t c = 0;
            for (size_t x = b; x < e; x++) c += t[x] != HOLE;
            cnt[i + 1] = c;
        });
        for (int i = 0; i < T; i++) cnt[i + 1] += cnt[i];
        if (cnt[T] != live_tokens) { fprintf(stderr, "zig_fast: stream has %zu tokens, expected %llu\n", cnt[T], (unsigned long long)live_tokens); abort(); }
        uint16_t *o = out.data();
        parallel_for(n, T, [&](size_t b, size_t e, int i) {
            size_t j = cnt[i];
            for (size_t x = b; x < e; x++)
                if (t[x] != HOLE) o[j++] = t[x];
        });
    }

    /* one merge: (a, b) -> X over the pair's live entries */
    std::vector<uint32_t> applied, touched, adv;
    std::vector<uint32_t> lcnt, rcnt, lseen, rseen;
    std::vector<uint32_t> lslot = std::vector<uint32_t>(65536), rslot = std::vector<uint32_t>(65536); /* token -> list index */

    void dec(uint32_t id, uint32_t pos, uint32_t stamp) {
        pcnt[id]--;
        if (pstamp[id] != stamp) { pstamp[id] = stamp; touched.push_back(id); }
        if (pos == pfo[id] && padv[id] != stamp) { padv[id] = stamp; adv.push_back(id); }
    }

    void apply(uint32_t pid, uint16_t X, uint32_t stamp) {
        const uint32_t key = pkey[pid];
        const uint16_t a = (uint16_t)key, b = (uint16_t)(key >> 16);
        applied.clear();
        touched.clear();
        adv.clear();
        const uint32_t *L0 = arena + poff[pid];
        for (uint32_t e = pcur[pid]; e < plen[pid]; e++) {
            uint32_t p = L0[e];
            if (tok[p] != a) continue;
            uint32_t q = nxt[p];
            if (q == NONE || tok[q] != b) continue;
            uint32_t L = prv[p], R = nxt[q];
            if (L != NONE && tok[L] != X) dec(km.find(key_of(tok[L], a)), L, stamp);
            dec(pid, p, stamp);
            if (R != NONE) dec(km.find(key_of(b, tok[R])), q, stamp);
            tok[p] = X;
            tok[q] = HOLE;
            nxt[p] = R;
            if (R != NONE) prv[R] = p;
            else tail = p;
            applied.push_back(p);
        }
        live_tokens -= applied.size();
        /* births: (tok[L], X) at L and (X, tok[R]) at p; an (X, X) is counted once, as a left pair */
        if (lcnt.size() < 65536) { lcnt.assign(65536, 0); rcnt.assign(65536, 0); }
        lseen.clear();
        rseen.clear();
        for (uint32_t p : applied) {
            uint32_t L = prv[p], R = nxt[p];
            if (L != NONE) { if (!lcnt[tok[L]]++) lseen.push_back(tok[L]); }
            if (R != NONE && tok[R] != X) { if (!rcnt[tok[R]]++) rseen.push_back(tok[R]); }
        }
        /* lay out the new lists, then scatter positions (applied is in position order, so each list
         * comes out sorted) */
        std::vector<uint64_t> loff(lseen.size()), roff(rseen.size());
        for (size_t i = 0; i < lseen.size(); i++) { lslot[lseen[i]] = (uint32_t)i; loff[i] = arena_top; arena_top += lcnt[lseen[i]]; }
        for (size_t i = 0; i < rseen.size(); i++) { rslot[rseen[i]] = (uint32_t)i; roff[i] = arena_top; arena_top += rcnt[rseen[i]]; }
        if (arena_top > arena_cap) { fprintf(stderr, "zig_fast: arena overflow\n"); abort(); }
        std::vector<uint64_t> lw(loff), rw(roff);
        for (uint32_t p : applied) {
            uint32_t L = prv[p], R = nxt[p];
            if (L != NONE) arena[lw[lslot[tok[L]]]++] = L;
            if (R != NONE && tok[R] != X) arena[rw[rslot[tok[R]]]++] = p;
        }
        /* the old pairs' counts and first occurrences */
        if (pcnt[pid] != 0) { fprintf(stderr, "zig_fast: top pair count %u after its merge\n", pcnt[pid]); abort(); }
        for (uint32_t id : adv) {
            if (pcnt[id] == 0) continue;
            uint32_t c = pcur[id];
            const uint32_t *L = arena + poff[id];
            while (c < plen[id] && !entry_live(pkey[id], L[c])) c++;
            if (c == plen[id]) { fprintf(stderr, "zig_fast: live pair without a live entry\n"); abort(); }
            pcur[id] = c;
            pfo[id] = L[c];
            mark(id);
        }
        for (uint32_t id : touched) {
            if (pcnt[id] == 0) { if (plive[id] != NONE) kill(id); continue; }
            heap.push_back((uint64_t)pcnt[id] << 32 | id);
            std::push_heap(heap.begin(), heap.end());
        }
        for (size_t i = 0; i < lseen.size(); i++) {
            uint16_t y = (uint16_t)lseen[i];
            new_pair(key_of(y, X), lcnt[y], loff[i], lcnt[y]);
            lcnt[y] = 0;
        }
        for (size_t i = 0; i < rseen.size(); i++) {
            uint16_t z = (uint16_t)rseen[i];
            new_pair(key_of(X, z), rcnt[z], roff[i], rcnt[z]);
            rcnt[z] = 0;
        }
    }

    /* 0 ok, 2 OOM / overflow, 4 a replay disagreed with a predicted winner (mismatch_k / _key) */
    int run(Pool *pool) {
        double t0 = now();
        if (!init()) return 2;
        t_init = now() - t0;
        const size_t cap = vocab - 256;
        std::vector<uint32_t> tied, tkeys;
        size_t ov = 0;
        for (uint32_t cur = 256; cur < vocab; cur++) {
            uint32_t k = cur - 256;
            if (pool && pool->mismatch_k.load() != NONE) break;
            uint32_t T = top(tied);
            size_t D = n_live;
            if (tied.empty() || D == 0) {
                fprintf(stderr, "No more pairs to merge. Stopping early.\n");
                break;
            }
            uint32_t win_id = tied[0];
            if (tied.size() > 1) {
                bool extra = extra_lookup();
                tkeys.clear();
                for (uint32_t id : tied) tkeys.push_back(pkey[id]);
                while (ov < overrides->size() && (*overrides)[ov].k < k) ov++;
                bool forced = ov < overrides->size() && (*overrides)[ov].k == k;
                uint32_t win_key;
                if (forced && no_replay) {  // (analysis tools only: decisions taken from a verified golden)
                    win_key = (*overrides)[ov].key;
                } else if (D <= sync_limit || !pool) {
                    double a0 = now();
                    std::shared_ptr<const Snap> sn = snapshot();
                    double a1 = now();
                    ReplayResult r = zig_replay(sn->v.data(), sn->n, extra, tkeys.data(), tkeys.size());
                    t_snap += a1 - a0;
                    t_sync += now() - a1;
                    if (r.winner == NONE) return 2;
                    win_key = r.winner;
                    ties_sync++;
                    log->line("tie %u ok %u %u %u %zu sync\n", k, r.winner, r.slot, r.cap, tkeys.size());
                } else {
                    win_key = forced ? (*overrides)[ov].key : predict(tied, extra);
                    Job j;
                    j.kind = 0;
                    j.k = k;
                    double a0 = now();
                    j.snap = snapshot();
                    t_snap += now() - a0;
                    j.tied = tkeys;
                    j.used = win_key;
                    j.extra = extra;
                    double a1 = now();
                    pool->submit(std::move(j));
                    t_wait += now() - a1;
                    ties_async++;
                }
                for (uint32_t id : tied)
                    if (pkey[id] == win_key) win_id = id;
                if (pkey[win_id] != win_key) return 2;
                for (uint32_t id : tied) /* the others stay candidates */
                    if (id != win_id) { heap.push_back((uint64_t)pcnt[id] << 32 | id); std::push_heap(heap.begin(), heap.end()); }
            }
            uint32_t key = pkey[win_id];
            out_triples[3 * k] = (uint16_t)key;
            out_triples[3 * k + 1] = (uint16_t)(key >> 16);
            out_triples[3 * k + 2] = (uint16_t)cur;
            out_counts[k] = T;
            out_ties[k] = (uint32_t)tied.size();
            out_distinct[k] = (uint32_t)D;
            if (pre_apply) pre_apply(*this, k, win_id, T, tied);
            double a0 = now();
            apply(win_id, (uint16_t)cur, k);
            t_apply += now() - a0;
            out_len_after[k] = live_tokens;
            merges_done = k + 1;
            log->line("%u %u %u %u %u %zu %zu %llu\n", k, key & 0xFFFF, key >> 16, cur, T, tied.size(), D,
                      (unsigned long long)live_tokens);
            if (fnv_every && merges_done % fnv_every == 0) {
                Job j;
                j.kind = 1;
                j.k = merges_done;
                double a1 = now();
                stream_copy(j.stream);
                t_copy += now() - a1;
                if (pool) pool->submit(std::move(j));
                else log->line("fnv %u %zu %016llx\n", j.k, j.stream.size(),
                               (unsigned long long)fnv64_u16(j.stream.data(), j.stream.size()));
            }
            (void)cap;
        }
        if (pool) {
            pool->drain();
            if (pool->mismatch_k.load() != NONE) {
                mismatch_k = pool->mismatch_k.load();
                mismatch_key = pool->mismatch_key.load();
                return 4;
            }
        }
        return 0;
    }
};

} // namespace

extern "C" {

/* Train like basic_tokenizer.zig:140-306 (see the header).  Returns 0 ok, 1 InvalidVocabSize,
 * 2 OutOfMemory / internal error.  out_len_after[k] = stream length after merge k.  out_final (may be
 * NULL) receives the final stream (capacity n).  `threads` >= 1 (workers = threads - 1); tied merges
 * with at most `sync_limit` live pairs are replayed before the merge, larger ones asynchronously.
 * out_info[0..3] = restarts, ties replayed synchronously, ties replayed by workers (final attempt). */
int zfast_train(const uint8_t *text, size_t n, uint32_t vocab, int threads, uint64_t sync_limit,
                uint32_t fnv_every, const char *progress, uint16_t *out_triples, uint64_t *out_counts,
                uint32_t *out_ties, uint32_t *out_distinct, uint64_t *out_len_after, size_t *out_n_merges,
                uint16_t *out_final, size_t *out_final_len, uint64_t *out_info) {
    *out_n_merges = 0;
    if (vocab < 256) return 1;
    if (n >= (1ULL << 32) - 1) return 2;
    if (threads < 1) threads = 1;
    Log log;
    if (progress) log.f = fopen(progress, "w");
    std::vector<Override> overrides;
    uint64_t restarts = 0;
    int rc;
    for (;;) {
        Trainer t;
        t.text = text;
        t.n = n;
        t.vocab = vocab;
        t.threads = threads;
        t.fnv_every = fnv_every;
        t.sync_limit = sync_limit;
        t.log = &log;
        t.overrides = &overrides;
        t.out_triples = out_triples;
        t.out_counts = out_counts;
        t.out_ties = out_ties;
        t.out_distinct = out_distinct;
        t.out_len_after = out_len_after;
        {
            Pool *pool = threads > 1 ? new Pool(threads - 1, 2 * (threads - 1), &log) : nullptr;
            rc = t.run(pool);
            delete pool;
        }
        if (rc == 4) {
            /* a literal replay disagreed with the predicted winner: fix that merge and start over */
            overrides.push_back(Override{t.mismatch_k, t.mismatch_key});
            std::sort(overrides.begin(), overrides.end(), [](const Override &x, const Override &y) { return x.k < y.k; });
            restarts++;
            log.line("restart %u %u\n", t.mismatch_k, t.mismatch_key);
            continue;
        }
        if (rc == 0) {
            std::vector<uint16_t> fin;
            t.stream_copy(fin);
            log.line("done %u %zu %016llx\n", t.merges_done, fin.size(),
                     (unsigned long long)fnv64_u16(fin.data(), fin.size()));
            if (out_final) memcpy(out_final, fin.data(), fin.size() * sizeof(uint16_t));
            if (out_final_len) *out_final_len = fin.size();
            *out_n_merges = t.merges_done;
            if (out_info) {
                out_info[0] = restarts;
                out_info[1] = t.ties_sync;
                out_info[2] = t.ties_async;
            }
            log.line("timing init %.2f apply %.2f snapshot %.2f sync_replay %.2f stream_copy %.2f queue_wait %.2f\n",
                     t.t_init, t.t_apply, t.t_snap, t.t_sync, t.t_copy, t.t_wait);
        }
        break;
    }
    if (log.f) fclose(log.f);
    return rc;
}

/* the restated Zig hash and sizing, for the CPU test against zig_ref.c */
uint64_t zfast_pair_hash(uint32_t key) { return zig_hash(key); }
uint32_t zfast_final_capacity(uint64_t d, int extra) { return zig_final_capacity(d, extra != 0); }

} // extern "C"

/*
 * oracle/zig_ref.c -- TEST INFRASTRUCTURE ONLY (the parity checker, never the product).
 *
 * Plain-C restatement of the reference BPE trainer in
 *   /root/reference/src/basic_tokenizer.zig
 * together with the parts of the Zig 0.13.0 standard library whose arithmetic decides
 * the result (README.md:19 pins "Zig version 0.13.0"; the std lib is not vendored):
 *   - std.hash.Wyhash (lib/std/hash/wyhash.zig), seed 0 via std.hash_map.getAutoHashFn,
 *   - std.HashMapUnmanaged (lib/std/hash_map.zig): power-of-two capacity, linear probing,
 *     max_load_percentage 80, minimal_capacity 8, growIfNeeded(1) on EVERY getOrPut
 *     (before the lookup), grow() re-inserting in old-slot order, Iterator = slot order,
 *   - std.mem.sort = std.sort.block (stable).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this.
 * The product (zig-bpe_amd/) never links or calls it.
 *
 * Parity pinning (see DESIGN.md "Oracle"):
 *   - Wyhash known-answer vectors from Zig's own wyhash.zig tests (zref_selftest).
 *   - /root/reference/merges.txt reproduced byte for byte from taylorswift.txt, V=300
 *     (tests/golden/c1_*; line 39 is a real top-count tie decided by hash-map order).
 *   - The five inline tests of basic_tokenizer.zig:351-461 restated in tests/test_oracle.py.
 *   The grow-on-lookup rule (hash_map.zig growIfNeeded) is not pinned by any reference
 *   artefact; it is restated from the Zig 0.13 source as documented in SURVEY.md App. A.3.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ------------------------------------------------------------------------------------ */
/* Zig 0.13 std.hash.Wyhash                                                             */
/* ------------------------------------------------------------------------------------ */
static const uint64_t WY_S0 = 0xa0761d6478bd642fULL, WY_S1 = 0xe7037ed1a0b428dbULL,
                      WY_S2 = 0x8ebc6af09c88c6e3ULL, WY_S3 = 0x589965cc75374cc3ULL;

static inline void wy_mum(uint64_t *a, uint64_t *b) {
    __uint128_t x = (__uint128_t)(*a) * (*b);
    *a = (uint64_t)x;
    *b = (uint64_t)(x >> 64);
}
static inline uint64_t wy_mix(uint64_t a, uint64_t b) { wy_mum(&a, &b); return a ^ b; }
static inline uint64_t wy_read(const uint8_t *p, int bytes) {
    uint64_t v = 0;
    for (int i = 0; i < bytes; i++) v |= (uint64_t)p[i] << (8 * i);
    return v;
}

/* Wyhash.hash(seed, input): init -> smallKey | rounds+final0+final1 -> final2 */
uint64_t zref_wyhash(uint64_t seed, const uint8_t *in, size_t len) {
    const uint64_t secret[4] = {WY_S0, WY_S1, WY_S2, WY_S3};
    uint64_t st[3];
    st[0] = seed ^ wy_mix(seed ^ secret[0], secret[1]);
    st[1] = st[0];
    st[2] = st[0];
    uint64_t a, b;
    if (len <= 16) {
        if (len >= 4) {
            size_t end = len - 4, quarter = (len >> 3) << 2;
            a = (wy_read(in, 4) << 32) | wy_read(in + quarter, 4);
            b = (wy_read(in + end, 4) << 32) | wy_read(in + end - quarter, 4);
        } else if (len > 0) {
            a = ((uint64_t)in[0] << 16) | ((uint64_t)in[len >> 1] << 8) | in[len - 1];
            b = 0;
        } else {
            a = 0;
            b = 0;
        }
    } else {
        size_t i = 0;
        if (len >= 48) {
            while (i + 48 < len) {
                for (int r = 0; r < 3; r++) {
                    uint64_t x = wy_read(in + i + 16 * r, 8), y = wy_read(in + i + 16 * r + 8, 8);
                    st[r] = wy_mix(x ^ secret[r + 1], y ^ st[r]);
                }
                i += 48;
            }
            st[0] ^= st[1] ^ st[2]; /* final0 */
        }
        /* final1 */
        const uint8_t *p = in + i;
        size_t rem = len - i, j = 0;
        while (j + 16 < rem) {
            st[0] = wy_mix(wy_read(p + j, 8) ^ secret[1], wy_read(p + j + 8, 8) ^ st[0]);
            j += 16;
        }
        a = wy_read(in + len - 16, 8);
        b = wy_read(in + len - 8, 8);
    }
    /* final2 */
    a ^= secret[1];
    b ^= st[0];
    wy_mum(&a, &b);
    return wy_mix(a ^ secret[0] ^ (uint64_t)len, b ^ secret[1]);
}

/* AutoHashMap(CharPair, usize) key hash: CharPair{first:u16, second:u16} has a unique
 * representation, so getAutoHashFn -> Wyhash.hash(0, asBytes(&key)) over
 * [first_lo, first_hi, second_lo, second_hi] (basic_tokenizer.zig:40-43, :265). */
uint64_t zref_pair_hash(uint16_t first, uint16_t second) {
    uint8_t k[4] = {(uint8_t)first, (uint8_t)(first >> 8), (uint8_t)second, (uint8_t)(second >> 8)};
    return zref_wyhash(0, k, 4);
}

/* ------------------------------------------------------------------------------------ */
/* Zig 0.13 std.HashMapUnmanaged(CharPair, usize, AutoContext, 80)                      */
/* ------------------------------------------------------------------------------------ */
typedef struct {
    uint32_t *keys;   /* first | second << 16 */
    uint64_t *vals;
    uint8_t *used;    /* metadata: used bit (no removals -> no tombstones) */
    uint32_t cap;     /* 0 before the first allocation */
    uint32_t size;
    uint32_t available;
} zmap;

static uint32_t zmap_max_load(uint32_t cap) { return (uint32_t)(((uint64_t)cap * 80) / 100); }
static uint32_t ceil_pow2(uint64_t x) {
    uint64_t p = 1;
    while (p < x) p <<= 1;
    return (uint32_t)p;
}
static uint32_t capacity_for_size(uint32_t size) { /* capacityForSize */
    return ceil_pow2(((uint64_t)size * 100) / 80 + 1);
}
/* zref_pair_hash with the 4-byte path of zref_wyhash unfolded (len 4: quarter 0, so a = b =
 * w << 32 | w; seed 0 gives a constant state); zref_selftest checks the two agree. */
static inline uint64_t key_hash(uint32_t k) {
    const uint64_t s = wy_mix(WY_S0, WY_S1); /* seed 0: 0 ^ mix(0 ^ s0, s1) */
    uint64_t a = ((uint64_t)k << 32 | k) ^ WY_S1, b = ((uint64_t)k << 32 | k) ^ s;
    wy_mum(&a, &b);
    return wy_mix(a ^ WY_S0 ^ 4u, b ^ WY_S1);
}

static void zmap_free(zmap *m) {
    free(m->keys);
    free(m->vals);
    free(m->used);
    memset(m, 0, sizeof(*m));
}

/* putAssumeCapacityNoClobber */
static void zmap_put_no_clobber(zmap *m, uint32_t key, uint64_t val) {
    uint32_t mask = m->cap - 1, idx = (uint32_t)(key_hash(key) & mask);
    while (m->used[idx]) idx = (idx + 1) & mask;
    m->used[idx] = 1;
    m->keys[idx] = key;
    m->vals[idx] = val;
    m->available--;
    m->size++;
}

/* grow(): allocate new_cap (>= minimal_capacity 8), re-insert in OLD SLOT order */
static void zmap_grow(zmap *m, uint32_t new_capacity) {
    uint32_t new_cap = new_capacity < 8 ? 8 : new_capacity;
    zmap n;
    memset(&n, 0, sizeof(n));
    n.cap = new_cap;
    n.keys = (uint32_t *)malloc(sizeof(uint32_t) * new_cap);
    n.vals = (uint64_t *)malloc(sizeof(uint64_t) * new_cap);
    n.used = (uint8_t *)calloc(new_cap, 1);
    n.available = zmap_max_load(new_cap);
    if (m->size != 0) {
        for (uint32_t i = 0; i < m->cap; i++) {
            if (!m->used[i]) continue;
            zmap_put_no_clobber(&n, m->keys[i], m->vals[i]);
            if (n.size == m->size) break;
        }
    }
    zmap_free(m);
    *m = n;
}

/* getOrPut(): growIfNeeded(1) FIRST (even if the key exists), then probe. */
static uint64_t *zmap_get_or_put(zmap *m, uint32_t key, int *found_existing) {
    if (1 > m->available) {
        uint32_t load = zmap_max_load(m->cap) - m->available;
        zmap_grow(m, capacity_for_size(load + 1));
    }
    uint32_t mask = m->cap - 1, idx = (uint32_t)(key_hash(key) & mask), limit = m->cap;
    while (m->used[idx] && limit != 0) {
        if (m->keys[idx] == key) {
            *found_existing = 1;
            return &m->vals[idx];
        }
        limit--;
        idx = (idx + 1) & mask;
    }
    m->available--;
    m->used[idx] = 1;
    m->keys[idx] = key;
    m->size++;
    *found_existing = 0;
    return &m->vals[idx];
}

/* ------------------------------------------------------------------------------------ */
/* stable sort by count descending (std.mem.sort == std.sort.block, stable)             */
/* ------------------------------------------------------------------------------------ */
typedef struct { uint32_t pair; uint64_t count; } pair_count;

static void merge_sort_desc(pair_count *a, pair_count *tmp, size_t n) {
    if (n < 2) return;
    size_t h = n / 2;
    merge_sort_desc(a, tmp, h);
    merge_sort_desc(a + h, tmp, n - h);
    size_t i = 0, j = h, k = 0;
    /* lessThan(a,b) = a.count > b.count; take right only when strictly "less" */
    while (i < h && j < n) tmp[k++] = (a[j].count > a[i].count) ? a[j++] : a[i++];
    while (i < h) tmp[k++] = a[i++];
    while (j < n) tmp[k++] = a[j++];
    memcpy(a, tmp, n * sizeof(pair_count));
}

/* ------------------------------------------------------------------------------------ */
/* TimeStats (src/utils/time_statistics.zig:4-13)                                       */
/* ------------------------------------------------------------------------------------ */
typedef struct {
    double sort_pairs_s, replace_pair_s, generate_pairs_s, count_pairs_s, total_s;
    uint64_t sort_pairs_calls, replace_pair_calls, generate_pairs_calls, count_pairs_calls;
    uint64_t pair_tokens; /* sum over iterations of n_t (pairs hashed = n_t - 1) */
    uint64_t tie_iterations;
} zref_stats;

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

/* ------------------------------------------------------------------------------------ */
/* BasicTokenizer.train (basic_tokenizer.zig:140-306)                                   */
/* ------------------------------------------------------------------------------------ */
/* Returns 0 ok, 1 InvalidVocabSize, 2 OutOfMemory.
 * out_triples: 3*(vocab-256) u16 {first, second, new_token}; out_counts: top count per merge;
 * out_ties: number of pairs sharing the top count per merge (may be NULL);
 * out_distinct: D_t per merge (may be NULL); max_merges caps the loop (0 = no cap) so that
 * a bounded CPU sample can be timed. */
/* FNV-1a 64 over the u16 stream's bytes (the long-run goldens record it per merge window). */
uint64_t zref_fnv64(const uint16_t *tok, size_t len) {
    uint64_t h = 0xcbf29ce484222325ULL;
    const uint8_t *p = (const uint8_t *)tok;
    for (size_t i = 0; i < 2 * len; i++) h = (h ^ p[i]) * 0x100000001b3ULL;
    return h;
}

/* zref_train with a progress log: when `progress` is non-NULL, one line per merge
 * "k first second new_token count ties distinct len_after" is appended and flushed, and every
 * `fnv_every` merges (0 = never) a line "fnv k len fnv64" of the stream after merge k, so a
 * multi-hour golden run keeps what it has computed if it is stopped. */
int zref_train_log(const uint8_t *text, size_t n, uint32_t vocab_size, int verbose, uint32_t max_merges,
                   uint16_t *out_triples, uint64_t *out_counts, uint32_t *out_ties, uint32_t *out_distinct,
                   size_t *out_n_merges, zref_stats *stats, uint16_t *out_tokens, size_t *out_n_tokens,
                   const char *progress, uint32_t fnv_every);

int zref_train(const uint8_t *text, size_t n, uint32_t vocab_size, int verbose, uint32_t max_merges,
               uint16_t *out_triples, uint64_t *out_counts, uint32_t *out_ties, uint32_t *out_distinct,
               size_t *out_n_merges, zref_stats *stats, uint16_t *out_tokens, size_t *out_n_tokens) {
    return zref_train_log(text, n, vocab_size, verbose, max_merges, out_triples, out_counts, out_ties,
                          out_distinct, out_n_merges, stats, out_tokens, out_n_tokens, NULL, 0);
}

int zref_train_log(const uint8_t *text, size_t n, uint32_t vocab_size, int verbose, uint32_t max_merges,
                   uint16_t *out_triples, uint64_t *out_counts, uint32_t *out_ties, uint32_t *out_distinct,
                   size_t *out_n_merges, zref_stats *stats, uint16_t *out_tokens, size_t *out_n_tokens,
                   const char *progress, uint32_t fnv_every) {
    zref_stats st;
    memset(&st, 0, sizeof(st));
    double t_train = now_s();
    *out_n_merges = 0;
    if (vocab_size < 256) { /* :147-149 */
        if (stats) *stats = st;
        return 1;
    }
    /* generateInitialTokens (:155-170) + copy in expandVocabulary (:173-175) */
    uint16_t *tok = (uint16_t *)malloc(sizeof(uint16_t) * (n ? n : 1));
    if (!tok) return 2;
    for (size_t i = 0; i < n; i++) tok[i] = text[i];
    FILE *plog = progress ? fopen(progress, "w") : NULL;
    size_t len = n;
    size_t pairs_cap = 0;
    uint32_t *pairs = NULL;
    pair_count *sorted = NULL, *tmp = NULL;
    size_t sorted_cap = 0;
    uint32_t merges_done = 0;

    for (uint32_t cur = 256; cur < vocab_size; cur++) {
        if (max_merges && merges_done >= max_merges) break;
        /* generateCodePointPairs (:234-255). The reference computes len-1 on usize and
         * panics (safe builds) for len == 0; we define it as "no pairs". */
        double t0 = now_s();
        size_t np = len >= 1 ? len - 1 : 0;
        if (np > pairs_cap) {
            pairs_cap = np;
            pairs = (uint32_t *)realloc(pairs, sizeof(uint32_t) * pairs_cap);
        }
        for (size_t i = 0; i < np; i++) pairs[i] = (uint32_t)tok[i] | ((uint32_t)tok[i + 1] << 16);
        double t1 = now_s();
        st.generate_pairs_s += t1 - t0;
        st.generate_pairs_calls++;
        /* countCodePointPairs (:257-278) */
        zmap m;
        memset(&m, 0, sizeof(m));
        for (size_t i = 0; i < np; i++) {
            int found;
            uint64_t *v = zmap_get_or_put(&m, pairs[i], &found);
            if (!found) *v = 1;
            else *v += 1;
        }
        double t2 = now_s();
        st.count_pairs_s += t2 - t1;
        st.count_pairs_calls++;
        st.pair_tokens += len;
        /* sortCodePointPairs (:280-306): iterator (slot order) then stable sort desc */
        if (m.size > sorted_cap) {
            sorted_cap = m.size;
            sorted = (pair_count *)realloc(sorted, sizeof(pair_count) * sorted_cap);
            tmp = (pair_count *)realloc(tmp, sizeof(pair_count) * sorted_cap);
        }
        size_t d = 0;
        for (uint32_t s = 0; s < m.cap; s++)
            if (m.used[s]) {
                sorted[d].pair = m.keys[s];
                sorted[d].count = m.vals[s];
                d++;
            }
        merge_sort_desc(sorted, tmp, d);
        double t3 = now_s();
        st.sort_pairs_s += t3 - t2;
        st.sort_pairs_calls++;
        zmap_free(&m);
        if (d == 0) { /* :188-191 */
            fprintf(stderr, "No more pairs to merge. Stopping early.\n");
            break;
        }
        pair_count top = sorted[0]; /* :193 */
        uint32_t ties = 1;
        while (ties < d && sorted[ties].count == top.count) ties++;
        if (ties > 1) st.tie_iterations++;
        uint16_t first = (uint16_t)top.pair, second = (uint16_t)(top.pair >> 16);
        if (verbose) /* printMergeInfo (:308-317) */
            fprintf(stderr, "merge %u/%u: (%u,%u) -> %u had %llu occurrences\n", cur - 256 + 1,
                    vocab_size - 256, first, second, cur, (unsigned long long)top.count);
        out_triples[3 * merges_done + 0] = first; /* merges.put (:199) */
        out_triples[3 * merges_done + 1] = second;
        out_triples[3 * merges_done + 2] = (uint16_t)cur;
        if (out_counts) out_counts[merges_done] = top.count;
        if (out_ties) out_ties[merges_done] = ties;
        if (out_distinct) out_distinct[merges_done] = (uint32_t)d;
        merges_done++;
        /* replaceTopPairWithNewToken (:207-232): left-to-right, non-overlapping */
        size_t i = 0, j = 0;
        while (i + 1 < len) {
            if (tok[i] == first && tok[i + 1] == second) {
                tok[j] = (uint16_t)cur;
                i += 2;
            } else {
                tok[j] = tok[i];
                i += 1;
            }
            j++;
        }
        if (i < len) tok[j++] = tok[i];
        len = j;
        st.replace_pair_s += now_s() - t3;
        st.replace_pair_calls++;
        if (plog) {
            fprintf(plog, "%u %u %u %u %llu %u %zu %zu\n", merges_done - 1, first, second, cur,
                    (unsigned long long)top.count, ties, d, len);
            if (fnv_every && merges_done % fnv_every == 0)
                fprintf(plog, "fnv %u %zu %016llx\n", merges_done, len,
                        (unsigned long long)zref_fnv64(tok, len));
            fflush(plog);
        }
    }
    if (plog) {
        fprintf(plog, "done %u %zu %016llx\n", merges_done, len, (unsigned long long)zref_fnv64(tok, len));
        fclose(plog);
    }
    st.total_s = now_s() - t_train;
    *out_n_merges = merges_done;
    if (out_tokens && out_n_tokens) {
        memcpy(out_tokens, tok, len * sizeof(uint16_t));
        *out_n_tokens = len;
    } else if (out_n_tokens) {
        *out_n_tokens = len;
    }
    if (stats) *stats = st;
    free(tok);
    free(pairs);
    free(sorted);
    free(tmp);
    return 0;
}

/* ONE iteration of expandVocabulary (basic_tokenizer.zig:183-204) on a given token stream:
 * generateCodePointPairs (:234-255) -> countCodePointPairs (:257-278) -> sortCodePointPairs
 * (:280-306) -> sortedCodePointPairs[0] (:193). Used by the parity tests to check the device's
 * merge k+1 on the device's own stream after k merges (any merge of C3/C4, where a full oracle
 * run is out of reach), and by bench.py's cpu_baseline to time a late merge.
 *   literal = 1: materialise the pairs array and stable-sort the slot-ordered entries, exactly as
 *                the reference does (the cost the CPU baseline prices);
 *   literal = 0: the same map, but pairs are hashed as they are read and the winner is taken as
 *                the first maximum in slot order -- what a stable sort by count descending puts
 *                at [0] -- so no n-sized or D-sized array is allocated.
 * Returns 0 ok, 2 OutOfMemory, 3 no pairs ("Stopping early", :188-191). */
int zref_step(const uint16_t *tok, size_t len, int literal, uint32_t *out_pair, uint64_t *out_count,
              uint32_t *out_ties, uint64_t *out_distinct, zref_stats *stats) {
    zref_stats st;
    memset(&st, 0, sizeof(st));
    double t0 = now_s();
    size_t np = len >= 1 ? len - 1 : 0;
    uint32_t *pairs = NULL;
    if (literal && np) {
        pairs = (uint32_t *)malloc(sizeof(uint32_t) * np);
        if (!pairs) return 2;
        for (size_t i = 0; i < np; i++) pairs[i] = (uint32_t)tok[i] | ((uint32_t)tok[i + 1] << 16);
    }
    double t1 = now_s();
    st.generate_pairs_s = t1 - t0;
    zmap m;
    memset(&m, 0, sizeof(m));
    for (size_t i = 0; i < np; i++) {
        int found;
        uint32_t key = pairs ? pairs[i] : ((uint32_t)tok[i] | ((uint32_t)tok[i + 1] << 16));
        uint64_t *v = zmap_get_or_put(&m, key, &found);
        if (!found) *v = 1;
        else *v += 1;
    }
    double t2 = now_s();
    st.count_pairs_s = t2 - t1;
    st.pair_tokens = len;
    free(pairs);
    size_t d = m.size;
    uint32_t best_pair = 0, ties = 0;
    uint64_t best = 0;
    if (literal && d) {
        pair_count *sorted = (pair_count *)malloc(sizeof(pair_count) * d);
        pair_count *tmp = (pair_count *)malloc(sizeof(pair_count) * d);
        if (!sorted || !tmp) { free(sorted); free(tmp); zmap_free(&m); return 2; }
        size_t k = 0;
        for (uint32_t s = 0; s < m.cap; s++)
            if (m.used[s]) { sorted[k].pair = m.keys[s]; sorted[k].count = m.vals[s]; k++; }
        merge_sort_desc(sorted, tmp, d);
        best_pair = sorted[0].pair;
        best = sorted[0].count;
        while (ties < d && sorted[ties].count == best) ties++;
        free(sorted);
        free(tmp);
    } else {
        for (uint32_t s = 0; s < m.cap; s++) {
            if (!m.used[s]) continue;
            if (m.vals[s] > best) { best = m.vals[s]; best_pair = m.keys[s]; ties = 1; }
            else if (m.vals[s] == best) ties++;
        }
    }
    st.sort_pairs_s = now_s() - t2;
    st.total_s = now_s() - t0;
    zmap_free(&m);
    if (stats) *stats = st;
    if (out_distinct) *out_distinct = d;
    if (d == 0) return 3;
    *out_pair = best_pair;
    *out_count = best;
    if (out_ties) *out_ties = ties;
    return 0;
}

/* Hash-map iteration order of the pair map built from `tokens` (countCodePointPairs +
 * iterator). Writes keys in slot order, their slots, counts; returns the final capacity. */
uint32_t zref_map_order(const uint16_t *tok, size_t len, uint32_t *out_keys, uint32_t *out_slots,
                        uint64_t *out_counts, size_t *out_d) {
    zmap m;
    memset(&m, 0, sizeof(m));
    size_t np = len >= 1 ? len - 1 : 0;
    for (size_t i = 0; i < np; i++) {
        int found;
        uint64_t *v = zmap_get_or_put(&m, (uint32_t)tok[i] | ((uint32_t)tok[i + 1] << 16), &found);
        if (!found) *v = 1;
        else *v += 1;
    }
    size_t d = 0;
    for (uint32_t s = 0; s < m.cap; s++)
        if (m.used[s]) {
            if (out_keys) out_keys[d] = m.keys[s];
            if (out_slots) out_slots[d] = s;
            if (out_counts) out_counts[d] = m.vals[s];
            d++;
        }
    *out_d = d;
    uint32_t cap = m.cap;
    zmap_free(&m);
    return cap;
}

/* ------------------------------------------------------------------------------------ */
/* BasicTokenizer.encode (basic_tokenizer.zig:71-88)                                    */
/* ------------------------------------------------------------------------------------ */
/* literal == 1: the reference's in-place orderedRemove loop, O(M*n^2) worst case.
 * literal == 0: the same left-greedy result with an O(n) compaction per merge. */
int zref_encode(const uint16_t *triples, size_t n_merges, const uint8_t *text, size_t n, int literal,
                uint16_t *out, size_t *out_len) {
    size_t len = n;
    for (size_t i = 0; i < n; i++) out[i] = text[i];
    for (size_t k = 0; k < n_merges; k++) {
        uint16_t a = triples[3 * k], b = triples[3 * k + 1], x = triples[3 * k + 2];
        if (literal) {
            size_t i = 0;
            while (i < len) {
                if (i + 1 < len && out[i] == a && out[i + 1] == b) {
                    out[i] = x;
                    memmove(out + i + 1, out + i + 2, (len - i - 2) * sizeof(uint16_t));
                    len--;
                } else {
                    i++;
                }
            }
        } else {
            /* identical to the literal loop, including x == a re-matching: after a hit the
             * literal loop re-tests position i (now x) against (a, b). */
            size_t i = 0, j = 0;
            while (i < len) {
                if (i + 1 < len && out[i] == a && out[i + 1] == b) {
                    if (x == a) { /* rare: new token equals first (it chains); defer to literal */
                        return zref_encode(triples, n_merges, text, n, 1, out, out_len);
                    }
                    out[j++] = x;
                    i += 2;
                } else {
                    out[j++] = out[i++];
                }
            }
            len = j;
        }
    }
    *out_len = len;
    return 0;
}

/* ------------------------------------------------------------------------------------ */
/* decode (basic_tokenizer.zig:90-138): first matching merge, recursive left then right */
/* ------------------------------------------------------------------------------------ */
static long find_merge(const uint16_t *triples, size_t n_merges, uint16_t tok) {
    for (size_t k = 0; k < n_merges; k++)
        if (triples[3 * k + 2] == tok) return (long)k;
    return -1;
}
static int decode_merge(const uint16_t *triples, size_t n_merges, long k, uint8_t *out, size_t cap,
                        size_t *len, int depth) {
    if (depth > 70000) return 3;
    for (int side = 0; side < 2; side++) {
        uint16_t t = triples[3 * k + side];
        if (t < 256) {
            if (*len >= cap) return 2;
            out[(*len)++] = (uint8_t)t;
        } else {
            long s = find_merge(triples, n_merges, t);
            if (s < 0) return 1;
            int rc = decode_merge(triples, n_merges, s, out, cap, len, depth + 1);
            if (rc) return rc;
        }
    }
    return 0;
}
/* 0 ok, 1 InvalidToken, 2 output capacity exceeded */
int zref_decode(const uint16_t *triples, size_t n_merges, const uint16_t *tokens, size_t n, uint8_t *out,
                size_t cap, size_t *out_len) {
    size_t len = 0;
    for (size_t i = 0; i < n; i++) {
        if (tokens[i] < 256) {
            if (len >= cap) return 2;
            out[len++] = (uint8_t)tokens[i];
        } else {
            long k = find_merge(triples, n_merges, tokens[i]);
            if (k < 0) return 1;
            int rc = decode_merge(triples, n_merges, k, out, cap, &len, 0);
            if (rc) return rc;
        }
    }
    *out_len = len;
    return 0;
}

/* Zig std.hash.Wyhash test vectors (lib/std/hash/wyhash.zig, Zig 0.13) + pair hashes.
 * Returns the number of failures. */
int zref_selftest(void) {
    struct { uint64_t seed; const char *in; uint64_t want; } v[] = {
        {0, "", 0x0409638ee2bde459ULL},
        {1, "a", 0xa8412d091b5fe0a9ULL},
        {2, "abc", 0x32dd92e4b2915153ULL},
        {3, "message digest", 0x8619124089a3a16bULL},
        {4, "abcdefghijklmnopqrstuvwxyz", 0x7a43afb61d7f5f40ULL},
        {5, "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789", 0xff42329b90e50d58ULL},
        {6, "12345678901234567890123456789012345678901234567890123456789012345678901234567890",
         0xc39cab13b115aad3ULL},
    };
    int fails = 0;
    for (size_t i = 0; i < sizeof(v) / sizeof(v[0]); i++)
        if (zref_wyhash(v[i].seed, (const uint8_t *)v[i].in, strlen(v[i].in)) != v[i].want) fails++;
    /* the map's unfolded key hash == Wyhash.hash(0, key bytes) */
    uint32_t k = 0x12345u;
    for (int i = 0; i < 4096; i++, k = k * 2654435761u + 12345u)
        if (key_hash(k) != zref_pair_hash((uint16_t)k, (uint16_t)(k >> 16))) { fails++; break; }
    return fails;
}

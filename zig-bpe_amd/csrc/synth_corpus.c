/*
 * Seeded synthetic corpora for the BPE trainer benchmarks and parity tests.
 * The reference ships one corpus (taylorswift.txt); configs C2-C5 need corpora that do not exist
 * offline, so they are generated here, deterministically from (kind, seed, n_bytes):
 *
 *   kind 0  "words": Zipf(s=1.1) pseudo-words over an English-like letter distribution,
 *           separated by spaces / punctuation / newlines. ASCII only (C2).
 *   kind 1  "words+utf8": as kind 0, with ~utf8_permille/1000 of the vocabulary made of
 *           multi-byte UTF-8 words (Latin-1 accents, Hangul, CJK, emoji) (C3/C4/C5 stand-in
 *           for a Wikipedia slice).
 *   kind 2  "uniform": uniform printable ASCII bytes (tie-break stress: most iterations tie).
 *   kind 3  "runs": long runs of a few symbols (self-pair (a,a) stress).
 *
 * The output is produced in independent 1 MiB chunks, each from its own PRNG stream, so the
 * bytes do not depend on the number of threads used.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>

typedef struct { uint64_t s[4]; } rng_t;
static uint64_t splitmix(uint64_t *x) {
    uint64_t z = (*x += 0x9e3779b97f4a7c15ULL);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}
static void rng_seed(rng_t *r, uint64_t seed) {
    uint64_t x = seed;
    for (int i = 0; i < 4; i++) r->s[i] = splitmix(&x);
}
static inline uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
static inline uint64_t rng_next(rng_t *r) { /* xoshiro256** */
    uint64_t *s = r->s, res = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
    s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3]; s[2] ^= t; s[3] = rotl(s[3], 45);
    return res;
}
static inline double rng_unit(rng_t *r) { return (rng_next(r) >> 11) * (1.0 / 9007199254740992.0); }
static inline uint32_t rng_below(rng_t *r, uint32_t n) { return (uint32_t)(((rng_next(r) >> 32) * n) >> 32); }

/* English letter frequencies (per mille, a..z) */
static const int LETTER_PM[26] = {82, 15, 28, 43, 127, 22, 20, 61, 70, 2, 8, 40, 24,
                                  67, 75, 19, 1, 60, 63, 91, 28, 10, 24, 2, 20, 1};

#define NWORDS 60000
#define MAXW 24
typedef struct {
    uint8_t bytes[NWORDS][MAXW];
    uint8_t len[NWORDS];
    /* alias table over word ranks, Zipf(1.1) */
    double prob[NWORDS];
    uint32_t alias[NWORDS];
} vocab_t;

static size_t put_utf8(uint8_t *o, uint32_t cp) {
    if (cp < 0x80) { o[0] = (uint8_t)cp; return 1; }
    if (cp < 0x800) { o[0] = 0xC0 | (cp >> 6); o[1] = 0x80 | (cp & 63); return 2; }
    if (cp < 0x10000) { o[0] = 0xE0 | (cp >> 12); o[1] = 0x80 | ((cp >> 6) & 63); o[2] = 0x80 | (cp & 63); return 3; }
    o[0] = 0xF0 | (cp >> 18); o[1] = 0x80 | ((cp >> 12) & 63); o[2] = 0x80 | ((cp >> 6) & 63); o[3] = 0x80 | (cp & 63);
    return 4;
}

static void build_vocab(vocab_t *v, uint64_t seed, int utf8_permille) {
    rng_t r;
    rng_seed(&r, seed ^ 0x766f636162ULL);
    int cdf[26], acc = 0;
    for (int i = 0; i < 26; i++) { acc += LETTER_PM[i]; cdf[i] = acc; }
    for (int w = 0; w < NWORDS; w++) {
        uint8_t *o = v->bytes[w];
        size_t L = 0;
        int utf = utf8_permille > 0 && (int)rng_below(&r, 1000) < utf8_permille;
        /* frequent words are short: length grows slowly with rank */
        int base = 1 + (w < 30 ? (int)rng_below(&r, 3) : w < 1000 ? 2 + (int)rng_below(&r, 4) : 3 + (int)rng_below(&r, 7));
        if (utf) {
            int script = (int)rng_below(&r, 4), n = 1 + (int)rng_below(&r, base > 4 ? 4 : base);
            for (int i = 0; i < n && L + 4 <= MAXW; i++) {
                uint32_t cp;
                switch (script) {
                case 0: cp = 0xE0 + rng_below(&r, 32); break;         /* Latin-1 accented */
                case 1: cp = 0xAC00 + rng_below(&r, 400); break;      /* Hangul syllables */
                case 2: cp = 0x4E00 + rng_below(&r, 600); break;      /* CJK ideographs */
                default: cp = 0x1F600 + rng_below(&r, 64); break;     /* emoji */
                }
                if (script == 0 && (i & 1)) { /* mix accents with letters */
                    int x = (int)rng_below(&r, acc), c = 0;
                    while (cdf[c] <= x) c++;
                    cp = 'a' + c;
                }
                L += put_utf8(o + L, cp);
            }
        } else {
            for (int i = 0; i < base && L < MAXW; i++) {
                int x = (int)rng_below(&r, acc), c = 0;
                while (cdf[c] <= x) c++;
                o[L++] = (uint8_t)('a' + c);
            }
            if (w % 17 == 5 && L > 0) o[0] = (uint8_t)(o[0] - 'a' + 'A'); /* some capitalised */
        }
        v->len[w] = (uint8_t)L;
    }
    /* Zipf(1.1) weights -> Vose alias table */
    double *p = (double *)malloc(sizeof(double) * NWORDS), sum = 0;
    for (int w = 0; w < NWORDS; w++) { p[w] = 1.0; double x = w + 1.0; p[w] = 1.0 / (x * pow(x, 0.1)); sum += p[w]; }
    uint32_t *small = (uint32_t *)malloc(sizeof(uint32_t) * NWORDS), *large = (uint32_t *)malloc(sizeof(uint32_t) * NWORDS);
    int ns = 0, nl = 0;
    for (int w = 0; w < NWORDS; w++) {
        p[w] = p[w] * NWORDS / sum;
        if (p[w] < 1.0) small[ns++] = w; else large[nl++] = w;
    }
    while (ns && nl) {
        uint32_t s = small[--ns], l = large[--nl];
        v->prob[s] = p[s];
        v->alias[s] = l;
        p[l] = (p[l] + p[s]) - 1.0;
        if (p[l] < 1.0) small[ns++] = l; else large[nl++] = l;
    }
    while (nl) { uint32_t l = large[--nl]; v->prob[l] = 1.0; v->alias[l] = l; }
    while (ns) { uint32_t s = small[--ns]; v->prob[s] = 1.0; v->alias[s] = s; }
    free(p); free(small); free(large);
}

typedef struct {
    const vocab_t *v;
    int kind;
    uint64_t seed;
    uint8_t *out;
    size_t n;
    size_t chunk0, chunk1;
} job_t;

#define CHUNK (1u << 20)

static void gen_chunk(const job_t *j, size_t c) {
    size_t beg = c * (size_t)CHUNK, end = beg + CHUNK;
    if (end > j->n) end = j->n;
    uint8_t *o = j->out;
    rng_t r;
    rng_seed(&r, j->seed * 0x100000001b3ULL + c * 0x9E3779B97F4A7C15ULL + 1);
    size_t p = beg;
    if (j->kind == 2) {
        for (; p < end; p++) o[p] = (uint8_t)(32 + rng_below(&r, 95));
        return;
    }
    if (j->kind == 3) {
        static const uint8_t sym[5] = {'a', 'a', 'b', ' ', '='};
        while (p < end) {
            uint8_t s = sym[rng_below(&r, 5)];
            uint32_t L = 1 + rng_below(&r, 1 + rng_below(&r, 64));
            for (uint32_t i = 0; i < L && p < end; i++) o[p++] = s;
        }
        return;
    }
    const vocab_t *v = j->v;
    while (p < end) {
        uint32_t w = rng_below(&r, NWORDS);
        if (rng_unit(&r) >= v->prob[w]) w = v->alias[w];
        for (int i = 0; i < v->len[w] && p < end; i++) o[p++] = v->bytes[w][i];
        uint32_t x = rng_below(&r, 1000);
        const char *sep = x < 850 ? " " : x < 910 ? ", " : x < 960 ? ". " : x < 980 ? ".\n" : x < 990 ? "\n" : x < 995 ? "! " : "? ";
        for (const char *s = sep; *s && p < end; s++) o[p++] = (uint8_t)*s;
    }
}

static void *worker(void *arg) {
    job_t *j = (job_t *)arg;
    for (size_t c = j->chunk0; c < j->chunk1; c++) gen_chunk(j, c);
    return NULL;
}

/* Returns 0 on success. kind/seed as above; utf8_permille applies to kind 1. */
int zbpe_synth_corpus(int kind, uint64_t seed, int utf8_permille, uint8_t *out, size_t n, int threads) {
    vocab_t *v = NULL;
    if (kind == 0 || kind == 1) {
        v = (vocab_t *)calloc(1, sizeof(vocab_t));
        if (!v) return 2;
        build_vocab(v, seed, kind == 1 ? utf8_permille : 0);
    } else if (kind != 2 && kind != 3) {
        return 1;
    }
    size_t nchunks = (n + CHUNK - 1) / CHUNK;
    if (threads < 1) threads = 1;
    if ((size_t)threads > nchunks) threads = (int)(nchunks ? nchunks : 1);
    job_t *jobs = (job_t *)calloc((size_t)threads, sizeof(job_t));
    pthread_t *th = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    for (int t = 0; t < threads; t++) {
        jobs[t] = (job_t){v, kind, seed, out, n, nchunks * t / threads, nchunks * (t + 1) / threads};
        pthread_create(&th[t], NULL, worker, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    free(jobs);
    free(th);
    free(v);
    return 0;
}

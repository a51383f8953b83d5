/*
 * A C consumer of include/zbpe.h: what the reference's CLI (src/main.zig:8-43) does, through the
 * C ABI alone, as a Zig `@cImport` binding would see it. Trains the given text at vocab 300, writes
 * merges.txt (serializeMerges, basic_tokenizer.zig:319-330), encodes and decodes the main.zig:25
 * string, prints the reference's time statistics. Exit status 0 when decode(encode(s)) == s.
 *
 *   main <taylorswift.txt> <merges.txt out>
 */
#define _POSIX_C_SOURCE 199309L
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "zbpe.h"

#define VOCAB 300

static long find_merge(const uint16_t *tri, size_t n, uint16_t tok) { /* findMerge: the first match */
    for (size_t k = 0; k < n; k++)
        if (tri[3 * k + 2] == tok) return (long)k;
    return -1;
}

/* decode (basic_tokenizer.zig:90-138): host-side, like the reference */
static int decode_tok(const uint16_t *tri, size_t n, uint16_t tok, uint8_t *out, size_t cap, size_t *len, int depth) {
    if (tok < 256) {
        if (*len >= cap) return 2;
        out[(*len)++] = (uint8_t)tok;
        return 0;
    }
    long k = find_merge(tri, n, tok);
    if (k < 0 || depth > 65536) return 1; /* error.InvalidToken */
    int rc = decode_tok(tri, n, tri[3 * k], out, cap, len, depth + 1);
    return rc ? rc : decode_tok(tri, n, tri[3 * k + 1], out, cap, len, depth + 1);
}

static int die(zbpe_ctx *ctx, const char *what, zbpe_status s) {
    fprintf(stderr, "%s failed (%d): %s\n", what, (int)s, zbpe_last_error(ctx));
    zbpe_destroy(ctx);
    return 2;
}

int main(int argc, char **argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: %s <text> <merges.txt out>\n", argv[0]);
        return 64;
    }
    FILE *f = fopen(argv[1], "rb");
    if (!f) { perror(argv[1]); return 66; }
    fseek(f, 0, SEEK_END);
    const long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    uint8_t *text = (uint8_t *)malloc((size_t)n + 1);
    if (!text || fread(text, 1, (size_t)n, f) != (size_t)n) { fclose(f); return 66; }
    fclose(f);

    printf("%s\n", zbpe_version());
    zbpe_ctx *ctx = NULL;
    zbpe_status s = zbpe_create(0, &ctx);
    if (s != ZBPE_OK) return die(ctx, "zbpe_create", s);

    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    uint16_t triples[3 * (VOCAB - 256)];
    uint64_t counts[VOCAB - 256];
    size_t n_merges = 0;
    zbpe_stats st;
    s = zbpe_train(ctx, text, (size_t)n, VOCAB, 0, triples, counts, &n_merges, &st);
    if (s != ZBPE_OK) return die(ctx, "zbpe_train", s);
    uint64_t bad = 1;
    s = zbpe_verify_counts(ctx, &bad);
    if (s != ZBPE_OK || bad) return die(ctx, "zbpe_verify_counts", s);
    size_t n_tok = 0;
    s = zbpe_tokens(ctx, NULL, 0, &n_tok);
    if (s != ZBPE_OK || n_tok != st.final_tokens) return die(ctx, "zbpe_tokens", s);

    FILE *m = fopen(argv[2], "wb"); /* serializeMerges */
    if (!m) { perror(argv[2]); zbpe_destroy(ctx); return 73; }
    for (size_t k = 0; k < n_merges; k++) fprintf(m, "%u,%u,%u\n", triples[3 * k], triples[3 * k + 1], triples[3 * k + 2]);
    fclose(m);

    const char *msg = "hello world!!!? (\xec\x95\x88\xeb\x85\x95\xed\x95\x98\xec\x84\xb8\xec\x9a\x94!) lol123 \xf0\x9f\x98\x89";
    const size_t mlen = strlen(msg);
    uint16_t enc[128];
    size_t n_enc = 0;
    s = zbpe_encode(ctx, triples, n_merges, (const uint8_t *)msg, mlen, enc, &n_enc);
    if (s != ZBPE_OK) return die(ctx, "zbpe_encode", s);
    for (size_t i = 0; i < n_enc; i++) printf("%u ", enc[i]);
    uint8_t dec[256];
    size_t n_dec = 0;
    for (size_t i = 0; i < n_enc; i++)
        if (decode_tok(triples, n_merges, enc[i], dec, sizeof dec, &n_dec, 0)) { zbpe_destroy(ctx); return 3; }
    printf("\n%.*s\n", (int)n_dec, (const char *)dec);
    clock_gettime(CLOCK_MONOTONIC, &t1);

    char stats_text[1024];
    size_t stats_len = 0;
    s = zbpe_format_time_stats(&st, stats_text, sizeof stats_text, &stats_len);
    if (s != ZBPE_OK) return die(ctx, "zbpe_format_time_stats", s);
    fputs(stats_text, stderr);
    printf("Training completed in %ld ms\n", (long)((t1.tv_sec - t0.tv_sec) * 1000 + (t1.tv_nsec - t0.tv_nsec) / 1000000));
    printf("merges %zu, final tokens %llu\n", n_merges, (unsigned long long)st.final_tokens);
    zbpe_destroy(ctx);
    free(text);
    return (n_dec == mlen && memcmp(dec, msg, mlen) == 0 && n_merges == VOCAB - 256) ? 0 : 1;
}

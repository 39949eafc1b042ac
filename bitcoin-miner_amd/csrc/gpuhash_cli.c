/* gpuhash_cli.c -- plain-C client of the C ABI (include/gpuhash.h), no Python/torch.
 *
 * It makes the same calls, in the same order, as the cgo binding in
 * integration/go/gpuhash/gpuhash.go.  That is the miner's sequence: open once, then per
 * Request (bitcoin/message.go:25-32) one gpuhash_min, answered as NewResult(hash, nonce)
 * (message.go:36-42), with the optional one-nonce self-check through gpuhash_hash_cpu
 * (== bitcoin.Hash, hash.go:11-15).
 *
 *   gpuhash_cli MSG LOWER UPPER        -> "Result <hash> <nonce>" (the client's output format)
 *   gpuhash_cli --range MSG LOWER COUNT -> one hash per line (gpuhash_hash_range)
 *   gpuhash_cli --version
 * Exit status: 0 ok, 2 usage, 3 library error (message on stderr), 4 self-check mismatch.
 */
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "gpuhash.h"

static int parse_u64(const char *s, uint64_t *out) {
    char *end = NULL;
    if (!s || !*s || *s == '-') return -1;
    unsigned long long v = strtoull(s, &end, 10);
    if (*end) return -1;
    *out = (uint64_t)v;
    return 0;
}

static int fail(const char *what, int rc) {
    fprintf(stderr, "%s: %s (rc=%d)\n", what, gpuhash_strerror(rc), rc);
    return 3;
}

int main(int argc, char **argv) {
    if (argc == 2 && strcmp(argv[1], "--version") == 0) {
        printf("%s\n", gpuhash_version());
        return 0;
    }
    const int range_mode = argc == 5 && strcmp(argv[1], "--range") == 0;
    if (!range_mode && argc != 4) {
        fprintf(stderr, "usage: %s MSG LOWER UPPER | --range MSG LOWER COUNT | --version\n", argv[0]);
        return 2;
    }
    const char *msg = argv[range_mode ? 2 : 1];
    uint64_t a, b;
    if (parse_u64(argv[range_mode ? 3 : 2], &a) || parse_u64(argv[range_mode ? 4 : 3], &b)) {
        fprintf(stderr, "bad number\n");
        return 2;
    }
    gpuhash_ctx *ctx = NULL;
    int rc = gpuhash_open(NULL, 0, &ctx);
    if (rc) return fail("gpuhash_open", rc);
    const size_t len = strlen(msg);
    int status = 0;
    if (range_mode) {
        uint64_t *out = (uint64_t *)malloc((size_t)(b ? b : 1) * sizeof(uint64_t));
        if (!out) { gpuhash_close(ctx); return 3; }
        rc = gpuhash_hash_range(ctx, (const uint8_t *)msg, len, a, b, out);
        if (rc) status = fail("gpuhash_hash_range", rc);
        for (uint64_t i = 0; !rc && i < b; i++) printf("%" PRIu64 "\n", out[i]);
        free(out);
    } else {
        uint64_t h = 0, n = 0;
        rc = gpuhash_min(ctx, (const uint8_t *)msg, len, a, b, &h, &n);
        if (rc) {
            status = fail("gpuhash_min", rc);
        } else if (gpuhash_hash_cpu((const uint8_t *)msg, len, n) != h) {
            fprintf(stderr, "self-check failed: Hash(msg, %" PRIu64 ") != %" PRIu64 "\n", n, h);
            status = 4;
        } else {
            printf("Result %" PRIu64 " %" PRIu64 "\n", h, n);
        }
    }
    gpuhash_close(ctx);
    return status;
}

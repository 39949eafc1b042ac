/*
 * oracle/cpu_baseline.c -- the reference miner's loop on the CPU, for bench.py's
 * cpu_baseline leg.
 *
 * TEST / BENCH INFRASTRUCTURE ONLY: bench.py times it as the CPU baseline and
 * tests/test_oracle.py checks it against oracle/hash_oracle.c.  The product path never
 * links or calls it.
 *
 * hash_oracle.c restates SHA-256 in plain C, which is the checker but slower than what
 * the reference would run: Go's crypto/sha256 has an amd64 assembly block function
 * (SHA-NI / AVX2).  This file times the spec'd loop (p1.pdf pp.12-14; the miner stub at
 * src/github.com/cmu440/bitcoin/miner/miner.go:15) with a comparable library SHA-256:
 * OpenSSL's SHA-256 from the system libcrypto (loaded at run time; SHA-NI where the
 * CPU has it), run per nonce on a freshly formatted and allocated "%s %d" buffer like
 * bitcoin.Hash (hash.go:12-14), ascending with strict '<'.  Optional threads scan
 * contiguous sub-ranges and merge with the lexicographic key (the SURVEY's "one
 * goroutine per core" variant).
 */
#include <dlfcn.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* The low-level SHA256_Init/Update/Final (the one-shot SHA256() of OpenSSL 3 fetches a
 * provider per call, which costs more than the hash and serialises threads).  The
 * context is opaque here: SHA256_CTX is 112 bytes. */
typedef struct { uint64_t words[16]; } sha_ctx;
typedef int (*init_fn)(sha_ctx *);
typedef int (*update_fn)(sha_ctx *, const void *, size_t);
typedef int (*final_fn)(unsigned char *, sha_ctx *);
typedef struct { init_fn init; update_fn update; final_fn final; } sha_lib;
typedef const sha_lib *sha256_fn;

static sha256_fn resolve(void) {
    static sha_lib lib;
    static int state = 0; /* 0 untried, 1 ok, -1 unavailable */
    if (state == 0) {
        state = -1;
        void *h = dlopen("libcrypto.so.3", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("libcrypto.so", RTLD_NOW | RTLD_LOCAL);
        if (h) {
            lib.init = (init_fn)dlsym(h, "SHA256_Init");
            lib.update = (update_fn)dlsym(h, "SHA256_Update");
            lib.final = (final_fn)dlsym(h, "SHA256_Final");
            if (lib.init && lib.update && lib.final) state = 1;
        }
    }
    return state == 1 ? &lib : NULL;
}

/* 1 if the library SHA-256 is available, else 0. */
int baseline_available(void) { return resolve() != NULL; }

static int fmt_u64(uint64_t v, char *buf) {
    char tmp[20];
    int n = 0;
    do { tmp[n++] = (char)('0' + (int)(v % 10u)); v /= 10u; } while (v);
    for (int i = 0; i < n; i++) buf[i] = tmp[n - 1 - i];
    return n;
}

static uint64_t hash_one(sha256_fn sha, const uint8_t *msg, size_t len, uint64_t nonce) {
    uint8_t *buf = (uint8_t *)malloc(len + 22); /* Sprintf + []byte: one allocation */
    unsigned char md[32];
    memcpy(buf, msg, len);
    buf[len] = ' ';
    int nd = fmt_u64(nonce, (char *)buf + len + 1);
    sha_ctx c;
    sha->init(&c); /* sha256.New() */
    sha->update(&c, buf, len + 1 + (size_t)nd); /* hasher.Write */
    sha->final(md, &c); /* hasher.Sum(nil) */
    free(buf);
    uint64_t h = 0;
    for (int i = 0; i < 8; i++) h = (h << 8) | md[i]; /* binary.BigEndian.Uint64(digest[0:8]) */
    return h;
}

uint64_t baseline_hash(const uint8_t *msg, size_t len, uint64_t nonce) {
    sha256_fn sha = resolve();
    return sha ? hash_one(sha, msg, len, nonce) : 0;
}

static int scan(const uint8_t *msg, size_t len, uint64_t lower, uint64_t upper, uint64_t *oh, uint64_t *on) {
    sha256_fn sha = resolve();
    if (!sha) return -2;
    uint64_t best = hash_one(sha, msg, len, lower), bn = lower;
    for (uint64_t n = lower; n != upper;) {
        n++;
        uint64_t h = hash_one(sha, msg, len, n);
        if (h < best) { best = h; bn = n; }
    }
    *oh = best;
    *on = bn;
    return 0;
}

typedef struct {
    const uint8_t *msg; size_t len; uint64_t lo, hi, h, n; int rc;
} span_t;

static void *worker(void *p) {
    span_t *s = (span_t *)p;
    s->rc = scan(s->msg, s->len, s->lo, s->hi, &s->h, &s->n);
    return NULL;
}

/* argmin over [lower, upper] of (Hash, nonce); 0 ok, -1 lower > upper, -2 no libcrypto */
int baseline_min(const uint8_t *msg, size_t len, uint64_t lower, uint64_t upper, int nthreads,
                 uint64_t *out_hash, uint64_t *out_nonce) {
    if (lower > upper) return -1;
    if (!resolve()) return -2;
    if (nthreads < 1) nthreads = 1;
    uint64_t span = upper - lower;
    if ((uint64_t)nthreads > span + 1u) nthreads = (int)(span + 1u);
    if (nthreads == 1) return scan(msg, len, lower, upper, out_hash, out_nonce);
    span_t *s = (span_t *)calloc((size_t)nthreads, sizeof(span_t));
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    if (!s || !th) { free(s); free(th); return -3; }
    uint64_t per = span / (uint64_t)nthreads + 1u, cur = lower;
    int used = 0;
    for (int i = 0; i < nthreads; i++) {
        uint64_t hi = (upper - cur < per - 1u) ? upper : cur + (per - 1u);
        s[i] = (span_t){msg, len, cur, hi, 0, 0, 0};
        pthread_create(&th[i], NULL, worker, &s[i]);
        used++;
        if (hi == upper) break;
        cur = hi + 1u;
    }
    int rc = 0;
    uint64_t bh = ~0ull, bn = ~0ull;
    for (int i = 0; i < used; i++) {
        pthread_join(th[i], NULL);
        if (s[i].rc) rc = s[i].rc;
        if (s[i].h < bh || (s[i].h == bh && s[i].n < bn)) { bh = s[i].h; bn = s[i].n; }
    }
    free(s);
    free(th);
    *out_hash = bh;
    *out_nonce = bn;
    return rc;
}

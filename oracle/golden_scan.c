/*
 * oracle/golden_scan.c -- fast multi-threaded CPU scan for the LARGE golden fixtures.
 *
 * TEST INFRASTRUCTURE ONLY.  tests/golden/make_golden.py runs it to produce the
 * expected (hash, nonce) of searches too big for hash_oracle.c in reasonable time
 * (config 4's [0, 2^40) and config 5's per-client [0, 2^36]); tests/test_oracle.py
 * checks it against hash_oracle.c and hashlib.  The product path never links or calls it.
 *
 * What it restates: the same thing as hash_oracle.c --
 *   bitcoin.Hash  src/github.com/cmu440/bitcoin/hash.go:11-15  (SHA-256 of
 *   msg ‖ ' ' ‖ "%d"(nonce), first 8 digest bytes big-endian), and the spec'd miner
 *   loop (p1.pdf pp.12-14, stub miner.go:15): argmin over the INCLUSIVE [lower, upper]
 *   of the key (hash, nonce), i.e. an ascending strict-'<' scan.
 * It is a THIRD, independent implementation of SHA-256: the x86 SHA extensions
 * (sha256rnds2 / sha256msg1 / sha256msg2, Intel SDM), so a golden produced here does
 * not share arithmetic with the plain-C oracle nor with the HIP kernels.  What it adds
 * over hash_oracle.c is speed only:
 *   - whole 64-byte blocks of msg+' ' before the first digit are compressed once
 *     (a midstate; FIPS 180-4 processes blocks in order, so this is exact);
 *   - the decimal digits are advanced in place (no re-formatting per nonce);
 *   - NB nonces are compressed interleaved to hide the SHA-NI latency;
 *   - threads take 2^22-nonce chunks from an atomic counter and merge with the key.
 * Chunks are split at powers of ten so the digit count is fixed inside a segment.
 */
#include <immintrin.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define NB 4                       /* nonces compressed together per thread */
#define CHUNK (1ull << 22)         /* nonces per work item */

static const uint32_t K256[64] __attribute__((aligned(16))) = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u,
    0x923f82a4u, 0xab1c5ed5u, 0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u,
    0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u, 0xe49b69c1u, 0xefbe4786u,
    0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u,
    0x06ca6351u, 0x14292967u, 0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u,
    0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u, 0xa2bfe8a1u, 0xa81a664bu,
    0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au,
    0x5b9cca4fu, 0x682e6ff3u, 0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u,
    0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

static const uint32_t IV[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                               0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};

/* state words a..h -> the SHA-NI register pair (ABEF, CDGH) */
static void to_ni(const uint32_t st[8], __m128i *abef, __m128i *cdgh) {
    __m128i t = _mm_loadu_si128((const __m128i *)st);        /* d c b a */
    __m128i s1 = _mm_loadu_si128((const __m128i *)(st + 4)); /* h g f e */
    t = _mm_shuffle_epi32(t, 0xB1);                            /* c d a b */
    s1 = _mm_shuffle_epi32(s1, 0x1B);                          /* e f g h */
    *abef = _mm_alignr_epi8(t, s1, 8);                         /* a b e f */
    *cdgh = _mm_blend_epi16(s1, t, 0xF0);                      /* c d g h */
}

static void from_ni(__m128i abef, __m128i cdgh, uint32_t st[8]) {
    __m128i t = _mm_shuffle_epi32(abef, 0x1B);   /* f e b a */
    cdgh = _mm_shuffle_epi32(cdgh, 0xB1);        /* d c h g */
    __m128i lo = _mm_blend_epi16(t, cdgh, 0xF0); /* d c b a */
    __m128i hi = _mm_alignr_epi8(cdgh, t, 8);    /* h g f e */
    _mm_storeu_si128((__m128i *)st, lo);
    _mm_storeu_si128((__m128i *)(st + 4), hi);
}

/* Big-endian 32-bit word loads of one 64-byte block (FIPS 180-4 5.2.1). */
static inline void load_block(const uint8_t *blk, __m128i m[4]) {
    const __m128i bswap = _mm_set_epi64x(0x0c0d0e0f08090a0bull, 0x0405060700010203ull);
    for (int i = 0; i < 4; i++)
        m[i] = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i *)(blk + 16 * i)), bswap);
}

/* NB independent compressions (FIPS 180-4 6.2.2), interleaved. */
static inline void compress_nb(__m128i abef[NB], __m128i cdgh[NB], __m128i w[NB][4]) {
    __m128i s0[NB], s1[NB];
    for (int b = 0; b < NB; b++) { s0[b] = abef[b]; s1[b] = cdgh[b]; }
    for (int g = 0; g < 16; g++) {
        const __m128i k = _mm_load_si128((const __m128i *)&K256[4 * g]);
        for (int b = 0; b < NB; b++) {
            __m128i kw = _mm_add_epi32(w[b][g & 3], k);
            s1[b] = _mm_sha256rnds2_epu32(s1[b], s0[b], kw);
            kw = _mm_shuffle_epi32(kw, 0x0E);
            s0[b] = _mm_sha256rnds2_epu32(s0[b], s1[b], kw);
        }
        if (g < 12) {
            /* W[4g+16 .. 4g+19] replaces W[4g .. 4g+3] in slot g&3 */
            for (int b = 0; b < NB; b++) {
                __m128i *q = w[b];
                __m128i t = _mm_sha256msg1_epu32(q[g & 3], q[(g + 1) & 3]);
                t = _mm_add_epi32(t, _mm_alignr_epi8(q[(g + 3) & 3], q[(g + 2) & 3], 4));
                q[g & 3] = _mm_sha256msg2_epu32(t, q[(g + 3) & 3]);
            }
        }
    }
    for (int b = 0; b < NB; b++) {
        abef[b] = _mm_add_epi32(abef[b], s0[b]);
        cdgh[b] = _mm_add_epi32(cdgh[b], s1[b]);
    }
}

static void compress1(uint32_t st[8], const uint8_t *blk) {
    __m128i abef[NB], cdgh[NB], w[NB][4];
    to_ni(st, &abef[0], &cdgh[0]);
    load_block(blk, w[0]);
    for (int b = 1; b < NB; b++) { abef[b] = abef[0]; cdgh[b] = cdgh[0]; memcpy(w[b], w[0], sizeof w[0]); }
    compress_nb(abef, cdgh, w);
    from_ni(abef[0], cdgh[0], st);
}

static int ndigits(uint64_t v) {
    int d = 1;
    while (v >= 10u) { v /= 10u; d++; }
    return d;
}

static void fmt_fixed(uint64_t v, int d, uint8_t *out) {
    for (int i = d - 1; i >= 0; i--) { out[i] = (uint8_t)('0' + v % 10u); v /= 10u; }
}

/* add k to the ASCII decimal number at p[0..d-1] (digit by digit with carry); the
 * caller guarantees no carry out of the top digit (segments never cross a power of ten) */
static inline void add_digits(uint8_t *p, int d, unsigned k) {
    for (int i = d - 1; k && i >= 0; i--) {
        unsigned v = (unsigned)(p[i] - '0') + k;
        p[i] = (uint8_t)('0' + v % 10u);
        k = v / 10u;
    }
}

typedef struct {
    const uint8_t *msg; size_t len;
    uint64_t lower, upper, nchunks;
    uint32_t mid[8];          /* state after the nonce-free prefix blocks */
    size_t nfull;             /* number of such blocks */
    _Atomic uint64_t next, done;
    pthread_mutex_t mu;
    uint64_t best_h, best_n;
    int progress, avx512;
} job_t;

static inline int better(uint64_t h, uint64_t n, uint64_t bh, uint64_t bn) {
    return h < bh || (h == bh && n < bn);
}

/* argmin over [lo, hi], every nonce with the same digit count d */
static void scan_segment(const job_t *J, uint64_t lo, uint64_t hi, int d, uint64_t *bh, uint64_t *bn) {
    const size_t tl = J->len + 1 - 64 * J->nfull;   /* prefix bytes in the tail blocks */
    const size_t L = J->len + 1 + (size_t)d;        /* hashed length */
    const int nblk = (tl + (size_t)d + 9 <= 64) ? 1 : 2;
    uint8_t buf[NB][128];
    for (int b = 0; b < NB; b++) {
        memset(buf[b], 0, sizeof buf[b]);
        size_t off = 64 * J->nfull;
        for (size_t i = 0; i < tl; i++) buf[b][i] = (i + off < J->len) ? J->msg[i + off] : ' ';
        buf[b][tl + (size_t)d] = 0x80;
        uint64_t bits = (uint64_t)L * 8u;
        for (int i = 0; i < 8; i++) buf[b][64 * nblk - 1 - i] = (uint8_t)(bits >> (8 * i));
        uint64_t n = lo + (uint64_t)b;
        if (n > hi) n = hi; /* pad with the last nonce: a duplicate key leaves the min unchanged */
        fmt_fixed(n, d, buf[b] + tl);
    }
    __m128i mid_abef, mid_cdgh;
    to_ni(J->mid, &mid_abef, &mid_cdgh);
    uint64_t h_best = *bh, n_best = *bn;
    for (uint64_t base = lo;; base += NB) {
        __m128i abef[NB], cdgh[NB], w[NB][4];
        for (int b = 0; b < NB; b++) { abef[b] = mid_abef; cdgh[b] = mid_cdgh; load_block(buf[b], w[b]); }
        compress_nb(abef, cdgh, w);
        if (nblk == 2) {
            for (int b = 0; b < NB; b++) load_block(buf[b] + 64, w[b]);
            compress_nb(abef, cdgh, w);
        }
        for (int b = 0; b < NB; b++) {
            uint64_t h = ((uint64_t)(uint32_t)_mm_extract_epi32(abef[b], 3) << 32) |
                         (uint32_t)_mm_extract_epi32(abef[b], 2);
            uint64_t n = base + (uint64_t)b;
            if (n > hi) n = hi;
            if (better(h, n, h_best, n_best)) { h_best = h; n_best = n; }
        }
        if (hi - base < NB) break;          /* this group reached hi */
        uint64_t left = hi - base - NB;     /* nonces after this group's first, minus NB */
        for (int b = 0; b < NB; b++) {
            if ((uint64_t)b <= left) add_digits(buf[b] + tl, d, NB);
            else { /* past hi: pin to hi */
                fmt_fixed(hi, d, buf[b] + tl);
            }
        }
    }
    *bh = h_best;
    *bn = n_best;
}

/* ---- AVX-512 path: 16 nonces per vector, NV vectors interleaved ------------------------
 * FIPS 180-4 6.2.2 written with vprord (rotate), vpternlogd (0x96 = xor3, 0xCA = Ch,
 * 0xE8 = Maj) and vpaddd; one nonce per 32-bit lane. */
#define NV 2
#define LANES (16 * NV)

__attribute__((target("avx512f")))
static inline void compress_v(__m512i st[NV][8], __m512i w[NV][16]) {
    __m512i a[NV], b[NV], c[NV], d[NV], e[NV], f[NV], g[NV], h[NV];
    for (int v = 0; v < NV; v++) {
        a[v] = st[v][0]; b[v] = st[v][1]; c[v] = st[v][2]; d[v] = st[v][3];
        e[v] = st[v][4]; f[v] = st[v][5]; g[v] = st[v][6]; h[v] = st[v][7];
    }
    for (int t = 0; t < 64; t++) {
        const __m512i k = _mm512_set1_epi32((int)K256[t]);
        for (int v = 0; v < NV; v++) {
            __m512i *W = w[v];
            if (t >= 16) {
                __m512i x = W[(t - 15) & 15], y = W[(t - 2) & 15];
                __m512i s0 = _mm512_ternarylogic_epi32(_mm512_ror_epi32(x, 7), _mm512_ror_epi32(x, 18),
                                                       _mm512_srli_epi32(x, 3), 0x96);
                __m512i s1 = _mm512_ternarylogic_epi32(_mm512_ror_epi32(y, 17), _mm512_ror_epi32(y, 19),
                                                       _mm512_srli_epi32(y, 10), 0x96);
                W[t & 15] = _mm512_add_epi32(_mm512_add_epi32(W[t & 15], s0),
                                             _mm512_add_epi32(W[(t - 7) & 15], s1));
            }
            __m512i S1 = _mm512_ternarylogic_epi32(_mm512_ror_epi32(e[v], 6), _mm512_ror_epi32(e[v], 11),
                                                   _mm512_ror_epi32(e[v], 25), 0x96);
            __m512i ch = _mm512_ternarylogic_epi32(e[v], f[v], g[v], 0xCA);
            __m512i t1 = _mm512_add_epi32(_mm512_add_epi32(h[v], S1),
                                          _mm512_add_epi32(ch, _mm512_add_epi32(W[t & 15], k)));
            __m512i S0 = _mm512_ternarylogic_epi32(_mm512_ror_epi32(a[v], 2), _mm512_ror_epi32(a[v], 13),
                                                   _mm512_ror_epi32(a[v], 22), 0x96);
            __m512i mj = _mm512_ternarylogic_epi32(a[v], b[v], c[v], 0xE8);
            h[v] = g[v]; g[v] = f[v]; f[v] = e[v]; e[v] = _mm512_add_epi32(d[v], t1);
            d[v] = c[v]; c[v] = b[v]; b[v] = a[v]; a[v] = _mm512_add_epi32(t1, _mm512_add_epi32(S0, mj));
        }
    }
    for (int v = 0; v < NV; v++) {
        st[v][0] = _mm512_add_epi32(st[v][0], a[v]); st[v][1] = _mm512_add_epi32(st[v][1], b[v]);
        st[v][2] = _mm512_add_epi32(st[v][2], c[v]); st[v][3] = _mm512_add_epi32(st[v][3], d[v]);
        st[v][4] = _mm512_add_epi32(st[v][4], e[v]); st[v][5] = _mm512_add_epi32(st[v][5], f[v]);
        st[v][6] = _mm512_add_epi32(st[v][6], g[v]); st[v][7] = _mm512_add_epi32(st[v][7], h[v]);
    }
}

static inline uint32_t be32(const uint8_t *p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

__attribute__((target("avx512f")))
static void scan_segment_avx512(const job_t *J, uint64_t lo, uint64_t hi, int d, uint64_t *bh, uint64_t *bn) {
    const size_t tl = J->len + 1 - 64 * J->nfull;
    const size_t L = J->len + 1 + (size_t)d;
    const int nblk = (tl + (size_t)d + 9 <= 64) ? 1 : 2;
    const int wlo = (int)(tl / 4), whi = (int)((tl + (size_t)d - 1) / 4); /* digit-bearing words */
    static __thread uint8_t buf[LANES][128];
    static __thread uint32_t wl[32][LANES] __attribute__((aligned(64)));
    for (int l = 0; l < LANES; l++) {
        memset(buf[l], 0, 128);
        size_t off = 64 * J->nfull;
        for (size_t i = 0; i < tl; i++) buf[l][i] = (i + off < J->len) ? J->msg[i + off] : ' ';
        buf[l][tl + (size_t)d] = 0x80;
        uint64_t bits = (uint64_t)L * 8u;
        for (int i = 0; i < 8; i++) buf[l][64 * nblk - 1 - i] = (uint8_t)(bits >> (8 * i));
        uint64_t n = lo + (uint64_t)l;
        if (n > hi) n = hi;
        fmt_fixed(n, d, buf[l] + tl);
        for (int i = 0; i < 16 * nblk; i++) wl[i][l] = be32(buf[l] + 4 * i);
    }
    uint64_t h_best = *bh, n_best = *bn;
    for (uint64_t base = lo;; base += LANES) {
        __m512i st[NV][8], w[NV][16];
        for (int v = 0; v < NV; v++) {
            for (int i = 0; i < 8; i++) st[v][i] = _mm512_set1_epi32((int)J->mid[i]);
            for (int i = 0; i < 16; i++) w[v][i] = _mm512_load_si512((const void *)&wl[i][16 * v]);
        }
        compress_v(st, w);
        if (nblk == 2) {
            for (int v = 0; v < NV; v++)
                for (int i = 0; i < 16; i++) w[v][i] = _mm512_load_si512((const void *)&wl[16 + i][16 * v]);
            compress_v(st, w);
        }
        uint32_t ha[LANES] __attribute__((aligned(64))), hb[LANES] __attribute__((aligned(64)));
        for (int v = 0; v < NV; v++) {
            _mm512_store_si512((void *)&ha[16 * v], st[v][0]);
            _mm512_store_si512((void *)&hb[16 * v], st[v][1]);
        }
        for (int l = 0; l < LANES; l++) {
            uint64_t h = ((uint64_t)ha[l] << 32) | hb[l];
            uint64_t n = base + (uint64_t)l;
            if (n > hi) n = hi;
            if (better(h, n, h_best, n_best)) { h_best = h; n_best = n; }
        }
        if (hi - base < LANES) break;
        uint64_t left = hi - base - LANES;
        for (int l = 0; l < LANES; l++) {
            if ((uint64_t)l <= left) add_digits(buf[l] + tl, d, LANES);
            else fmt_fixed(hi, d, buf[l] + tl);
            for (int i = wlo; i <= whi; i++) wl[i][l] = be32(buf[l] + 4 * i);
        }
    }
    *bh = h_best;
    *bn = n_best;
}

static int have_avx512(void) {
    unsigned a, b, c, d;
    __asm__ volatile("cpuid" : "=a"(a), "=b"(b), "=c"(c), "=d"(d) : "a"(7), "c"(0));
    return (b >> 16) & 1u;
}

static void scan_range(const job_t *J, uint64_t lo, uint64_t hi, uint64_t *bh, uint64_t *bn) {
    uint64_t cur = lo;
    for (;;) {
        int d = ndigits(cur);
        uint64_t seg_hi = hi;
        if (d < 20) {
            uint64_t p10 = 1;
            for (int i = 0; i < d; i++) p10 *= 10u;
            if (p10 - 1u < seg_hi) seg_hi = p10 - 1u;
        }
        if (J->avx512) scan_segment_avx512(J, cur, seg_hi, d, bh, bn);
        else scan_segment(J, cur, seg_hi, d, bh, bn);
        if (seg_hi == hi) return;
        cur = seg_hi + 1u;
    }
}

static void *worker(void *p) {
    job_t *J = (job_t *)p;
    uint64_t bh = ~0ull, bn = ~0ull;
    for (;;) {
        uint64_t c = atomic_fetch_add(&J->next, 1);
        if (c >= J->nchunks) break;
        uint64_t lo = J->lower + c * CHUNK;
        uint64_t hi = (J->upper - lo < CHUNK - 1u) ? J->upper : lo + CHUNK - 1u;
        scan_range(J, lo, hi, &bh, &bn);
        uint64_t dn = atomic_fetch_add(&J->done, 1) + 1;
        if (J->progress && (dn % 4096u == 0 || dn == J->nchunks)) {
            fprintf(stderr, "golden_scan: %llu/%llu chunks\n", (unsigned long long)dn,
                    (unsigned long long)J->nchunks);
        }
    }
    pthread_mutex_lock(&J->mu);
    if (better(bh, bn, J->best_h, J->best_n)) { J->best_h = bh; J->best_n = bn; }
    pthread_mutex_unlock(&J->mu);
    return NULL;
}

/* 1 if this CPU has the SHA extensions (the only instructions here beyond SSE4.1). */
int golden_available(void) {
    unsigned a, b, c, d;
    __asm__ volatile("cpuid" : "=a"(a), "=b"(b), "=c"(c), "=d"(d) : "a"(7), "c"(0));
    return (b >> 29) & 1u;
}

/* bitcoin.Hash(msg, nonce) through this implementation (for the cross-checks). */
uint64_t golden_hash(const uint8_t *msg, size_t len, uint64_t nonce) {
    size_t L = len + 1 + (size_t)ndigits(nonce);
    size_t nb = (L + 9 + 63) / 64;
    uint8_t *buf = (uint8_t *)calloc(nb * 64, 1);
    memcpy(buf, msg, len);
    buf[len] = ' ';
    fmt_fixed(nonce, ndigits(nonce), buf + len + 1);
    buf[L] = 0x80;
    for (int i = 0; i < 8; i++) buf[nb * 64 - 1 - i] = (uint8_t)(((uint64_t)L * 8u) >> (8 * i));
    uint32_t st[8];
    memcpy(st, IV, sizeof st);
    for (size_t i = 0; i < nb; i++) compress1(st, buf + 64 * i);
    free(buf);
    return ((uint64_t)st[0] << 32) | st[1];
}

/* argmin of (Hash(msg, n), n) over the inclusive [lower, upper]; 0 ok, -1 lower > upper,
 * -2 no SHA extensions. */
int golden_min(const uint8_t *msg, size_t len, uint64_t lower, uint64_t upper, int nthreads,
               int progress, uint64_t *out_hash, uint64_t *out_nonce) {
    if (lower > upper) return -1;
    if (!golden_available()) return -2;
    job_t J;
    memset(&J, 0, sizeof J);
    J.msg = msg; J.len = len; J.lower = lower; J.upper = upper;
    J.nchunks = (upper - lower) / CHUNK + 1u;
    J.nfull = (len + 1) / 64;
    memcpy(J.mid, IV, sizeof J.mid);
    if (J.nfull) {
        uint8_t *pre = (uint8_t *)malloc(64 * J.nfull);
        for (size_t i = 0; i < 64 * J.nfull; i++) pre[i] = i < len ? msg[i] : ' ';
        for (size_t i = 0; i < J.nfull; i++) compress1(J.mid, pre + 64 * i);
        free(pre);
    }
    atomic_init(&J.next, 0);
    atomic_init(&J.done, 0);
    pthread_mutex_init(&J.mu, NULL);
    J.best_h = ~0ull; J.best_n = ~0ull;
    J.progress = progress;
    J.avx512 = have_avx512() && !getenv("GOLDEN_SCAN_NO_AVX512");
    if (nthreads < 1) nthreads = 1;
    if ((uint64_t)nthreads > J.nchunks) nthreads = (int)J.nchunks;
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    for (int i = 0; i < nthreads; i++) pthread_create(&th[i], NULL, worker, &J);
    for (int i = 0; i < nthreads; i++) pthread_join(th[i], NULL);
    free(th);
    pthread_mutex_destroy(&J.mu);
    *out_hash = J.best_h;
    *out_nonce = J.best_n;
    return 0;
}

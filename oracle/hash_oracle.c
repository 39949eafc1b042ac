/*
 * oracle/hash_oracle.c -- CPU restatement of the reference hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / the timed CPU
 * baseline.  The product path (libgpuhash.so) never links or calls it.
 *
 * What it restates (reference = mohitreddy1996/BitCoin-Miner, Go):
 *   - bitcoin.Hash            src/github.com/cmu440/bitcoin/hash.go:11-15
 *       hasher := sha256.New()                                   (hash.go:12)
 *       hasher.Write([]byte(fmt.Sprintf("%s %d", msg, nonce)))   (hash.go:13)
 *       return binary.BigEndian.Uint64(hasher.Sum(nil))           (hash.go:14)
 *     The SHA-256 itself is Go's stdlib crypto/sha256 (unvendored, version unpinned,
 *     SURVEY.md 8(c)); it implements FIPS 180-4, which is restated here from the
 *     standard: IV, K[64], 64 rounds, 0x80 + zero pad + 64-bit big-endian bit length.
 *     "%d" of a uint64 = unsigned decimal, no sign, no padding, "0" for zero.
 *   - The miner's min-hash loop, specified (not implemented) in p1.pdf pp.12-14 and
 *     stubbed at src/github.com/cmu440/bitcoin/miner/miner.go:15: for every nonce n in
 *     the INCLUSIVE range [Lower, Upper] (message.go:25-32) keep the least Hash, with
 *     ties going to the lowest nonce (ascending scan with strict '<', north_star).
 *
 * Pinning: the handout known-answer values (p1.pdf p.12) are checked by
 * tests/test_oracle.py together with an independent hashlib (OpenSSL) restatement
 * (oracle/hash_oracle.py).  The Go reference itself cannot be built in this image
 * (no Go toolchain; see DESIGN.md "Oracle").
 *
 * Deliberately naive: every call re-formats the message and re-hashes it from the
 * IV, exactly like hash.go -- this is also what bench.py times as the CPU baseline
 * ("port" of the reference loop).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static const uint32_t K256[64] = {
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

static inline uint32_t ror(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

/* FIPS 180-4 section 6.2.2: one compression of a 64-byte block into st[8]. */
static void compress(uint32_t st[8], const uint8_t blk[64]) {
    uint32_t w[64];
    for (int t = 0; t < 16; t++)
        w[t] = ((uint32_t)blk[4 * t] << 24) | ((uint32_t)blk[4 * t + 1] << 16) |
               ((uint32_t)blk[4 * t + 2] << 8) | (uint32_t)blk[4 * t + 3];
    for (int t = 16; t < 64; t++) {
        uint32_t s0 = ror(w[t - 15], 7) ^ ror(w[t - 15], 18) ^ (w[t - 15] >> 3);
        uint32_t s1 = ror(w[t - 2], 17) ^ ror(w[t - 2], 19) ^ (w[t - 2] >> 10);
        w[t] = w[t - 16] + s0 + w[t - 7] + s1;
    }
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
    uint32_t e = st[4], f = st[5], g = st[6], h = st[7];
    for (int t = 0; t < 64; t++) {
        uint32_t S1 = ror(e, 6) ^ ror(e, 11) ^ ror(e, 25);
        uint32_t ch = (e & f) ^ (~e & g);
        uint32_t t1 = h + S1 + ch + K256[t] + w[t];
        uint32_t S0 = ror(a, 2) ^ ror(a, 13) ^ ror(a, 22);
        uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
        uint32_t t2 = S0 + mj;
        h = g; g = f; f = e; e = d + t1;
        d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d;
    st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

/* Full SHA-256 (FIPS 180-4 5.1.1 padding), digest as 8 state words. */
void oracle_sha256(const uint8_t *data, size_t len, uint32_t out[8]) {
    uint32_t st[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                      0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
    size_t off = 0;
    for (; off + 64 <= len; off += 64) compress(st, data + off);
    uint8_t tail[128];
    size_t rem = len - off;
    memset(tail, 0, sizeof tail);
    if (rem) memcpy(tail, data + off, rem);
    tail[rem] = 0x80;
    size_t tl = (rem + 1 + 8 <= 64) ? 64 : 128;
    uint64_t bits = (uint64_t)len * 8u;
    for (int i = 0; i < 8; i++) tail[tl - 1 - i] = (uint8_t)(bits >> (8 * i));
    compress(st, tail);
    if (tl == 128) compress(st, tail + 64);
    memcpy(out, st, sizeof st);
}

/* fmt "%d" of a uint64 (hash.go:13): returns the number of digits written. */
static int fmt_u64(uint64_t v, char *buf) {
    char tmp[20];
    int n = 0;
    do { tmp[n++] = (char)('0' + (int)(v % 10u)); v /= 10u; } while (v);
    for (int i = 0; i < n; i++) buf[i] = tmp[n - 1 - i];
    return n;
}

/* bitcoin.Hash(msg, nonce), hash.go:11-15.  Allocates like the Go code does
 * (Sprintf + []byte): one heap buffer per call. */
uint64_t oracle_hash(const uint8_t *msg, size_t len, uint64_t nonce) {
    uint8_t *buf = (uint8_t *)malloc(len + 22);
    memcpy(buf, msg, len);
    buf[len] = ' ';
    int nd = fmt_u64(nonce, (char *)buf + len + 1);
    uint32_t d[8];
    oracle_sha256(buf, len + 1 + (size_t)nd, d);
    free(buf);
    return ((uint64_t)d[0] << 32) | d[1]; /* binary.BigEndian.Uint64(digest[0:8]) */
}

/* The spec'd miner loop (p1.pdf pp.12-14): ascending scan of [lower, upper]
 * inclusive, strict '<' so the lowest nonce wins ties.  Returns 0, or -1 when
 * lower > upper (undefined in the reference; an error in gpuhash.h). */
int oracle_min(const uint8_t *msg, size_t len, uint64_t lower, uint64_t upper,
               uint64_t *out_hash, uint64_t *out_nonce) {
    if (lower > upper) return -1;
    uint64_t best = oracle_hash(msg, len, lower), bn = lower;
    for (uint64_t n = lower; n != upper;) {
        n++;
        uint64_t h = oracle_hash(msg, len, n);
        if (h < best) { best = h; bn = n; }
    }
    *out_hash = best;
    *out_nonce = bn;
    return 0;
}

typedef struct {
    const uint8_t *msg; size_t len; uint64_t lo, hi, h, n;
} span_t;

static void *span_worker(void *p) {
    span_t *s = (span_t *)p;
    oracle_min(s->msg, s->len, s->lo, s->hi, &s->h, &s->n);
    return NULL;
}

/* Same result as oracle_min, computed over `nthreads` contiguous sub-ranges and
 * merged with the lexicographic (hash, nonce) key -- used to make the large
 * golden fixtures (tests/golden/make_golden.py) and the multi-core CPU baseline. */
int oracle_min_mt(const uint8_t *msg, size_t len, uint64_t lower, uint64_t upper,
                  int nthreads, uint64_t *out_hash, uint64_t *out_nonce) {
    if (lower > upper) return -1;
    if (nthreads < 1) nthreads = 1;
    uint64_t span = upper - lower; /* count - 1, never overflows */
    if ((uint64_t)nthreads > span + 1u) nthreads = (int)(span + 1u);
    span_t *s = (span_t *)calloc((size_t)nthreads, sizeof(span_t));
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    uint64_t per = span / (uint64_t)nthreads + 1u, cur = lower;
    int used = 0;
    for (int i = 0; i < nthreads; i++) {
        s[i].msg = msg; s[i].len = len; s[i].lo = cur;
        uint64_t rest = upper - cur;
        s[i].hi = (rest < per - 1u || i == nthreads - 1) ? upper : cur + per - 1u;
        pthread_create(&th[i], NULL, span_worker, &s[i]);
        used++;
        if (s[i].hi == upper) break;
        cur = s[i].hi + 1u;
    }
    uint64_t bh = UINT64_MAX, bn = UINT64_MAX;
    for (int i = 0; i < used; i++) {
        pthread_join(th[i], NULL);
        if (s[i].h < bh || (s[i].h == bh && s[i].n < bn)) { bh = s[i].h; bn = s[i].n; }
    }
    free(s); free(th);
    *out_hash = bh;
    *out_nonce = bn;
    return 0;
}

/* Every hash of [lower, lower+count) into out[] -- the per-nonce parity check
 * against gpuhash_hash_range(). */
void oracle_hash_range(const uint8_t *msg, size_t len, uint64_t lower, uint64_t count,
                       uint64_t *out) {
    for (uint64_t i = 0; i < count; i++) out[i] = oracle_hash(msg, len, lower + i);
}

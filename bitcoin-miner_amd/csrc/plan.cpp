// plan.cpp -- host-side layout planner (see plan.h for the decomposition).
//
// Semantics restated from the reference:
//   * hashed bytes = msg ‖ 0x20 ‖ decimal(n), "%s %d" of hash.go:13; decimal has no
//     sign, no padding, "0" for zero, up to 20 digits for a uint64.
//   * SHA-256 per FIPS 180-4 (Go stdlib crypto/sha256, called at hash.go:12-14).
//   * result = first 8 digest bytes big-endian = (H0 << 32) | H1 (hash.go:14).
//   * search range is INCLUSIVE [Lower, Upper] (bitcoin/message.go:25-32, p1.pdf p.14).
#include "plan.h"

#include <algorithm>
#include <cmath>
#include <cstring>

namespace gpuhash {

const uint32_t kK[64] = {
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

void sha256_expand(uint32_t w[64]) {
    for (int t = 16; t < 64; t++) {
        uint32_t s0 = ror(w[t - 15], 7) ^ ror(w[t - 15], 18) ^ (w[t - 15] >> 3);
        uint32_t s1 = ror(w[t - 2], 17) ^ ror(w[t - 2], 19) ^ (w[t - 2] >> 10);
        w[t] = w[t - 16] + s0 + w[t - 7] + s1;
    }
}

void sha256_rounds(uint32_t st[8], const uint32_t w[64], int t_begin, int t_end) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6],
             h = st[7];
    for (int t = t_begin; t < t_end; t++) {
        uint32_t S1 = ror(e, 6) ^ ror(e, 11) ^ ror(e, 25);
        uint32_t ch = (e & f) ^ (~e & g);
        uint32_t t1 = h + S1 + ch + kK[t] + w[t];
        uint32_t S0 = ror(a, 2) ^ ror(a, 13) ^ ror(a, 22);
        uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
        h = g; g = f; f = e; e = d + t1;
        d = c; c = b; b = a; a = t1 + S0 + mj;
    }
    st[0] = a; st[1] = b; st[2] = c; st[3] = d; st[4] = e; st[5] = f; st[6] = g; st[7] = h;
}

void sha256_compress(uint32_t st[8], const uint32_t w16[16]) {
    uint32_t w[64], s[8];
    std::memcpy(w, w16, 64);
    sha256_expand(w);
    std::memcpy(s, st, 32);
    sha256_rounds(s, w, 0, 64);
    for (int i = 0; i < 8; i++) st[i] += s[i];
}

int num_digits(uint64_t n) {
    int d = 1;
    while (n >= 10u) { n /= 10u; d++; }
    return d;
}

uint64_t pow10u(int k) {
    uint64_t p = 1;
    for (int i = 0; i < k; i++) p *= 10u;
    return p;
}

uint32_t ascii4(uint32_t x) {
    uint32_t d0 = x % 10u, d1 = (x / 10u) % 10u, d2 = (x / 100u) % 10u, d3 = (x / 1000u) % 10u;
    return 0x30303030u | (d3 << 24) | (d2 << 16) | (d1 << 8) | d0;
}

static inline uint32_t be32(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

// msg ‖ ' ' ‖ dec(nonce), padded, hashed with this file's compress.  Used for the C-ABI
// gpuhash_hash_cpu() convenience (the Go shim's one-nonce self-check) only.
uint64_t hash_host(const uint8_t* msg, uint64_t len, uint64_t nonce) {
    char dig[20];
    int nd = 0;
    uint64_t v = nonce;
    do { dig[nd++] = (char)('0' + (int)(v % 10u)); v /= 10u; } while (v);
    uint64_t L = len + 1 + (uint64_t)nd;
    uint64_t nblk = (L + 9 + 63) / 64;
    std::vector<uint8_t> buf(nblk * 64, 0);
    if (len) std::memcpy(buf.data(), msg, len);
    buf[len] = ' ';
    for (int i = 0; i < nd; i++) buf[len + 1 + i] = (uint8_t)dig[nd - 1 - i];
    buf[L] = 0x80;
    uint64_t bits = L * 8u;
    for (int i = 0; i < 8; i++) buf[nblk * 64 - 1 - i] = (uint8_t)(bits >> (8 * i));
    uint32_t st[8];
    std::memcpy(st, kIV, 32);
    for (uint64_t b = 0; b < nblk; b++) {
        uint32_t w[16];
        for (int i = 0; i < 16; i++) w[i] = be32(&buf[b * 64 + 4 * i]);
        sha256_compress(st, w);
    }
    return ((uint64_t)st[0] << 32) | st[1];
}

namespace {

struct GroupLayout {
    int d, J, q, s, C2, EX;
    int u;       // 1: a tail-digit layout -- d counts the digits of k = nonce / 10, the
                 //    last digit follows them as a constant message byte (plan.h)
    int q1;      // C2 = 2: digits of W_1 (q = 4 + q1)
    uint64_t B;  // index of the block holding the last digit
};

// `span` = nonces of this digit group in the search (0 = unknown: assume a full group).
GroupLayout layout_for(uint64_t m, int d, uint64_t span = 0, int policy = kLayoutAuto) {
    GroupLayout g{};
    g.d = d;
    uint64_t L = m + 1 + (uint64_t)d;
    uint64_t f_abs = m + 1, e_abs = L - 1;
    g.B = e_abs / 64;
    int e = (int)(e_abs % 64);
    g.J = e / 4;
    uint64_t wstart = 64 * g.B + 4 * (uint64_t)g.J;
    g.q = (int)(e_abs - std::max(wstart, f_abs) + 1);
    g.EX = e >= 55;
    int before = d - g.q;
    g.s = std::min(std::min(kMaxLane, before), kMaxLaunchDigits - g.q);
    if (g.s < 0) g.s = 0;
    g.u = 0;
    uint64_t blkB = 64 * g.B;
    // digit bytes of block B that precede word J
    uint64_t nbB = (f_abs >= wstart) ? 0 : wstart - std::max(f_abs, blkB);
    g.C2 = (uint64_t)g.s > nbB;
    // J = 1 with lanes spilling into block B-1: W_0 is four digits, W_1 holds q digits.
    // Three layouts can run such a digit group:
    //   C2 = 1 (classic)    lanes in W_0 + block B-1, W_1 per nonce: every nonce pays
    //                       block B's schedule, ~31.7 GH/s;
    //   C2 = 2 (two-word)   lanes = block B-1 digits, the loop takes W_0 and W_1: block B's
    //                       schedule is wave-uniform (built in LDS per 64 loop values),
    //                       45.2-45.7 GH/s on full 256-lane rows, but a lane covers up to
    //                       10^8 loop values, so narrow searches leave rows partly empty;
    //   C2 = 3 (lane table) lanes = the W_0/W_1 digits (>= 10^5 values: rows always fill),
    //                       each lane keeps block B's schedule in registers, the loop runs
    //                       over the block B-1 values whose chaining values the host
    //                       precomputes: 44-46.3 GH/s, >= C2 = 2 on every measured layout,
    //                       full rows included (profiles/r03_sweep_lt_vs_u2.jsonl).
    // The policy rule is stated once, in include/gpuhash.h above GPUHASH_LAYOUT_AUTO
    // (tests/test_plan.py checks this function against it): the lane table's p-table
    // costs 64 B and one compression per block B-1 value, so AUTO and LANETABLE cap it at
    // kMaxLtTable (= GPUHASH_LANETABLE_MAX) values, beyond which C2 = 2 rows are full anyway.
    if (g.C2 && g.J == 1) {
        const int nb1 = d - 4 - g.q;  // digits in block B-1 and earlier
        const uint64_t RQ = pow10u(4 + g.q);
        const uint64_t nloop = span ? (span - 1) / RQ + 2 : pow10u(std::min(nb1, 6));
        const bool lt_too_big = nb1 >= 3 && nloop > kMaxLtTable;
        int c2 = 3;
        if (policy == kLayoutClassic) c2 = 1;
        else if (policy == kLayoutUniform) c2 = nb1 >= 3 ? 2 : 3;
        else if (policy == kLayoutLaneTable) c2 = lt_too_big ? 2 : 3;
        else {
            // a row of the lane table builds block B's schedule once (~550 VALU) for every
            // loop value it then hashes: below ~2 loop values the classic layout's
            // per-nonce schedule (~1,300 VALU per nonce) is cheaper
            // (profiles/r03_planner_regret.jsonl: 26.2 vs 29.0 GH/s at 0.7 loop values)
            if (span && span < 2 * RQ) c2 = 1;
            else c2 = lt_too_big ? 2 : 3;
        }
        if (c2 == 2) {
            g.C2 = 2;
            g.q1 = g.q;
            g.q = 4 + g.q;
            g.s = std::min(std::min(kMaxLane, nb1), kMaxLaunchDigitsU2 - g.q);
        } else if (c2 == 3) {
            g.C2 = 3;
            g.q1 = g.q;
            g.q = 4 + g.q;
            g.s = std::min(kMaxLane, nb1);
        }
    }
    return g;
}

// Tail-digit layout of plain digit group d (plan.h): when its last digit-bearing word W_J
// holds one digit and W_{J-1} four, the nonces = t (mod 10) of the group are searched as
// k = nonce / 10 with t a constant byte after k's digits, so the loop word is W_{J-1}
// (R = 10^4) instead of W_J (R = 10: a row's setup -- lane words, two rounds, the
// schedule terms that do not read the loop word, ~255 VALU per lane -- amortised over 10
// nonces costs ~2.6%, tools/q1_probe.py).  The per-nonce work is the J-1 kernel's, one
// round more.  Returns false when the group does not qualify.
bool tail_layout(uint64_t m, int d, const GroupLayout& g, GroupLayout& out) {
    if (g.C2 || g.q != 1 || g.J < 2 || d < 6) return false;
    GroupLayout k = layout_for(m, d - 1);
    // the same final block, k's last digit ending W_{J-1}, four loop digits, no spill into
    // block B-1; the extra-block flag follows the real length (k's last byte is one
    // before the tail's, and 4 | tail byte, so both read >= 55 alike)
    if (k.C2 || k.B != g.B || k.J != g.J - 1 || k.q != 4 || k.EX != g.EX) return false;
    if (k.EX && k.J < 13) return false;
    k.u = 1;
    out = k;
    return true;
}

// The layout plan_range runs digit group d with when the search covers `span` of its
// nonces (0 = all of them / unknown): layout_for under the policy's base, then the
// tail-digit layout when it qualifies and the policy and span allow it.  Returns whether
// the tail-digit layout was taken (`g` is then that layout).
bool group_layout(uint64_t len, int d, uint64_t span, int policy, GroupLayout& g) {
    g = layout_for(len, d, span, policy & kLayoutMask);
    GroupLayout gt;
    const bool tail = !(policy & kLayoutTailNever) &&
                      ((policy & kLayoutTailAlways) || span == 0 || span >= kTailMinSpan) &&
                      tail_layout(len, d, g, gt);
    if (tail) g = gt;
    return tail;
}

// Relative VALU work per nonce of a layout: one final-block compression, +0.7 for the
// extra constant block, + the per-lane block B-1 compression amortised over R nonces.
// (measured per-layout rates, profiles/r01_layout_sweep.jsonl: plain 32-39 GH/s,
// uniform-schedule C2 ~45, extra padding block ~20.5)
double layout_cost(const GroupLayout& g) {
    double c = 1.0;
    if (g.EX) c += 0.7;
    if (g.C2 == 2 || g.C2 == 3 || (g.C2 == 1 && g.J == 0)) c = 0.75;
    if (g.C2 == 3) return c + 0.6 / (double)pow10u(g.s);  // per-row schedule over the loop
    if (g.C2) c += 0.9 / (double)pow10u(g.q);
    else c += 0.2 / (double)std::min<uint64_t>(pow10u(g.q), 100);
    return c;
}

inline uint32_t low_bytes_mask(int nbytes) {
    if (nbytes <= 0) return 0u;
    if (nbytes >= 4) return 0xFFFFFFFFu;
    return (1u << (8 * nbytes)) - 1u;
}

// Chaining state after the leading blocks that hold message bytes only (they are the
// same for every digit group and launch of a search, so plan_range compresses them once).
struct Prefix {
    uint64_t blocks = 0;  // floor(m / 64): block `blocks` is the first that holds ' '
    uint32_t st[8];
};

Prefix make_prefix(const uint8_t* msg, uint64_t m) {
    Prefix p;
    std::memcpy(p.st, kIV, 32);
    p.blocks = m / 64;
    for (uint64_t b = 0; b < p.blocks; b++) {
        uint32_t w[16];
        for (int i = 0; i < 16; i++) w[i] = be32(msg + b * 64 + 4 * (uint64_t)i);
        sha256_compress(p.st, w);
    }
    return p;
}

// [lo, hi]: the launch's nonces, or for a tail-digit layout (g.u = 1) its k = nonce / 10
// values, whose nonces end in the digit `tail`.
void build_launch(const uint8_t* msg, uint64_t m, const Prefix& pre, const GroupLayout& g, uint64_t H,
                  uint64_t lo, uint64_t hi, uint32_t rchunk_max, Launch& out, bool host_ptab,
                  uint32_t tail = 0) {
    const int d = g.d, q = g.q, s = g.s, h = d - s - q;
    const uint64_t L = m + 1 + (uint64_t)d + (uint64_t)g.u;
    const uint64_t nblk = g.B + 1 + (uint64_t)g.EX;
    const uint64_t first_var = g.C2 ? g.B - 1 : g.B;
    // pre.blocks <= first_var: the first digit is at byte m+1, and block B-1 of a C2
    // layout holds digits, so it cannot lie wholly inside the message
    const uint64_t p0 = pre.blocks, base = 64 * p0;
    std::vector<uint8_t> buf((nblk - p0) * 64, 0);  // blocks p0 .. nblk-1
    if (m > base) std::memcpy(buf.data(), msg + base, m - base);
    buf[m - base] = ' ';
    // the h leading digits (H has exactly h digits; H == 0 when h == 0)
    uint64_t v = H;
    for (int i = h - 1; i >= 0; i--) { buf[m + 1 + (uint64_t)i - base] = (uint8_t)('0' + v % 10u); v /= 10u; }
    // lane + loop digit bytes stay 0: the kernel ORs ASCII into them
    if (g.u) buf[L - 1 - base] = (uint8_t)('0' + tail);
    buf[L - base] = 0x80;
    uint64_t bits = L * 8u;
    for (int i = 0; i < 8; i++) buf[(nblk - p0) * 64 - 1 - (uint64_t)i] = (uint8_t)(bits >> (8 * i));
    auto words = [&](uint64_t blk, uint32_t w[16]) {
        for (int i = 0; i < 16; i++) w[i] = be32(&buf[(blk - p0) * 64 + 4 * (uint64_t)i]);
    };

    LaunchDesc& D = out.desc;
    std::memset(&D, 0, sizeof D);
    uint32_t st[8];
    std::memcpy(st, pre.st, 32);
    for (uint64_t b = p0; b < first_var; b++) {
        uint32_t w[16];
        words(b, w);
        sha256_compress(st, w);
    }
    words(g.B, D.U);
    if (g.C2) {
        std::memcpy(D.CV1, st, 32);
        words(g.B - 1, D.U1);
        uint32_t w[64] = {0};
        std::memcpy(w, D.U1, 64);  // rounds 0..13 read only W0..W13 (uniform)
        uint32_t s1[8];
        std::memcpy(s1, st, 32);
        sha256_rounds(s1, w, 0, 14);
        std::memcpy(D.S1, s1, 32);
    } else {
        std::memcpy(D.CV, st, 32);
        uint32_t w[64] = {0};
        std::memcpy(w, D.U, 64);
        uint32_t s0[8];
        std::memcpy(s0, st, 32);
        if (g.J >= 2) sha256_rounds(s0, w, 0, g.J - 2);
        std::memcpy(D.S0, s0, 32);
    }
    if (g.EX) {
        uint32_t w[64];
        words(g.B + 1, w);
        sha256_expand(w);
        for (int t = 0; t < 64; t++) D.KWX[t] = kK[t] + w[t];
    }
    D.mask_lo = low_bytes_mask(std::min(s, 4));
    D.mask_hi = low_bytes_mask(s - 4);
    D.qmask = low_bytes_mask(g.C2 >= 2 ? g.q1 : q);
    D.R1 = g.C2 >= 2 ? (uint32_t)pow10u(g.q1) : 1u;
    const int e = (int)((L - 1 - (uint64_t)g.u) % 64);  // the last (loop) digit's byte
    D.loop_shift = (uint32_t)(3 - e % 4) * 8u;
    if (g.C2 == 3) {
        // lane table: lanes = the q digits of W_0/W_1 (x in [x_a, x_b]), loop = the s digits
        // at the end of block B-1 (p in [p_a, p_b]); [lo, hi] is a rectangle (plan_range)
        const uint64_t U = pow10u(s + q), RQ = pow10u(q);
        const uint64_t off_lo = lo - H * U, off_hi = hi - H * U;
        const uint64_t p_a = off_lo / RQ, p_b = off_hi / RQ;
        const uint32_t NP = (uint32_t)(p_b - p_a + 1);
        D.RQ = (uint32_t)RQ;
        D.R = NP;
        D.rchunk = NP;
        D.nrchunks = 1;
        D.p_first = (uint32_t)(off_lo % RQ);
        D.p_last = (uint32_t)(off_hi % RQ);
        D.r_first = 0;
        D.r_last = NP - 1u;
        D.base = H * U + p_a * RQ;
        D.lt_p0 = (uint32_t)p_a;
        D.stride = 1u;
        D.tail = 0u;
        out.stride = 1u;
        out.nptab = 16u * NP;
        // p-table: block B-1 with the s loop digits of p (its last s bytes), compressed
        // from CV1, then round 0 of block B up to its K+W term.  The library builds it on
        // the device (k_ptab, the same steps); the host copy is for the CPU replay.
        out.ptab.clear();
        if (host_ptab) out.ptab.assign(16ull * NP, 0u);
        std::vector<uint8_t> blk(64);
        std::memcpy(blk.data(), &buf[(g.B - 1 - p0) * 64], 64);
        for (uint32_t k = 0; host_ptab && k < NP; k++) {
            uint64_t v = p_a + k;
            for (int i = s - 1; i >= 0; i--) { blk[64 - (size_t)s + (size_t)i] = (uint8_t)('0' + v % 10u); v /= 10u; }
            uint32_t w[16], cv[8];
            for (int i = 0; i < 16; i++) w[i] = be32(&blk[4 * (size_t)i]);
            std::memcpy(cv, D.CV1, 32);
            sha256_compress(cv, w);
            uint32_t* e8 = &out.ptab[16ull * k];
            std::memcpy(e8, cv, 32);
            const uint32_t a = cv[0], b = cv[1], c = cv[2], ee = cv[4], f = cv[5], gg = cv[6], h = cv[7];
            e8[8] = h + (ror(ee, 6) ^ ror(ee, 11) ^ ror(ee, 25)) + ((ee & f) ^ (~ee & gg));
            e8[9] = (ror(a, 2) ^ ror(a, 13) ^ ror(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
        }
        out.J = g.J; out.C2 = g.C2; out.EX = g.EX;
        out.d = d; out.q = q; out.s = s;
        out.c = 2;
        out.lo = lo; out.hi = hi;
        out.nblocks = (D.p_last - D.p_first) / (uint32_t)kBlock + 1u;
        return;
    }
    out.ptab.clear();
    out.nptab = 0;
    const uint64_t R = pow10u(q), P = pow10u(s);
    D.R = (uint32_t)R;
    // r values per work item: ~100 keeps every workgroup short (a few ms at full load)
    // so a launch's tail is small, and still amortises the per-item setup (lane words,
    // hoisted schedule terms; for C2 the lane block B-1, ~1.1k ops) to ~1-11 ops/nonce.
    uint32_t rc = rchunk_max ? rchunk_max : 100u;
    D.rchunk = (uint32_t)std::min<uint64_t>(R, rc);
    D.nrchunks = (uint32_t)((R + D.rchunk - 1) / D.rchunk);
    D.p_first = (uint32_t)((lo / R) % P);
    D.r_first = (uint32_t)(lo % R);
    D.p_last = (uint32_t)((hi / R) % P);
    D.r_last = (uint32_t)(hi % R);
    D.base = H * R * P;
    D.stride = g.u ? 10u : 1u;
    D.tail = tail;

    out.J = g.J; out.C2 = g.C2; out.EX = g.EX;
    out.d = d + g.u; out.q = q; out.s = s;
    out.c = ((m + 1) / 64 != (L - 1) / 64) ? 2 : 1;
    out.stride = D.stride;
    out.lo = lo * D.stride + tail; out.hi = hi * D.stride + tail;
    uint32_t npb = (D.p_last - D.p_first) / (uint32_t)kBlock + 1u;
    out.nblocks = npb * D.nrchunks;
}

}  // namespace

void plan_range(const uint8_t* msg, uint64_t len, uint64_t lower, uint64_t upper,
                std::vector<Launch>& out, uint32_t rchunk_max, int policy, bool host_ptab) {
    const int dlo = num_digits(lower), dhi = num_digits(upper);
    const Prefix pre = make_prefix(msg, len);
    for (int d = dlo; d <= dhi; d++) {
        uint64_t a = d == 1 ? 0 : pow10u(d - 1);
        uint64_t b = d == 20 ? UINT64_MAX : pow10u(d) - 1;
        a = std::max(a, lower);
        b = std::min(b, upper);
        if (a > b) continue;
        const uint64_t span = b - a == UINT64_MAX ? 0 : b - a + 1;
        GroupLayout g;
        const bool tail = group_layout(len, d, span, policy, g);
        if (tail) {
            const GroupLayout& gt = g;
            // ten launch sets, one per last digit t: k = nonce / 10 over the nonces = t (mod
            // 10) of [a, b] (a >= 10^(d-1) >= 10, so every k has d-1 digits)
            for (uint32_t t = 0; t < 10; t++) {
                if (b < t) continue;
                // ceil((a - t) / 10) without overflowing at a = 2^64-1
                const uint64_t ka = a <= t ? 0 : (a - t) / 10 + ((a - t) % 10 != 0), kb = (b - t) / 10;
                if (ka > kb) continue;
                const uint64_t Uk = pow10u(gt.s + gt.q);
                for (uint64_t H = ka / Uk;; H++) {
                    Launch l;
                    build_launch(msg, len, pre, gt, H, std::max(ka, H * Uk),
                                 H == kb / Uk ? kb : H * Uk + (Uk - 1), rchunk_max, l, host_ptab, t);
                    out.push_back(std::move(l));
                    if (H == kb / Uk) break;
                }
            }
            continue;
        }
        const uint64_t U = pow10u(g.s + g.q);
        const uint64_t Hf = a / U, Hl = b / U;
        for (uint64_t H = Hf;; H++) {
            uint64_t lo = std::max(a, H * U);
            uint64_t hi = (H == Hl) ? b : H * U + (U - 1);
            if (g.C2 == 3) {
                // lane table: each launch must be a rectangle (loop values p) x (lane
                // values x) -- a partial first p, the full p's, a partial last p -- of at
                // most kMaxLtLoop p values
                const uint64_t RQ = pow10u(g.q), base = H * U;
                uint64_t o = lo - base;
                const uint64_t oe = hi - base;
                while (o <= oe) {
                    const uint64_t p = o / RQ, x = o % RQ;
                    uint64_t end;  // last offset of this rectangle
                    if (x != 0 || oe / RQ == p) {
                        end = std::min(oe, p * RQ + RQ - 1);  // within one p
                    } else {
                        uint64_t pe = oe / RQ;  // full p's up to pe (pe's row may be partial)
                        if (oe % RQ != RQ - 1) pe--;
                        pe = std::min(pe, p + kMaxLtLoop - 1);
                        end = pe * RQ + RQ - 1;
                    }
                    Launch l;
                    build_launch(msg, len, pre, g, H, base + o, base + end, rchunk_max, l, host_ptab);
                    out.push_back(std::move(l));
                    o = end + 1;
                }
            } else {
                Launch l;
                build_launch(msg, len, pre, g, H, lo, hi, rchunk_max, l, host_ptab);
                out.push_back(std::move(l));
            }
            if (H == Hl) break;
        }
    }
}

double group_cost(uint64_t msg_len, int d, uint64_t span, int policy) {
    GroupLayout g;
    group_layout(msg_len, d, span, policy, g);
    return layout_cost(g);
}

double plan_cost(const std::vector<Launch>& plan) {
    double c = 0;
    for (const Launch& l : plan) {
        GroupLayout g{};
        g.d = l.d; g.J = l.J; g.q = l.q; g.s = l.s; g.C2 = l.C2; g.EX = l.EX;
        c += (double)((l.hi - l.lo) / l.stride + 1) * layout_cost(g);
    }
    return c;
}

std::vector<Shard> shard_range(uint64_t msg_len, uint64_t lower, uint64_t upper, int n, int policy) {
    std::vector<Shard> sh((size_t)std::max(n, 1));
    if (n <= 1) { sh[0] = {lower, upper, 0}; return sh; }
    struct G { uint64_t a, b; long double w; };
    std::vector<G> gs;
    long double total = 0;
    // A shard runs its part of a digit group with the layout plan_range picks for THAT
    // part (the tail-digit launches and the J = 1 straddle choice depend on the span the
    // call covers): each group is priced at the span a shard typically holds
    // of it, min(the group's span in the range, the range / n).
    const long double per_shard = ((long double)(upper - lower) + 1.0L) / (long double)n;
    for (int d = num_digits(lower); d <= num_digits(upper); d++) {
        uint64_t a = d == 1 ? 0 : pow10u(d - 1), b = d == 20 ? UINT64_MAX : pow10u(d) - 1;
        a = std::max(a, lower); b = std::min(b, upper);
        if (a > b) continue;
        const long double est = std::min(((long double)(b - a) + 1.0L), std::ceil(per_shard));
        const uint64_t span = est >= 18446744073709551616.0L ? 0 : (uint64_t)est;
        long double w = (long double)group_cost(msg_len, d, span, policy);
        gs.push_back({a, b, w});
        total += ((long double)(b - a) + 1.0L) * w;
    }
    // cut points: first nonce of shard k (k = 1..n-1) at cumulative cost k·total/n
    std::vector<uint64_t> cut((size_t)n + 1);
    cut[0] = lower;
    size_t gi = 0;
    long double acc = 0;
    for (int k = 1; k < n; k++) {
        long double target = total * (long double)k / (long double)n;
        while (gi < gs.size()) {
            long double gc = ((long double)(gs[gi].b - gs[gi].a) + 1.0L) * gs[gi].w;
            if (acc + gc >= target) break;
            acc += gc;
            gi++;
        }
        uint64_t c;
        if (gi >= gs.size()) {
            c = upper;
        } else {
            long double off = (target - acc) / gs[gi].w;
            uint64_t o = (uint64_t)off;
            uint64_t span = gs[gi].b - gs[gi].a;
            if (o > span) o = span;
            c = gs[gi].a + o;
        }
        cut[(size_t)k] = std::max(c, cut[(size_t)k - 1]);
    }
    // shard k = [cut[k], cut[k+1]-1]; the last shard ends at upper
    for (int k = 0; k < n; k++) {
        uint64_t lo = cut[(size_t)k];
        if (k == n - 1) { sh[(size_t)k] = {lo, upper, 0}; break; }
        uint64_t nx = cut[(size_t)k + 1];
        if (nx == lo) sh[(size_t)k] = {0, 0, 1};
        else sh[(size_t)k] = {lo, nx - 1, 0};
    }
    // the last shard must not be empty-by-overlap: if cut[n-1] > upper cannot happen
    return sh;
}

}  // namespace gpuhash

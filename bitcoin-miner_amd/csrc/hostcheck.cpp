// hostcheck.cpp -- TEST-ONLY CPU view of the planner (libgpuhash_hostcheck.so).
//
// Exposes the launch plan the HIP library would execute and replays, in plain C++,
// the data flow a scan kernel performs for ONE nonce from that launch's descriptor
// (uniform words, lane/loop digit insertion, precomputed S0/S1/CV midstates, extra
// padding block).  tests/test_plan.py compares it against the oracle on CPU so that a
// wrong host precomputation is caught without a GPU.  Not linked into libgpuhash.so
// and never used to produce a search result.
#include <cstring>
#include <vector>

#include "plan.h"

using namespace gpuhash;

static int g_policy = kLayoutAuto;

extern "C" {

// Layout policy used by every plan_* / hostcheck_* call below (plan.h LayoutPolicy).
void hostcheck_set_layout_policy(int policy) { g_policy = policy; }

struct gpuhash_plan_info {
    int J, C2, EX, d, q, s;
    uint64_t lo, hi, base;
    uint32_t nblocks, R, rchunk, nrchunks, p_first, p_last, r_first, r_last;
    uint32_t stride, tail;  // tail-digit launches: nonces = tail (mod stride) in [lo, hi]
};

int gpuhash_plan_count(const uint8_t* msg, uint64_t len, uint64_t lower, uint64_t upper,
                       uint32_t rchunk) {
    if (lower > upper) return -1;
    std::vector<Launch> v;
    plan_range(msg, len, lower, upper, v, rchunk, g_policy);
    return (int)v.size();
}

int gpuhash_plan_get(const uint8_t* msg, uint64_t len, uint64_t lower, uint64_t upper,
                     uint32_t rchunk, int idx, gpuhash_plan_info* out) {
    if (lower > upper || !out) return -1;
    std::vector<Launch> v;
    plan_range(msg, len, lower, upper, v, rchunk, g_policy);
    if (idx < 0 || idx >= (int)v.size()) return -1;
    const Launch& l = v[(size_t)idx];
    const LaunchDesc& D = l.desc;
    *out = gpuhash_plan_info{l.J, l.C2, l.EX, l.d, l.q, l.s, l.lo, l.hi, D.base, l.nblocks,
                             D.R, D.rchunk, D.nrchunks, D.p_first, D.p_last, D.r_first, D.r_last,
                             D.stride, D.tail};
    return 0;
}

// Whole plan in one call: fills up to cap entries, returns the launch count.
int gpuhash_plan_all(const uint8_t* msg, uint64_t len, uint64_t lower, uint64_t upper,
                     uint32_t rchunk, gpuhash_plan_info* out, int cap) {
    if (lower > upper) return -1;
    std::vector<Launch> v;
    plan_range(msg, len, lower, upper, v, rchunk, g_policy);
    for (int i = 0; i < (int)v.size() && i < cap; i++) {
        const Launch& l = v[(size_t)i];
        const LaunchDesc& D = l.desc;
        out[i] = gpuhash_plan_info{l.J, l.C2, l.EX, l.d, l.q, l.s, l.lo, l.hi, D.base, l.nblocks,
                                   D.R, D.rchunk, D.nrchunks, D.p_first, D.p_last, D.r_first, D.r_last,
                                   D.stride, D.tail};
    }
    return (int)v.size();
}

int gpuhash_shard(uint64_t msg_len, uint64_t lower, uint64_t upper, int n, uint64_t* lo,
                  uint64_t* hi, int* empty) {
    if (lower > upper || n < 1) return -1;
    std::vector<Shard> s = shard_range(msg_len, lower, upper, n, g_policy);
    for (int i = 0; i < n; i++) {
        lo[i] = s[(size_t)i].lo;
        hi[i] = s[(size_t)i].hi;
        empty[i] = s[(size_t)i].empty;
    }
    return 0;
}

// The cost model's price of the plan of [lower, upper] (plan_cost): what a shard of that
// range really costs under the layouts plan_range picks for it.
double gpuhash_plan_cost(const uint8_t* msg, uint64_t len, uint64_t lower, uint64_t upper) {
    if (lower > upper) return -1;
    std::vector<Launch> v;
    plan_range(msg, len, lower, upper, v, 0, g_policy);
    return plan_cost(v);
}

// Replays the kernel's per-nonce computation from launch `idx`'s descriptor.
int hostcheck_desc_hash(const uint8_t* msg, uint64_t len, uint64_t lower, uint64_t upper,
                        uint32_t rchunk, int idx, uint64_t nonce, uint64_t* out) {
    std::vector<Launch> v;
    plan_range(msg, len, lower, upper, v, rchunk, g_policy, /*host_ptab=*/true);
    if (idx < 0 || idx >= (int)v.size()) return -1;
    const Launch& l = v[(size_t)idx];
    const LaunchDesc& D = l.desc;
    if (nonce < l.lo || nonce > l.hi) return -2;
    if (l.C2 == 3) {
        // lane table: x = lane value (W_0/W_1 digits), r = loop value (p-table entry)
        const uint64_t off = nonce - D.base;
        const uint32_t r = (uint32_t)(off / D.RQ), x = (uint32_t)(off % D.RQ);
        if (x < D.p_first || x > D.p_last || r >= D.R) return -3;  // not a rectangle
        const uint32_t* P = &l.ptab[16ull * r];
        uint32_t W[64], st[8];
        std::memcpy(W, D.U, 64);
        W[0] |= ascii4(x / D.R1);
        W[1] |= (ascii4(x % D.R1) & D.qmask) << D.loop_shift;
        sha256_expand(W);
        std::memcpy(st, P, 32);
        // round 0 from the table's partial sums (as the kernel's ut_hash), then 1..63
        const uint32_t kw0 = kK[0] + W[0];
        uint32_t s1[8] = {P[8] + P[9] + kw0, st[0], st[1], st[2], st[3] + P[8] + kw0, st[4], st[5], st[6]};
        sha256_rounds(s1, W, 1, 64);
        *out = ((uint64_t)(P[0] + s1[0]) << 32) | (uint32_t)(P[1] + s1[1]);
        return 0;
    }
    // tail-digit launch: the kernel iterates k = nonce / stride; the tail digit is a
    // constant byte of D.U
    if (nonce % D.stride != D.tail) return -2;
    const uint64_t off = nonce / D.stride - D.base;
    const uint32_t p = (uint32_t)(off / D.R), r = (uint32_t)(off % D.R);
    const uint32_t alo = ascii4(p % 10000u), ahi = ascii4((p / 10000u) % 10000u);
    uint32_t W[64], st[8], cv[8];
    std::memcpy(W, D.U, 64);
    const int J = l.J;
    if (l.C2) {
        uint32_t V[64];
        std::memcpy(V, D.U1, 64);
        if (J == 0 || l.C2 == 2) { V[15] |= alo & D.mask_lo; V[14] |= ahi & D.mask_hi; }
        else { V[15] |= ahi & D.mask_hi; W[0] |= alo & D.mask_lo; }
        sha256_expand(V);
        std::memcpy(st, D.S1, 32);
        sha256_rounds(st, V, 14, 64);
        for (int i = 0; i < 8; i++) cv[i] = D.CV1[i] + st[i];
        std::memcpy(st, cv, 32);
        if (J == 1 && l.C2 == 1) sha256_rounds(st, W, 0, 1);  // W[1..] unused by round 0
    } else {
        std::memcpy(st, D.S0, 32);
        std::memcpy(cv, D.CV, 32);
        if (J >= 2) {
            W[J - 2] |= ahi & D.mask_hi;
            W[J - 1] |= alo & D.mask_lo;
            sha256_rounds(st, W, J - 2, J);
        } else if (J == 1) {
            W[0] |= alo & D.mask_lo;
            sha256_rounds(st, W, 0, 1);
        }
    }
    int t0 = J;
    if (l.C2 == 2) {  // two loop words: W_0 = 4 digits of r / R1, W_1 = digits of r % R1
        W[0] = D.U[0] | ascii4(r / D.R1);
        W[1] = D.U[1] | ((ascii4(r % D.R1) & D.qmask) << D.loop_shift);
        t0 = 0;
    } else {
        W[J] = D.U[J] | ((ascii4(r) & D.qmask) << D.loop_shift);
    }
    sha256_expand(W);
    sha256_rounds(st, W, t0, 64);
    uint32_t y[8];
    for (int i = 0; i < 8; i++) y[i] = cv[i] + st[i];
    if (l.EX) {
        uint32_t s2[8];
        std::memcpy(s2, y, 32);
        uint32_t kwx_minus_k[64];
        for (int t = 0; t < 64; t++) kwx_minus_k[t] = D.KWX[t] - kK[t];
        sha256_rounds(s2, kwx_minus_k, 0, 64);
        for (int i = 0; i < 8; i++) y[i] += s2[i];
    }
    *out = ((uint64_t)y[0] << 32) | y[1];
    return 0;
}

}  // extern "C"

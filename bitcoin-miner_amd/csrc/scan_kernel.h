// scan_kernel.h -- gfx950 nonce-scan kernel template (included by kernels_*.hip).
//
// One workgroup = 256 lanes × one chunk of loop values r.  Each lane owns one lane
// value p (its digits fill message words J-1 / J-2, or block B-1 for C2 layouts) and
// iterates r (the digits of the LAST digit-bearing word W_J of the final block):
//
//   per work item (once):  lane words, the lane-only rounds before J, block B-1 for
//                           C2, and every schedule/round term that does not read W_J
//                           (compile-time dependency analysis `kDep` + LICM)
//   per nonce (hot loop):   W_J = U_J | ascii(r) << shift  -- wave-UNIFORM, SALU
//                           rounds J..63 on VALU, schedule words that depend on W_J,
//                           H0 = IV/CV-folded a64; one v_cmp against a wave-uniform
//                           pruning threshold T; rare slow path does the exact
//                           lexicographic (hash, nonce) update in scalar registers.
//
// Everything is integer VALU: v_alignbit_b32 rotates, v_bitop3_b32 (XOR3 0x96, CH
// 0xCA, MAJ 0xE8), v_add3_u32.  No LDS or HBM traffic in the loop; one 16-byte
// candidate per workgroup at the end (appended only if it beats the threshold).
//
// Semantics: bitcoin.Hash (src/github.com/cmu440/bitcoin/hash.go:11-15), argmin over
// the inclusive range with the lowest nonce winning ties (spec'd loop p1.pdf pp.12-14,
// north_star).  The pruning is exact: T only ever holds the high word of a hash some
// valid nonce already achieved, and ties on the high word take the slow path.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "kernels.h"
#include "plan.h"

// Code phase of the per-nonce loop bodies.  The same instruction stream runs ~3.5% faster
// when the loop body starts at 4 mod 8 bytes than at 0 mod 8 (measured on config 2, J = 2,
// J = 13 and config 3, profiles/r01_loop_phase.jsonl; the mechanism is in the instruction
// fetch of the mixed 4-/8-byte encodings).  Without this, any edit before the loop flips
// the phase at random.  ".p2align 3" + one s_nop pins it at 4 mod 8 for one or two s_nop
// per iteration (~0.1%).  -DGPUHASH_LOOP_PHASE=0 / -1 selects phase 0 / no pinning; the
// kernels_misc.hip layouts (classic straddle, extra block), insensitive to the phase,
// build with -1.
#ifndef GPUHASH_LOOP_PHASE
#define GPUHASH_LOOP_PHASE 4
#endif
#if GPUHASH_LOOP_PHASE == 4
#define GPUHASH_LOOP_ALIGN() asm volatile(".p2align 3\n\ts_nop 0")
#elif GPUHASH_LOOP_PHASE == 0
#define GPUHASH_LOOP_ALIGN() asm volatile(".p2align 3")
#else
#define GPUHASH_LOOP_ALIGN() ((void)0)
#endif

namespace gpuhash {

namespace dev {

__device__ constexpr uint32_t K[64] = {
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

// Per-lane (VGPR) primitives: one VALU op each on gfx950.
__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) {
    return __builtin_amdgcn_alignbit(x, x, n);
}
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t ch(uint32_t e, uint32_t f, uint32_t g) {
    return __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA);
}
__device__ __forceinline__ uint32_t maj(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
}
__device__ __forceinline__ uint32_t bS0(uint32_t a) { return xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22)); }
__device__ __forceinline__ uint32_t bS1(uint32_t e) { return xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25)); }
__device__ __forceinline__ uint32_t bs0(uint32_t x) { return xor3(rotr(x, 7), rotr(x, 18), x >> 3); }
__device__ __forceinline__ uint32_t bs1(uint32_t x) { return xor3(rotr(x, 17), rotr(x, 19), x >> 10); }

// Wave-uniform primitives: plain C so the compiler keeps them on SALU.
__device__ __forceinline__ uint32_t urotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
// (LLVM issues the uniform sigma0(W_J) as v_alignbit with SGPR sources; pinning it on
// SALU measured 2.6% slower on config 2: tools/tuning_hooks.patch)
__device__ __forceinline__ uint32_t us0(uint32_t x) { return urotr(x, 7) ^ urotr(x, 18) ^ (x >> 3); }
__device__ __forceinline__ uint32_t us1(uint32_t x) { return urotr(x, 17) ^ urotr(x, 19) ^ (x >> 10); }

__device__ __forceinline__ uint32_t ascii4(uint32_t x) {
    uint32_t x1 = x / 10u, x2 = x1 / 10u, x3 = x2 / 10u;
    uint32_t d0 = x - x1 * 10u, d1 = x1 - x2 * 10u, d2 = x2 - x3 * 10u, d3 = x3 % 10u;
    return 0x30303030u | (d3 << 24) | (d2 << 16) | (d1 << 8) | d0;
}

// kDep<J>[t]: does schedule word W_t depend on the per-nonce word W_J?
template <int J>
struct DepTable {
    bool v[64];
    constexpr DepTable() : v() {
        for (int t = 0; t < 16; t++) v[t] = (t == J);
        for (int t = 16; t < 64; t++) v[t] = v[t - 2] || v[t - 7] || v[t - 15] || v[t - 16];
    }
};

template <int B, int E, class F>
__device__ __forceinline__ void sfor(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        sfor<B + 1, E>(f);
    }
}

struct State {
    uint32_t a, b, c, d, e, f, g, h;
};

// One generic round with K[t] + W folded into `kw`.
__device__ __forceinline__ void round_kw(State& s, uint32_t kw) {
    uint32_t t1 = s.h + kw + ch(s.e, s.f, s.g) + bS1(s.e);
    uint32_t t2 = bS0(s.a) + maj(s.a, s.b, s.c);
    s.h = s.g; s.g = s.f; s.f = s.e; s.e = s.d + t1;
    s.d = s.c; s.c = s.b; s.b = s.a; s.a = t1 + t2;
}

// A round whose K+W is wave-uniform (an SGPR) and whose h is per-lane.  A 2-input VALU
// add with a scalar operand issues at the slow rate; left to itself LLVM
// reads `kw` in the 2-input h + kw.  Here it goes into the 3-input add, slow class
// anyway, so the round's 2-input adds read VGPRs only.  The K+W-table layout (config 3)
// runs +1.8% with it; the plain, extra-block and lane-table rounds with a uniform K+W run
// 0.3-3.8% SLOWER with it (tools/tuning_hooks.patch; profiles/r04_fold_variants.jsonl),
// so only ut_hash's table rounds use it.
__device__ __forceinline__ void round_ukw(State& s, uint32_t kw) {
    uint32_t x;
    asm("v_add3_u32 %0, %1, %2, %3" : "=v"(x) : "v"(s.h), "s"(kw), "v"(ch(s.e, s.f, s.g)));
    uint32_t t1 = x + bS1(s.e);
    uint32_t t2 = bS0(s.a) + maj(s.a, s.b, s.c);
    s.h = s.g; s.g = s.f; s.f = s.e; s.e = s.d + t1;
    s.d = s.c; s.c = s.b; s.b = s.a; s.a = t1 + t2;
}

// Message expansion of a block whose words are all per-lane or uniform (no W_J):
// used for block B-1 of C2 layouts, once per work item.
__device__ __forceinline__ void expand_full(uint32_t (&w)[64]) {
    sfor<16, 64>([&](auto tc) {
        constexpr int t = decltype(tc)::value;
        w[t] = w[t - 16] + bs0(w[t - 15]) + w[t - 7] + bs1(w[t - 2]);
    });
}

}  // namespace dev

// Running best of one wave (wave-uniform, lives in SGPRs): exact lexicographic
// (hash, nonce) key and the pruning word T (high word of the best hash seen anywhere).
struct WaveBest {
    unsigned long long h, n;
    uint32_t T;
};

// Rounds 0..63 of block B when its whole message schedule is wave-uniform (C2 layouts
// whose loop digits are the only digits in block B): kw[t] = K[t] + W_t comes from a
// table, the per-lane input is the state s after block B-1 (= cv), so a nonce costs 64
// rounds and no schedule work.  Round 0 reuses the per-row part `inv0` (everything but
// kw[0]); round 63 skips e and folds CV0.
// Rounds t in [SK0, SK1) have a wave-uniform kw(t) (scalar loads) and a per-lane h.
template <int SK0, int SK1, class KW>
__device__ __forceinline__ void ut_hash(const dev::State& s, const uint32_t (&cv)[8], uint32_t inv0,
                                        uint32_t t20, KW&& kw, uint32_t& H0, uint32_t& H1) {
    using namespace dev;
    dev::State x = s;
    const uint32_t k0 = kw(0);
    x.h = x.g; x.g = x.f; x.f = x.e; x.e = (x.d + inv0) + k0;
    x.d = x.c; x.c = x.b; x.b = x.a; x.a = (inv0 + t20) + k0;
    sfor<1, 63>([&](auto tc) {
        constexpr int t = decltype(tc)::value;
        if constexpr (t >= SK0 && t < SK1) round_ukw(x, kw(t));
        else round_kw(x, kw(t));
    });
    const uint32_t t1 = x.h + kw(63) + cv[0] + ch(x.e, x.f, x.g) + bS1(x.e);
    H0 = t1 + bS0(x.a) + maj(x.a, x.b, x.c);
    H1 = cv[1] + x.a;
}

// One row of one launch: 256 consecutive lane values p (row) x loop values [r0, r1).
//
// C2 = 0: lane digits in words J-2, J-1 of block B, loop digits in W_J.
// C2 = 1: lane digits spill into block B-1 (compressed per lane, once per row); for J = 0
//         block B holds only loop digits, so its schedule is the per-r table `ktab`
//         (built by k_ktab, read with scalar loads).
// C2 = 2: (J = 1) block B's W_0 and W_1 hold only LOOP digits (r = W_0 digits * R1 + W_1
//         digits) and the lanes vary block B-1 only; the uniform schedules of 64 loop
//         values at a time are built by wave 0 into LDS and shared by the 4 waves.
template <int J, int C2, bool EX, int MODE>
__device__ __forceinline__ void scan_row(const LaunchDesc& D, uint32_t row, uint32_t r0, uint32_t r1,
                                         WaveBest& wb, unsigned long long* __restrict__ dump,
                                         unsigned long long dump_lo, const uint32_t* __restrict__ ktab) {
    using namespace dev;
    constexpr DepTable<J> kDep{};
    constexpr bool UT = C2 == 2 || (C2 == 1 && J == 0);  // uniform block-B schedule
    const uint32_t p = D.p_first + row * 256u + threadIdx.x;
    // A wave whose 64 lanes all lie past the launch's last lane value (the tail of a
    // partial last row) has no nonce to hash: it skips the row (up to 3.4x on one-row
    // C2 = 2 searches, profiles/r02_partial_rows.jsonl).  Only the C2 = 2 loop has
    // barriers (its LDS batches), so there an idle wave still walks the batches but
    // hashes nothing.  (Rotating which wave takes which 64-lane block per workgroup, to
    // spread the idle slots over the SIMDs, measured 1-4% slower on partial rows.)
    const bool wave_idle =
        __builtin_amdgcn_readfirstlane(D.p_first + row * 256u + (threadIdx.x & ~63u)) > D.p_last;
    if constexpr (C2 != 2) {
        if (wave_idle) return;
    }

    // ---- once per row: lane words and everything that does not read W_J ----
    const uint32_t alo = ascii4(p % 10000u);
    const uint32_t ahi = ascii4((p / 10000u) % 10000u);
    uint32_t W[16];
#pragma unroll
    for (int i = 0; i < 16; i++) W[i] = D.U[i];
    State s;
    uint32_t cv[8];
    if constexpr (C2 != 0) {
        uint32_t V[64];
#pragma unroll
        for (int i = 0; i < 16; i++) V[i] = D.U1[i];
        if constexpr (UT) {  // every lane digit sits at the end of block B-1
            V[15] |= alo & D.mask_lo;
            V[14] |= ahi & D.mask_hi;
        } else {
            V[15] |= ahi & D.mask_hi;
            W[0] |= alo & D.mask_lo;
        }
        expand_full(V);
        s = State{D.S1[0], D.S1[1], D.S1[2], D.S1[3], D.S1[4], D.S1[5], D.S1[6], D.S1[7]};
        sfor<14, 64>([&](auto tc) {
            constexpr int t = decltype(tc)::value;
            round_kw(s, K[t] + V[t]);
        });
        cv[0] = D.CV1[0] + s.a; cv[1] = D.CV1[1] + s.b; cv[2] = D.CV1[2] + s.c; cv[3] = D.CV1[3] + s.d;
        cv[4] = D.CV1[4] + s.e; cv[5] = D.CV1[5] + s.f; cv[6] = D.CV1[6] + s.g; cv[7] = D.CV1[7] + s.h;
        s = State{cv[0], cv[1], cv[2], cv[3], cv[4], cv[5], cv[6], cv[7]};
        if constexpr (!UT && J == 1) round_kw(s, K[0] + W[0]);
    } else {
        s = State{D.S0[0], D.S0[1], D.S0[2], D.S0[3], D.S0[4], D.S0[5], D.S0[6], D.S0[7]};
#pragma unroll
        for (int i = 0; i < 8; i++) cv[i] = D.CV[i];
        if constexpr (J >= 2) {
            W[J - 2] |= ahi & D.mask_hi;
            W[J - 1] |= alo & D.mask_lo;
            round_kw(s, K[J - 2] + W[J - 2]);
            round_kw(s, K[J - 1] + W[J - 1]);
        } else if constexpr (J == 1) {
            W[0] |= alo & D.mask_lo;
            round_kw(s, K[0] + W[0]);
        }
    }
    // UT layouts: round 0 of block B without its K+W term (per row)
    uint32_t inv0 = 0, t20 = 0;
    if constexpr (UT) {
        inv0 = s.h + bS1(s.e) + ch(s.e, s.f, s.g);
        t20 = bS0(s.a) + maj(s.a, s.b, s.c);
    }

    // Edge handling: only the first / last lane of a launch has a partial r range, and
    // lanes past p_last are idle.  Checked only in the (rare) slow path.
    const bool lane_ok = p <= D.p_last;
    const uint32_t rlo = (p == D.p_first) ? D.r_first : 0u;
    const uint32_t rhi = (p == D.p_last) ? D.r_last : D.R - 1u;

    // Per-nonce bookkeeping: dump (MODE 1) or the exact lexicographic running best with
    // the wave-uniform pruning test (MODE 0).
    auto finish = [&](uint32_t r, uint32_t H0, uint32_t H1) {
#ifdef GPUHASH_TIE_TEST_BITS
        // Test-only build (libgpuhash_tietest.so): keep only the top bits of the hash so
        // equal keys are common and every reduction level's lowest-nonce rule is exercised.
        H0 >>= (32 - GPUHASH_TIE_TEST_BITS);
        H1 = 0;
#endif
        if constexpr (MODE == 1) {
            if (lane_ok && r >= rlo && r <= rhi) {
                // k = D.base + p·R + r; nonce = k·stride + tail (tail-digit launches, plan.h)
                unsigned long long n = (D.base + (unsigned long long)p * D.R + r) * D.stride + D.tail;
                dump[n - dump_lo] = ((unsigned long long)H0 << 32) | H1;
            }
        } else {
            unsigned long long m = __builtin_amdgcn_ballot_w64(H0 <= wb.T);
            if (m) {  // wave-uniform, rare once T has settled
                const bool ok = lane_ok && r >= rlo && r <= rhi;
                m = __builtin_amdgcn_ballot_w64(H0 <= wb.T && ok);
                while (m) {
                    const int l = __builtin_ctzll(m);
                    m &= m - 1;
                    const uint32_t h0 = __builtin_amdgcn_readlane(H0, l);
                    const uint32_t h1 = __builtin_amdgcn_readlane(H1, l);
                    const uint32_t pl = __builtin_amdgcn_readlane(p, l);
                    const unsigned long long hh = ((unsigned long long)h0 << 32) | h1;
                    const unsigned long long nn = (D.base + (unsigned long long)pl * D.R + r) * D.stride + D.tail;
                    if (hh < wb.h || (hh == wb.h && nn < wb.n)) {
                        wb.h = hh;
                        wb.n = nn;
                        wb.T = h0 < wb.T ? h0 : wb.T;
                    }
                }
            }
        }
    };

    if constexpr (C2 == 2) {
        // 64 loop values per batch: wave 0 lane j builds the K+W schedule of r = rb + j
        // (row stride 68 words keeps 16-byte alignment for the broadcast reads).
        __shared__ uint4 sh_kw[64][17];
        for (uint32_t rb = r0; rb < r1; rb += 64u) {
            const uint32_t nb = r1 - rb < 64u ? r1 - rb : 64u;
            __syncthreads();  // the previous batch has been consumed by every wave
            if (threadIdx.x < nb) {
                const uint32_t r = rb + threadIdx.x;
                const uint32_t m = r / D.R1, q = r - m * D.R1;
                uint32_t w[64];
#pragma unroll
                for (int i = 0; i < 16; i++) w[i] = D.U[i];
                w[0] |= ascii4(m);
                w[1] |= (ascii4(q) & D.qmask) << D.loop_shift;
                expand_full(w);
#pragma unroll
                for (int i = 0; i < 16; i++)
                    sh_kw[threadIdx.x][i] = make_uint4(K[4 * i] + w[4 * i], K[4 * i + 1] + w[4 * i + 1],
                                                       K[4 * i + 2] + w[4 * i + 2], K[4 * i + 3] + w[4 * i + 3]);
            }
            __syncthreads();
            for (uint32_t j = 0; j < (wave_idle ? 0u : nb); j++) {
                const uint4* kr = sh_kw[j];
                uint32_t H0, H1;
                ut_hash<0, 0>(s, cv, inv0, t20, [&](int t) {   // kw from LDS: per-lane
                    const uint4 v = kr[t >> 2];
                    return (t & 3) == 0 ? v.x : (t & 3) == 1 ? v.y : (t & 3) == 2 ? v.z : v.w;
                }, H0, H1);
                finish(rb + j, H0, H1);
            }
        }
        return;
    }

#pragma unroll 1  // one nonce per iteration (unrolling x2 measured no gain, r01_variants)
    for (uint32_t r = r0; r < r1; r++) {
        GPUHASH_LOOP_ALIGN();
        uint32_t H0, H1;
        if constexpr (UT) {
            const uint32_t* __restrict__ kw = ktab + D.tab_off + 64u * r;
            ut_hash<1, 63>(s, cv, inv0, t20, [&](int t) { return kw[t]; }, H0, H1);
        } else {
            const uint32_t WJ = D.U[J] | ((ascii4(r) & D.qmask) << D.loop_shift);
            uint32_t w[64];
#pragma unroll
            for (int i = 0; i < 16; i++) w[i] = W[i];
            w[J] = WJ;
            // schedule word t, computed just before round t uses it (so only the ~16
            // words of the sliding window are live, not all 48): loop-invariant terms
            // are summed first so LICM hoists them out of the r-loop
            auto sched = [&](auto tc) {
                constexpr int t = decltype(tc)::value;
                constexpr bool d2 = kDep.v[t - 2], d7 = kDep.v[t - 7], d15 = kDep.v[t - 15], d16 = kDep.v[t - 16];
                uint32_t x2, x15;
                if constexpr (t - 2 == J) x2 = us1(w[t - 2]); else x2 = bs1(w[t - 2]);
                if constexpr (t - 15 == J) x15 = us0(w[t - 15]); else x15 = bs0(w[t - 15]);
                uint32_t inv = (d2 ? 0u : x2) + (d7 ? 0u : w[t - 7]) + (d15 ? 0u : x15) + (d16 ? 0u : w[t - 16]);
                uint32_t var = (d2 ? x2 : 0u) + (d7 ? w[t - 7] : 0u) + (d15 ? x15 : 0u) + (d16 ? w[t - 16] : 0u);
                w[t] = inv + var;
            };
            State x = s;
            {   // round J: everything but W_J is loop-invariant
                uint32_t inv = x.h + bS1(x.e) + ch(x.e, x.f, x.g) + K[J];
                uint32_t t2 = bS0(x.a) + maj(x.a, x.b, x.c);
                x.h = x.g; x.g = x.f; x.f = x.e; x.e = (x.d + inv) + WJ;
                x.d = x.c; x.c = x.b; x.b = x.a; x.a = (inv + t2) + WJ;
            }
            sfor<J + 1, 63>([&](auto tc) {
                constexpr int t = decltype(tc)::value;
                if constexpr (t < 16) {
                    round_kw(x, K[t] + w[t]);   // uniform word: K+W folds
                } else {
                    sched(tc);
                    round_kw(x, w[t] + K[t]);
                }
            });
            sched(std::integral_constant<int, 63>{});
            if constexpr (!EX) {
                // round 63: e is dead; fold CV0 into the constant so a64 + CV0 is free
                uint32_t t1 = x.h + w[63] + (K[63] + cv[0]) + ch(x.e, x.f, x.g) + bS1(x.e);
                H0 = t1 + bS0(x.a) + maj(x.a, x.b, x.c);
                H1 = cv[1] + x.a;
            } else {
                round_kw(x, w[63] + K[63]);
                State y{cv[0] + x.a, cv[1] + x.b, cv[2] + x.c, cv[3] + x.d,
                        cv[4] + x.e, cv[5] + x.f, cv[6] + x.g, cv[7] + x.h};
                const uint32_t y0 = y.a, y1 = y.b;
                sfor<0, 63>([&](auto tc) {
                    constexpr int t = decltype(tc)::value;
                    round_kw(y, D.KWX[t]);
                });
                uint32_t t1 = y.h + D.KWX[63] + ch(y.e, y.f, y.g) + bS1(y.e);
                H0 = y0 + t1 + bS0(y.a) + maj(y.a, y.b, y.c);
                H1 = y1 + y.a;
            }
        }
        finish(r, H0, H1);
    }
}

// C2 = 3 (lane table): one row = 256 consecutive values x of block B's W_0/W_1 digits,
// one per lane, x loop values r = the block B-1 digits, p = p_a + r.  Per row each lane
// builds block B's K+W schedule for its x ONCE (kept in registers: the rows of C2 = 2
// could share one schedule across a wave only because its lanes varied block B-1); per
// loop value the wave reads block B-1's chaining value and round 0's partial sums from
// the host's p-table (scalar loads) and every lane runs block B's 64 rounds, as ut_hash.
// nonce = D.base + r * D.RQ + x.
template <int MODE>
__device__ __forceinline__ void scan_row_lt(const LaunchDesc& D, uint32_t row, uint32_t r0, uint32_t r1,
                                            WaveBest& wb, unsigned long long* __restrict__ dump,
                                            unsigned long long dump_lo, const uint32_t* __restrict__ ptab) {
    using namespace dev;
    const uint32_t x = D.p_first + row * 256u + threadIdx.x;
    const bool wave_idle =
        __builtin_amdgcn_readfirstlane(D.p_first + row * 256u + (threadIdx.x & ~63u)) > D.p_last;
    if (wave_idle) return;
    const bool lane_ok = x <= D.p_last;
    uint32_t kw[64];
    {
        const uint32_t hi4 = x / D.R1, lo = x - hi4 * D.R1;
        uint32_t w[64];
#pragma unroll
        for (int i = 0; i < 16; i++) w[i] = D.U[i];
        w[0] |= ascii4(hi4);
        w[1] |= (ascii4(lo) & D.qmask) << D.loop_shift;
        expand_full(w);
#pragma unroll
        for (int t = 0; t < 64; t++) kw[t] = K[t] + w[t];
    }
#pragma unroll 1
    for (uint32_t r = r0; r < r1; r++) {
        const uint32_t* __restrict__ P = ptab + D.tab_off + 16u * r;
        uint32_t cv[8];
#pragma unroll
        for (int i = 0; i < 8; i++) cv[i] = P[i];
        const State s{cv[0], cv[1], cv[2], cv[3], cv[4], cv[5], cv[6], cv[7]};
        uint32_t H0, H1;
        ut_hash<0, 0>(s, cv, P[8], P[9], [&](int t) { return kw[t]; }, H0, H1);
#ifdef GPUHASH_TIE_TEST_BITS
        H0 >>= (32 - GPUHASH_TIE_TEST_BITS);
        H1 = 0;
#endif
        if constexpr (MODE == 1) {
            if (lane_ok) dump[D.base + (unsigned long long)r * D.RQ + x - dump_lo] = ((unsigned long long)H0 << 32) | H1;
        } else {
            unsigned long long m = __builtin_amdgcn_ballot_w64(H0 <= wb.T);
            if (m) {  // wave-uniform, rare once T has settled
                m = __builtin_amdgcn_ballot_w64(H0 <= wb.T && lane_ok);
                while (m) {
                    const int l = __builtin_ctzll(m);
                    m &= m - 1;
                    const uint32_t h0 = __builtin_amdgcn_readlane(H0, l);
                    const uint32_t h1 = __builtin_amdgcn_readlane(H1, l);
                    const uint32_t xl = __builtin_amdgcn_readlane(x, l);
                    const unsigned long long hh = ((unsigned long long)h0 << 32) | h1;
                    const unsigned long long nn = D.base + (unsigned long long)r * D.RQ + xl;
                    if (hh < wb.h || (hh == wb.h && nn < wb.n)) {
                        wb.h = hh;
                        wb.n = nn;
                        wb.T = h0 < wb.T ? h0 : wb.T;
                    }
                }
            }
        }
    }
}

__device__ __forceinline__ unsigned long long uniform64(unsigned long long v) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return ((unsigned long long)hi << 32) | lo;
}

// Persistent scan over every launch descriptor of one kernel variant.
//
// Work = rows x loop values, linearised in "row-iterations" (one r value for a whole
// 256-lane row): descriptor i owns [offs[i], offs[i+1]).  Workgroups (a grid sized to
// the resident capacity) grab contiguous pieces with one atomicAdd -- guided
// self-scheduling: piece = clamp(remaining / (2 * grid), gmin, gmax) -- so early pieces
// amortise the per-row setup and the last ones are short, which keeps the tail of the
// launch to ~gmin iterations.  The wave-uniform best (and its pruning word) persists
// across pieces; each workgroup appends one 16-byte candidate at the end if it found one.
// Tuning hook (tools/build_variants.sh): -DGPUHASH_WAVES_PER_EU=N asks for >= N waves per
// SIMD, i.e. a VGPR budget of 512/N.  Off in the product build.
#ifdef GPUHASH_WAVES_PER_EU
#define GPUHASH_SCAN_ATTR __attribute__((amdgpu_waves_per_eu(GPUHASH_WAVES_PER_EU)))
#else
#define GPUHASH_SCAN_ATTR
#endif
template <int J, int C2, bool EX, int MODE>
__global__ __launch_bounds__(256) GPUHASH_SCAN_ATTR void k_scan(const LaunchDesc* __restrict__ descs,
                                              const unsigned long long* __restrict__ offs,
                                              int ndesc, unsigned long long* __restrict__ work,
                                              unsigned int gmin, unsigned int gmax,
                                              unsigned long long* __restrict__ thresh,
                                              Cand* __restrict__ cands,
                                              unsigned int* __restrict__ ncand,
                                              unsigned long long* __restrict__ dump,
                                              unsigned long long dump_lo,
                                              const uint32_t* __restrict__ ktab) {
    static_assert(J >= 0 && J < 16, "loop word index");
    static_assert(!C2 || J <= 1, "C2 layouts have the loop word at J <= 1");
    static_assert(C2 != 2 || J == 1, "two-word uniform loop only with the loop word at J = 1");
    static_assert(C2 != 3 || (J == 1 && !EX), "lane table only with the loop word at J = 1");
    static_assert(!EX || J >= 13, "extra padding block only when the last digit is at byte >= 55");
    __shared__ unsigned long long sh_grab[2];
    __shared__ unsigned long long sh_best[4][2];
    const uint32_t tid = threadIdx.x;
    const unsigned long long total = offs[ndesc];

    // clock evidence: workgroup 0 (resident for the whole persistent launch) samples the
    // shader clock counter and the 100 MHz real-time counter at its start and its end,
    // into the 4 words after the group's work counter (no extra kernel argument: one
    // measurably changed the hot loop's SGPR assignment and cost 3.5%)
    unsigned long long* const clk = work + 1;
    if (blockIdx.x == 0 && tid == 0) {
        clk[0] = __builtin_amdgcn_s_memtime();
        clk[1] = __builtin_amdgcn_s_memrealtime();
    }
    WaveBest wb{~0ull, ~0ull, 0xFFFFFFFFu};
    for (;;) {
        if (tid == 0) {
            const unsigned long long cur = __hip_atomic_load(work, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned long long rem = cur < total ? total - cur : 0ull;
            unsigned long long g = rem / (2ull * gridDim.x);
            g = g < gmin ? gmin : (g > gmax ? gmax : g);
            sh_grab[0] = atomicAdd(work, g);
            sh_grab[1] = g;
        }
        __syncthreads();
        unsigned long long x = uniform64(sh_grab[0]);
        const unsigned long long g = uniform64(sh_grab[1]);
        __syncthreads();
        if (x >= total) break;
        const unsigned long long end = x + g < total ? x + g : total;
        if constexpr (MODE == 0) {
            const unsigned long long tv = __hip_atomic_load(thresh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t t = __builtin_amdgcn_readfirstlane((uint32_t)(tv >> 32));
            wb.T = t < wb.T ? t : wb.T;
        }
        while (x < end) {
            int i = 0;
            while (i + 1 < ndesc && offs[i + 1] <= x) i++;
            const LaunchDesc& D = descs[i];
            const uint32_t rel = (uint32_t)(x - offs[i]);  // < rows * R <= 2^32 (plan.h)
            const uint32_t row = rel / D.R, r0 = rel - row * D.R;
            const unsigned long long left = end - x;
            const uint32_t r1 = (unsigned long long)(D.R - r0) < left ? D.R : r0 + (uint32_t)left;
            if constexpr (C2 == 3) scan_row_lt<MODE>(D, row, r0, r1, wb, dump, dump_lo, ktab);
            else scan_row<J, C2, EX, MODE>(D, row, r0, r1, wb, dump, dump_lo, ktab);
            x += r1 - r0;
        }
    }

    if (blockIdx.x == 0 && tid == 0) {
        clk[2] = __builtin_amdgcn_s_memtime();
        clk[3] = __builtin_amdgcn_s_memrealtime();
    }
    if constexpr (MODE == 0) {
        const uint32_t wave = tid >> 6;
        if ((tid & 63u) == 0) { sh_best[wave][0] = wb.h; sh_best[wave][1] = wb.n; }
        __syncthreads();
        if (tid == 0) {
            unsigned long long bh = sh_best[0][0], bn = sh_best[0][1];
#pragma unroll
            for (int i = 1; i < 4; i++) {
                if (sh_best[i][0] < bh || (sh_best[i][0] == bh && sh_best[i][1] < bn)) {
                    bh = sh_best[i][0];
                    bn = sh_best[i][1];
                }
            }
            if (bh != ~0ull || bn != ~0ull) {
                atomicMin(thresh, bh);
                const unsigned int idx = atomicAdd(ncand, 1u);
                cands[idx].hash = bh;
                cands[idx].nonce = bn;
            }
        }
    }
}

}  // namespace gpuhash

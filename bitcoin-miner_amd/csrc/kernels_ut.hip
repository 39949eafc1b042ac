// kernels_ut.hip -- k_scan instances of the K+W-table uniform-schedule layout (C2 = 1,
// J = 0: block B holds loop digits only), the lane-table layout (C2 = 3,
// J = 1) and the table builder k_ktab.
// Built with -mllvm -amdgpu-sched-strategy=max-ilp (Makefile): +2.1% on config 3 over
// the default options (profiles/r01_variants.jsonl).
#include "scan_decl.h"
#include "scan_kernel.h"

namespace gpuhash {

// Uniform schedule table of a C2/J=0 descriptor (one thread per loop value r):
// tab[64*r + t] = K[t] + W_t, W = block B's uniform words with r's ASCII digits in W_0.
__global__ __launch_bounds__(256) void k_ktab(const LaunchDesc* __restrict__ desc,
                                              uint32_t* __restrict__ tab, uint32_t R) {
    using namespace dev;
    const uint32_t r = blockIdx.x * 256u + threadIdx.x;
    if (r >= R) return;
    const LaunchDesc& D = *desc;
    uint32_t w[64];
#pragma unroll
    for (int i = 0; i < 16; i++) w[i] = D.U[i];
    w[0] |= (ascii4(r) & D.qmask) << D.loop_shift;
    expand_full(w);
    uint32_t* out = tab + 64ull * r;
#pragma unroll
    for (int t = 0; t < 64; t++) out[t] = K[t] + w[t];
}

// p-table of a lane-table (C2 = 3) descriptor (one thread per loop value k < D.R, one
// blockIdx.y per descriptor): block B-1 = its uniform words U1 with the s digits of
// p = lt_p0 + k at its end, compressed from the uniform state S1 after rounds 0..13 (those
// read no digit), + CV1 -> block B's input state cv; then round 0 of block B without its
// K+W term: inv0 = h + S1(e) + Ch(e, f, g), t20 = S0(a) + Maj(a, b, c).
__global__ __launch_bounds__(256) void k_ptab(const LaunchDesc* __restrict__ descs, uint32_t* __restrict__ tab) {
    using namespace dev;
    const LaunchDesc& D = descs[blockIdx.y];
    const uint32_t k = blockIdx.x * 256u + threadIdx.x;
    if (k >= D.R) return;
    const uint32_t p = D.lt_p0 + k;
    uint32_t V[64];
#pragma unroll
    for (int i = 0; i < 16; i++) V[i] = D.U1[i];
    V[15] |= ascii4(p % 10000u) & D.mask_lo;
    V[14] |= ascii4((p / 10000u) % 10000u) & D.mask_hi;
    expand_full(V);
    State s{D.S1[0], D.S1[1], D.S1[2], D.S1[3], D.S1[4], D.S1[5], D.S1[6], D.S1[7]};
    sfor<14, 64>([&](auto tc) {
        constexpr int t = decltype(tc)::value;
        round_kw(s, K[t] + V[t]);
    });
    const uint32_t cv[8] = {D.CV1[0] + s.a, D.CV1[1] + s.b, D.CV1[2] + s.c, D.CV1[3] + s.d,
                            D.CV1[4] + s.e, D.CV1[5] + s.f, D.CV1[6] + s.g, D.CV1[7] + s.h};
    uint32_t* out = tab + D.tab_off + 16u * k;
#pragma unroll
    for (int i = 0; i < 8; i++) out[i] = cv[i];
    out[8] = cv[7] + bS1(cv[4]) + ch(cv[4], cv[5], cv[6]);
    out[9] = bS0(cv[0]) + maj(cv[0], cv[1], cv[2]);
}

}  // namespace gpuhash

GPUHASH_INSTANTIATE_SCAN(0, 1, false, 0);
GPUHASH_INSTANTIATE_SCAN(0, 1, false, 1);
// C2 = 3: the lane-table straddle layout (scan_row_lt), uniform-table family too
GPUHASH_INSTANTIATE_SCAN(1, 3, false, 0);
GPUHASH_INSTANTIATE_SCAN(1, 3, false, 1);

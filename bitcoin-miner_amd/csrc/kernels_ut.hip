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

}  // namespace gpuhash

GPUHASH_INSTANTIATE_SCAN(0, 1, false, 0);
GPUHASH_INSTANTIATE_SCAN(0, 1, false, 1);
// C2 = 3: the lane-table straddle layout (scan_row_lt), uniform-table family too
GPUHASH_INSTANTIATE_SCAN(1, 3, false, 0);
GPUHASH_INSTANTIATE_SCAN(1, 3, false, 1);

// scan_decl.h -- declarations of the scan kernels for the dispatch TU (kernels.hip).
//
// The k_scan instances are compiled in three TUs with the code-generation options each
// layout family measured best with (tools/variant_bench.py):
//   kernels_plain.hip  C2 = 0, no extra block: 8 waves/SIMD (63 VGPRs, no spills)
//   kernels_ut.hip     C2 = 1, J = 0 (K+W table layouts), C2 = 3 (lane table) + k_ktab:
//                      max-ILP scheduling
//   kernels_misc.hip   C2 = 1/J = 1, C2 = 2, extra-block layouts: max-ILP scheduling
// kernels.hip launches them through these declarations only, so nothing is implicitly
// instantiated there.
#pragma once
#include <stdint.h>

#include "kernels.h"
#include "plan.h"

namespace gpuhash {

template <int J, int C2, bool EX, int MODE>
__global__ void k_scan(const LaunchDesc* __restrict__ descs, const unsigned long long* __restrict__ offs,
                       int ndesc, unsigned long long* __restrict__ work, unsigned int gmin,
                       unsigned int gmax, unsigned long long* __restrict__ thresh,
                       Cand* __restrict__ cands, unsigned int* __restrict__ ncand,
                       unsigned long long* __restrict__ dump, unsigned long long dump_lo,
                       const uint32_t* __restrict__ ktab);

__global__ void k_ktab(const LaunchDesc* __restrict__ desc, uint32_t* __restrict__ tab, uint32_t R);
__global__ void k_ptab(const LaunchDesc* __restrict__ descs, uint32_t* __restrict__ tab);

}  // namespace gpuhash

// Explicit instantiation of one k_scan instance (used by the kernels_*.hip TUs).
#define GPUHASH_INSTANTIATE_SCAN(J, C2, EX, MODE)                                                    \
    template __global__ void gpuhash::k_scan<J, C2, EX, MODE>(                                       \
        const gpuhash::LaunchDesc* __restrict__, const unsigned long long* __restrict__, int,        \
        unsigned long long* __restrict__, unsigned int, unsigned int,                                \
        unsigned long long* __restrict__, gpuhash::Cand* __restrict__, unsigned int* __restrict__,   \
        unsigned long long* __restrict__, unsigned long long, const uint32_t* __restrict__)

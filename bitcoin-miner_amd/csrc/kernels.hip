// kernels.hip -- instantiates the gfx950 scan kernels and the candidate reduce.
#include "kernels.h"
#include "scan_kernel.h"

namespace gpuhash {

// Second pass: fold the appended per-workgroup candidates into the running best
// (lexicographic (hash, nonce), lowest nonce on ties) and reset the append counter.
__global__ __launch_bounds__(1024) void k_reduce(Cand* __restrict__ cands,
                                                 unsigned int* __restrict__ ncand,
                                                 Cand* __restrict__ best) {
    __shared__ unsigned long long sh[1024][2];
    const unsigned int n = *ncand;
    unsigned long long bh = ~0ull, bn = ~0ull;
    for (unsigned int i = threadIdx.x; i < n; i += 1024u) {
        const unsigned long long h = cands[i].hash, x = cands[i].nonce;
        if (h < bh || (h == bh && x < bn)) { bh = h; bn = x; }
    }
    sh[threadIdx.x][0] = bh;
    sh[threadIdx.x][1] = bn;
    __syncthreads();
    for (unsigned int s = 512; s > 0; s >>= 1) {
        if (threadIdx.x < s) {
            const unsigned long long h = sh[threadIdx.x + s][0], x = sh[threadIdx.x + s][1];
            if (h < sh[threadIdx.x][0] || (h == sh[threadIdx.x][0] && x < sh[threadIdx.x][1])) {
                sh[threadIdx.x][0] = h;
                sh[threadIdx.x][1] = x;
            }
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const unsigned long long h = sh[0][0], x = sh[0][1];
        if (h < best->hash || (h == best->hash && x < best->nonce)) {
            best->hash = h;
            best->nonce = x;
        }
        *ncand = 0u;
    }
}

template <int J, bool C2, bool EX, int MODE>
static hipError_t go(const Launch& l, const ScanArgs& a) {
    hipLaunchKernelGGL((k_scan<J, C2, EX, MODE>), dim3(l.nblocks), dim3(256), 0, a.stream, l.desc,
                       a.thresh, a.cands, a.ncand, a.dump, a.dump_lo);
    return hipGetLastError();
}

template <int MODE>
static hipError_t dispatch(const Launch& l, const ScanArgs& a) {
    if (l.C2) {
        switch (l.J) {
            case 0: return go<0, true, false, MODE>(l, a);
            case 1: return go<1, true, false, MODE>(l, a);
            default: return hipErrorInvalidValue;
        }
    }
    if (l.EX) {
        switch (l.J) {
            case 13: return go<13, false, true, MODE>(l, a);
            case 14: return go<14, false, true, MODE>(l, a);
            case 15: return go<15, false, true, MODE>(l, a);
            default: return hipErrorInvalidValue;
        }
    }
    switch (l.J) {
        case 0: return go<0, false, false, MODE>(l, a);
        case 1: return go<1, false, false, MODE>(l, a);
        case 2: return go<2, false, false, MODE>(l, a);
        case 3: return go<3, false, false, MODE>(l, a);
        case 4: return go<4, false, false, MODE>(l, a);
        case 5: return go<5, false, false, MODE>(l, a);
        case 6: return go<6, false, false, MODE>(l, a);
        case 7: return go<7, false, false, MODE>(l, a);
        case 8: return go<8, false, false, MODE>(l, a);
        case 9: return go<9, false, false, MODE>(l, a);
        case 10: return go<10, false, false, MODE>(l, a);
        case 11: return go<11, false, false, MODE>(l, a);
        case 12: return go<12, false, false, MODE>(l, a);
        case 13: return go<13, false, false, MODE>(l, a);
        case 14: return go<14, false, false, MODE>(l, a);
        case 15: return go<15, false, false, MODE>(l, a);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_scan(const Launch& l, int mode, const ScanArgs& a) {
    return mode == 0 ? dispatch<0>(l, a) : dispatch<1>(l, a);
}

hipError_t launch_reduce(Cand* cands, unsigned int* ncand, Cand* best, hipStream_t stream) {
    hipLaunchKernelGGL(k_reduce, dim3(1), dim3(1024), 0, stream, cands, ncand, best);
    return hipGetLastError();
}

}  // namespace gpuhash

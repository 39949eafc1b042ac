// kernels.hip -- launch dispatch for the gfx950 scan kernels (instantiated in
// kernels_{plain,ut,misc}.hip, see scan_decl.h) and the candidate reduce.
#include <atomic>

#include "kernels.h"
#include "scan_decl.h"

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

template <int J, int C2, bool EX, int MODE>
static auto kfn() {
    return &k_scan<J, C2, EX, MODE>;
}

template <int J, int C2, bool EX, int MODE>
static hipError_t go(const ScanArgs& a) {
    hipLaunchKernelGGL((k_scan<J, C2, EX, MODE>), dim3(a.grid), dim3(256), 0, a.stream, a.descs,
                       a.offs, a.ndesc, a.work, a.gmin, a.gmax, a.thresh, a.cands, a.ncand, a.dump,
                       a.dump_lo, a.ktab);
    return hipGetLastError();
}

template <int J, int C2, bool EX, int MODE>
static unsigned int occ(int device) {
    // cached per (variant, device): resident blocks per CU x CUs.  Device threads may
    // race to fill an entry; they compute the same value.
    static std::atomic<unsigned int> cache[64];
    if (device < 0 || device >= 64) return 0;
    unsigned int v = cache[device].load(std::memory_order_relaxed);
    if (!v) {
        int nb = 0, cus = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)kfn<J, C2, EX, MODE>(), 256, 0) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess)
            return 0;
        v = (unsigned int)(nb > 0 ? nb : 1) * (unsigned int)cus;
        cache[device].store(v, std::memory_order_relaxed);
    }
    return v;
}

// Expands a runtime (J, C2, EX) into the matching template instance and applies F.
template <int MODE, class F>
static auto with_variant(int J, int C2, int EX, F&& f) {
    if (C2 == 3) return f.template operator()<1, 3, false, MODE>();
    if (C2 == 2) return f.template operator()<1, 2, false, MODE>();
    if (C2) {
        switch (J) {
            case 0: return f.template operator()<0, 1, false, MODE>();
            default: return f.template operator()<1, 1, false, MODE>();
        }
    }
    if (EX) {
        switch (J) {
            case 13: return f.template operator()<13, 0, true, MODE>();
            case 14: return f.template operator()<14, 0, true, MODE>();
            default: return f.template operator()<15, 0, true, MODE>();
        }
    }
    switch (J) {
        case 0: return f.template operator()<0, 0, false, MODE>();
        case 1: return f.template operator()<1, 0, false, MODE>();
        case 2: return f.template operator()<2, 0, false, MODE>();
        case 3: return f.template operator()<3, 0, false, MODE>();
        case 4: return f.template operator()<4, 0, false, MODE>();
        case 5: return f.template operator()<5, 0, false, MODE>();
        case 6: return f.template operator()<6, 0, false, MODE>();
        case 7: return f.template operator()<7, 0, false, MODE>();
        case 8: return f.template operator()<8, 0, false, MODE>();
        case 9: return f.template operator()<9, 0, false, MODE>();
        case 10: return f.template operator()<10, 0, false, MODE>();
        case 11: return f.template operator()<11, 0, false, MODE>();
        case 12: return f.template operator()<12, 0, false, MODE>();
        default: return f.template operator()<13, 0, false, MODE>();
    }
}

static bool valid_variant(int J, int C2, int EX) {
    if (C2 == 2 || C2 == 3) return !EX && J == 1;
    if (C2) return C2 == 1 && !EX && (J == 0 || J == 1);
    if (EX) return J >= 13 && J <= 15;
    return J >= 0 && J <= 13;  // J = 14, 15 always need the extra block
}

struct Launcher {
    const ScanArgs& a;
    template <int J, int C2, bool EX, int MODE>
    hipError_t operator()() const { return go<J, C2, EX, MODE>(a); }
};

struct Occupancy {
    int device;
    template <int J, int C2, bool EX, int MODE>
    unsigned int operator()() const { return occ<J, C2, EX, MODE>(device); }
};

unsigned int grid_for(int J, int C2, int EX, int mode, int device) {
    if (!valid_variant(J, C2, EX)) return 0;
    return mode == 0 ? with_variant<0>(J, C2, EX, Occupancy{device})
                     : with_variant<1>(J, C2, EX, Occupancy{device});
}

hipError_t launch_scan(int J, int C2, int EX, int mode, const ScanArgs& a) {
    if (!valid_variant(J, C2, EX) || a.grid == 0 || a.ndesc <= 0) return hipErrorInvalidValue;
    return mode == 0 ? with_variant<0>(J, C2, EX, Launcher{a}) : with_variant<1>(J, C2, EX, Launcher{a});
}

hipError_t launch_ktab(const LaunchDesc* d_desc, uint32_t* tab, uint32_t R, hipStream_t stream) {
    if (!d_desc || !tab || R == 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_ktab, dim3((R + 255u) / 256u), dim3(256), 0, stream, d_desc, tab, R);
    return hipGetLastError();
}

hipError_t launch_ptab(const LaunchDesc* d_descs, int ndesc, uint32_t* tab, hipStream_t stream) {
    if (!d_descs || !tab || ndesc <= 0) return hipErrorInvalidValue;
    // kMaxLtLoop = 1024 loop values per descriptor: 4 workgroups of 256 per descriptor
    hipLaunchKernelGGL(k_ptab, dim3(kMaxLtLoop / 256u, (unsigned)ndesc), dim3(256), 0, stream, d_descs, tab);
    return hipGetLastError();
}

hipError_t launch_reduce(Cand* cands, unsigned int* ncand, Cand* best, hipStream_t stream) {
    hipLaunchKernelGGL(k_reduce, dim3(1), dim3(1024), 0, stream, cands, ncand, best);
    return hipGetLastError();
}

}  // namespace gpuhash

// kernels.h -- host-side entry points of kernels.hip.
#pragma once
#include <hip/hip_runtime.h>

#include "plan.h"

namespace gpuhash {

// One search candidate: a (hash, nonce) key, compared lexicographically.
struct Cand {
    unsigned long long hash;
    unsigned long long nonce;
};

struct ScanArgs {
    hipStream_t stream;
    const LaunchDesc* descs;         // device: the group's launch descriptors
    const unsigned long long* offs;  // device: ndesc+1 prefix offsets in row-iterations
    int ndesc;
    unsigned long long* work;        // device: guided-scheduling counter (zeroed per launch),
                                     // followed by 4 clock words the kernel fills: s_memtime /
                                     // s_memrealtime of workgroup 0 at its start and its end
    unsigned int gmin, gmax;         // piece size bounds (r values per grab)
    unsigned long long* thresh;      // pruning threshold (monotone atomicMin), per job
    Cand* cands;                     // appended per-workgroup candidates
    unsigned int* ncand;             // append counter
    unsigned long long* dump;        // MODE 1 only: per-nonce hashes
    unsigned long long dump_lo;      // MODE 1 only: nonce of dump[0]
    const uint32_t* ktab;            // C2/J=0 only: per-r K+W tables (see LaunchDesc::tab_off)
    unsigned int grid;               // workgroups (<= resident capacity, see grid_for)
};

// Resident workgroups of 256 threads for the (J, C2, EX, mode) kernel on this device.
unsigned int grid_for(int J, int C2, int EX, int mode, int device);

// One persistent launch of the (J, C2, EX) variant over a.descs[0..ndesc).
hipError_t launch_scan(int J, int C2, int EX, int mode, const ScanArgs& a);
// Fills the uniform K+W table of a C2/J=0 descriptor: tab[64*r + t] = K[t] + W_t(r),
// r in [0, D.R), for block B's words U with the loop digits of r inserted into W_0.
hipError_t launch_ktab(const LaunchDesc* d_desc, uint32_t* tab, uint32_t R, hipStream_t stream);
// Fills the p-tables of ndesc lane-table (C2 = 3) descriptors: for descriptor i and k < R,
// tab[desc.tab_off + 16k ...] = block B-1's chaining value for p = lt_p0 + k, then round 0's
// partial sums inv0, t20 of block B (scan_row_lt).
hipError_t launch_ptab(const LaunchDesc* d_descs, int ndesc, uint32_t* tab, hipStream_t stream);
hipError_t launch_reduce(Cand* cands, unsigned int* ncand, Cand* best, hipStream_t stream);

}  // namespace gpuhash

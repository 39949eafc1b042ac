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
    unsigned long long* thresh;  // pruning threshold (monotone atomicMin), per job
    Cand* cands;                 // appended per-workgroup candidates
    unsigned int* ncand;         // append counter
    unsigned long long* dump;    // MODE 1 only: per-nonce hashes
    unsigned long long dump_lo;  // MODE 1 only: nonce of dump[0]
};

// mode 0 = argmin scan, 1 = per-nonce hash dump
hipError_t launch_scan(const Launch& l, int mode, const ScanArgs& a);
hipError_t launch_reduce(Cand* cands, unsigned int* ncand, Cand* best, hipStream_t stream);

}  // namespace gpuhash

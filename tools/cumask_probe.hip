// cumask_probe.hip -- is gfx950's 4-cycle issue of rotate-bearing VALU streams a pipeline
// property or a power/current limit?  The same streams as
// tools/issue_probe.hip (8 independent chains, 32-instruction bodies, 8 waves per SIMD)
// run on streams restricted by a CU mask to 4, 16, 64 and all CUs.  A power or di/dt limit
// (chip- or XCD-wide) would let a few active CUs issue faster per CU than the whole chip;
// a pipeline property gives the same per-CU rate at every count.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/cumask_probe tools/cumask_probe.hip
//   tools/bin/cumask_probe [iters]      -> one JSON line per (stream, active CUs)
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#define CHK(x)                                                                    \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

// 32 instructions per body on chains %0..%7 (i % 8), %9/%10 loop-invariant VGPRs
#define XOR4 "v_xor_b32 %0, %9, %0\n\tv_xor_b32 %1, %9, %1\n\tv_xor_b32 %2, %9, %2\n\tv_xor_b32 %3, %9, %3\n\t" \
             "v_xor_b32 %4, %9, %4\n\tv_xor_b32 %5, %9, %5\n\tv_xor_b32 %6, %9, %6\n\tv_xor_b32 %7, %9, %7\n\t"
#define ALIGN8 "v_alignbit_b32 %0, %0, %9, 7\n\tv_alignbit_b32 %1, %1, %9, 7\n\tv_alignbit_b32 %2, %2, %9, 7\n\tv_alignbit_b32 %3, %3, %9, 7\n\t" \
               "v_alignbit_b32 %4, %4, %9, 7\n\tv_alignbit_b32 %5, %5, %9, 7\n\tv_alignbit_b32 %6, %6, %9, 7\n\tv_alignbit_b32 %7, %7, %9, 7\n\t"
// SHA-like: per chain 3 rotates, 1 xor3, 1 add3, 1 add (the round's mix), 48 instructions
#define SHA1(c) "v_alignbit_b32 " c ", " c ", %9, 6\n\tv_alignbit_b32 " c ", " c ", %9, 11\n\tv_alignbit_b32 " c ", " c ", %9, 25\n\t" \
                "v_bitop3_b32 " c ", " c ", %9, %10 bitop3:0x96\n\tv_add3_u32 " c ", " c ", %9, %10\n\tv_add_u32 " c ", %9, " c "\n\t"
#define SHA8 SHA1("%0") SHA1("%1") SHA1("%2") SHA1("%3") SHA1("%4") SHA1("%5") SHA1("%6") SHA1("%7")

template <int KIND>
__global__ __launch_bounds__(256) void k_probe(unsigned* out, unsigned long long* clk, int iters) {
    unsigned a = threadIdx.x, b = a * 3u + 1u, c = a * 5u + 2u, d = a * 7u + 3u, e = a * 11u + 4u,
             f = a * 13u + 5u, g = a * 17u + 6u, h = a * 19u + 7u;
    unsigned k1 = threadIdx.x * 2654435761u + 1u, k2 = k1 ^ 0x5bd1e995u;
    unsigned s = __builtin_amdgcn_readfirstlane(k1);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; i++) {
        if constexpr (KIND == 0) {
            asm volatile(XOR4 XOR4 XOR4 XOR4
                         : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h)
                         : "s"(s), "v"(k1), "v"(k2));
        } else if constexpr (KIND == 1) {
            asm volatile(ALIGN8 ALIGN8 ALIGN8 ALIGN8
                         : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h)
                         : "s"(s), "v"(k1), "v"(k2));
        } else {
            asm volatile(SHA8
                         : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h)
                         : "s"(s), "v"(k1), "v"(k2));
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = a ^ b ^ c ^ d ^ e ^ f ^ g ^ h;
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

template <int KIND>
static void run(const char* name, int ninstr, int ncu_active, int cus, int iters) {
    // CU mask: the first ncu_active bits (the hardware's CU numbering; only the count matters)
    std::vector<uint32_t> mask((cus + 31) / 32, 0u);
    for (int i = 0; i < ncu_active; i++) mask[i / 32] |= 1u << (i % 32);
    hipStream_t st;
    CHK(hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data()));
    const int per_cu = 8, blocks = ncu_active * per_cu;  // 8 x 256 threads = 8 waves per SIMD
    unsigned* out;
    unsigned long long* clk;
    CHK(hipMalloc(&out, (size_t)blocks * 256 * 4));
    CHK(hipMalloc(&clk, (size_t)blocks * 16));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k_probe<KIND>, dim3(blocks), dim3(256), 0, st, out, clk, iters / 10);
    CHK(hipStreamSynchronize(st));
    float best = 1e30f;
    for (int rep = 0; rep < 3; rep++) {
        CHK(hipEventRecord(e0, st));
        hipLaunchKernelGGL(k_probe<KIND>, dim3(blocks), dim3(256), 0, st, out, clk, iters);
        CHK(hipGetLastError());
        CHK(hipEventRecord(e1, st));
        CHK(hipEventSynchronize(e1));
        float ms;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
    }
    std::vector<unsigned long long> h((size_t)blocks * 2);
    CHK(hipMemcpy(h.data(), clk, (size_t)blocks * 16, hipMemcpyDeviceToHost));
    double ghz = 0;
    for (int b = 0; b < blocks; b++) ghz += (double)h[2 * b] / (double)h[2 * b + 1] * 0.1;
    ghz /= blocks;
    const double lane_instr = (double)blocks * 256.0 * ninstr * iters;
    printf("{\"stream\": \"%s\", \"active_cus\": %d, \"waves_per_simd\": %d, \"ms\": %.3f, \"clock_ghz\": %.3f, "
           "\"lane_instr_per_active_cu_per_clk\": %.2f}\n",
           name, ncu_active, per_cu, best, ghz, lane_instr / (best * 1e-3) / (ncu_active * ghz * 1e9));
    fflush(stdout);
    CHK(hipFree(out));
    CHK(hipFree(clk));
    CHK(hipEventDestroy(e0));
    CHK(hipEventDestroy(e1));
    CHK(hipStreamDestroy(st));
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 20000;
    hipDeviceProp_t p;
    CHK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    for (int n : {4, 16, 64, cus}) {
        if (n > cus) continue;
        // fewer active CUs -> proportionally fewer blocks: scale iterations so each run is
        // long enough to time
        const int it = n == cus ? iters : iters * 2;
        run<0>("xor x32", 32, n, cus, it);
        run<1>("alignbit x32", 32, n, cus, it);
        run<2>("sha-mix 3 alignbit + xor3 + add3 + add, x8", 48, n, cus, it);
    }
    return 0;
}

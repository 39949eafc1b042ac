// mode_probe.hip -- is the gfx950 "slow VALU" state per wave or per SIMD, and how long
// does it last?  (tools/gen_issue_probe.py showed that one v_alignbit among 7 fast ops
// makes the whole stream run at the 4-cycle rate.)
//
// Kernels (512-thread blocks = 2 waves per SIMD per block, 4 blocks per CU):
//   k_split<M>: waves 0-3 of a block run M-instruction bodies of pure v_xor, waves 4-7 of
//               pure v_alignbit, so every SIMD hosts both kinds; reports each kind's
//               cycles per instruction from its own s_memtime.
//   k_runs<S, F>: every wave runs S alignbit then F xor per iteration (long runs).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1);} } while (0)

#define X8(op) op("v10") op("v11") op("v12") op("v13") op("v14") op("v15") op("v16") op("v17")
#define XOR(r) "v_xor_b32 " r ", v40, " r "\n\t"
#define ALN(r) "v_alignbit_b32 " r ", " r ", v40, 7\n\t"
#define CLOB "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v40"

template <int KIND>  // 0 = xor, 1 = align
__device__ __forceinline__ void body32() {
    if constexpr (KIND == 0) asm volatile(X8(XOR) X8(XOR) X8(XOR) X8(XOR) ::: CLOB);
    else asm volatile(X8(ALN) X8(ALN) X8(ALN) X8(ALN) ::: CLOB);
}

__device__ __forceinline__ void init_regs(unsigned x) {
    asm volatile("v_mov_b32 v10, %0\n\tv_mov_b32 v11, %0\n\tv_mov_b32 v12, %0\n\tv_mov_b32 v13, %0\n\t"
                 "v_mov_b32 v14, %0\n\tv_mov_b32 v15, %0\n\tv_mov_b32 v16, %0\n\tv_mov_b32 v17, %0\n\t"
                 "v_mov_b32 v40, %0" :: "v"(x) : CLOB);
}

// MODE 0: waves 0-3 xor, 4-7 align.  MODE 1: all xor.  MODE 2: all align.
template <int MODE>
__global__ __launch_bounds__(512) void k_split(unsigned long long* cyc, int iters) {
    init_regs(threadIdx.x * 2654435761u);
    const int wave = threadIdx.x >> 6;
    const bool is_xor = MODE == 1 || (MODE == 0 && wave < 4);
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (is_xor) { for (int i = 0; i < iters; i++) body32<0>(); }
    else { for (int i = 0; i < iters; i++) body32<1>(); }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) cyc[(blockIdx.x * 8 + wave) * 2] = t1 - t0, cyc[(blockIdx.x * 8 + wave) * 2 + 1] = is_xor;
}

template <int S, int F>
__global__ __launch_bounds__(512) void k_runs(unsigned long long* cyc, int iters) {
    init_regs(threadIdx.x * 2654435761u);
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int j = 0; j < S / 32; j++) body32<1>();
#pragma unroll
        for (int j = 0; j < F / 32; j++) body32<0>();
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const int wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) cyc[(blockIdx.x * 8 + wave) * 2] = t1 - t0, cyc[(blockIdx.x * 8 + wave) * 2 + 1] = 0;
}

typedef void (*KFn)(unsigned long long*, int);

static void run(KFn k, const char* name, int per_cu, int iters, int instr_per_iter) {
    hipDeviceProp_t p; CHK(hipGetDeviceProperties(&p, 0));
    int cus = p.multiProcessorCount, blocks = cus * per_cu;
    unsigned long long* d; CHK(hipMalloc(&d, (size_t)blocks * 8 * 16));
    hipLaunchKernelGGL(k, dim3(blocks), dim3(512), 0, 0, d, iters / 10);
    CHK(hipDeviceSynchronize());
    hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    CHK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(k, dim3(blocks), dim3(512), 0, 0, d, iters);
    CHK(hipEventRecord(e1, 0)); CHK(hipEventSynchronize(e1));
    float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
    unsigned long long* h = (unsigned long long*)malloc((size_t)blocks * 8 * 16);
    CHK(hipMemcpy(h, d, (size_t)blocks * 8 * 16, hipMemcpyDeviceToHost));
    double cx = 0, ca = 0; long nx = 0, na = 0;
    for (int w = 0; w < blocks * 8; w++) {
        if (h[2 * w + 1]) { cx += (double)h[2 * w]; nx++; } else { ca += (double)h[2 * w]; na++; }
    }
    // cycles per instruction of ONE wave (s_memtime counts shader clocks)
    double total = (double)iters * instr_per_iter;
    printf("{\"probe\": \"%s\", \"ms\": %.3f, \"xor_wave_cyc_per_instr\": %.2f, \"other_wave_cyc_per_instr\": %.2f}\n",
           name, ms, nx ? cx / nx / total : 0.0, na ? ca / na / total : 0.0);
    fflush(stdout);
    free(h); CHK(hipFree(d)); CHK(hipEventDestroy(e0)); CHK(hipEventDestroy(e1));
}

int main(int argc, char** argv) {
    int per_cu = argc > 1 ? atoi(argv[1]) : 4, iters = argc > 2 ? atoi(argv[2]) : 20000;
    run(k_split<1>, "all xor", per_cu, iters, 32);
    run(k_split<2>, "all align", per_cu, iters, 32);
    run(k_split<0>, "split: waves 0-3 xor, 4-7 align", per_cu, iters, 32);
    run(k_runs<32, 32>, "runs 32 align + 32 xor", per_cu, iters / 2, 64);
    run(k_runs<32, 96>, "runs 32 align + 96 xor", per_cu, iters / 4, 128);
    run(k_runs<32, 224>, "runs 32 align + 224 xor", per_cu, iters / 8, 256);
    run(k_runs<64, 448>, "runs 64 align + 448 xor", per_cu, iters / 16, 512);
    return 0;
}

// valu_peak.hip -- measures the gfx950 int32 VALU issue rate for the instructions the
// SHA-256 scan kernel is made of, so the roofline peak used by bench.py is a measured
// number, not a datasheet guess.
//
//   ./valu_peak [blocks_per_cu] [iters]
// prints one JSON line per instruction kind: lane-ops/s, lane-ops per CU per clock, and
// the in-kernel shader clock (s_memtime / s_memrealtime).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x)                                                                        \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } \
    } while (0)

// 8 independent chains x 4 instructions = 32 VALU per iteration.
#define S_ALIGN(r) "v_alignbit_b32 " r ", " r ", " r ", 7\n\t"
#define S_BITOP3(r) "v_bitop3_b32 " r ", " r ", %8, " r " bitop3:0x96\n\t"
#define S_ADD3(r) "v_add3_u32 " r ", " r ", %8, " r "\n\t"
#define S_ADD(r) "v_add_u32 " r ", %8, " r "\n\t"
#define S_LSHR(r) "v_lshrrev_b32 " r ", 3, " r "\n\t"
#define S_XOR(r) "v_xor_b32 " r ", %8, " r "\n\t"
#define S_MIX(r) S_ALIGN(r) S_BITOP3(r) S_ADD3(r) S_ADD(r)
#define X4(S, r) S(r) S(r) S(r) S(r)
#define BODY(S) X4(S, "%0") X4(S, "%1") X4(S, "%2") X4(S, "%3") X4(S, "%4") X4(S, "%5") X4(S, "%6") X4(S, "%7")
#define BODY_MIX S_MIX("%0") S_MIX("%1") S_MIX("%2") S_MIX("%3") S_MIX("%4") S_MIX("%5") S_MIX("%6") S_MIX("%7")

template <int KIND>
__global__ __launch_bounds__(256) void k_valu(unsigned* out, unsigned long long* clk, int iters, unsigned seed) {
    unsigned a = threadIdx.x ^ seed, b = a * 3u, c = a * 5u, d = a * 7u, e = a * 11u, f = a * 13u,
             g = a * 17u, h = a * 19u;
    unsigned s = __builtin_amdgcn_readfirstlane(seed | 1u);
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; i++) {
#define ASM(B) asm volatile(B : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h) : "s"(s))
        if constexpr (KIND == 0) ASM(BODY_MIX);
        if constexpr (KIND == 1) ASM(BODY(S_ALIGN));
        if constexpr (KIND == 2) ASM(BODY(S_BITOP3));
        if constexpr (KIND == 3) ASM(BODY(S_ADD3));
        if constexpr (KIND == 4) ASM(BODY(S_ADD));
        if constexpr (KIND == 5) ASM(BODY(S_LSHR));
        if constexpr (KIND == 6) ASM(BODY(S_XOR));
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = a ^ b ^ c ^ d ^ e ^ f ^ g ^ h;
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

static const char* kNames[] = {"mix(alignbit,bitop3,add3,add)", "v_alignbit_b32", "v_bitop3_b32",
                               "v_add3_u32", "v_add_u32", "v_lshrrev_b32", "v_xor_b32"};

template <int KIND>
static void run(int per_cu, int iters) {
    hipDeviceProp_t p;
    CHK(hipGetDeviceProperties(&p, 0));
    int cus = p.multiProcessorCount;
    int blocks = cus * per_cu;
    unsigned* out;
    unsigned long long* clk;
    CHK(hipMalloc(&out, (size_t)blocks * 256 * 4));
    CHK(hipMalloc(&clk, (size_t)blocks * 16));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k_valu<KIND>, dim3(blocks), dim3(256), 0, 0, out, clk, iters / 10, 1u);
    CHK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 3; rep++) {
        CHK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(k_valu<KIND>, dim3(blocks), dim3(256), 0, 0, out, clk, iters, 2u + rep);
        CHK(hipEventRecord(e1, 0));
        CHK(hipEventSynchronize(e1));
        float ms;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
    }
    unsigned long long* h = (unsigned long long*)malloc((size_t)blocks * 16);
    CHK(hipMemcpy(h, clk, (size_t)blocks * 16, hipMemcpyDeviceToHost));
    double ghz = 0;
    for (int b = 0; b < blocks; b++) ghz += (double)h[2 * b] / (double)h[2 * b + 1] * 0.1;  // 100 MHz RTC
    ghz /= blocks;
    double ops = (double)blocks * 256.0 * 32.0 * (double)iters;
    double rate = ops / (best * 1e-3);
    printf("{\"kind\": \"%s\", \"cus\": %d, \"blocks_per_cu\": %d, \"ms\": %.3f, \"lane_ops_per_s\": %.4e, "
           "\"clock_ghz\": %.3f, \"lane_ops_per_cu_per_clk\": %.2f}\n",
           kNames[KIND], cus, per_cu, best, rate, ghz, rate / (cus * ghz * 1e9));
    fflush(stdout);
    free(h);
    CHK(hipFree(out));
    CHK(hipFree(clk));
}

int main(int argc, char** argv) {
    int per_cu = argc > 1 ? atoi(argv[1]) : 8;
    int iters = argc > 2 ? atoi(argv[2]) : 100000;
    run<0>(per_cu, iters);
    run<1>(per_cu, iters);
    run<2>(per_cu, iters);
    run<3>(per_cu, iters);
    run<4>(per_cu, iters);
    run<5>(per_cu, iters);
    run<6>(per_cu, iters);
    return 0;
}

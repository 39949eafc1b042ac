// valu_peak.hip -- measures the gfx950 int32 VALU issue rate for the instructions the
// SHA-256 scan kernel is made of (v_alignbit_b32, v_bitop3_b32, v_add3_u32, v_add_u32),
// so the roofline peak in bench.py is a measured number, not a datasheet guess.
//
//   ./valu_peak [blocks_per_cu] [iters]
// prints one JSON line: lane-ops/s, per-CU lane-ops per clock, in-kernel clock (GHz).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x)                                                                        \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } \
    } while (0)

// 8 independent chains x 4 instruction kinds = 32 VALU per iteration.
#define STEP(r)                                   \
    "v_alignbit_b32 " r ", " r ", " r ", 7\n\t"   \
    "v_bitop3_b32 " r ", " r ", %8, " r " bitop3:0x96\n\t" \
    "v_add3_u32 " r ", " r ", %8, " r "\n\t"      \
    "v_add_u32 " r ", " r ", %8\n\t"

__global__ __launch_bounds__(256) void k_valu(unsigned* out, unsigned long long* clk, int iters, unsigned seed) {
    unsigned a = threadIdx.x ^ seed, b = a * 3u, c = a * 5u, d = a * 7u, e = a * 11u, f = a * 13u,
             g = a * 17u, h = a * 19u;
    unsigned s = seed | 1u;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; i++) {
        asm volatile(STEP("%0") STEP("%1") STEP("%2") STEP("%3") STEP("%4") STEP("%5") STEP("%6") STEP("%7")
                     : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h)
                     : "s"(s));
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = a ^ b ^ c ^ d ^ e ^ f ^ g ^ h;
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

int main(int argc, char** argv) {
    int per_cu = argc > 1 ? atoi(argv[1]) : 8;
    int iters = argc > 2 ? atoi(argv[2]) : 200000;
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
    hipLaunchKernelGGL(k_valu, dim3(blocks), dim3(256), 0, 0, out, clk, iters / 10, 1u);  // warm
    CHK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 3; rep++) {
        CHK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(k_valu, dim3(blocks), dim3(256), 0, 0, out, clk, iters, 2u + rep);
        CHK(hipEventRecord(e1, 0));
        CHK(hipEventSynchronize(e1));
        float ms;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
    }
    unsigned long long* h = (unsigned long long*)malloc((size_t)blocks * 16);
    CHK(hipMemcpy(h, clk, (size_t)blocks * 16, hipMemcpyDeviceToHost));
    double ghz = 0;
    for (int b = 0; b < blocks; b++) ghz += (double)h[2 * b] / (double)h[2 * b + 1] * 0.1;  // memrealtime = 100 MHz
    ghz /= blocks;
    double ops = (double)blocks * 256.0 * 32.0 * (double)iters;  // lane-ops
    double rate = ops / (best * 1e-3);
    printf("{\"cus\": %d, \"blocks_per_cu\": %d, \"iters\": %d, \"ms\": %.3f, \"lane_ops_per_s\": %.4e, "
           "\"clock_ghz\": %.3f, \"lane_ops_per_cu_per_clk\": %.2f, \"peak_at_2p4ghz_T\": %.2f}\n",
           cus, per_cu, iters, best, rate, ghz, rate / (cus * ghz * 1e9), rate / (cus * ghz * 1e9) * cus * 2.4e9 / 1e12);
    return 0;
}

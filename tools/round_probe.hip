// round_probe.hip -- does the ORDER of a SHA-256 round's instructions change the gfx950
// VALU rate?  (issue probes: one v_alignbit among fast ops drags them to the 4-cycle rate;
// fast ops are v_add/v_xor and v_bitop3 when it alternates with 2-operand ops.)
//
// Each kernel runs B independent nonces per lane through 64 rounds (K as literals, W
// folded, like the uniform-schedule layouts) and reports nonce-rounds per clock per CU.
//   ORDER 0: C++ round (compiler schedules; v_add3/v_bitop3 as in scan_kernel.h)
//   ORDER 1: asm, one nonce after another, the compiler's instruction set (6 alignbit,
//            4 bitop3, 2 add3, 2 add), natural order
//   ORDER 2: asm, clustered: all 6*B alignbits first, then per nonce 10 fast ops
//            alternating bitop3 / v_add_u32 (no add3)
//   ORDER 3: asm, clustered like 2 but the fast block keeps the 4 bitop3 together
//   ORDER 4: asm, per nonce [6 alignbit][10 fast alternating] (clusters of one nonce)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1);} } while (0)

__device__ constexpr uint32_t KC[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

#define ALN(d, s, n) asm volatile("v_alignbit_b32 %0, %1, %1, " #n : "=v"(d) : "v"(s))
#define BOP(d, a, b, c, imm) asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:" #imm : "=v"(d) : "v"(a), "v"(b), "v"(c))
#define ADD(d, a, b) asm volatile("v_add_u32 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b))
#define ADDK(d, a, k) asm volatile("v_add_u32 %0, %1, %2" : "=v"(d) : "i"(k), "v"(a))
#define ADD3(d, a, b, c) asm volatile("v_add3_u32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c))
#define ADD3K(d, a, b, k) asm volatile("v_add3_u32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "s"(k))

struct St { uint32_t a, b, c, d, e, f, g, h; };

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }

__device__ __forceinline__ void shift(St& s, uint32_t e2, uint32_t a2) {
    s.h = s.g; s.g = s.f; s.f = s.e; s.e = e2;
    s.d = s.c; s.c = s.b; s.b = s.a; s.a = a2;
}

template <int B, int ORDER, int T>
__device__ __forceinline__ void round_b(St (&s)[B]) {
    constexpr uint32_t k = KC[T];
    if constexpr (ORDER == 0) {
#pragma unroll
        for (int i = 0; i < B; i++) {
            uint32_t t1 = s[i].h + k + __builtin_amdgcn_bitop3_b32(s[i].e, s[i].f, s[i].g, 0xCA) +
                          xor3(rotr(s[i].e, 6), rotr(s[i].e, 11), rotr(s[i].e, 25));
            uint32_t t2 = xor3(rotr(s[i].a, 2), rotr(s[i].a, 13), rotr(s[i].a, 22)) +
                          __builtin_amdgcn_bitop3_b32(s[i].a, s[i].b, s[i].c, 0xE8);
            shift(s[i], s[i].d + t1, t1 + t2);
        }
    } else if constexpr (ORDER == 1) {
#pragma unroll
        for (int i = 0; i < B; i++) {
            uint32_t r0, r1, r2, r3, r4, r5, S1, S0, CH, MJ, t, e2, a2;
            ALN(r0, s[i].e, 6); ALN(r1, s[i].e, 11); ALN(r2, s[i].e, 25);
            BOP(S1, r0, r1, r2, 0x96);
            BOP(CH, s[i].e, s[i].f, s[i].g, 0xCA);
            ADDK(t, s[i].h, k);
            ADD3(t, t, CH, S1);
            ALN(r3, s[i].a, 2); ALN(r4, s[i].a, 13); ALN(r5, s[i].a, 22);
            BOP(S0, r3, r4, r5, 0x96);
            BOP(MJ, s[i].a, s[i].b, s[i].c, 0xE8);
            ADD(e2, s[i].d, t);
            ADD3(a2, t, S0, MJ);
            shift(s[i], e2, a2);
        }
    } else {
        uint32_t r[B][6];
        if constexpr (ORDER == 4) {
#pragma unroll
            for (int i = 0; i < B; i++) {
                ALN(r[i][0], s[i].e, 6); ALN(r[i][1], s[i].e, 11); ALN(r[i][2], s[i].e, 25);
                ALN(r[i][3], s[i].a, 2); ALN(r[i][4], s[i].a, 13); ALN(r[i][5], s[i].a, 22);
                uint32_t S1, S0, CH, MJ, t, e2, a2;
                ADDK(t, s[i].h, k);
                BOP(S1, r[i][0], r[i][1], r[i][2], 0x96);
                ADD(t, t, S1);
                BOP(CH, s[i].e, s[i].f, s[i].g, 0xCA);
                ADD(t, t, CH);
                BOP(S0, r[i][3], r[i][4], r[i][5], 0x96);
                ADD(e2, s[i].d, t);
                BOP(MJ, s[i].a, s[i].b, s[i].c, 0xE8);
                ADD(a2, t, S0);
                ADD(a2, a2, MJ);
                shift(s[i], e2, a2);
            }
        } else {
#pragma unroll
            for (int i = 0; i < B; i++) {
                ALN(r[i][0], s[i].e, 6); ALN(r[i][1], s[i].e, 11); ALN(r[i][2], s[i].e, 25);
                ALN(r[i][3], s[i].a, 2); ALN(r[i][4], s[i].a, 13); ALN(r[i][5], s[i].a, 22);
            }
#pragma unroll
            for (int i = 0; i < B; i++) {
                uint32_t S1, S0, CH, MJ, t, e2, a2;
                if constexpr (ORDER == 2) {
                    ADDK(t, s[i].h, k);
                    BOP(S1, r[i][0], r[i][1], r[i][2], 0x96);
                    ADD(t, t, S1);
                    BOP(CH, s[i].e, s[i].f, s[i].g, 0xCA);
                    ADD(t, t, CH);
                    BOP(S0, r[i][3], r[i][4], r[i][5], 0x96);
                    ADD(e2, s[i].d, t);
                    BOP(MJ, s[i].a, s[i].b, s[i].c, 0xE8);
                    ADD(a2, t, S0);
                    ADD(a2, a2, MJ);
                } else {
                    BOP(S1, r[i][0], r[i][1], r[i][2], 0x96);
                    BOP(CH, s[i].e, s[i].f, s[i].g, 0xCA);
                    BOP(S0, r[i][3], r[i][4], r[i][5], 0x96);
                    BOP(MJ, s[i].a, s[i].b, s[i].c, 0xE8);
                    ADDK(t, s[i].h, k);
                    ADD(t, t, S1);
                    ADD(t, t, CH);
                    ADD(e2, s[i].d, t);
                    ADD(a2, t, S0);
                    ADD(a2, a2, MJ);
                }
                shift(s[i], e2, a2);
            }
        }
    }
}

template <int B, int ORDER, int T0, int T1>
__device__ __forceinline__ void rounds(St (&s)[B]) {
    if constexpr (T0 < T1) {
        round_b<B, ORDER, T0>(s);
        rounds<B, ORDER, T0 + 1, T1>(s);
    }
}

template <int B, int ORDER>
__global__ __launch_bounds__(256) void k_rounds(uint32_t* out, unsigned long long* clk, int iters, uint32_t seed) {
    St s[B];
#pragma unroll
    for (int i = 0; i < B; i++) {
        uint32_t x = (blockIdx.x * 256u + threadIdx.x) * 2654435761u ^ seed ^ (i * 0x9e3779b9u);
        s[i] = St{x, x * 3u + 1u, x * 5u + 2u, x * 7u + 3u, x * 11u + 4u, x * 13u + 5u, x * 17u + 6u, x * 19u + 7u};
    }
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; it++) rounds<B, ORDER, 0, 64>(s);
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < B; i++) acc ^= s[i].a ^ s[i].e;
    out[blockIdx.x * 256u + threadIdx.x] = acc;
    if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}

typedef void (*KFn)(uint32_t*, unsigned long long*, int, uint32_t);

static void run(KFn k, const char* name, int B, int per_cu, int iters) {
    hipDeviceProp_t p; CHK(hipGetDeviceProperties(&p, 0));
    int cus = p.multiProcessorCount, blocks = cus * per_cu;
    uint32_t* out; unsigned long long* clk;
    CHK(hipMalloc(&out, (size_t)blocks * 256 * 4)); CHK(hipMalloc(&clk, (size_t)blocks * 16));
    hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, clk, iters / 10 + 1, 1u);
    CHK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 3; rep++) {
        CHK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, clk, iters, 2u + rep);
        CHK(hipEventRecord(e1, 0)); CHK(hipEventSynchronize(e1));
        float ms; CHK(hipEventElapsedTime(&ms, e0, e1)); if (ms < best) best = ms;
    }
    unsigned long long* h = (unsigned long long*)malloc((size_t)blocks * 16);
    CHK(hipMemcpy(h, clk, (size_t)blocks * 16, hipMemcpyDeviceToHost));
    double ghz = 0; for (int b = 0; b < blocks; b++) ghz += (double)h[2*b] / (double)h[2*b+1] * 0.1; ghz /= blocks;
    double nonce_rounds = (double)blocks * 256.0 * B * 64.0 * iters;
    double per_clk_cu = nonce_rounds / (best * 1e-3) / (cus * ghz * 1e9);
    // 64 rounds per nonce -> GH/s if a nonce were rounds only
    printf("{\"kernel\": \"%s\", \"B\": %d, \"blocks_per_cu\": %d, \"ms\": %.3f, \"clock_ghz\": %.3f, "
           "\"nonce_rounds_per_clk_cu\": %.3f, \"simd_cycles_per_round\": %.2f, \"GHs_64rounds\": %.2f}\n",
           name, B, per_cu, best, ghz, per_clk_cu, 4.0 * 64.0 / per_clk_cu, nonce_rounds / 64.0 / (best * 1e-3) / 1e9);
    fflush(stdout); free(h); CHK(hipFree(out)); CHK(hipFree(clk)); CHK(hipEventDestroy(e0)); CHK(hipEventDestroy(e1));
}

int main(int argc, char** argv) {
    int iters = argc > 1 ? atoi(argv[1]) : 2000;
    for (int per_cu : {8, 4}) {
        run(k_rounds<1, 0>, "cxx", 1, per_cu, iters);
        run(k_rounds<2, 0>, "cxx", 2, per_cu, iters / 2);
        run(k_rounds<1, 1>, "asm natural", 1, per_cu, iters);
        run(k_rounds<1, 4>, "asm per-nonce clusters", 1, per_cu, iters);
        run(k_rounds<2, 4>, "asm per-nonce clusters", 2, per_cu, iters / 2);
        run(k_rounds<2, 2>, "asm clustered alt", 2, per_cu, iters / 2);
        run(k_rounds<4, 2>, "asm clustered alt", 4, per_cu, iters / 4);
        run(k_rounds<2, 3>, "asm clustered grouped", 2, per_cu, iters / 2);
        run(k_rounds<4, 3>, "asm clustered grouped", 4, per_cu, iters / 4);
    }
    return 0;
}

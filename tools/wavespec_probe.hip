// wavespec_probe.hip -- does splitting SHA-256 across two specialised waves beat one wave
// doing all of it on gfx950?  (build the wave-specialised variant
// instead of costing it.)
//
// Background: v_alignbit_b32 (the only one-instruction rotate) and
// v_add3_u32 issue at the 4-cycle wave64 rate, and a wave whose stream contains them runs
// its 2-cycle instructions (v_xor, v_add_u32, v_lshrrev, ...) at 4 cycles too; pure-xor
// and pure-alignbit waves sharing a SIMD partly overlap (tools/mode_probe.hip).  So: put
// the rotates in one wave, the adds and boolean functions in another, exchange through
// LDS every round.
//
// Both kernels compute the same thing: for every nonce n in [0, N) one generic SHA-256
// compression of the block W_i = n ^ C_i (all 16 words per-nonce, so nothing folds),
// from the IV, all 64 rounds and 48 schedule words; per lane the least (H0 << 32 | H1)
// and a checksum (sum of H0 ^ H1) -- the host compares both kernels with a CPU
// restatement on a small N, then times them on a large one.
//
//   k_base      256-thread workgroups, one nonce per lane per iteration: the production
//               kernel's instruction forms (alignbit rotates, bitop3 xor3/ch/maj, add3).
//   k_spec<P>   128-thread workgroups = one wave pair.  Wave R (rotates): Sigma0(a),
//               Sigma1(e), sigma0(W_t-15), sigma1(W_t-2) -- alignbit + bitop3 + lshr only.
//               Wave F (the rest): Ch, Maj, the schedule sums and every round addition,
//               as two-input v_add_u32 (2-cycle class).  Per round F sends (a, e, W_t)
//               and R sends (S0, S1, s0, s1) through LDS.  2P nonces per lane are in
//               flight in two groups, software-pipelined: in step s, R works on group
//               s & 1 while F works on the other group, one barrier per step (129 steps
//               per 2P nonces), so neither wave waits on the other's latency within a step.
//
//   wavespec_probe <N_log2> [iters_check]   -> one JSON line per kernel
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <type_traits>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1);} } while (0)

static const uint32_t hK[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};
static const uint32_t hIV[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                                0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};

__device__ constexpr uint32_t K[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};
__device__ constexpr uint32_t IV[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                                       0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
// per-word message constants: W_i = n ^ MC(i)
__host__ __device__ constexpr uint32_t MC(int i) { return 0x9e3779b9u * (uint32_t)(2 * i + 1); }

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }
__device__ __forceinline__ uint32_t ch(uint32_t e, uint32_t f, uint32_t g) { return __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA); }
__device__ __forceinline__ uint32_t maj(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8); }
__device__ __forceinline__ uint32_t bS0(uint32_t a) { return xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22)); }
__device__ __forceinline__ uint32_t bS1(uint32_t e) { return xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25)); }
__device__ __forceinline__ uint32_t bs0(uint32_t x) { return xor3(rotr(x, 7), rotr(x, 18), x >> 3); }
__device__ __forceinline__ uint32_t bs1(uint32_t x) { return xor3(rotr(x, 17), rotr(x, 19), x >> 10); }
// two-input add, kept as such (the compiler would otherwise fuse pairs into v_add3_u32)
__device__ __forceinline__ uint32_t add2(uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_add_u32_e32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

template <int B, int E, class F>
__device__ __forceinline__ void sfor(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        sfor<B + 1, E>(f);
    }
}

struct Acc {
    unsigned long long best, sum;
};
__device__ __forceinline__ void acc_add(Acc& A, uint32_t H0, uint32_t H1) {
    const unsigned long long h = ((unsigned long long)H0 << 32) | H1;
    A.best = h < A.best ? h : A.best;
    A.sum += (unsigned long long)(H0 ^ H1);
}

// ---------------------------------------------------------------- baseline: one wave
__global__ __launch_bounds__(256) void k_base(unsigned long long* out, uint32_t iters) {
    const uint32_t gid = blockIdx.x * 256u + threadIdx.x;
    Acc A{~0ull, 0ull};
#pragma unroll 1
    for (uint32_t it = 0; it < iters; it++) {
        const uint32_t n = gid * iters + it;
        uint32_t w[16];
#pragma unroll
        for (int i = 0; i < 16; i++) w[i] = n ^ MC(i);
        uint32_t a = IV[0], b = IV[1], c = IV[2], d = IV[3], e = IV[4], f = IV[5], g = IV[6], h = IV[7];
        sfor<0, 64>([&](auto tc) {
            constexpr int t = decltype(tc)::value;
            if constexpr (t >= 16)
                w[t & 15] = w[t & 15] + bs0(w[(t - 15) & 15]) + w[(t - 7) & 15] + bs1(w[(t - 2) & 15]);
            const uint32_t t1 = h + (K[t] + w[t & 15]) + ch(e, f, g) + bS1(e);
            const uint32_t t2 = bS0(a) + maj(a, b, c);
            h = g; g = f; f = e; e = d + t1;
            d = c; c = b; b = a; a = t1 + t2;
        });
        acc_add(A, IV[0] + a, IV[1] + b);
    }
    out[2 * gid] = A.best;
    out[2 * gid + 1] = A.sum;
}

// ---------------------------------------------------------------- specialised wave pair
template <int P>
struct Lds {
    uint32_t toR[2][P][3][64];  // F -> R: a, e, W_t
    uint32_t toF[2][P][4][64];  // R -> F: S0, S1, s0, s1
};

template <int P>
__global__ __launch_bounds__(128) void k_spec(unsigned long long* out, uint32_t iters) {
    __shared__ Lds<P> L;
    const uint32_t lane = threadIdx.x & 63u;
    const bool isF = threadIdx.x < 64u;  // wave 0 = F, wave 1 = R (wave-uniform)
    const uint32_t gl = blockIdx.x * 64u + lane;  // global lane; 2P nonces per iteration
    Acc A{~0ull, 0ull};
#pragma unroll 1
    for (uint32_t it = 0; it < iters; it++) {
        // nonce of group g, slot p
        auto nonce = [&](int g, int p) { return (gl * iters + it) * (2u * P) + (uint32_t)(g * P + p); };
        if (isF) {
            uint32_t st[2][P][8], w[2][P][16];
#pragma unroll
            for (int g = 0; g < 2; g++)
#pragma unroll
                for (int p = 0; p < P; p++) {
#pragma unroll
                    for (int i = 0; i < 8; i++) st[g][p][i] = IV[i];
#pragma unroll
                    for (int i = 0; i < 16; i++) w[g][p][i] = nonce(g, p) ^ MC(i);
                }
            // step s: F runs round t = (s - 1) >> 1 of group (s + 1) & 1
            sfor<0, 129>([&](auto sc) {
                constexpr int s = decltype(sc)::value;
                if constexpr (s >= 1) {
                    constexpr int g = (s + 1) & 1, t = (s - 1) >> 1;
#pragma unroll
                    for (int p = 0; p < P; p++) {
                        uint32_t* x = st[g][p];
                        uint32_t* W = w[g][p];
                        const uint32_t S0 = L.toF[g][p][0][lane], S1 = L.toF[g][p][1][lane];
                        if constexpr (t >= 16) {
                            const uint32_t s0 = L.toF[g][p][2][lane], s1 = L.toF[g][p][3][lane];
                            W[t & 15] = add2(add2(W[t & 15], s0), add2(W[(t - 7) & 15], s1));
                        }
                        const uint32_t kw = W[t & 15] + K[t];  // VOP2 with a literal
                        const uint32_t t1 = add2(add2(x[7], kw), add2(ch(x[4], x[5], x[6]), S1));
                        const uint32_t na = add2(t1, add2(S0, maj(x[0], x[1], x[2])));
                        const uint32_t ne = add2(x[3], t1);
                        x[7] = x[6]; x[6] = x[5]; x[5] = x[4]; x[4] = ne;
                        x[3] = x[2]; x[2] = x[1]; x[1] = x[0]; x[0] = na;
                        if constexpr (t < 63) {
                            L.toR[g][p][0][lane] = na;
                            L.toR[g][p][1][lane] = ne;
                            if constexpr (t >= 16) L.toR[g][p][2][lane] = W[t & 15];
                        }
                    }
                }
                __syncthreads();
            });
#pragma unroll
            for (int g = 0; g < 2; g++)
#pragma unroll
                for (int p = 0; p < P; p++) acc_add(A, IV[0] + st[g][p][0], IV[1] + st[g][p][1]);
        } else {
            uint32_t w[2][P][16];
#pragma unroll
            for (int g = 0; g < 2; g++)
#pragma unroll
                for (int p = 0; p < P; p++)
#pragma unroll
                    for (int i = 0; i < 16; i++) w[g][p][i] = nonce(g, p) ^ MC(i);
            // step s: R runs round t = s >> 1 of group s & 1
            sfor<0, 129>([&](auto sc) {
                constexpr int s = decltype(sc)::value;
                if constexpr ((s >> 1) < 64) {
                    constexpr int g = s & 1, t = s >> 1;
#pragma unroll
                    for (int p = 0; p < P; p++) {
                        uint32_t* W = w[g][p];
                        uint32_t a, e;
                        if constexpr (t == 0) {
                            a = IV[0]; e = IV[4];
                        } else {
                            a = L.toR[g][p][0][lane]; e = L.toR[g][p][1][lane];
                            if constexpr (t - 1 >= 16) W[(t - 1) & 15] = L.toR[g][p][2][lane];
                        }
                        L.toF[g][p][0][lane] = bS0(a);
                        L.toF[g][p][1][lane] = bS1(e);
                        if constexpr (t >= 16) {
                            L.toF[g][p][2][lane] = bs0(W[(t - 15) & 15]);
                            L.toF[g][p][3][lane] = bs1(W[(t - 2) & 15]);
                        }
                    }
                }
                __syncthreads();
            });
        }
    }
    if (isF) {
        out[2 * gl] = A.best;
        out[2 * gl + 1] = A.sum;
    }
}

// ---------------------------------------------------------------- host
static void cpu_ref(uint64_t N, unsigned long long* best, unsigned long long* sum) {
    *best = ~0ull;
    *sum = 0;
    for (uint64_t n = 0; n < N; n++) {
        uint32_t w[64];
        for (int i = 0; i < 16; i++) w[i] = (uint32_t)n ^ MC(i);
        auto ror = [](uint32_t x, int k) { return (x >> k) | (x << (32 - k)); };
        for (int t = 16; t < 64; t++)
            w[t] = w[t - 16] + (ror(w[t - 15], 7) ^ ror(w[t - 15], 18) ^ (w[t - 15] >> 3)) + w[t - 7] +
                   (ror(w[t - 2], 17) ^ ror(w[t - 2], 19) ^ (w[t - 2] >> 10));
        uint32_t a = hIV[0], b = hIV[1], c = hIV[2], d = hIV[3], e = hIV[4], f = hIV[5], g = hIV[6], h = hIV[7];
        for (int t = 0; t < 64; t++) {
            uint32_t t1 = h + (ror(e, 6) ^ ror(e, 11) ^ ror(e, 25)) + ((e & f) ^ (~e & g)) + hK[t] + w[t];
            uint32_t t2 = (ror(a, 2) ^ ror(a, 13) ^ ror(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
            h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
        }
        uint32_t H0 = hIV[0] + a, H1 = hIV[1] + b;
        unsigned long long v = ((unsigned long long)H0 << 32) | H1;
        if (v < *best) *best = v;
        *sum += (unsigned long long)(H0 ^ H1);
    }
}

template <class Launch>
static void run(const char* name, uint64_t lanes, uint32_t iters, uint64_t nonces, int reps, Launch launch,
                bool check, unsigned long long want_best, unsigned long long want_sum) {
    unsigned long long* d;
    CHK(hipMalloc(&d, lanes * 16));
    launch(d, iters);  // warm-up
    CHK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    CHK(hipEventRecord(e0, 0));
    for (int r = 0; r < reps; r++) launch(d, iters);
    CHK(hipEventRecord(e1, 0));
    CHK(hipEventSynchronize(e1));
    float ms;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    unsigned long long* h = (unsigned long long*)malloc(lanes * 16);
    CHK(hipMemcpy(h, d, lanes * 16, hipMemcpyDeviceToHost));
    unsigned long long best = ~0ull, sum = 0;
    for (uint64_t i = 0; i < lanes; i++) {
        best = h[2 * i] < best ? h[2 * i] : best;
        sum += h[2 * i + 1];
    }
    const double ghs = (double)nonces * reps / (ms * 1e-3) / 1e9;
    printf("{\"kernel\": \"%s\", \"nonces\": %llu, \"ms_per_launch\": %.3f, \"GHs\": %.3f, \"best\": %llu, "
           "\"checksum\": %llu, \"check\": %s}\n",
           name, (unsigned long long)nonces, ms / reps, ghs, best, sum,
           check ? ((best == want_best && sum == want_sum) ? "\"ok\"" : "\"MISMATCH\"") : "null");
    fflush(stdout);
    free(h);
    CHK(hipFree(d));
    CHK(hipEventDestroy(e0));
    CHK(hipEventDestroy(e1));
}

int main(int argc, char** argv) {
    const int lg = argc > 1 ? atoi(argv[1]) : 32;  // log2 nonces of the timed runs
    const int reps = argc > 2 ? atoi(argv[2]) : 3;
    // correctness: 2^20 nonces against the CPU restatement
    {
        const uint64_t N = 1ull << 20;
        unsigned long long wb, ws;
        cpu_ref(N, &wb, &ws);
        const uint32_t it = 16;
        run("k_base", N / it, it, N, 1, [&](unsigned long long* d, uint32_t i) {
            k_base<<<(unsigned)(N / it / 256), 256>>>(d, i); }, true, wb, ws);
        run("k_spec<1>", N / it / 2, it, N, 1, [&](unsigned long long* d, uint32_t i) {
            k_spec<1><<<(unsigned)(N / it / 2 / 64), 128>>>(d, i); }, true, wb, ws);
        run("k_spec<2>", N / it / 4, it, N, 1, [&](unsigned long long* d, uint32_t i) {
            k_spec<2><<<(unsigned)(N / it / 4 / 64), 128>>>(d, i); }, true, wb, ws);
    }
    const uint64_t N = 1ull << lg;
    const uint32_t it = 256;
    run("k_base", N / it, it, N, reps, [&](unsigned long long* d, uint32_t i) {
        k_base<<<(unsigned)(N / it / 256), 256>>>(d, i); }, false, 0, 0);
    run("k_spec<1>", N / it / 2, it, N, reps, [&](unsigned long long* d, uint32_t i) {
        k_spec<1><<<(unsigned)(N / it / 2 / 64), 128>>>(d, i); }, false, 0, 0);
    run("k_spec<2>", N / it / 4, it, N, reps, [&](unsigned long long* d, uint32_t i) {
        k_spec<2><<<(unsigned)(N / it / 4 / 64), 128>>>(d, i); }, false, 0, 0);
    return 0;
}

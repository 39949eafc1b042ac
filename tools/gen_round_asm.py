#!/usr/bin/env python3
"""Generates tools/round_asm.hip: SHA-256 rounds in hand-placed gfx950 asm (fixed VGPRs,
no compiler scheduling or hazard nops), B independent nonces per lane, to measure how the
ORDER of a round's instructions sets the VALU rate.

Per round and nonce the work is the same (6 v_alignbit; Sigma0/Sigma1/Ch/Maj as 4
v_bitop3; the adds either as the compiler emits them -- 2 v_add3 + 2 v_add -- or as 6
2-operand v_add_u32), only the order and the add forms differ:

  nat    per nonce: rot(e) x3, S1, Ch, t=h+Ch, t=add3(t,S1,K), rot(a) x3, S0, Maj,
         e'=d+t, a'=add3(Maj,t,S0)                        (the compiler's stream)
  clu    all 6B alignbits, then per nonce 10 fast ops alternating bitop3 / v_add_u32
  clu3   all 6B alignbits, then per nonce the 4 bitop3 + 2 add3 + 2 add (no split adds)
  pn     per nonce: 6 alignbits then its 10 fast ops (clusters of one nonce)
K comes from an SGPR (`s`, the uniform-schedule layouts' table) or a literal (`l`).
"""
import os

K = [0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5]
BASE = 8  # first VGPR we own


def gen_body(B, order, kform):
    # registers: state 8 per nonce, rot 6 per nonce, t 1 per nonce
    st = [[BASE + 15 * i + j for j in range(8)] for i in range(B)]
    rot = [[BASE + 15 * i + 8 + j for j in range(6)] for i in range(B)]
    tt = [BASE + 15 * i + 14 for i in range(B)]
    lines = []
    v = lambda r: f"v{r}"

    def kop(rnd):
        return f"s{20 + rnd}" if kform == "s" else hex(K[rnd])

    for rnd in range(8):
        def rots_e(i):
            a, b, c, d, e, f, g, h = st[i]
            return [f"v_alignbit_b32 {v(rot[i][0])}, {v(e)}, {v(e)}, 6",
                    f"v_alignbit_b32 {v(rot[i][1])}, {v(e)}, {v(e)}, 11",
                    f"v_alignbit_b32 {v(rot[i][2])}, {v(e)}, {v(e)}, 25"]

        def rots_a(i):
            a = st[i][0]
            return [f"v_alignbit_b32 {v(rot[i][3])}, {v(a)}, {v(a)}, 2",
                    f"v_alignbit_b32 {v(rot[i][4])}, {v(a)}, {v(a)}, 13",
                    f"v_alignbit_b32 {v(rot[i][5])}, {v(a)}, {v(a)}, 22"]

        def fast_alt(i):
            a, b, c, d, e, f, g, h = st[i]
            r = rot[i]
            t = tt[i]
            # S1 -> r0, Ch -> r1, S0 -> r3, Maj -> r4; e' -> d's reg, a' -> h's reg
            if kform == "s":
                first = f"v_add_u32 {v(t)}, {kop(rnd)}, {v(h)}"
            else:
                first = f"v_add_u32 {v(t)}, {kop(rnd)}, {v(h)}"
            return [first,
                    f"v_bitop3_b32 {v(r[0])}, {v(r[0])}, {v(r[1])}, {v(r[2])} bitop3:0x96",
                    f"v_add_u32 {v(t)}, {v(t)}, {v(r[0])}",
                    f"v_bitop3_b32 {v(r[1])}, {v(e)}, {v(f)}, {v(g)} bitop3:0xca",
                    f"v_add_u32 {v(t)}, {v(t)}, {v(r[1])}",
                    f"v_bitop3_b32 {v(r[3])}, {v(r[3])}, {v(r[4])}, {v(r[5])} bitop3:0x96",
                    f"v_add_u32 {v(d)}, {v(d)}, {v(t)}",
                    f"v_bitop3_b32 {v(r[4])}, {v(a)}, {v(b)}, {v(c)} bitop3:0xe8",
                    f"v_add_u32 {v(h)}, {v(t)}, {v(r[3])}",
                    f"v_add_u32 {v(h)}, {v(h)}, {v(r[4])}"]

        def fast_add3(i):
            a, b, c, d, e, f, g, h = st[i]
            r = rot[i]
            t = tt[i]
            k = kop(rnd)
            kadd = (f"v_add3_u32 {v(t)}, {v(t)}, {v(r[0])}, {k}" if kform == "s"
                    else None)
            out = [f"v_bitop3_b32 {v(r[0])}, {v(r[0])}, {v(r[1])}, {v(r[2])} bitop3:0x96",
                   f"v_bitop3_b32 {v(r[1])}, {v(e)}, {v(f)}, {v(g)} bitop3:0xca",
                   f"v_add_u32 {v(t)}, {v(h)}, {v(r[1])}"]
            if kform == "s":
                out.append(kadd)
            else:  # no literal in VOP3 on gfx9: fold K by a VOP2 literal add first
                out[-1:] = [f"v_add_u32 {v(t)}, {k}, {v(h)}", f"v_add3_u32 {v(t)}, {v(t)}, {v(r[0])}, {v(r[1])}"]
            out += [f"v_bitop3_b32 {v(r[3])}, {v(r[3])}, {v(r[4])}, {v(r[5])} bitop3:0x96",
                    f"v_bitop3_b32 {v(r[4])}, {v(a)}, {v(b)}, {v(c)} bitop3:0xe8",
                    f"v_add_u32 {v(d)}, {v(d)}, {v(t)}",
                    f"v_add3_u32 {v(h)}, {v(r[4])}, {v(t)}, {v(r[3])}"]
            return out

        if order == "nat":
            for i in range(B):
                f3 = fast_add3(i)
                # interleave like the compiler: rot(e), S1, Ch, adds, rot(a), S0, Maj, adds
                lines += rots_e(i) + f3[:4 if kform == "s" else 4] + rots_a(i) + f3[4:]
        elif order == "clu":
            for i in range(B):
                lines += rots_e(i) + rots_a(i)
            for i in range(B):
                lines += fast_alt(i)
        elif order == "clu3":
            for i in range(B):
                lines += rots_e(i) + rots_a(i)
            for i in range(B):
                lines += fast_add3(i)
        elif order == "pn":
            for i in range(B):
                lines += rots_e(i) + rots_a(i) + fast_alt(i)
        elif order == "cluI":  # all rotates, then the fast ops of all nonces interleaved
            for i in range(B):
                lines += rots_e(i) + rots_a(i)
            fs = [fast_alt(i) for i in range(B)]
            for j in range(10):
                for i in range(B):
                    lines.append(fs[i][j])
        else:
            raise ValueError(order)
        # rename: new[i] = old[i-1]
        for i in range(B):
            o = st[i]
            st[i] = [o[7], o[0], o[1], o[2], o[3], o[4], o[5], o[6]]
    nregs = 15 * B
    return lines, nregs


VARIANTS = []
for kform in ["s", "l"]:
    for B in [1, 2, 4]:
        for order in ["nat", "clu", "clu3", "pn", "cluI"]:
            if B == 1 and order in ("pn", "cluI"):
                continue
            VARIANTS.append((B, order, kform))
VARIANTS.append((8, "clu", "s"))
VARIANTS.append((8, "cluI", "s"))

out = ['// GENERATED by tools/gen_round_asm.py -- SHA-256 round-order VALU probe (gfx950)',
       '#include <hip/hip_runtime.h>', '#include <stdint.h>', '#include <stdio.h>', '#include <stdlib.h>',
       '#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\\n", #x, hipGetErrorString(e_)); exit(1);} } while (0)']
for idx, (B, order, kform) in enumerate(VARIANTS):
    lines, nregs = gen_body(B, order, kform)
    regs = [f"v{r}" for r in range(BASE, BASE + nregs)]
    clob = ", ".join(f'"{r}"' for r in regs)
    sclob = ", ".join(f'"s{20 + i}"' for i in range(8))
    init = "\\n\\t".join(f"v_xor_b32 {r}, {hex(0x1000193 * (j + 1) & 0xffffffff)}, %0" for j, r in enumerate(regs))
    sinit = "\\n\\t".join(f"s_mov_b32 s{20 + i}, {hex(K[i])}" for i in range(8))
    fold = "\\n\\t".join(f"v_xor_b32 %0, %0, {r}" for r in regs)
    body = "\\n\\t".join(lines)
    out.append(f'''
// B={B} order={order} K={kform}: {len(lines)} VALU per 8 rounds
__global__ __launch_bounds__(256) void k{idx}(uint32_t* out, unsigned long long* clk, int iters, uint32_t seed) {{
    uint32_t x = (blockIdx.x * 256u + threadIdx.x) * 2654435761u ^ seed;
    asm volatile("{init}\\n\\t{sinit}" :: "v"(x) : {clob}, {sclob});
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; i++) asm volatile("{body}" ::: {clob}, {sclob});
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t acc = 0;
    asm volatile("{fold}" : "+v"(acc) :: {clob});
    out[blockIdx.x * 256u + threadIdx.x] = acc;
    if (threadIdx.x == 0) {{ clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }}
}}''')
out.append('''
typedef void (*KFn)(uint32_t*, unsigned long long*, int, uint32_t);
static void run(KFn k, const char* name, int B, int ninstr, int per_cu, int iters) {
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
    double nr = (double)blocks * 256.0 * B * 8.0 * iters;  // nonce-rounds
    double per_clk_cu = nr / (best * 1e-3) / (cus * ghz * 1e9);
    double lane_instr = (double)blocks * 256.0 * ninstr * iters / (best * 1e-3) / (cus * ghz * 1e9);
    printf("{\\"variant\\": \\"%s\\", \\"B\\": %d, \\"blocks_per_cu\\": %d, \\"ms\\": %.3f, \\"clock_ghz\\": %.3f, "
           "\\"instr_per_round\\": %.2f, \\"simd_cycles_per_round\\": %.2f, \\"lane_instr_per_clk_cu\\": %.2f, \\"GHs_64rounds\\": %.2f}\\n",
           name, B, per_cu, best, ghz, (double)ninstr / (8.0 * B), 256.0 / per_clk_cu, lane_instr,
           nr / 64.0 / (best * 1e-3) / 1e9);
    fflush(stdout); free(h); CHK(hipFree(out)); CHK(hipFree(clk)); CHK(hipEventDestroy(e0)); CHK(hipEventDestroy(e1));
}
int main(int argc, char** argv) {
    int iters = argc > 1 ? atoi(argv[1]) : 4000;
    int per_cu = argc > 2 ? atoi(argv[2]) : 8;''')
for idx, (B, order, kform) in enumerate(VARIANTS):
    n = len(gen_body(B, order, kform)[0])
    # keep resident waves comparable: 8 blocks/CU up to B=4 (60 VGPRs), fewer at B=8
    out.append(f'    run(k{idx}, "{order}/K{kform}", {B}, {n}, per_cu, iters / {B});')
out.append('    return 0;\n}')
open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "round_asm.hip"), "w").write("\n".join(out) + "\n")

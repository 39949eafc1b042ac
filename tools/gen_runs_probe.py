#!/usr/bin/env python3
"""Generates tools/runs_probe.hip: does a SHA-256 round issue faster when its fast-class
instructions run in long runs with NO scalar operand?

Round 1's round-order probe (tools/gen_round_asm.py) grouped the 6B rotates of B nonces
ahead of their "fast" ops and saw no gain -- but each nonce's fast run opened with
`v_add_u32 t, K, h`, K a literal or SGPR, and DESIGN 4.1 lists any fast op with a scalar
operand as slow-class: every fast run carried slow ops.  Here K+W sits in a VGPR (as it
would when the schedule word is stored pre-added), so the fast runs hold only v_bitop3
and two-VGPR v_add_u32.

Variants (B independent nonces per lane, 8 rounds per loop iteration):
  nat    the compiler's per-nonce order, 14 instr/round (3 v_add3, 1 v_add)
  cluV   all 6B v_alignbit, then per nonce 10 fast ops (4 v_bitop3 + 6 v_add_u32)
  cluIV  all 6B v_alignbit, then the 10B fast ops interleaved across nonces
  cluA   all 6B v_alignbit, then per nonce 4 v_bitop3 + 2 v_add3 + 2 v_add_u32 (14/round)
and pure calibration streams (independent ops, 8 per lane register group):
  p_align, p_xor, p_add, p_bitop3_3v (3 distinct VGPRs), p_mix (the cluIV fast mix only)
Prints one JSON line per variant: lane-instructions per CU per clock at the in-kernel
clock, and SIMD cycles per nonce-round.
"""
import os

BASE = 8
NREG_NONCE = 16  # 8 state + 6 rot + t + kw


def sha_body(B, order):
    st = [[BASE + NREG_NONCE * i + j for j in range(8)] for i in range(B)]
    rot = [[BASE + NREG_NONCE * i + 8 + j for j in range(6)] for i in range(B)]
    tt = [BASE + NREG_NONCE * i + 14 for i in range(B)]
    kw = [BASE + NREG_NONCE * i + 15 for i in range(B)]
    v = lambda r: f"v{r}"
    lines = []
    for rnd in range(8):
        def rots(i):
            a, e = st[i][0], st[i][4]
            r = rot[i]
            return [f"v_alignbit_b32 {v(r[0])}, {v(e)}, {v(e)}, 6",
                    f"v_alignbit_b32 {v(r[1])}, {v(e)}, {v(e)}, 11",
                    f"v_alignbit_b32 {v(r[2])}, {v(e)}, {v(e)}, 25",
                    f"v_alignbit_b32 {v(r[3])}, {v(a)}, {v(a)}, 2",
                    f"v_alignbit_b32 {v(r[4])}, {v(a)}, {v(a)}, 13",
                    f"v_alignbit_b32 {v(r[5])}, {v(a)}, {v(a)}, 22"]

        def fast10(i):  # 4 bitop3 + 6 two-VGPR adds, no scalar operand
            a, b, c, d, e, f, g, h = st[i]
            r, t, k = rot[i], tt[i], kw[i]
            return [f"v_add_u32 {v(t)}, {v(k)}, {v(h)}",
                    f"v_bitop3_b32 {v(r[0])}, {v(r[0])}, {v(r[1])}, {v(r[2])} bitop3:0x96",
                    f"v_add_u32 {v(t)}, {v(t)}, {v(r[0])}",
                    f"v_bitop3_b32 {v(r[1])}, {v(e)}, {v(f)}, {v(g)} bitop3:0xca",
                    f"v_add_u32 {v(t)}, {v(t)}, {v(r[1])}",
                    f"v_bitop3_b32 {v(r[3])}, {v(r[3])}, {v(r[4])}, {v(r[5])} bitop3:0x96",
                    f"v_add_u32 {v(d)}, {v(d)}, {v(t)}",
                    f"v_bitop3_b32 {v(r[4])}, {v(a)}, {v(b)}, {v(c)} bitop3:0xe8",
                    f"v_add_u32 {v(h)}, {v(t)}, {v(r[3])}",
                    f"v_add_u32 {v(h)}, {v(h)}, {v(r[4])}"]

        def fast8(i):  # 4 bitop3 + 2 add3 + 2 add, K+W in a VGPR
            a, b, c, d, e, f, g, h = st[i]
            r, t, k = rot[i], tt[i], kw[i]
            return [f"v_bitop3_b32 {v(r[0])}, {v(r[0])}, {v(r[1])}, {v(r[2])} bitop3:0x96",
                    f"v_bitop3_b32 {v(r[1])}, {v(e)}, {v(f)}, {v(g)} bitop3:0xca",
                    f"v_add_u32 {v(t)}, {v(h)}, {v(k)}",
                    f"v_add3_u32 {v(t)}, {v(t)}, {v(r[0])}, {v(r[1])}",
                    f"v_bitop3_b32 {v(r[3])}, {v(r[3])}, {v(r[4])}, {v(r[5])} bitop3:0x96",
                    f"v_bitop3_b32 {v(r[4])}, {v(a)}, {v(b)}, {v(c)} bitop3:0xe8",
                    f"v_add_u32 {v(d)}, {v(d)}, {v(t)}",
                    f"v_add3_u32 {v(h)}, {v(r[4])}, {v(t)}, {v(r[3])}"]

        if order == "nat":
            for i in range(B):
                rr, f8 = rots(i), fast8(i)
                lines += rr[:3] + f8[:4] + rr[3:] + f8[4:]
        elif order == "cluV":
            for i in range(B):
                lines += rots(i)
            for i in range(B):
                lines += fast10(i)
        elif order == "cluIV":
            for i in range(B):
                lines += rots(i)
            fs = [fast10(i) for i in range(B)]
            for j in range(10):
                for i in range(B):
                    lines.append(fs[i][j])
        elif order == "cluA":
            for i in range(B):
                lines += rots(i)
            for i in range(B):
                lines += fast8(i)
        else:
            raise ValueError(order)
        for i in range(B):
            o = st[i]
            st[i] = [o[7], o[0], o[1], o[2], o[3], o[4], o[5], o[6]]
    return lines, NREG_NONCE * B, 8 * B  # lines, VGPRs, nonce-rounds per iteration


def pure_body(kind):
    # 32 independent destinations v8..v39 over sources v40..v47, 64 ops per iteration
    v = lambda r: f"v{r}"
    lines = []
    for j in range(64):
        d, s0, s1, s2 = 8 + j % 32, 40 + j % 8, 40 + (j + 3) % 8, 40 + (j + 5) % 8
        if kind == "p_align":
            lines.append(f"v_alignbit_b32 {v(d)}, {v(s0)}, {v(s0)}, 7")
        elif kind == "p_xor":
            lines.append(f"v_xor_b32 {v(d)}, {v(s0)}, {v(d)}")
        elif kind == "p_add":
            lines.append(f"v_add_u32 {v(d)}, {v(s0)}, {v(d)}")
        elif kind == "p_bitop3_3v":
            lines.append(f"v_bitop3_b32 {v(d)}, {v(s0)}, {v(s1)}, {v(s2)} bitop3:0x96")
        elif kind == "p_mix":  # 4 bitop3 (3 distinct) : 6 add, like cluIV's fast part
            if j % 10 in (1, 3, 5, 7):
                lines.append(f"v_bitop3_b32 {v(d)}, {v(s0)}, {v(s1)}, {v(d)} bitop3:0x96")
            else:
                lines.append(f"v_add_u32 {v(d)}, {v(s0)}, {v(d)}")
        else:
            raise ValueError(kind)
    return lines, 40, 0


VARIANTS = []
for kind in ["p_align", "p_xor", "p_add", "p_bitop3_3v", "p_mix"]:
    VARIANTS.append((kind, 0))
for B in [1, 2, 4, 8]:
    for order in ["nat", "cluV", "cluIV", "cluA"]:
        VARIANTS.append((order, B))

out = ['// GENERATED by tools/gen_runs_probe.py -- fast-run / scalar-operand VALU probe (gfx950)',
       '#include <hip/hip_runtime.h>', '#include <stdint.h>', '#include <stdio.h>', '#include <stdlib.h>',
       '#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\\n", #x, hipGetErrorString(e_)); exit(1);} } while (0)']
meta = []
for idx, (name, B) in enumerate(VARIANTS):
    if B == 0:
        lines, nregs, nr = pure_body(name)
        regs = [f"v{r}" for r in range(8, 48)]
    else:
        lines, nregs, nr = sha_body(B, name)
        regs = [f"v{r}" for r in range(BASE, BASE + nregs)]
    meta.append((name, B, len(lines), nr, len(regs)))
    clob = ", ".join(f'"{r}"' for r in regs)
    init = "\\n\\t".join(f"v_xor_b32 {r}, {hex(0x1000193 * (j + 1) & 0xffffffff)}, %0" for j, r in enumerate(regs))
    fold = "\\n\\t".join(f"v_xor_b32 %0, %0, {r}" for r in regs)
    body = "\\n\\t".join(lines)
    out.append(f'''
// {name} B={B}: {len(lines)} VALU per iteration, {len(regs)} VGPRs
__global__ __launch_bounds__(256) void k{idx}(uint32_t* out, unsigned long long* clk, int iters, uint32_t seed) {{
    uint32_t x = (blockIdx.x * 256u + threadIdx.x) * 2654435761u ^ seed;
    asm volatile("{init}" :: "v"(x) : {clob});
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; i++) asm volatile("{body}" ::: {clob});
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t acc = 0;
    asm volatile("{fold}" : "+v"(acc) :: {clob});
    out[blockIdx.x * 256u + threadIdx.x] = acc;
    if (threadIdx.x == 0) {{ clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }}
}}''')
out.append('''
typedef void (*KFn)(uint32_t*, unsigned long long*, int, uint32_t);
static void run(KFn k, const char* name, int B, int ninstr, int nr, int per_cu, int iters) {
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
    double lane_instr = (double)blocks * 256.0 * ninstr * iters / (best * 1e-3) / (cus * ghz * 1e9);
    double cyc_round = nr ? (double)ninstr / nr * 256.0 / lane_instr : 0.0;  // SIMD cycles per nonce-round
    printf("{\\"variant\\": \\"%s\\", \\"B\\": %d, \\"blocks_per_cu\\": %d, \\"ms\\": %.3f, \\"clock_ghz\\": %.3f, "
           "\\"instr_per_round\\": %.2f, \\"lane_instr_per_clk_cu\\": %.2f, \\"simd_cycles_per_round\\": %.2f}\\n",
           name, B, per_cu, best, ghz, nr ? (double)ninstr / nr : 0.0, lane_instr, cyc_round);
    fflush(stdout); free(h); CHK(hipFree(out)); CHK(hipFree(clk)); CHK(hipEventDestroy(e0)); CHK(hipEventDestroy(e1));
}
int main(int argc, char** argv) {
    int iters = argc > 1 ? atoi(argv[1]) : 4000;''')
for idx, (name, B, n, nr, nv) in enumerate(meta):
    # resident waves: 8 per SIMD while VGPRs allow (<= 64), else what fits (512 / VGPRs)
    waves = min(8, 512 // ((nv + 8 + 7) // 8 * 8))
    per_cu = waves  # 256-thread blocks: one wave per SIMD each
    its = f"iters / {max(B, 1)}" if B else "iters"
    out.append(f'    run(k{idx}, "{name}", {B}, {n}, {nr}, {per_cu}, {its});')
out.append('    return 0;\n}')
open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "runs_probe.hip"), "w").write("\n".join(out) + "\n")

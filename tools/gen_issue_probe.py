#!/usr/bin/env python3
"""Generates tools/issue_probe.hip: VALU issue-rate probes for ORDERED instruction
sequences (which forms pair, which interleavings reach the 2-cycle rate).

Each kernel runs 8 independent chains (%0..%7) through a 32-instruction body given as a
list of (form, chain) in issue order; %8 is an SGPR, %9/%10 are loop-invariant VGPRs.
Output: lane-ops per CU per clock at the in-kernel shader clock.
"""
import os

# instruction forms; {c} = chain register, K1/K2 = invariant VGPRs, S = SGPR
F = {
    "xor": "v_xor_b32 {c}, %9, {c}",
    "xor_s": "v_xor_b32 {c}, %8, {c}",
    "add": "v_add_u32 {c}, %9, {c}",
    "add_lit": "v_add_u32 {c}, 0x428a2f98, {c}",
    "and": "v_and_b32 {c}, %9, {c}",
    "or": "v_or_b32 {c}, %9, {c}",
    "lshr": "v_lshrrev_b32 {c}, 3, {c}",
    "lshr_v": "v_lshrrev_b32 {c}, %9, {c}",
    "lshl": "v_lshlrev_b32 {c}, 3, {c}",
    "lshl_v": "v_lshlrev_b32 {c}, %9, {c}",
    "align": "v_alignbit_b32 {c}, {c}, %9, 7",
    "align_same": "v_alignbit_b32 {c}, {c}, {c}, 7",
    "bitop3": "v_bitop3_b32 {c}, {c}, %9, %10 bitop3:0x96",
    "bitop3_s": "v_bitop3_b32 {c}, {c}, %8, %10 bitop3:0x96",
    "add3": "v_add3_u32 {c}, {c}, %9, %10",
    "add3_s": "v_add3_u32 {c}, {c}, %8, %10",
    "add_e64": "v_add_u32_e64 {c}, {c}, %9",
    "xor_e64": "v_xor_b32_e64 {c}, {c}, %9",
    "mov": "v_mov_b32 {c}, %9",
    "pk_add_u16": "v_pk_add_u16 {c}, {c}, %9",
    "bitop3_2": "v_bitop3_b32 {c}, {c}, %9, {c} bitop3:0x96",
    "bitop3_ch": "v_bitop3_b32 {c}, {c}, %9, %10 bitop3:0xca",
    "add3_2": "v_add3_u32 {c}, {c}, %9, {c}",
    "add3_c": "v_add3_u32 {c}, {c}, %9, 7",
    "align3": "v_alignbit_b32 {c}, %9, {c}, 7",
    "align_v": "v_alignbit_b32 {c}, {c}, %9, %10",
    "alignbyte": "v_alignbyte_b32 {c}, {c}, %9, 1",
    "perm": "v_perm_b32 {c}, {c}, %9, %10",
    "bfi": "v_bfi_b32 {c}, {c}, %9, %10",
    "lshl_or": "v_lshl_or_b32 {c}, {c}, 3, %9",
    "lshl_add": "v_lshl_add_u32 {c}, {c}, 3, %9",
    "sub": "v_sub_u32 {c}, %9, {c}",
    "ashr": "v_ashrrev_i32 {c}, 3, {c}",
    "not": "v_not_b32 {c}, {c}",
    "xnor": "v_xnor_b32 {c}, %9, {c}",
    "max": "v_max_u32 {c}, %9, {c}",
    "mul24": "v_mul_u32_u24 {c}, %9, {c}",
    "add_f32": "v_add_f32 {c}, %9, {c}",
    "fma_f32": "v_fma_f32 {c}, {c}, %9, %10",
    "pk_add_f32": "v_pk_add_f32 {c}[0:1], {c}[0:1], %9[0:1]",
}


def seq_repeat(form, n=32):
    return [(form, i % 8) for i in range(n)]


def seq_pattern(pattern, n=32):
    """pattern: list of forms; instruction i uses pattern[i % len] on chain i % 8."""
    return [(pattern[i % len(pattern)], i % 8) for i in range(n)]


SEQS = []
for f in ["xor", "xor_s", "add", "add_lit", "and", "lshr", "lshr_v", "lshl", "lshl_v", "align",
          "align_same", "bitop3", "bitop3_s", "add3", "add3_s", "add_e64", "xor_e64", "mov",
          "pk_add_u16"]:
    SEQS.append((f, seq_repeat(f)))
SEQS += [
    ("alt align,xor", seq_pattern(["align", "xor"])),
    ("alt align,add", seq_pattern(["align", "add"])),
    ("alt bitop3,xor", seq_pattern(["bitop3", "xor"])),
    ("alt add3,add", seq_pattern(["add3", "add"])),
    ("alt align,lshr", seq_pattern(["align", "lshr"])),
    ("pairs xor,xor,align,align", seq_pattern(["xor", "xor", "align", "align"])),
    ("quads xor x4,align x4", seq_pattern(["xor"] * 4 + ["align"] * 4)),
    ("1 align : 3 vop2", seq_pattern(["align", "xor", "add", "and"])),
    ("vop2 mix xor,add,and,lshr", seq_pattern(["xor", "add", "and", "lshr"])),
    ("alt bitop3,add", seq_pattern(["bitop3", "add"])),
    ("alt bitop3,add_lit", seq_pattern(["bitop3", "add_lit"])),
    ("alt bitop3,lshr", seq_pattern(["bitop3", "lshr"])),
    ("alt bitop3,and", seq_pattern(["bitop3", "and"])),
    ("alt bitop3_ch,xor", seq_pattern(["bitop3_ch", "xor"])),
    ("alt bitop3_2,xor", seq_pattern(["bitop3_2", "xor"])),
    ("alt bitop3,bitop3_2", seq_pattern(["bitop3", "bitop3_2"])),
    ("alt add3,xor", seq_pattern(["add3", "xor"])),
    ("alt add3_2,xor", seq_pattern(["add3_2", "xor"])),
    ("alt add3_c,xor", seq_pattern(["add3_c", "xor"])),
    ("alt align,bitop3", seq_pattern(["align", "bitop3"])),
    ("alt align3,xor", seq_pattern(["align3", "xor"])),
    ("alt align_v,xor", seq_pattern(["align_v", "xor"])),
    ("alt lshl,xor", seq_pattern(["lshl", "xor"])),
    ("alt bfi,xor", seq_pattern(["bfi", "xor"])),
    ("alt perm,xor", seq_pattern(["perm", "xor"])),
    ("alt xor_s,xor", seq_pattern(["xor_s", "xor"])),
    ("alt bitop3_s,xor", seq_pattern(["bitop3_s", "xor"])),
    ("align,xor,xor,bitop3", seq_pattern(["align", "xor", "xor", "bitop3"])),
    ("align,bitop3,xor,xor", seq_pattern(["align", "bitop3", "xor", "xor"])),
    ("bitop3,xor,xor", seq_pattern(["bitop3", "xor", "xor"], 33)[:32]),
    ("bitop3,bitop3,xor,xor", seq_pattern(["bitop3", "bitop3", "xor", "xor"])),
    ("sha-ish: align x3,bitop3,add3,add", seq_pattern(["align", "align", "align", "bitop3", "add3", "add"], 36)[:32]),
    ("dep: bitop3 then xor same chain", [("bitop3" if i % 2 == 0 else "xor", (i // 2) % 8) for i in range(32)]),
    ("dep: align then xor same chain", [("align" if i % 2 == 0 else "xor", (i // 2) % 8) for i in range(32)]),
]
for f in ["bitop3_2", "bitop3_ch", "add3_2", "add3_c", "align3", "align_v", "alignbyte", "perm", "bfi",
          "lshl_or", "lshl_add", "sub", "ashr", "not", "xnor", "max", "mul24", "add_f32", "fma_f32"]:
    SEQS.append((f, seq_repeat(f)))


def body(seq):
    lines = []
    for form, c in seq:
        lines.append(F[form].format(c=f"%{c}"))
    return "\\n\\t".join(lines)


out = ['// GENERATED by tools/gen_issue_probe.py -- ordered-sequence VALU issue probe (gfx950)',
       '#include <hip/hip_runtime.h>', '#include <stdio.h>', '#include <stdlib.h>',
       '#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\\n", #x, hipGetErrorString(e_)); exit(1);} } while (0)']
for i, (name, seq) in enumerate(SEQS):
    n = len(seq)
    out.append(f'''
__global__ __launch_bounds__(256) void k{i}(unsigned* out, unsigned long long* clk, int iters, unsigned seed) {{
    unsigned a = threadIdx.x ^ seed, b = a * 3u + 1u, c = a * 5u + 2u, d = a * 7u + 3u, e = a * 11u + 4u, f = a * 13u + 5u, g = a * 17u + 6u, h = a * 19u + 7u;
    unsigned k1 = threadIdx.x * 2654435761u + seed, k2 = k1 ^ 0x5bd1e995u;
    unsigned s = __builtin_amdgcn_readfirstlane(seed * 2654435761u | 1u);
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; i++) {{
        asm volatile("{body(seq)}" : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h) : "s"(s), "v"(k1), "v"(k2));
    }}
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = a ^ b ^ c ^ d ^ e ^ f ^ g ^ h;
    if (threadIdx.x == 0) {{ clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }}
}}
static const int n{i} = {n};''')
out.append('''
typedef void (*KFn)(unsigned*, unsigned long long*, int, unsigned);
static void run(KFn k, const char* name, int ninstr, int per_cu, int iters) {
    hipDeviceProp_t p; CHK(hipGetDeviceProperties(&p, 0));
    int cus = p.multiProcessorCount, blocks = cus * per_cu;
    unsigned* out; unsigned long long* clk;
    CHK(hipMalloc(&out, (size_t)blocks * 256 * 4)); CHK(hipMalloc(&clk, (size_t)blocks * 16));
    hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, clk, iters / 10, 1u);
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
    double rate = (double)blocks * 256.0 * ninstr * iters / (best * 1e-3);
    printf("{\\"seq\\": \\"%s\\", \\"blocks_per_cu\\": %d, \\"ms\\": %.3f, \\"clock_ghz\\": %.3f, \\"lane_ops_per_cu_per_clk\\": %.2f}\\n",
           name, per_cu, best, ghz, rate / (cus * ghz * 1e9));
    fflush(stdout); free(h); CHK(hipFree(out)); CHK(hipFree(clk)); CHK(hipEventDestroy(e0)); CHK(hipEventDestroy(e1));
}
int main(int argc, char** argv) {
    int per_cu = argc > 1 ? atoi(argv[1]) : 8, iters = argc > 2 ? atoi(argv[2]) : 20000;''')
for i, (name, seq) in enumerate(SEQS):
    out.append(f'    run(k{i}, "{name}", n{i}, per_cu, iters);')
out.append('    return 0;\n}')
open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "issue_probe.hip"), "w").write("\n".join(out) + "\n")

#!/bin/bash
# tools/build_phase_variants.sh -- code-phase sweep of the plain-layout loop:
# tools/variants/ph<P> = the product build with the plain kernels' per-nonce loop body at
# P mod 64 bytes (.p2align 6 + P/4 s_nop at the loop top), P = 4, 12, ..., 60;
# tools/variants/product = the Makefile build (.p2align 3 + 1 s_nop: 4 mod 8).  The probe
# macro is patched into a scratch copy of csrc/, so the product sources (and the build id
# the committed PMC summaries are matched against) stay as they are.  For
# tools/variant_bench.py.  CPU only.
set -eu
cd "$(dirname "$0")/.."
HIPCC=/opt/rocm/bin/hipcc
B=bitcoin-miner_amd/build
SRC=$(mktemp -d)
trap 'rm -rf "$SRC"' EXIT
cp bitcoin-miner_amd/csrc/* "$SRC/"
python3 - "$SRC/scan_kernel.h" <<'PY'
import sys
p = sys.argv[1]
s = open(p).read()
old = '#define GPUHASH_LOOP_ALIGN() asm volatile(".p2align 3\\n\\ts_nop 0")'
assert old in s
new = ('#define GPUHASH_PS2(x) #x\n#define GPUHASH_PS(x) GPUHASH_PS2(x)\n'
       '#define GPUHASH_LOOP_ALIGN() asm volatile(".p2align 6\\n\\t.rept " GPUHASH_PS(GPUHASH_PHASE64) "/4\\n\\ts_nop 0\\n\\t.endr")')
open(p, "w").write(s.replace(old, new))
PY
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -I$SRC -Wno-unused-result -Wno-unused-value"
mkdir -p tools/variants/product
cp bitcoin-miner_amd/lib/libgpuhash.so tools/variants/product/
for P in ${PHASES:-4 12 20 28 36 44 52 60}; do
    (
    out=tools/variants/ph$P
    mkdir -p "$out"
    $HIPCC $F -DGPUHASH_WAVES_PER_EU=8 -DGPUHASH_PHASE64=$P -c "$SRC/kernels_plain.hip" -o "$out/kernels_plain.o"
    $HIPCC --offload-arch=gfx950 -shared -fPIC -o "$out/libgpuhash.so" $B/kernels.o "$out/kernels_plain.o" \
        $B/kernels_ut.o $B/kernels_misc.o $B/gpuhash.o $B/plan_hip.o -lpthread
    rm -f "$out"/*.o
    echo "built ph$P"
    ) &
done
wait

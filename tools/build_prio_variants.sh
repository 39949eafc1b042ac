#!/bin/bash
# tools/build_prio_variants.sh -- static wave priorities (round 4): builds the product
# library (tools/variants/product) and the same per-family build with s_setprio(P) in
# every odd workgroup of the scan kernels (tools/variants/prio<P>), for
# tools/variant_bench.py.  The guide's VALU arbiter picks the ready wave by priority, then
# age; a static split changes which waves' instruction classes interleave on a SIMD.
# The hook is inserted into a temporary copy of csrc/ (the product sources, and so the
# product build id, stay untouched).  CPU only.
set -eu
cd "$(dirname "$0")/.."
HIPCC=/opt/rocm/bin/hipcc
TMP=$(mktemp -d)
trap 'rm -rf "$TMP"' EXIT
cp -r bitcoin-miner_amd/csrc "$TMP/csrc"
python3 - "$TMP/csrc/scan_kernel.h" <<'PY'
import sys
p = sys.argv[1]
s = open(p).read()
anchor = "    WaveBest wb{~0ull, ~0ull, 0xFFFFFFFFu};\n    for (;;) {"
assert anchor in s
s = s.replace(anchor, "    if (blockIdx.x & 1u) __builtin_amdgcn_s_setprio(GPUHASH_SETPRIO);\n" + anchor)
open(p, "w").write(s)
PY
INC="-Iinclude -I$TMP/csrc"
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC $INC -Wno-unused-result -Wno-unused-value"
mkdir -p tools/variants/product
cp bitcoin-miner_amd/lib/libgpuhash.so tools/variants/product/
for P in 1 3; do
    out=tools/variants/prio$P
    mkdir -p "$out"
    D=-DGPUHASH_SETPRIO=$P
    $HIPCC $F $D -c $TMP/csrc/kernels.hip -o "$out/kernels.o" &
    $HIPCC $F $D -DGPUHASH_WAVES_PER_EU=8 -c $TMP/csrc/kernels_plain.hip -o "$out/kernels_plain.o" &
    $HIPCC $F $D -mllvm -amdgpu-sched-strategy=max-ilp -c $TMP/csrc/kernels_ut.hip -o "$out/kernels_ut.o" &
    $HIPCC $F $D -mllvm -amdgpu-sched-strategy=max-ilp -DGPUHASH_LOOP_PHASE=-1 -c $TMP/csrc/kernels_misc.hip -o "$out/kernels_misc.o" &
    $HIPCC $F -c $TMP/csrc/gpuhash.cpp -o "$out/gpuhash.o" &
    $HIPCC $F -x c++ -c $TMP/csrc/plan.cpp -o "$out/plan.o" &
    wait
    $HIPCC --offload-arch=gfx950 -shared -fPIC -o "$out/libgpuhash.so" "$out"/kernels*.o "$out/gpuhash.o" "$out/plan.o" -lpthread
    rm -f "$out"/*.o
    echo "built prio$P"
done

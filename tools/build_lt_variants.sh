#!/bin/bash
# tools/build_lt_variants.sh -- code-phase A/B for the lane-table loop:
# tools/variants/product = the Makefile build (loop unpinned), tools/variants/ltalign =
# the same with the lane-table loop body pinned at 4 mod 8 bytes (-DGPUHASH_LT_ALIGN), for
# tools/variant_bench.py.  CPU only.
set -eu
cd "$(dirname "$0")/.."
HIPCC=/opt/rocm/bin/hipcc
# the tuning hooks live in tools/tuning_hooks.patch (not in the product sources): applied
# to a temporary copy of csrc/, so the product sources and build id stay untouched
TMP=$(mktemp -d)
trap 'rm -rf "$TMP"' EXIT
mkdir -p "$TMP/bitcoin-miner_amd"
cp -r bitcoin-miner_amd/csrc "$TMP/bitcoin-miner_amd/csrc"
patch -s -p1 -d "$TMP" < tools/tuning_hooks.patch
INC="-Iinclude -I$TMP/bitcoin-miner_amd/csrc"
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC $INC -Wno-unused-result -Wno-unused-value"
out=tools/variants/ltalign
mkdir -p "$out" tools/variants/product
cp bitcoin-miner_amd/lib/libgpuhash.so tools/variants/product/
$HIPCC $F -c $TMP/bitcoin-miner_amd/csrc/kernels.hip -o "$out/kernels.o" &
$HIPCC $F -DGPUHASH_WAVES_PER_EU=8 -c $TMP/bitcoin-miner_amd/csrc/kernels_plain.hip -o "$out/kernels_plain.o" &
$HIPCC $F -mllvm -amdgpu-sched-strategy=max-ilp -DGPUHASH_LT_ALIGN -c $TMP/bitcoin-miner_amd/csrc/kernels_ut.hip -o "$out/kernels_ut.o" &
$HIPCC $F -mllvm -amdgpu-sched-strategy=max-ilp -DGPUHASH_LOOP_PHASE=-1 -c $TMP/bitcoin-miner_amd/csrc/kernels_misc.hip -o "$out/kernels_misc.o" &
$HIPCC $F -c bitcoin-miner_amd/csrc/gpuhash.cpp -o "$out/gpuhash.o" &
$HIPCC $F -x c++ -c bitcoin-miner_amd/csrc/plan.cpp -o "$out/plan.o" &
wait
$HIPCC --offload-arch=gfx950 -shared -fPIC -o "$out/libgpuhash.so" "$out"/kernels*.o "$out/gpuhash.o" "$out/plan.o" -lpthread
rm -f "$out"/*.o
echo "built ltalign"

#!/bin/bash
# tools/build_salu_variants.sh -- prices the 44 s_mov_b32 that re-materialise K constants
# in SGPRs in every iteration of the config-2 loop: builds the product
# library (tools/variants/product) and the same build with 44 MORE scalar instructions per
# iteration (-DGPUHASH_EXTRA_SALU, tools/variants/salu44) for tools/variant_bench.py.  If
# doubling the loop's scalar instructions costs nothing measurable, removing the 44 s_movs
# cannot gain anything either.  CPU only.
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
out=tools/variants/salu44
mkdir -p "$out" tools/variants/product
cp bitcoin-miner_amd/lib/libgpuhash.so tools/variants/product/
$HIPCC $F -c $TMP/bitcoin-miner_amd/csrc/kernels.hip -o "$out/kernels.o" &
$HIPCC $F -DGPUHASH_WAVES_PER_EU=8 -DGPUHASH_EXTRA_SALU -c $TMP/bitcoin-miner_amd/csrc/kernels_plain.hip -o "$out/kernels_plain.o" &
$HIPCC $F -mllvm -amdgpu-sched-strategy=max-ilp -c $TMP/bitcoin-miner_amd/csrc/kernels_ut.hip -o "$out/kernels_ut.o" &
$HIPCC $F -mllvm -amdgpu-sched-strategy=max-ilp -DGPUHASH_LOOP_PHASE=-1 -c $TMP/bitcoin-miner_amd/csrc/kernels_misc.hip -o "$out/kernels_misc.o" &
$HIPCC $F -c bitcoin-miner_amd/csrc/gpuhash.cpp -o "$out/gpuhash.o" &
$HIPCC $F -x c++ -c bitcoin-miner_amd/csrc/plan.cpp -o "$out/plan.o" &
wait
$HIPCC --offload-arch=gfx950 -shared -fPIC -o "$out/libgpuhash.so" "$out"/kernels*.o "$out/gpuhash.o" "$out/plan.o" -lpthread
rm -f "$out"/*.o
echo "built salu44"

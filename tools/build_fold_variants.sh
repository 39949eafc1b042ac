#!/bin/bash
# tools/build_fold_variants.sh -- scalar operands out of the 2-input adds (round 4):
# tools/variants/product = the Makefile build; the others are the same per-family build
# with the tuning hooks of tools/tuning_hooks.patch (round_ukw: a wave-uniform K+W goes into the
# round's v_add3 instead of its 2-input h + kw; GPUHASH_SALU_SIGMA: the uniform
# sigma0(W_J) on SALU), for tools/variant_bench.py (profiles/r04_fold_variants.jsonl):
#   fold  every hook    plain  plain-layout rounds   ex  extra block   lt  lane table
#   salu  sigma0(W_J) on SALU
# The K+W-table rounds (config 3) use round_ukw in the product build.  CPU only.
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
mkdir -p tools/variants/product
cp bitcoin-miner_amd/lib/libgpuhash.so tools/variants/product/
for name in ${FOLD_VARIANTS:-fold salu plain ex lt}; do
    out=tools/variants/$name
    mkdir -p "$out"
    case $name in
        fold) D="-DGPUHASH_SALU_SIGMA -DGPUHASH_FOLD_PLAIN -DGPUHASH_FOLD_EX -DGPUHASH_FOLD_LT" ;;
        salu) D="-DGPUHASH_SALU_SIGMA" ;;
        plain) D="-DGPUHASH_FOLD_PLAIN" ;;
        ex) D="-DGPUHASH_FOLD_EX" ;;
        lt) D="-DGPUHASH_FOLD_LT" ;;
        *) echo "unknown variant $name" >&2; exit 2 ;;
    esac
    $HIPCC $F $D -c $TMP/bitcoin-miner_amd/csrc/kernels.hip -o "$out/kernels.o" &
    $HIPCC $F $D -DGPUHASH_WAVES_PER_EU=8 -c $TMP/bitcoin-miner_amd/csrc/kernels_plain.hip -o "$out/kernels_plain.o" &
    $HIPCC $F $D -mllvm -amdgpu-sched-strategy=max-ilp -c $TMP/bitcoin-miner_amd/csrc/kernels_ut.hip -o "$out/kernels_ut.o" &
    $HIPCC $F $D -mllvm -amdgpu-sched-strategy=max-ilp -DGPUHASH_LOOP_PHASE=-1 -c $TMP/bitcoin-miner_amd/csrc/kernels_misc.hip -o "$out/kernels_misc.o" &
    $HIPCC $F -c bitcoin-miner_amd/csrc/gpuhash.cpp -o "$out/gpuhash.o" &
    $HIPCC $F -x c++ -c bitcoin-miner_amd/csrc/plan.cpp -o "$out/plan.o" &
    wait
    $HIPCC --offload-arch=gfx950 -shared -fPIC -o "$out/libgpuhash.so" "$out"/kernels*.o "$out/gpuhash.o" "$out/plan.o" -lpthread
    if [ -n "${KEEP_OBJ:-}" ]; then mkdir -p "$KEEP_OBJ/$name" && cp "$out"/kernels*.o "$KEEP_OBJ/$name/"; fi
    rm -f "$out"/*.o
    echo "built $name"
done

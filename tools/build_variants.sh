#!/bin/bash
# tools/build_variants.sh -- builds libgpuhash.so variants with one set of LLVM scheduling
# / occupancy options for every kernel TU into tools/variants/<name>/, plus the product
# build (per-TU options, Makefile), for tools/variant_bench.py.  CPU only.
set -eu
cd "$(dirname "$0")/.."
HIPCC=/opt/rocm/bin/hipcc
INC="-Iinclude -Ibitcoin-miner_amd/csrc"
build() {  # build <name> <extra flags...>
    local name=$1; shift
    local out=tools/variants/$name
    mkdir -p "$out"
    for k in kernels kernels_plain kernels_ut kernels_misc; do
        $HIPCC --offload-arch=gfx950 -O3 -std=c++17 -fPIC $INC "$@" -c bitcoin-miner_amd/csrc/$k.hip -o "$out/$k.o"
    done
    $HIPCC --offload-arch=gfx950 -O3 -std=c++17 -fPIC $INC -c bitcoin-miner_amd/csrc/gpuhash.cpp -o "$out/gpuhash.o"
    $HIPCC --offload-arch=gfx950 -O3 -std=c++17 -fPIC $INC -x c++ -c bitcoin-miner_amd/csrc/plan.cpp -o "$out/plan.o"
    $HIPCC --offload-arch=gfx950 -shared -fPIC -o "$out/libgpuhash.so" "$out"/kernels*.o "$out/gpuhash.o" "$out/plan.o" -lpthread
    rm -f "$out"/*.o
    echo "built $name"
}
# the product build (per-family options from the Makefile) next to uniform-option builds
mkdir -p tools/variants/product && cp bitcoin-miner_amd/lib/libgpuhash.so tools/variants/product/
build base &
build occ8 -DGPUHASH_WAVES_PER_EU=8 &
build maxilp -mllvm -amdgpu-sched-strategy=max-ilp &
build occ8_maxilp -DGPUHASH_WAVES_PER_EU=8 -mllvm -amdgpu-sched-strategy=max-ilp &
wait

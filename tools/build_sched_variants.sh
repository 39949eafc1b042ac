#!/bin/bash
# tools/build_sched_variants.sh -- instruction-order sweep of the plain-layout kernels
# (config 2's family): each variant rebuilds kernels_plain.hip with the product flags
# (8 waves/SIMD) plus one LLVM machine-scheduler option and links it with the product's
# other objects (bitcoin-miner_amd/build/, run `make` first), into
# tools/variants/<name>/libgpuhash.so for tools/variant_bench.py.  Round 4 found that a
# hand-placed v_add3 in ten rounds of the plain loop moved config 2 by 3%, so
# the order LLVM picks is worth a sweep.  (-misched=si never finished in 30 min;
# gcn-iterative-ilp / -minreg crash the compiler on this TU.)  CPU only.
set -eu
cd "$(dirname "$0")/.."
HIPCC=/opt/rocm/bin/hipcc
# the ahead<L> variants need the GPUHASH_SCHED_AHEAD hook (tools/sched_ahead.patch: schedule
# word t+L written before round t), applied to a temporary copy of the sources so the
# product sources, and so the product build id, stay untouched
TMP=$(mktemp -d)
trap 'rm -rf "$TMP"' EXIT
mkdir -p "$TMP/bitcoin-miner_amd"
cp -r bitcoin-miner_amd/csrc "$TMP/bitcoin-miner_amd/csrc"
patch -s -p1 -d "$TMP" < tools/tuning_hooks.patch  # sched_ahead.patch is written against it
patch -s -p1 -d "$TMP" < tools/sched_ahead.patch
INC="-Iinclude -I$TMP/bitcoin-miner_amd/csrc"
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC $INC -Wno-unused-result -Wno-unused-value -DGPUHASH_WAVES_PER_EU=8"
B=bitcoin-miner_amd/build
mkdir -p tools/variants/product
cp bitcoin-miner_amd/lib/libgpuhash.so tools/variants/product/
declare -A OPT=(
  [s_nomisched]="-mllvm -enable-misched=0"
  [s_nopostra]="-mllvm -disable-post-ra"
  [s_trackers]="-mllvm -amdgpu-use-amdgpu-trackers"
  [s_bias100]="-mllvm -amdgpu-schedule-metric-bias=100"
  [s_nohrp]="-mllvm -amdgpu-disable-unclustered-high-rp-reschedule"
  [s_noclus]="-mllvm -amdgpu-disable-clustered-low-occupancy-reschedule"
  [s_memclause]="-mllvm -amdgpu-sched-strategy=max-memory-clause"
  [ahead1]="-DGPUHASH_SCHED_AHEAD=1"
  [ahead2]="-DGPUHASH_SCHED_AHEAD=2"
  [ahead3]="-DGPUHASH_SCHED_AHEAD=3"
  [ahead5]="-DGPUHASH_SCHED_AHEAD=5"
)
names=${SCHED_VARIANTS:-${!OPT[@]}}
for name in $names; do
  (
    out=tools/variants/$name
    mkdir -p "$out"
    if $HIPCC $F ${OPT[$name]} -c $TMP/bitcoin-miner_amd/csrc/kernels_plain.hip -o "$out/kernels_plain.o" 2> "$out/build.log"; then
      $HIPCC --offload-arch=gfx950 -shared -fPIC -o "$out/libgpuhash.so" $B/kernels.o "$out/kernels_plain.o" \
          $B/kernels_ut.o $B/kernels_misc.o $B/gpuhash.o $B/plan_hip.o -lpthread
      [ -n "${KEEP_OBJ:-}" ] && mkdir -p "$KEEP_OBJ/$name" && cp "$out/kernels_plain.o" "$KEEP_OBJ/$name/"
      rm -f "$out/kernels_plain.o"
      echo "built $name"
    else
      echo "FAILED $name: $(tail -2 "$out/build.log")"; rm -rf "$out"
    fi
  ) &
  while [ "$(jobs -r | wc -l)" -ge 6 ]; do sleep 1; done
done
wait

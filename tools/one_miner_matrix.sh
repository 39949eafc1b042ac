#!/bin/bash
# ONE GPU-backed miner at the reference's LSP parameters (2 s epochs,
# EpochLimit 5, window 1), 4 clients x [0, 2^35], 10% read and write drops on every role;
# job size x depth with no speculative copies, then the server's defaults.  One JSON line
# per run (tools/system_bench.py) to $OUT.
set -u
OUT=${OUT:-gpurun_out/r06_one_miner.jsonl}
mkdir -p "$(dirname "$OUT")"
run() {
  timeout -k 10 240 python -u tools/system_bench.py --clients 4 --bits 35 --miners 1 --kill-after -1 "$@" \
    >> "$OUT" 2> "gpurun_out/one_miner_$(date +%s%N).err"
  rc=$?
  echo "run $* -> rc $rc" >&2
  [ $rc -eq 0 ] || exit $rc
}
for bits in 34 35 36; do
  for depth in 1 2; do
    run --job-bits $bits --depth $depth --copies 1 --label "2^$bits depth $depth, no copies"
  done
done
for k in 1 2 3; do
  run --label "server defaults (run $k)"
done

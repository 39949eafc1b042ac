#!/bin/bash
# Round-6 GPU session 1: the one-miner matrix at the reference's LSP parameters, then the
# message-length sweep (INTEGRATION.md's rate table).  Each step has its own time limit.
set -u
mkdir -p gpurun_out
bash tools/one_miner_matrix.sh || exit $?
timeout -k 10 420 python -u tools/length_sweep.py > gpurun_out/r06_length_sweep.jsonl 2> gpurun_out/r06_length_sweep.err

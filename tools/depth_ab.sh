set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for rep in 1 2; do
  for d in 1 2; do
    GPUHASH_MINER_DEPTH=$d timeout -k 10 300 python -u tools/system_bench.py > gpurun_out/ab_d${d}_r${rep}.log 2>&1 || exit $?
    echo "depth $d rep $rep: $(grep '"workload"' gpurun_out/ab_d${d}_r${rep}.log | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["system_GHs"], d["jobs_requeued"], d["all_results_verified"])')"
  done
done

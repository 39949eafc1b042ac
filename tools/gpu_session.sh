#!/bin/bash
# tools/gpu_session.sh STEP... -- runs GPU steps on the gpurun box, each under its own
# time limit, logging to gpurun_out/.  A plain failure (exit 1, e.g. a failing test)
# lets the next step run; a fault, abort, segfault, time limit or kill stops the session.
# Steps: valid | validcopies | validcopies37 | valid37 | c5ref | c5diag200 | hostwait | c5diag | c5stream | c5poll | lsweep | inproc8s | dist8s | fma | cumask | family | inproc8c4 | valu | go | test | soak | smoke | bench | bench3 | bench4 | prof4 | c4full | dist8c4 | dist2 | inproc | latency | prof | pmc | pmc3 | pmc4 | sweep | variants | partial | regret | sys5
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
# the build id of the library this session runs (profiles are matched against it)
python3 -c "import sys; sys.path.insert(0, 'bitcoin-miner_amd'); import gpuhash; print(gpuhash.build_id())" \
    > "$OUT/build_id.txt" 2>/dev/null || echo unknown > "$OUT/build_id.txt"

run() {  # run <name> <seconds> <cmd...>
    local name=$1 secs=$2
    shift 2
    echo "== $name: $*" | tee -a "$OUT/session.log"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc" | tee -a "$OUT/session.log"
    tail -n 5 "$OUT/$name.log"
    case $rc in
        0|1|2|5) return 0 ;;
        *) echo "== stopping: $name ended with rc=$rc" | tee -a "$OUT/session.log"; exit $rc ;;
    esac
}

for step in "$@"; do
    case $step in
        fma) run fma 180 ./tools/bin/fma_probe 20000 ;;
        valu) run valu 120 ./tools/bin/valu_peak 8 50000; run valu1 120 ./tools/bin/valu_peak 1 50000 ;;
        probe) run probe8 300 ./tools/bin/valu_probe 8 20000 ;;
        listctr) run listctr 120 rocprofv3 -L ;;
        clocks) { rocm-smi --showclocks; amd-smi metric --clock 2>&1 | head -40; } > "$OUT/clocks.log" 2>&1; cat "$OUT/clocks.log" | head -30 ;;
        go) { command -v go && go version; } > "$OUT/go.log" 2>&1; echo "go: $(cat $OUT/go.log)" ;;
        test) run pytest_gpu 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ;;
        valid) run validate_des 900 python -u tools/validate_des.py --runs "${VALID_RUNS:-10}" --out "$OUT/r06_validate_des_runs.jsonl" ;;
        validnew) run validate_des_defaults 900 python -u tools/validate_des.py --runs "${VALID_RUNS:-10}" --policies defaults --out "$OUT/r06_validate_des_runs_defaults2.jsonl" ;;
        validcopies) run validate_des_copies 900 python -u tools/validate_des.py --runs "${VALID_RUNS:-10}" --policies single,defaults --out "$OUT/r06_validate_des_runs_copies.jsonl" ;;
        validcopies37) run validate_des_copies_2p37 600 python -u tools/validate_des.py --runs "${VALID_RUNS:-4}" --bits 37 --seeds 100 --policies single,defaults --out "$OUT/r06_validate_des_runs_copies_2p37.jsonl" ;;
        valid37) run validate_des_2p37 600 python -u tools/validate_des.py --runs "${VALID_RUNS:-4}" --bits 37 --seeds 100 --out "$OUT/r06_validate_des_runs_2p37.jsonl" ;;
        killprobe) run kill_probe 400 python -u tools/kill_probe.py --rounds "${KILL_ROUNDS:-4}" ;;
        c5ref) run c5ref 500 env GPUHASH_DIAG_DIR="$OUT/c5ref" python -u -m pytest tests/test_gpu_system.py -m gpu -x -v -s --timeout 450 --timeout-method thread -k reference_lsp_params ;;
        systest) run pytest_sys 600 python -u -m pytest tests/test_gpu_system.py -m gpu -x -v --timeout 300 --timeout-method thread ;;
        smoke) run smoke 180 python -c "import __graft_entry__ as g; g.smoke()" ;;
        hostwait) run hostwait 400 python -u tools/host_wait_probe.py --procs "${HW_PROCS:-8}" --modes "${HW_MODES:-stream,event,poll}" ;;
        c5diag) run c5diag${C5TAG:-} 400 env GPUHASH_DIAG_DIR="$OUT/c5${C5TAG:-}" python -u -m pytest tests/test_gpu_system.py -m gpu -x -v -s --timeout 300 --timeout-method thread -k config5_full_size ;;
        c5stream) for i in $(seq 1 "${C5_REPEAT:-8}"); do
                      run c5stream_$i 200 env GPUHASH_HOST_WAIT=stream GPUHASH_DIAG_DIR="$OUT/c5stream_$i" python -u -m pytest tests/test_gpu_system.py -m gpu -x -v -s --timeout 180 --timeout-method thread -k config5_full_size
                  done ;;
        c5poll) run c5poll 400 env GPUHASH_HOST_WAIT=poll GPUHASH_DIAG_DIR="$OUT/c5poll" python -u -m pytest tests/test_gpu_system.py -m gpu -x -v -s --timeout 300 --timeout-method thread -k config5_full_size ;;
        benchwait) for i in 1 2; do for m in stream poll; do
                       run benchwait_${m}_$i 200 env GPUHASH_HOST_WAIT=$m python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --search off
                   done; done ;;
        bench) run bench 300 python -u bench.py --steps 10 --warmup 2 ;;
        inproc8s) run inproc8s 300 python -u bench.py --inproc 0,0,0,0,0,0,0,0 --steps 2 --warmup 1 --no-cpu-baseline ;;
        dist8s) run dist8s 400 env GPUHASH_SHARE_GPU=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29549 bench.py --gpus 8 --steps 1 --warmup 1 ;;
        inproc40) run inproc40 300 python -u bench.py --inproc 0,0 --steps 2 --warmup 1 --no-cpu-baseline ;;
        nccl1) run nccl1 300 env GPUHASH_FORCE_DIST=1 GPUHASH_DIST_BACKEND=nccl python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu-baseline ;;
        dist2) run dist2 300 env GPUHASH_SHARE_GPU=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 ;;
        inproc) run inproc2 300 python -u bench.py --inproc 0,0 --steps 3 --warmup 1 --no-cpu-baseline ;;
        latency) run latency 120 python -u tools/latency.py ;;
        ranks) run ranks 300 python -u tools/rank_windows.py --ranks "${RANKS:-0,1,2,3,4,5,6,7}" ;;
        sweep) run sweep 600 python -u tools/layout_sweep.py ;;
        lsweep) run lsweep 900 python -u tools/length_sweep.py ;;
        regret) run regret 600 python -u tools/planner_regret.py ;;
        partial) run partial 600 python -u tools/partial_row_probe.py "${VROUNDS:-2}" "${VARIANTS:-old,new}" ;;
        variants) run variants 600 python -u tools/variant_bench.py "${VROUNDS:-3}" "${VARIANTS:-old,new}" ;;
        sys5) run sys5 900 python -u tools/system_bench.py ;;
        sys5n) run sys5n 900 python -u tools/system_bench.py --native ;;
        sys5c) run sys5c 900 python -u tools/system_bench.py --compiled ;;
        sys5a) run sys5a 900 python -u tools/system_bench.py --adaptive
               run sys5an 900 python -u tools/system_bench.py --adaptive --native ;;
        cumask) run cumask 120 ./tools/bin/cumask_probe 20000 ;;
        family) run family 300 python3 -u tools/family_issue.py
                cp "$OUT/family.log" "$OUT/fam.jsonl"
                run family_pmc 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d "$OUT/fam_pmc" -o pmc --output-format csv -- python3 tools/family_issue.py --once
                run family_sum 60 python3 tools/family_issue.py --summarize "$OUT/fam_pmc" "$OUT/fam.jsonl" ;;
        inproc8c4) run inproc8c4 300 python -u bench.py --inproc 0,0,0,0,0,0,0,0 --config 4 --steps 1 --warmup 1 --no-cpu-baseline ;;
        soak) run soak $(( ${SOAK_SECONDS:-90} + 60 )) python -u tools/soak.py "${SOAK_SECONDS:-90}" "${SOAK_SEED:-2026}" ;;
        c4full) run c4full 400 python -u tools/config4_full.py ;;
        dist8c4) run dist8c4 400 env GPUHASH_SHARE_GPU=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29547 bench.py --gpus 8 --config 4 --steps 1 --warmup 0 ;;
        bench3) run bench3 300 python -u bench.py --config 3 --steps 5 --warmup 1 ;;
        bench4) run bench4 300 python -u bench.py --config 4 --steps 2 --warmup 1 ;;
        prof4) run prof_c4 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c4" -o bench --output-format csv -- python3 bench.py --config 4 --steps 1 --warmup 1 --no-cpu-baseline --no-search ;;
        prof) run prof 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o bench --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-search ;;
        pmc) run pmc_valu 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d "$OUT/pmc1" -o pmc --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-search
             run pmc_derived 120 rocprofv3 --pmc VALUBusy VALUUtilization -d "$OUT/pmc4" -o pmc --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-search
             run pmc_hbm 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc2" -o pmc --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-search
             run pmc_wr 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc3" -o pmc --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-search ;;
        pmc3) B3="python3 bench.py --config 3 --steps 2 --warmup 1 --no-cpu-baseline --no-search"
              run prof_c3 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c3" -o bench --output-format csv -- $B3
              run pmc_valu_c3 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d "$OUT/pmc1_c3" -o pmc --output-format csv -- $B3
              run pmc_derived_c3 120 rocprofv3 --pmc VALUBusy VALUUtilization -d "$OUT/pmc4_c3" -o pmc --output-format csv -- $B3
              run pmc_hbm_c3 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc2_c3" -o pmc --output-format csv -- $B3
              run pmc_wr_c3 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc3_c3" -o pmc --output-format csv -- $B3 ;;
        pmc4) B4="python3 bench.py --config 4 --steps 1 --warmup 1 --no-cpu-baseline --no-search"
              run prof_c4 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c4" -o bench --output-format csv -- $B4
              run pmc_valu_c4 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d "$OUT/pmc1_c4" -o pmc --output-format csv -- $B4
              run pmc_derived_c4 120 rocprofv3 --pmc VALUBusy VALUUtilization -d "$OUT/pmc4_c4" -o pmc --output-format csv -- $B4
              run pmc_hbm_c4 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc2_c4" -o pmc --output-format csv -- $B4
              run pmc_wr_c4 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc3_c4" -o pmc --output-format csv -- $B4 ;;
        *) echo "unknown step $step"; exit 2 ;;
    esac
done
echo "== session done"

#!/bin/bash
# Profiles of the driver's headline command (run on the GPU box from the repo root):
#   1. rocprofv3 --kernel-trace --stats of `python3 bench.py --gpus 1 --steps 20 --warmup 5`
#      (with --no-dp1: the 1-rank data-parallel leg runs in a child process of its own, profiled in 4)
#   2. two separate PMC passes (FETCH_SIZE, WRITE_SIZE) of the serve path alone at 20 steps
#      per launch (tools/pmc_traffic.py turns them into HBM bytes per launch)
#   3. the same for the cfg3 training step (bench.py --mode train)
#   4. kernel stats of the 1-rank data-parallel step (bench.py --dp1-child)
#   5. MFMA busy of the cfg5 bf16 stress step (SQ_VALU_MFMA_BUSY_CYCLES and GRBM_GUI_ACTIVE, one pass
#      each; tools/pmc_mfma.py turns them into matrix-pipe utilisation per kernel)
# Every step under its own time limit; the script stops at the first failure.
set -e
OUT=${1:-gpurun_out/prof}
mkdir -p "$OUT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-dp1 > "$OUT/bench_under_rocprof.json" 2> "$OUT/bench_under_rocprof.err"
SERVE="python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-streams --no-eval --no-data --no-api --no-stress --train-steps 0 --no-cpu"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- $SERVE > "$OUT/fetch.json" 2> "$OUT/fetch.err"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- $SERVE > "$OUT/write.json" 2> "$OUT/write.err"
# 3. the cfg3 fused training step (single GPU), kernel stats + the same two PMC passes
TRAIN="python3 bench.py --gpus 1 --mode train --steps 64 --warmup 16 --no-cpu"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/train_trace" -o run -- $TRAIN > "$OUT/train_under_rocprof.json" 2> "$OUT/train_under_rocprof.err"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/train_fetch" -o run -- $TRAIN > "$OUT/train_fetch.json" 2> "$OUT/train_fetch.err"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/train_write" -o run -- $TRAIN > "$OUT/train_write.json" 2> "$OUT/train_write.err"
# 4. the data-parallel step's form on a 1-rank RCCL group (what every rank runs at N > 1)
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/dp1_trace" -o run -- \
    python3 bench.py --dp1-child --train-steps 400 > "$OUT/dp1_under_rocprof.json" 2> "$OUT/dp1_under_rocprof.err"
# 5. matrix-pipe utilisation of the cfg5 bf16 stress step
STRESS="python3 bench.py --gpus 1 --mode stress --steps 16 --warmup 4 --no-cpu"
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d "$OUT/stress_mfma" -o run -- $STRESS > "$OUT/stress_mfma.json" 2> "$OUT/stress_mfma.err"
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE --output-format csv -d "$OUT/stress_grbm" -o run -- $STRESS > "$OUT/stress_grbm.json" 2> "$OUT/stress_grbm.err"
echo profile-done

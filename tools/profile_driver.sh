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
#   6. the same MFMA-busy passes of the serve command (the headline k_serve6<4,3,2,10> and the lone
#      batch-64 request's kernel, both launched by it)
#   7. cfg5: which unit the bf16 GEMM saturates (LDS bank conflicts / LDS cycles / LDS issue stalls;
#      TA and TCP busy), one pass per counter block
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
# 6. matrix-pipe utilisation of the serve command's kernels
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d "$OUT/serve_mfma" -o run -- $SERVE > "$OUT/serve_mfma.json" 2> "$OUT/serve_mfma.err"
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE --output-format csv -d "$OUT/serve_grbm" -o run -- $SERVE > "$OUT/serve_grbm.json" 2> "$OUT/serve_grbm.err"
# 7. cfg5 unit counters (SQ block: LDS; TA / TCP blocks: the vector-memory address and data paths)
timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d "$OUT/stress_lds" -o run -- $STRESS > "$OUT/stress_lds.json" 2> "$OUT/stress_lds.err" || echo "stress_lds pass failed"
timeout -s KILL 60 rocprofv3 --pmc TA_TA_BUSY_sum TA_BUFFER_LOAD_WAVEFRONTS_sum --output-format csv -d "$OUT/stress_ta" -o run -- $STRESS > "$OUT/stress_ta.json" 2> "$OUT/stress_ta.err" || echo "stress_ta pass failed"
timeout -s KILL 60 rocprofv3 --pmc TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_GATE_EN1_sum TCP_TD_TCP_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum --output-format csv -d "$OUT/stress_tcp" -o run -- $STRESS > "$OUT/stress_tcp.json" 2> "$OUT/stress_tcp.err" || echo "stress_tcp pass failed"
echo profile-done

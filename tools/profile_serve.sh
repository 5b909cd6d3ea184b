#!/bin/bash
# The headline's profiles alone (steps 1, 2 and 6 of tools/profile_driver.sh): rocprofv3 kernel
# stats of the driver's command, the serve path's FETCH_SIZE / WRITE_SIZE passes, and its
# matrix-pipe busy passes -- for a change that touches only the serve kernels.  Stops at the first
# failure; every step under its own time limit.
set -e
OUT=${1:-gpurun_out/prof}
mkdir -p "$OUT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-dp1 > "$OUT/bench_under_rocprof.json" 2> "$OUT/bench_under_rocprof.err"
SERVE="python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-streams --no-eval --no-data --no-api --no-stress --train-steps 0 --no-cpu"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- $SERVE > "$OUT/fetch.json" 2> "$OUT/fetch.err"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- $SERVE > "$OUT/write.json" 2> "$OUT/write.err"
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d "$OUT/serve_mfma" -o run -- $SERVE > "$OUT/serve_mfma.json" 2> "$OUT/serve_mfma.err"
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE --output-format csv -d "$OUT/serve_grbm" -o run -- $SERVE > "$OUT/serve_grbm.json" 2> "$OUT/serve_grbm.err"
echo profile-done

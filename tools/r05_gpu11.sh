# round 5, GPU call 11: own-slice K-combine A/B, then rocprofv3 kernel stats + PMC passes of the
# driver's command, the cfg3 step, the 1-rank DP step and cfg5 (tools/profile_driver.sh)
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_t11
L=3d-pose-baseline_amd
tools/gpu_steps.sh $OUT \
 "!serve_own_ab|300|python -u tools/lib_ab.py $L/libp3d.so $L/libp3d_own.so 4 tools/serve_ab.py" \
 "!profile|1000|bash tools/profile_driver.sh $OUT/prof"

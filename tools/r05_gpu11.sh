# round 5, GPU call 11: rocprofv3 kernel stats + PMC passes of the driver's command, the cfg3 step,
# the 1-rank DP step and cfg5 (tools/profile_driver.sh)
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r05_t11
timeout -k 10 1000 bash tools/profile_driver.sh gpurun_out/r05_t11/prof > gpurun_out/r05_t11/profile.log 2>&1

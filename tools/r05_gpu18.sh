# round 5, GPU call 18: rocprofv3 kernel stats + PMC passes (tools/profile_driver.sh) on the round's
# final kernels
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r05_t18
timeout -k 10 1000 bash tools/profile_driver.sh gpurun_out/r05_t18/prof > gpurun_out/r05_t18/profile.log 2>&1

# round 5, GPU call 33: host-runtime knobs on the headline's timed region -- the host's active
# (spinning) wait for the completion signal (ROC_ACTIVE_WAIT_TIMEOUT) and kernel arguments in device
# memory (HIP_FORCE_DEV_KERNARG)
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_t33
tools/gpu_steps.sh $OUT \
 "!wait_ab|500|python -u tools/env_ab.py - ROC_ACTIVE_WAIT_TIMEOUT=1000 3 tools/serve_ab.py" \
 "!kernarg_ab|500|python -u tools/env_ab.py - HIP_FORCE_DEV_KERNARG=1 3 tools/serve_ab.py"

# round 5, GPU call 13: phase timeline of the fused weight-gradient launch
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_t13
L=3d-pose-baseline_amd
tools/gpu_steps.sh $OUT \
 "!trace_wgrad|120|P3D_LIB=\$PWD/$L/libp3d_trace.so python -u tools/trace_wgrad.py"

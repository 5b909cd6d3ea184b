# round 5, GPU call 15: k_serve6 phase trace with the output-phase and ring-fill stamps
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_t15
L=3d-pose-baseline_amd
tools/gpu_steps.sh $OUT \
 "!trace6|120|P3D_LIB=\$PWD/$L/libp3d_trace.so python -u tools/trace_serve6.py 20 10"

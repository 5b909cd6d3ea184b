# round 5, GPU call 24: timelines of the pair form (trace builds): plain and with the pipelined
# epilogue, and the single-unit form from the same build for reference
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_t24
T1=$PWD/3d-pose-baseline_amd/libp3d_trace_np.so
T2=$PWD/3d-pose-baseline_amd/libp3d_trace.so
tools/gpu_steps.sh $OUT \
 "!trace_pair|150|env P3D_LIB=$T1 P3D_SERVE6_PAIR=1 python -u tools/trace_serve6.py 20 10" \
 "!trace_pipe|150|env P3D_LIB=$T2 P3D_SERVE6_PAIR=1 python -u tools/trace_serve6.py 20 10" \
 "!trace_rt10|150|env P3D_LIB=$T1 P3D_SERVE6_PAIR=0 python -u tools/trace_serve6.py 20 10"

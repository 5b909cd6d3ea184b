# round 5, GPU call 27: timeline of the pair form with the ring running on across blocks (trace build)
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_t27
T=$PWD/3d-pose-baseline_amd/libp3d_trace.so
tools/gpu_steps.sh $OUT \
 "!trace_pair|150|env P3D_LIB=$T P3D_SERVE6_PAIR=1 python -u tools/trace_serve6.py 20 10" \
 "!trace_rt10|150|env P3D_LIB=$T P3D_SERVE6_PAIR=0 python -u tools/trace_serve6.py 20 10"

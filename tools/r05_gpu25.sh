# round 5, GPU call 25: the pair form, prologue without spills, flags polled ahead of the tail
# -- bitwise against the single-unit form, A/B of the serve line against the single-unit form
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_t25
PL=$PWD/3d-pose-baseline_amd/libp3d_pair.so
tools/gpu_steps.sh $OUT \
 "!paircheck|150|env P3D_LIB=$PL python -u tools/serve_pair_check.py" \
 "!pair_ab|500|env P3D_LIB=$PL python -u tools/env_ab.py P3D_SERVE6_PAIR=0 P3D_SERVE6_PAIR=1 4 tools/serve_ab.py" && \
tools/gpu_steps.sh $OUT \
 "!trace_pair|150|env P3D_LIB=$PWD/3d-pose-baseline_amd/libp3d_trace.so P3D_SERVE6_PAIR=1 python -u tools/trace_serve6.py 20 10"

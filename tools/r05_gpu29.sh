# round 5, GPU call 29: the pair form (committed sources) against the single-unit form, 6 rounds
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_t29
PL=$PWD/3d-pose-baseline_amd/libp3d_pair.so
tools/gpu_steps.sh $OUT \
 "!pair_ab|700|env P3D_LIB=$PL python -u tools/env_ab.py P3D_SERVE6_PAIR=0 P3D_SERVE6_PAIR=1 6 tools/serve_ab.py"

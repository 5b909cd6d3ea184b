# round 5, GPU call 26: the pair form with the ring running on across blocks
# -- bitwise against the single-unit form, A/B of the serve line against the single-unit form
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_t26
PL=$PWD/3d-pose-baseline_amd/libp3d_pair.so
tools/gpu_steps.sh $OUT \
 "!paircheck|150|env P3D_LIB=$PL python -u tools/serve_pair_check.py" \
 "!pair_ab|500|env P3D_LIB=$PL python -u tools/env_ab.py P3D_SERVE6_PAIR=0 P3D_SERVE6_PAIR=1 4 tools/serve_ab.py"

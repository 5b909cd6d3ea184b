# round 5, GPU call 22: the k_serve6 pair form (P3D_SERVE6_PAIR=1, libp3d_pair.so) -- bitwise against
# the single-unit form, A/B of the serve line, the serve tests under it
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_t22
PL=$PWD/3d-pose-baseline_amd/libp3d_pair.so
tools/gpu_steps.sh $OUT \
 "!paircheck|150|env P3D_LIB=$PL python -u tools/serve_pair_check.py" \
 "!pair_ab|500|env P3D_LIB=$PL python -u tools/env_ab.py P3D_SERVE6_PAIR=0 P3D_SERVE6_PAIR=1 4 tools/serve_ab.py" \
 "!pair_servetests|300|env P3D_LIB=$PL P3D_SERVE6_PAIR=1 python -u -m pytest tests/test_gpu_serve.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider"

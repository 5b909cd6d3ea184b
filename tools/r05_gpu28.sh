# round 5, GPU call 28: the output phase in two MFMA chains (every k_serve6 form) and the pair form:
# bitwise pair check, the serve tests on the new build, the new build against the previous one
# (single-unit form), and the pair form against the single-unit form
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_t28
PL=$PWD/3d-pose-baseline_amd/libp3d_pair.so
PV=$PWD/3d-pose-baseline_amd/libp3d_prev.so
tools/gpu_steps.sh $OUT \
 "!paircheck|150|env P3D_LIB=$PL python -u tools/serve_pair_check.py" \
 "!servetests|300|env P3D_LIB=$PL python -u -m pytest tests/test_gpu_serve.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider" \
 "!lib_ab|500|python -u tools/lib_ab.py $PV $PL 3 tools/serve_ab.py" \
 "!pair_ab|500|env P3D_LIB=$PL python -u tools/env_ab.py P3D_SERVE6_PAIR=0 P3D_SERVE6_PAIR=1 3 tools/serve_ab.py"

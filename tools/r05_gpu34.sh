# round 5, GPU call 34: the pair form for 128-row-per-XCD launches too (16 steps: two 64-row units,
# k_serve6<4,3,2,4,true>) -- bitwise check, the serve tests, A/B at 16 steps
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_t34
PL=$PWD/3d-pose-baseline_amd/libp3d_pair.so
tools/gpu_steps.sh $OUT \
 "!paircheck|150|env P3D_LIB=$PL python -u tools/serve_pair_check.py" \
 "!servetests|300|env P3D_LIB=$PL python -u -m pytest tests/test_gpu_serve.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider" \
 "!ab16|500|env P3D_LIB=$PL python -u tools/env_ab.py P3D_SERVE6_PAIR=0 P3D_SERVE6_PAIR=1 4 tools/serve_ab.py --steps 16"

# round 5, GPU call 19: the weight-gradient grid with its small layers dispatched last, A/B and the
# fused/unfused bit-identity tests
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_t19
tools/gpu_steps.sh $OUT \
 '!train_tests|300|python -u -m pytest tests/test_gpu_parity.py -q -x -k "fused_train_step or train_step" --timeout 120 --timeout-method thread -p no:cacheprovider' \
 '!train_small_ab|300|python -u tools/env_ab.py P3D_WGRAD_SMALL_LAST=0 P3D_WGRAD_SMALL_LAST=1 4 tools/train_ab.py'

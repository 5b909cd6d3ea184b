# round 5, GPU call 12: the attached weight-gradient form (layer l+1's dW + Adam tiles riding layer
# l's data-gradient launch; 256-thread workgroups so a data-gradient tile and a weight-gradient
# tile share a CU) against the default tail launch; its bit-identity test first
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_t12
tools/gpu_steps.sh $OUT \
 '!attach_tests|300|python -u -m pytest tests/test_gpu_parity.py -q -x -k "fused_train_step_bit_identical" --timeout 120 --timeout-method thread -p no:cacheprovider' \
 '!train_attach_ab|300|python -u tools/env_ab.py P3D_WGRAD_ATTACH=0 P3D_WGRAD_ATTACH=1 3 tools/train_ab.py'

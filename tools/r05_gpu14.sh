# round 5, GPU call 14: the fused Adam's w / m / v requested before the contraction (1 or 2 of a
# thread's 4 rows) against the default, with the weight-gradient trace of the 2-row form
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_t14
L=3d-pose-baseline_amd
tools/gpu_steps.sh $OUT \
 "!train_we2_ab|300|python -u tools/lib_ab.py $L/libp3d.so $L/libp3d_we2.so 3 tools/train_ab.py" \
 "!train_we1_ab|300|python -u tools/lib_ab.py $L/libp3d.so $L/libp3d_we1.so 3 tools/train_ab.py"

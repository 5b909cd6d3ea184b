# round 5, GPU call 32: block 0's weight slots before the input hand-off, the output weights under
# the last store drain (libp3d_pair.so) -- bitwise check, A/B against the final tree's library
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_t32
PL=$PWD/3d-pose-baseline_amd/libp3d_pair.so
PV=$PWD/3d-pose-baseline_amd/libp3d_prev.so
tools/gpu_steps.sh $OUT \
 "!paircheck|150|env P3D_LIB=$PL python -u tools/serve_pair_check.py" \
 "!lib_ab|600|python -u tools/lib_ab.py $PV $PL 5 tools/serve_ab.py"

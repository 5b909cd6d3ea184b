# round 5, GPU call 8: the kernel-argument fetch probe, the fused weight-gradient kernel at 5 vs 4
# workgroups per CU, the phase trace of the default build, then the GPU suite
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_t8
L=3d-pose-baseline_amd
tools/gpu_steps.sh $OUT \
 '!kernarg_probe|60|tools/kernarg_probe' \
 "!train_wg_ab|300|python -u tools/lib_ab.py $L/libp3d_wg4.so $L/libp3d.so 3 tools/train_ab.py" \
 "!trace6|120|P3D_LIB=\$PWD/$L/libp3d_trace.so python -u tools/trace_serve6.py 20 10" \
 '!gputests|600|python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider'

# round 5, GPU call 16: the output-weight prefetch issued after the flag publish (vs before the
# drain), all four first weight slots prefetched off-contraction (PD = 4), trace of the new build
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_t16
L=3d-pose-baseline_amd
tools/gpu_steps.sh $OUT \
 '!serve_tests|300|python -u -m pytest tests/test_gpu_serve.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider' \
 "!serve_pub_ab|300|python -u tools/lib_ab.py $L/libp3d_prev.so $L/libp3d.so 4 tools/serve_ab.py" \
 "!serve_pd4_ab|300|python -u tools/lib_ab.py $L/libp3d.so $L/libp3d_pd4.so 4 tools/serve_ab.py" \
 "!trace6|120|P3D_LIB=\$PWD/$L/libp3d_trace.so python -u tools/trace_serve6.py 20 10"

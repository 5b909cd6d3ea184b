# round 5, GPU call 3: k_serve6 with the output layer as its own phase (tests, A/B against the
# previous build, phase trace) and the direct-load bf16 GEMM (tests, A/B against k_gemm_bf16p)
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_t3
tools/gpu_steps.sh $OUT \
 '!serve_tests|300|python -u -m pytest tests/test_gpu_serve.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider' \
 '!bf16_tests|300|python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "bf16" --timeout 120 --timeout-method thread -p no:cacheprovider' \
 '!serve_ab|400|python -u tools/lib_ab.py 3d-pose-baseline_amd/libp3d_base.so 3d-pose-baseline_amd/libp3d.so 4 tools/serve_ab.py' \
 '!stress_ab|300|python -u tools/env_ab.py P3D_BF16_DIRECT=0 P3D_BF16_DIRECT=1 3 tools/stress_ab.py' \
 '!trace6|120|P3D_LIB=$PWD/3d-pose-baseline_amd/libp3d_trace.so python -u tools/trace_serve6.py 20 10'

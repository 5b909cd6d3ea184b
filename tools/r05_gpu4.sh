# round 5, GPU call 4: k_serve6 output-phase A/B + trace; then the bf16 tests (the direct-load form
# last, with the runtime's error log on) and the cfg5 A/B
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_t4
md5sum 3d-pose-baseline_amd/*.so > $OUT.md5 2>/dev/null || true
tools/gpu_steps.sh $OUT \
 '!serve_ab|400|python -u tools/lib_ab.py 3d-pose-baseline_amd/libp3d_base.so 3d-pose-baseline_amd/libp3d.so 4 tools/serve_ab.py' \
 '!trace6|120|P3D_LIB=$PWD/3d-pose-baseline_amd/libp3d_trace.so python -u tools/trace_serve6.py 20 10' \
 '!bf16_tests|300|python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "bf16 and not direct" --timeout 120 --timeout-method thread -p no:cacheprovider' \
 '!direct_tests|200|AMD_LOG_LEVEL=1 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -x -k "bf16_direct and 512" --timeout 120 --timeout-method thread -p no:cacheprovider'

# round 5, GPU call 5: output-phase fix A/B (base -> wg), late epoch A/B (wg -> le), 4-deep
# activation ring A/B (le -> da4), argument pinning A/B (le -> pin -> cpin), fused weight-gradient at 4 per CU A/B (base -> wg), cfg5
# direct-load A/B, phase trace, the GPU suite
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_t5
L=3d-pose-baseline_amd
tools/gpu_steps.sh $OUT \
 "!serve_ab|400|python -u tools/lib_ab.py $L/libp3d_base.so $L/libp3d_wg.so 3 tools/serve_ab.py" \
 "!serve_le_ab|400|python -u tools/lib_ab.py $L/libp3d_wg.so $L/libp3d_le.so 3 tools/serve_ab.py" \
 "!serve_pin_ab|400|python -u tools/lib_ab.py $L/libp3d_le.so $L/libp3d_pin.so 3 tools/serve_ab.py" \
 "!serve_cpin_ab|400|python -u tools/lib_ab.py $L/libp3d_pin.so $L/libp3d_cpin.so 3 tools/serve_ab.py" \
 "!serve_da4_ab|400|python -u tools/lib_ab.py $L/libp3d_le.so $L/libp3d_da4.so 3 tools/serve_ab.py" \
 "!train_ab|400|python -u tools/lib_ab.py $L/libp3d_base.so $L/libp3d_wg.so 3 tools/train_ab.py" \
 '!stress_ab|300|python -u tools/env_ab.py P3D_BF16_DIRECT=0 P3D_BF16_DIRECT=1 3 tools/stress_ab.py' \
 "!trace6|120|P3D_LIB=\$PWD/$L/libp3d_trace.so python -u tools/trace_serve6.py 20 10" \
 '!gputests|600|python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider'

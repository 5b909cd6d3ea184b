# round 5, GPU call 10: regression A/B of the serve prologue change, the GPU suite, smoke, the
# driver's bench command on the round's kernels, phase trace
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_t10
L=3d-pose-baseline_amd
tools/gpu_steps.sh $OUT \
 "!serve_pf2_ab|300|python -u tools/lib_ab.py $L/libp3d_prev.so $L/libp3d.so 4 tools/serve_ab.py" \
 '!gputests|600|python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider' \
 '!smoke|300|python -u -c "import __graft_entry__ as g; g.smoke(); print(\"smoke-ok\")"' \
 '!driver_bench|400|python3 -u bench.py --gpus 1 --steps 20 --warmup 5' \
 "!trace6|120|P3D_LIB=\$PWD/$L/libp3d_trace.so python -u tools/trace_serve6.py 20 10"

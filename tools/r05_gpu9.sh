# round 5, GPU call 9: serve prologue A/B (clamped unconditional first-unit requests vs the previous
# build), phase trace, the GPU suite, the driver's bench command on the round's kernels
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_t9
L=3d-pose-baseline_amd
tools/gpu_steps.sh $OUT \
 "!serve_pf_ab|300|python -u tools/lib_ab.py $L/libp3d_prev.so $L/libp3d.so 5 tools/serve_ab.py" \
 "!trace6|120|P3D_LIB=\$PWD/$L/libp3d_trace.so python -u tools/trace_serve6.py 20 10" \
 '!gputests|600|python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider' \
 '!smoke|300|python -u -c "import __graft_entry__ as g; g.smoke(); print(\"smoke-ok\")"' \
 '!driver_bench|400|python -u bench.py'

# round 5, GPU call 35: the final tree -- the GPU
# suite, smoke, the driver's bench command
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_t35
tools/gpu_steps.sh $OUT \
 '!gputests|700|python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider' \
 '!smoke|300|python -u -c "import __graft_entry__ as g; g.smoke(); print(\"smoke-ok\")"' \
 '!driver_bench|400|python3 -u bench.py --gpus 1 --steps 20 --warmup 5' \
 '!pair_check|150|python -u tools/serve_pair_check.py'

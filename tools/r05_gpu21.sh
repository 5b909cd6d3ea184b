# round 5, GPU call 21: the GPU suite and smoke on the tree as it stands (rendezvous ports now below
# the ephemeral range), and the driver's bench command
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_t21
tools/gpu_steps.sh $OUT \
 '!gputests|600|python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider' \
 '!smoke|300|python -u -c "import __graft_entry__ as g; g.smoke(); print(\"smoke-ok\")"' \
 '!driver_bench|400|python3 -u bench.py --gpus 1 --steps 20 --warmup 5'

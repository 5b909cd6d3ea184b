# round 5, GPU call 30: the pair form as the default -- the GPU suite, smoke, the driver's bench
# command, and the headline's profiles (tools/profile_serve.sh)
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_t30
tools/gpu_steps.sh $OUT \
 '!gputests|700|python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider' \
 '!smoke|300|python -u -c "import __graft_entry__ as g; g.smoke(); print(\"smoke-ok\")"' \
 '!driver_bench|400|python3 -u bench.py --gpus 1 --steps 20 --warmup 5' \
 '!profile|900|bash tools/profile_serve.sh gpurun_out/r05_t30/prof'

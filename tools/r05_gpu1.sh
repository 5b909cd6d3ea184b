set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
tools/gpu_steps.sh gpurun_out/r05_t1 \
 '!gputests|900|python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider' \
 '!smoke|120|python -u -c "import __graft_entry__ as g; g.smoke()"' \
 '!bench|300|python3 bench.py --gpus 1 --steps 20 --warmup 5'

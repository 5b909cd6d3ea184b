# round 5, GPU call 20: output phase writing only its live tiles to LDS (A/B), then the GPU suite and
# smoke on the tree as it stands
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_t20
L=3d-pose-baseline_amd
tools/gpu_steps.sh $OUT \
 "!serve_live_ab|300|python -u tools/lib_ab.py $L/libp3d_prev.so $L/libp3d.so 4 tools/serve_ab.py" \
 '!gputests|600|python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider' \
 '!smoke|300|python -u -c "import __graft_entry__ as g; g.smoke(); print(\"smoke-ok\")"'

set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/ -x -q -m gpu > gpurun_out/t5.log 2>&1 || { tail -40 gpurun_out/t5.log; exit 1; }
tail -1 gpurun_out/t5.log
timeout -k 10 300 python bench.py --streams 1 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json

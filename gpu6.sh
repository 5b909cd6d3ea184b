set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k bf16 > gpurun_out/t6.log 2>&1 || { tail -40 gpurun_out/t6.log; exit 1; }
tail -1 gpurun_out/t6.log
timeout -k 10 300 python bench.py --mode stress --steps 64 --warmup 16 > gpurun_out/bench_stress.json 2> gpurun_out/bench_stress.err || { tail -20 gpurun_out/bench_stress.err; exit 1; }
cat gpurun_out/bench_stress.json

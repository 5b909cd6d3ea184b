set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k bf16 > gpurun_out/t7.log 2>&1 || { tail -40 gpurun_out/t7.log; exit 1; }
tail -1 gpurun_out/t7.log
for S in 2 3 4; do
P3D_BF16_STAGES=$S timeout -k 10 300 python bench.py --mode stress --steps 64 --warmup 16 > gpurun_out/bs$S.json 2> gpurun_out/bs$S.err || { tail -20 gpurun_out/bs$S.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bs$S.json'));print($S, d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline']['avg_us'])"
done

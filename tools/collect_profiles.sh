#!/bin/bash
# Copy the summaries of one tools/profile_driver.sh run into profiles/ (tracked):
#   tools/collect_profiles.sh gpurun_out/<call>/prof r05_v1
set -e
P=$1
T=profiles/$2
cp "$P/trace/run_kernel_stats.csv" "${T}_bench_kernel_stats.csv"
cp "$P/bench_under_rocprof.json" "${T}_bench_under_rocprof.json"
cp "$P/train_trace/run_kernel_stats.csv" "${T}_train_kernel_stats.csv"
cp "$P/train_under_rocprof.json" "${T}_train_under_rocprof.json"
cp "$P/dp1_trace/run_kernel_stats.csv" "${T}_dp1_kernel_stats.csv"
cp "$P/dp1_under_rocprof.json" "${T}_dp1_under_rocprof.json"
python tools/pmc_traffic.py "$P/fetch" "$P/write" serve --config mode=infer --config steps_per_launch=20 > "${T}_pmc_traffic_serve.json"
python tools/pmc_traffic.py "$P/train_fetch" "$P/train_write" --config mode=train --config batch=64 > "${T}_pmc_traffic_train.json"
python tools/pmc_mfma.py "$P/serve_mfma" "$P/serve_grbm" serve6 > "${T}_pmc_mfma_serve.json"
python tools/pmc_mfma.py "$P/stress_mfma" "$P/stress_grbm" bf16 > "${T}_pmc_mfma_stress.json"
python tools/pmc_units.py "$P" bf16p > "${T}_pmc_units_stress.json"
ls -la ${T}_*

# round 5, GPU call 2: GPU tests on the rebuilt library, a k_serve6 phase trace (-DP3D_TRACE build),
# the rocprofv3 driver profiles (kernel stats, FETCH/WRITE, MFMA-busy of serve and cfg5, cfg5 unit
# counters), the counter list
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_t2
tools/gpu_steps.sh $OUT \
 '!gputests|600|python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider' \
 '!trace6|120|P3D_LIB=$PWD/3d-pose-baseline_amd/libp3d_trace.so python -u tools/trace_serve6.py 20 10' \
 'counters|60|rocprofv3 -L' \
 '!profile|900|bash tools/profile_driver.sh gpurun_out/r05_t2/prof'

# round 5, GPU call 7: A/Bs of the k_serve6 / k_gemv_chain / layer-kernel options against the default
# build (more rounds where call 6 was within noise), the work-copy phase trace, then the GPU suite
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_t7
L=3d-pose-baseline_amd
tools/gpu_steps.sh $OUT \
 "!serve_pin_ab|300|python -u tools/lib_ab.py $L/libp3d_nopin.so $L/libp3d.so 5 tools/serve_ab.py" \
 "!b1_pin_ab|300|python -u tools/lib_ab.py $L/libp3d_nopin.so $L/libp3d.so 3 tools/b1_ab.py" \
 "!serve_pre_ab|300|python -u tools/lib_ab.py $L/libp3d_nopre.so $L/libp3d.so 4 tools/serve_ab.py" \
 "!serve_comb_ab|300|python -u tools/lib_ab.py $L/libp3d.so $L/libp3d_comb.so 4 tools/serve_ab.py" \
 "!train_lay_ab|300|python -u tools/lib_ab.py $L/libp3d.so $L/libp3d_lay.so 3 tools/train_ab.py" \
 "!serve_da4_ab|300|python -u tools/lib_ab.py $L/libp3d.so $L/libp3d_da4.so 3 tools/serve_ab.py" \
 "!trace6w|120|P3D_LIB=\$PWD/$L/libp3d_trace_w.so python -u tools/trace_serve6.py 20 10" \
 '!gputests|600|python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider'

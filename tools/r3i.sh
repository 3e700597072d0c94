set -e
O=gpurun_out/r3j; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "conv or deconv or upsample" > $O/t_conv.log 2>&1
KB_F16_ONLY=1 KB_CONV_TILES=auto,h2,h2s3 timeout -k 10 300 python -u tools/kbench.py conv > $O/kb_conv.log 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/b_new1.json 2>/dev/null
RF_CONV_HALO2=0 timeout -k 10 200 python bench.py --no-cpu-baseline > $O/b_old1.json 2>/dev/null
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/b_new2.json 2>/dev/null
RF_CONV_HALO2=0 timeout -k 10 200 python bench.py --no-cpu-baseline > $O/b_old2.json 2>/dev/null
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_parity_gpu.py -k "baseline_configs or production_taps" > $O/t_parity.log 2>&1
echo ok

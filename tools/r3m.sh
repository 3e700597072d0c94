set -e
O=gpurun_out/r3m; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "conv_halo2 or final_head" > $O/t.log 2>&1
KB_F16_ONLY=1 KB_CONV_TILES=h2,h2s3,h2s5,h2db3 timeout -k 10 300 python -u tools/kbench.py conv > $O/kb.log 2>&1
echo ok

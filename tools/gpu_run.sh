set -e
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py tests/test_parity_gpu.py -q -x > gpurun_out/t.log 2>&1
timeout -k 10 300 python tools/kbench.py gemm > gpurun_out/kb_gemm.log 2>&1

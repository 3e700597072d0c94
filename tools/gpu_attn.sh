set -e
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py -q -x -k "attn or attention or swin or gemm" > gpurun_out/t.log 2>&1
for k in 3 28 2; do RF_ATTN_KERNEL=$k timeout -k 10 200 python tools/kbench.py attn > gpurun_out/kb_$k.log 2>&1; done
timeout -k 10 300 python tools/kbench.py gemm > gpurun_out/kb_gemm.log 2>&1

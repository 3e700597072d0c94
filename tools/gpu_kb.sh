set -e
mkdir -p gpurun_out
timeout -k 10 300 python tools/kbench.py ${1:-gemm} > gpurun_out/kb_${1:-gemm}.log 2>&1

# A/B: current library vs renderformer_amd/lib/librfhip_old.so on the same box (kbench $1)
set -e
mkdir -p gpurun_out
timeout -k 10 300 python tools/kbench.py ${1:-gemm} > gpurun_out/kb_A.log 2>&1
RF_LIB=$PWD/renderformer_amd/lib/librfhip_old.so timeout -k 10 300 python tools/kbench.py ${1:-gemm} > gpurun_out/kb_B.log 2>&1
timeout -k 10 300 python tools/kbench.py ${1:-gemm} > gpurun_out/kb_A2.log 2>&1

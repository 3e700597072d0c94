# kernel micro-benchmarks: bash tools/gpu_kb.sh <tag> <kbench mode> (env KB_* passed through)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-kb}
mkdir -p $O
cd $R
timeout -k 10 600 python -u tools/kbench.py ${2:-gemm} > $O/kb.log 2>&1
echo done

# A/B of two builds of librfhip on the attention kernel: bash tools/gpu_libab.sh <tag> <old.so>
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-libab}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attn or attention" -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1
for i in 1 2; do
ABL=0 RF_LIB=$R/$2 timeout -k 10 200 python tools/attn_ablate.py > $O/old$i.log 2>&1
ABL=0 timeout -k 10 200 python tools/attn_ablate.py > $O/new$i.log 2>&1
done
echo done

set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-split}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "attn or attention" -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1
ABL=0,512,0,512 timeout -k 10 300 python tools/attn_ablate.py > $O/abl.log 2>&1
timeout -k 10 300 python tools/attn_ablate.py stamps 32 > $O/st_split.log 2>&1
timeout -k 10 300 python tools/attn_ablate.py stamps 288 > $O/st_unsplit.log 2>&1
echo done

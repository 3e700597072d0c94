set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-st}
mkdir -p $O
cd $R
timeout -k 10 120 python tools/attn_ablate.py stamps 32 > $O/stamps.log 2>&1
echo done

set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-sk}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attention or swin" -x -q --timeout 120 --timeout-method thread > $O/t_attn.log 2>&1
timeout -k 10 120 python tools/attn_ablate.py stamps 32 > $O/stamps.log 2>&1
timeout -k 10 120 python tools/attn_ablate.py stamps 96 >> $O/stamps.log 2>&1
timeout -k 10 300 python tools/attn_ablate.py > $O/ablate.log 2>&1
echo done

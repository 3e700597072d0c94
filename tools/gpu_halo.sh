set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-halo}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "conv or dpt" -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1
KB_F16_ONLY=1 KB_CONV_TILES=128,1288,256,auto RF_CONV_HALO=1 timeout -k 10 300 python tools/kbench.py conv > $O/kb_halo.log 2>&1
KB_F16_ONLY=1 KB_CONV_TILES=auto RF_CONV_HALO=0 timeout -k 10 300 python tools/kbench.py conv > $O/kb_gather.log 2>&1
echo done

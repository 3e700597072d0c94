set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-cv}
mkdir -p $O
cd $R
KB_F16_ONLY=1 KB_CONV_GEMM=1 KB_CONV_TILES=256,256ph,auto timeout -k 10 300 python tools/kbench.py conv > $O/kb_conv.log 2>&1
echo done

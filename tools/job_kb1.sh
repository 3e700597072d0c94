set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/fold; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "upsample or border or final_head or conv_halo2" > $O/t_k.log 2>&1
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_parity_gpu.py > $O/t_parity.log 2>&1
for v in 1 0; do
(cd /tmp && TMPDIR=/tmp RF_DPT_FOLD=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof$v -o run -- python3 $R/bench.py --profile --steps 5 --warmup 2 --no-cpu-baseline > $O/prof$v.log 2>&1)
python3 tools/prof_summary.py $(find $O/prof$v -name '*.db' -print -quit) 7 60 > $O/summary$v.txt 2>&1 || true
done
bash tools/gpu.sh ab fold "RF_DPT_FOLD=1" "RF_DPT_FOLD=0"
echo ok

set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/small4; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "conv or deconv" > $O/t_conv.log 2>&1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_parity_gpu.py -k "baseline_configs or production_taps or pipeline_matches" > $O/t_parity.log 2>&1
for v in 1 0; do
(cd /tmp && TMPDIR=/tmp RF_CONV_SMALL=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof$v -o run -- python3 $R/bench.py --profile --steps 5 --warmup 2 --no-cpu-baseline > $O/prof$v.log 2>&1)
python3 tools/prof_summary.py $(find $O/prof$v -name '*.db' -print -quit) 7 60 > $O/summary$v.txt 2>&1 || true
done
bash tools/gpu.sh ab small4 "RF_CONV_SMALL=1" "RF_CONV_SMALL=0"
echo ok

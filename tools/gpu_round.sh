# Full round check on one GPU box: gpu tests, bench (with CPU baseline), kernel-trace stats,
# and the two HBM-traffic PMC passes (FETCH_SIZE / WRITE_SIZE each in its own run).
# usage: bash tools/gpu_round.sh <tag>
set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-run}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --profile --steps 5 --warmup 2 > $O/prof.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --profile --steps 2 --warmup 1 > $O/pmc_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --profile --steps 2 --warmup 1 > $O/pmc_write.log 2>&1
cd $R
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python tools/attn_ablate.py stamps > $O/attn_clock.log 2>&1
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_mfma -o run -- python3 $R/tools/attn_ablate.py pmc 5 > $O/pmc_mfma.log 2>&1
echo done

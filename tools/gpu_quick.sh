# Quick GPU check: gpu tests, bench, kernel-trace stats.  usage: bash tools/gpu_quick.sh <tag> [bench args]
set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-run}; shift || true
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rP > $O/tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py "$@" > $O/bench.json 2> $O/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --profile --steps 5 --warmup 2 "$@" > $O/prof.log 2>&1
echo done

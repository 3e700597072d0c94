# kernel micro-bench sweep: bash tools/gpu_kb2.sh <tag> <what...>
set -e
R=$GRAFT_REPO_ROOT
TAG=$1; shift
mkdir -p $R/gpurun_out/$TAG
for W in "$@"; do
  timeout -k 10 400 python tools/kbench.py $W > $R/gpurun_out/$TAG/kb_$W.log 2>&1
done

# A/B of one env switch on the full bench in one call: bash tools/gpu_ab.sh <tag> "<envA>" "<envB>"
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-ab}
mkdir -p $O
cd $R
for i in 1 2; do
env $2 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_a$i.json 2> $O/bench_a.err
env $3 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_b$i.json 2> $O/bench_b.err
done
echo done

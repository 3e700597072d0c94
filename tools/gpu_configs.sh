# other SURVEY 8d configurations on one GPU (no CPU baseline): bunny N, 1024^2, multi-view, batched scenes
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-cfg}
mkdir -p $O
cd $R
timeout -k 10 200 python bench.py --no-cpu-baseline --tris 6209 > $O/bunny.json 2> $O/bunny.err
timeout -k 10 300 python bench.py --no-cpu-baseline --res 1024 --steps 5 --warmup 2 > $O/r1024.json 2> $O/r1024.err
timeout -k 10 300 python bench.py --no-cpu-baseline --views 4 --steps 5 --warmup 2 > $O/v4.json 2> $O/v4.err
timeout -k 10 300 python bench.py --no-cpu-baseline --scenes 4 --steps 5 --warmup 2 > $O/s4.json 2> $O/s4.err
timeout -k 10 200 python bench.py --no-cpu-baseline --config base --res 256 > $O/base256.json 2> $O/base256.err
echo done

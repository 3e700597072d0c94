set -e
O=gpurun_out/r3c; mkdir -p $O
T="python -u -m pytest -x -q --timeout 900 --timeout-method thread"
timeout -k 10 900 $T tests/test_examples.py -m gpu -s > $O/t_ex.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
timeout -k 10 600 python bench.py --no-cpu-baseline --workload c4 --steps 2 --warmup 1 > $O/c4.json 2> $O/c4.err
timeout -k 10 600 python bench.py --no-cpu-baseline --workload c5 --steps 2 --warmup 1 > $O/c5.json 2> $O/c5.err
timeout -k 10 600 python bench.py --no-cpu-baseline --workload c5 --view-chunk 3 --steps 2 --warmup 1 > $O/c5_3.json 2>> $O/c5.err
timeout -k 10 600 python bench.py --no-cpu-baseline --workload c5 --view-chunk 24 --steps 2 --warmup 1 > $O/c5_all.json 2>> $O/c5.err
echo ok

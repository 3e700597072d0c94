set -e
O=gpurun_out/r3d; mkdir -p $O
T="python -u -m pytest -x -q --timeout 600 --timeout-method thread"
timeout -k 10 600 $T tests/test_kernels_gpu.py -k "f16 or rmsnorm or swin or gemm_f32" > $O/t_kern.log 2>&1
timeout -k 10 900 $T tests/test_parity_gpu.py -k "production_taps or baseline_configs or pipeline_matches" -s > $O/t_par.log 2>&1 || true
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
RF_OPERANDS=bf16 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_bf16.json 2>> $O/bench.err
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench2.json 2>> $O/bench.err
echo ok

set -e
O=gpurun_out/r2s4_sk2; mkdir -p $O
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_kernels_gpu.py tests/test_parity_gpu.py -k "attention or attn or stream or parity or baseline" > $O/t_attn.log 2>&1
ABL=0,u,512 timeout -k 10 200 python tools/attn_ablate.py > $O/ablate.log 2>&1
timeout -k 10 120 python tools/attn_ablate.py stamps 32 > $O/stamps_sched.log 2>&1
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_s$i.json 2>>$O/bench.err
  RF_ATTN_SCHED=0 timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_u$i.json 2>>$O/bench.err
done
echo done

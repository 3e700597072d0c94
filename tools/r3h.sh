set -e
O=gpurun_out/r3h; mkdir -p $O
export KB_SHAPES="s1 qkv,s1 out,s1 w2,s2 q,s2 out,s2 w2"
timeout -k 10 300 python -u tools/kbench.py coldgemm > $O/cold_auto.log 2>&1
RF_GEMM_SKPH=1 timeout -k 10 300 python -u tools/kbench.py coldgemm > $O/cold_skph.log 2>&1
unset KB_SHAPES
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/b_a1.json 2>/dev/null
RF_GEMM_SKPH=1 timeout -k 10 200 python bench.py --no-cpu-baseline > $O/b_b1.json 2>/dev/null
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/b_a2.json 2>/dev/null
RF_GEMM_SKPH=1 timeout -k 10 200 python bench.py --no-cpu-baseline > $O/b_b2.json 2>/dev/null
echo ok

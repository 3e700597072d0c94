# One runner for every GPU-box job (run through gpurun from the repo root):
#   bash tools/gpu.sh <task> <tag> [args...]      outputs under gpurun_out/<tag>/
# tasks
#   check            GPU test suite + default bench (20 steps)
#   round            round evidence: tests, bench (+ CPU baseline), smoke, kernel-trace stats, HBM traffic
#                    (FETCH_SIZE / WRITE_SIZE, one --pmc pass each), attention MFMA counters and in-kernel clock
#   roundnt          the same without the GPU test suite (run `check` or the suite on its own first)
#   prof [bench args]  rocprofv3 kernel-trace stats of a short bench run
#   trace            kernel + HIP API + memory-copy trace of a 2-frame bench run (no counters)
#   attn             attention GPU tests, ablation timings, per-segment stamps
#   ab "<envA>" "<envB>"   the bench twice under each of two env settings, interleaved
#   kb <mode>...     tools/kbench.py micro-benchmarks (KB_* env passed through)
#   configs          the other SURVEY 8d configurations (bunny, 1024^2, 4 views, 4 scenes, v1-base 256^2)
#   c5               config 5 (24 views at 1024^2), bf16 and MX fp8
#   pmc <script args...>   SQ counter passes (one rocprofv3 run each) over one python command
#   l2               per-kernel L2 hit rates of a short bench run (TCC_HIT_sum / TCC_MISS_sum, tools/pmc_l2.py)
#   attnab           attention GPU tests, then interleaved ablation timings of the RF_ATTN_DBG variants in $ABL
#   fold             the DPT fold A/B: kernel-trace of the frame with RF_DPT_FOLD=1 and 0, then the bench A/B
#   c4               config 4: bench.py --workload c4 (64 example scenes) and batch_infer.py end to end (tools/batch_e2e.py)
#   new              GPU tests of this round's new kernels / entry points (4-wave GEMM, hk conv, native stages), the
#                    quad GEMM study leg, then a kernel-trace profile of the default bench
#   vpmc [legs]      kbench legs (default: vendor) under FETCH / WRITE / L2-hit / MFMA-busy counter passes
#   convab           halo2 vs conv3x3_hk_kernel on the 512^2 / 256^2 DPT convolutions
#   libab            the current library vs $BASE (default renderformer_amd/lib/librfhip_base.so, a build of another
#                    tree): GPU tests on the current one, then interleaved stage-1 attention timings, per-role stamps
#                    and bench runs of both (RF_LIB selects the library)
#   pnab             the deferred RMSNorm: GPU tests, kbench prenorm A/B vs $BASE, interleaved bench runs of both
#   libkb            kbench prenorm + bench of this library and $BASE, interleaved
#   quadstudy        tools/kbench.py quad on the study build: the 4-wave GEMM at MT128x192 / MT160x256 (register or
#                    LDS-DMA staging, whole tiles or stream-K) vs the default engine on the projection shapes
#   swin             Swin / q/k-norm-fold GPU tests, kernel-trace profile and one run of the default bench
#   profab           kernel-trace profiles of the default bench under each env setting in $ENVS (';'-separated)
#   vendor           kernel-trace of the vendor GEMM library vs the engine on the frame's projection shapes
#                    (tools/kbench.py vendor: study only, nothing of it is linked into librfhip)
# Every GPU step runs under its own timeout and the steps are chained with && (set -e): the first failure
# (fault, abort, time limit) ends the job.
set -e
TASK=$1
TAG=${2:-$1}
shift 2 || shift $#
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
prof_run() {  # rocprofv3 needs a cwd and TMPDIR it can write
    (cd /tmp && TMPDIR=/tmp "$@")
}
case $TASK in
check)
    timeout -k 10 900 $T tests -m gpu > $O/tests.log 2>&1
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err ;;
round|roundnt)
    if [ $TASK = round ]; then timeout -k 10 900 $T tests -m gpu > $O/tests.log 2>&1; fi
    timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
    prof_run timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --profile --steps 5 --warmup 2 > $O/prof.log 2>&1
    prof_run timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --profile --steps 2 --warmup 1 > $O/pmc_fetch.log 2>&1
    prof_run timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --profile --steps 2 --warmup 1 > $O/pmc_write.log 2>&1
    RF_TRAFFIC_OUT=$O/attn_stage1_traffic.json python tools/pmc_traffic.py $(find $O/pmc_fetch -name '*counter_collection.csv' -print -quit) $(find $O/pmc_write -name '*counter_collection.csv' -print -quit) $O/pmc_traffic.json > $O/pmc_traffic.txt 2>&1
    STUDY=$R/renderformer_amd/lib/librfhip_study.so  # the stamp build (RF_ATTN_DBG=32) is a study variant
    if [ -f $STUDY ]; then RF_LIB=$STUDY timeout -k 10 300 python tools/attn_ablate.py stamps > $O/attn_clock.log 2>&1; fi
    prof_run timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_mfma -o run -- python3 $R/tools/attn_ablate.py pmc 5 > $O/pmc_mfma.log 2>&1 ;;
prof)
    prof_run timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --profile --steps 5 --warmup 2 "$@" > $O/prof.log 2>&1 ;;
trace)
    prof_run timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --memory-copy-trace -d $O/trace -o run -- python3 $R/bench.py --profile --steps 2 --warmup 1 > $O/trace.log 2>&1 ;;
attn)
    timeout -k 10 300 $T tests/test_kernels_gpu.py -k "attention or swin or attn" > $O/t_attn.log 2>&1
    timeout -k 10 300 python tools/attn_ablate.py > $O/ablate.log 2>&1
    timeout -k 10 120 python tools/attn_ablate.py stamps 32 > $O/stamps.log 2>&1 ;;
ab)
    for i in 1 2; do
        env $1 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_a$i.json 2>> $O/bench.err
        env $2 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_b$i.json 2>> $O/bench.err
    done ;;
kb)
    for W in "$@"; do timeout -k 10 400 python -u tools/kbench.py $W > $O/kb_$W.log 2>&1; done ;;
configs)
    timeout -k 10 200 python bench.py --no-cpu-baseline --tris 6209 > $O/bunny.json 2> $O/configs.err
    timeout -k 10 300 python bench.py --no-cpu-baseline --res 1024 --steps 5 --warmup 2 > $O/r1024.json 2>> $O/configs.err
    timeout -k 10 300 python bench.py --no-cpu-baseline --views 4 --steps 5 --warmup 2 > $O/v4.json 2>> $O/configs.err
    timeout -k 10 300 python bench.py --no-cpu-baseline --scenes 4 --steps 5 --warmup 2 > $O/s4.json 2>> $O/configs.err
    timeout -k 10 200 python bench.py --no-cpu-baseline --config base --res 256 > $O/base256.json 2>> $O/configs.err ;;
c5)
    timeout -k 10 400 python bench.py --workload c5 --steps 3 --warmup 1 > $O/c5bf16.json 2> $O/c5.err
    timeout -k 10 400 python bench.py --workload c5 --fp8 --steps 3 --warmup 1 > $O/c5fp8.json 2>> $O/c5.err ;;
pmc)
    i=0
    for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
             "SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM"; do
        i=$((i+1))
        prof_run timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $O/p$i -o run -- python3 "$@" > $O/p$i.log 2>&1
    done ;;
l2)
    prof_run timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/pmc -o run -- python3 $R/bench.py --profile --steps 2 --warmup 1 > $O/pmc.log 2>&1
    python tools/pmc_l2.py $(find $O/pmc -name '*counter_collection.csv' -print -quit) 30 > $O/l2.txt ;;
attnab)
    timeout -k 10 300 $T tests/test_kernels_gpu.py -k "attention or attn" > $O/t_attn.log 2>&1
    ABL=${ABL:-0,1024} timeout -k 10 300 python -u tools/attn_ablate.py > $O/ablate.log 2>&1 ;;
fold)
    for v in 1 0; do
        (export RF_DPT_FOLD=$v; prof_run timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof$v -o run -- python3 $R/bench.py --profile --steps 5 --warmup 2 --no-cpu-baseline > $O/prof$v.log 2>&1)
    done
    bash tools/gpu.sh ab $TAG "RF_DPT_FOLD=1" "RF_DPT_FOLD=0" ;;
c4)
    timeout -k 10 400 python bench.py --workload c4 --steps 3 --warmup 1 > $O/c4.json 2> $O/c4.err
    timeout -k 10 500 python -u tools/batch_e2e.py 64 1 > $O/e2e.log 2>&1 ;;
new)
    timeout -k 10 600 $T tests/test_kernels_gpu.py -k "quad or hk or border_bias or c32 or f16_operands" > $O/t_new.log 2>&1
    timeout -k 10 300 $T tests/test_parity_gpu.py -k "native" > $O/t_native.log 2>&1
    timeout -k 10 400 python -u tools/kbench.py quad > $O/quad.log 2>&1
    prof_run timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --profile --steps 5 --warmup 2 > $O/prof.log 2>&1 ;;
vpmc)  # kbench legs ($@, default vendor) under counter passes (FETCH / WRITE / L2 hit / MFMA busy); KB_* passed through
    for LEG in ${@:-vendor}; do
        i=0
        for P in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES"; do
            i=$((i+1))
            prof_run timeout -s KILL 180 rocprofv3 --pmc $P --output-format csv -d $O/${LEG}_p$i -o run -- python3 $R/tools/kbench.py $LEG > $O/${LEG}_p$i.log 2>&1
        done
        python tools/pmc_kernels.py $(find $O/${LEG}_p1 $O/${LEG}_p2 $O/${LEG}_p3 $O/${LEG}_p4 -name '*counter_collection.csv') > $O/${LEG}_pmc.txt 2>&1
    done ;;
convab)  # the 512^2 / 256^2 DPT convolutions on halo2 vs conv3x3_hk_kernel
    KB_F16_ONLY=1 KB_CONV_HW=512,256 KB_CONV_TILES=h2,hk timeout -k 10 300 python -u tools/kbench.py conv > $O/convab.log 2>&1 ;;
libab)
    BASE=${BASE:-$R/renderformer_amd/lib/librfhip_base.so}
    timeout -k 10 900 $T tests -m gpu > $O/tests.log 2>&1
    for i in 1 2; do
        ABL=0 timeout -k 10 200 python -u tools/attn_ablate.py > $O/attn_new$i.log 2>&1
        ABL=0 RF_LIB=$BASE timeout -k 10 200 python -u tools/attn_ablate.py > $O/attn_base$i.log 2>&1
    done
    STUDY=$R/renderformer_amd/lib/librfhip_study.so  # the stamp build (RF_ATTN_DBG=32) of the current tree
    if [ -f $STUDY ]; then RF_LIB=$STUDY timeout -k 10 120 python tools/attn_ablate.py stamps > $O/stamps_new.log 2>&1; fi
    if [ -n "$BASE_STUDY" ]; then RF_LIB=$BASE_STUDY timeout -k 10 120 python tools/attn_ablate.py stamps > $O/stamps_base.log 2>&1; fi
    for i in 1 2; do
        timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_new$i.json 2>> $O/bench.err
        RF_LIB=$BASE timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_base$i.json 2>> $O/bench.err
    done ;;
pnab)  # deferred RMSNorm: its GPU tests, the kbench prenorm A/B on this library and the plain GEMMs on $BASE, then
       # interleaved bench runs of both libraries
    BASE=${BASE:-$R/renderformer_amd/lib/librfhip_base.so}
    timeout -k 10 900 $T tests/test_prenorm_gpu.py tests/test_parity_gpu.py -m gpu > $O/tests.log 2>&1
    timeout -k 10 300 python -u tools/kbench.py prenorm > $O/kb_new.log 2>&1
    KB_PLAIN_ONLY=1 RF_LIB=$BASE timeout -k 10 300 python -u tools/kbench.py prenorm > $O/kb_base.log 2>&1
    for i in 1 2; do
        timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_new$i.json 2>> $O/bench.err
        RF_LIB=$BASE timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_base$i.json 2>> $O/bench.err
    done ;;
libkb)  # the kbench prenorm A/B and bench runs of this library and $BASE, interleaved (two rounds each)
    BASE=${BASE:-$R/renderformer_amd/lib/librfhip_base.so}
    for i in 1 2; do
        timeout -k 10 300 python -u tools/kbench.py prenorm > $O/kb_new$i.log 2>&1
        RF_LIB=$BASE timeout -k 10 300 python -u tools/kbench.py prenorm > $O/kb_base$i.log 2>&1
    done
    for i in 1 2; do
        timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_new$i.json 2>> $O/bench.err
        RF_LIB=$BASE timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_base$i.json 2>> $O/bench.err
    done ;;
qkn)  # q/k norm: its GPU tests, kbench norms (split A/B), bench
    timeout -k 10 600 $T tests/test_kernels_gpu.py -k "qk_norm or rmsnorm" -m gpu > $O/tests.log 2>&1
    timeout -k 10 300 python -u tools/kbench.py norms > $O/norms.log 2>&1
    timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err ;;
costab)  # stage-1 attention timing + per-role stamps under the stream-K cost-model constants in $COSTS (';'-separated
         # RF_ATTN_COST values "tile,pro,pub,merge,store"; "-" = the built-in constants)
    STUDY=$R/renderformer_amd/lib/librfhip_study.so
    IFS=';' read -ra CS <<< "${COSTS:--}"
    for i in 1 2; do
        for c in "${CS[@]}"; do
            if [ "$c" = "-" ]; then unset RF_ATTN_COST; else export RF_ATTN_COST=$c; fi
            ABL=0 timeout -k 10 200 python -u tools/attn_ablate.py > $O/attn_${c//,/_}_$i.log 2>&1
            if [ $i = 1 ] && [ -f $STUDY ]; then RF_LIB=$STUDY timeout -k 10 120 python tools/attn_ablate.py stamps > $O/stamps_${c//,/_}.log 2>&1; fi
        done
    done
    unset RF_ATTN_COST ;;
quadstudy)  # the 4-wave GEMM (study build) at the library's tiles vs the default engine on the projection shapes
    KB_SHAPES=${KB_SHAPES:-"s1 qkv,s1 out,s1 w2,s2 out,s2 w2"} KB_QUAD=${KB_QUAD:-"0,1@128x192,2@128x192,1d@128x192,1@160x256,2@160x256,1d@160x256"} \
        RF_LIB=$R/renderformer_amd/lib/librfhip_study.so timeout -k 10 600 python -u tools/kbench.py quad > $O/quad.log 2>&1 ;;
swin)  # Swin / q/k-norm-fold GPU tests, then a kernel-trace profile of the default bench and one bench run
    timeout -k 10 600 $T tests/test_kernels_gpu.py tests/test_prenorm_gpu.py -k "swin or qkn" -m gpu > $O/tests.log 2>&1
    prof_run timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --profile --steps 5 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1
    timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err ;;
profab)  # kernel-trace profiles of the default bench under each ';'-separated env setting in $ENVS ("-" = none)
    IFS=';' read -ra ES <<< "${ENVS:--}"
    i=0
    for e in "${ES[@]}"; do
        i=$((i+1))
        if [ "$e" = "-" ]; then e=""; fi
        (export $e; prof_run timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof$i -o run -- python3 $R/bench.py --profile --steps 5 --warmup 2 --no-cpu-baseline > $O/prof$i.log 2>&1)
    done ;;
vendor)
    prof_run timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/vend -o run -- python3 $R/tools/kbench.py vendor > $O/vendor.log 2>&1 ;;
*)
    echo "unknown task $TASK" >&2; exit 2 ;;
esac
echo done

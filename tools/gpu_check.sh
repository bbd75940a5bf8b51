#!/bin/bash
# GPU-box check sequence (run through gpurun).  Every GPU step has its own time
# limit; a crash / abort / timeout (exit code > 1) ends the script right there.
# Usage: tools/gpu_check.sh [steps...]   steps: smoke tests bench layers sweep prof
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
# autotuned plans of the bench run are recorded here and reused by the profiling steps
export PO2Q_TUNE_FILE=$PWD/gpurun_out/tune.json
STEPS=${*:-smoke tests bench}

run() {  # name timeout cmd...
    local name=$1 t=$2
    shift 2
    local t0=$(date +%s)
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc $(( $(date +%s) - t0 ))s" | tee -a gpurun_out/status.txt
    tail -n 5 "gpurun_out/$name.log"
    if [ $rc -gt 1 ]; then
        echo "stopping: $name exited with $rc"
        exit $rc
    fi
    return 0
}

for s in $STEPS; do
    case $s in
        smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
        tests) run pytest_gpu 900 python -m pytest tests -m gpu -q -rf -x
               if ! grep -q " passed" gpurun_out/pytest_gpu.log || grep -q "failed\|error" gpurun_out/pytest_gpu.log; then
                   echo "stopping: GPU tests did not pass"; exit 1
               fi ;;
        convtests) run convtests 600 python -u -m pytest tests/test_gpu_conv.py -m gpu -x -q --timeout 300 --timeout-method thread
               if ! grep -q " passed" gpurun_out/convtests.log || grep -q "failed\|error" gpurun_out/convtests.log; then
                   echo "stopping: conv GPU tests did not pass"; exit 1
               fi ;;
        bench) run bench 600 python bench.py ;;
        benchnp) run benchnp 600 python bench.py --steps 5 --warmup 2 --no-pair --no-cpu-baseline ;;
        models) run models_c2 300 python tools/model_bench.py --model resnet56 --image 32 --classes 10 --graph
                run models_c3 300 python tools/model_bench.py --model mobilenet --image 32 --classes 10 --quantizer po2+ --graph
                run models_c5 300 python tools/model_bench.py --model mobilevit --image 256 --batch 64 --quantizer po2+ --bits 2 --graph
                run models_c4 300 python tools/model_bench.py --model resnet56 --image 224 --only-fused ;;
        profmb) run profmb 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profmb -o run \
                  -- python tools/model_bench.py --model mobilenet --image 32 --classes 10 --quantizer po2+ --only-fused ;;
        profvit) run profvit 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profvit -o run \
                  -- python tools/model_bench.py --model mobilevit --image 256 --batch 64 --quantizer po2+ --bits 2 --only-fused --graph ;;
        profr56) run profr56 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profr56 -o run \
                  -- python tools/model_bench.py --model resnet56 --image 224 --only-fused ;;
        bwdtests) run bwdtests 600 python -u -m pytest tests/test_gpu_backward.py tests/test_qat.py -m gpu -x -q --timeout 300 --timeout-method thread
               if ! grep -q " passed" gpurun_out/bwdtests.log || grep -q "failed\|error" gpurun_out/bwdtests.log; then
                   echo "stopping: backward GPU tests did not pass"; exit 1
               fi ;;
        dwtests) run dwtests 600 python -u -m pytest tests/test_gpu_depthwise.py -m gpu -x -q --timeout 300 --timeout-method thread
               if ! grep -q " passed" gpurun_out/dwtests.log || grep -q "failed\|error" gpurun_out/dwtests.log; then
                   echo "stopping: depthwise GPU tests did not pass"; exit 1
               fi ;;
        chaintests) run chaintests 600 python -u -m pytest tests/test_gpu_chain.py -m gpu -x -q --timeout 300 --timeout-method thread
               if ! grep -q " passed" gpurun_out/chaintests.log || grep -q "failed\|error" gpurun_out/chaintests.log; then
                   echo "stopping: chain tests failed"; exit 3; fi ;;
        c64res) run c64res 600 python -u -m pytest tests/test_gpu_conv.py -m gpu -x -q --timeout 300 --timeout-method thread -k "c64_residual or fused_epilogue"
               if ! grep -q " passed" gpurun_out/c64res.log || grep -q "failed\|error" gpurun_out/c64res.log; then
                   echo "stopping: c64res failed"; exit 3; fi ;;
        pairtests) run pairtests 600 python -u -m pytest tests/test_gpu_pair.py -m gpu -x -q --timeout 300 --timeout-method thread
               if ! grep -q " passed" gpurun_out/pairtests.log || grep -q "failed\|error" gpurun_out/pairtests.log; then
                   echo "stopping: pair GPU tests did not pass"; exit 1
               fi ;;
        pairb) run pairb 300 python tools/pair_bench.py ;;
        pairstg) run pairstg 300 env PAIR_C32=0 PAIR_VARIANTS=123,10123,10023,23 python tools/pair_bench.py ;;
        pairablate) run pairablate 300 python tools/pair_ablate.py ;;
        pairpd) run pairpd 300 env PAIR_C32=0 PAIR_VARIANTS=23,33,43,123,133,143 python tools/pair_bench.py ;;
        abc32) for r in 1 2; do
                   run abc32_off_$r 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-cifar
                   run abc32_on_$r 300 env PO2Q_PAIR_C32=1 python bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-cifar
               done ;;
        pairq) run pairq 300 env PAIR_C32=0 PAIR_VARIANTS=123,20023 python tools/pair_bench.py ;;
        abab) for r in 1 2; do for v in 123 20023; do
                   run abab_${v}_$r 300 env PO2Q_PAIR_VARIANT=$v python bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-cifar --no-models
               done; done ;;
        benchq) run benchq 300 python bench.py --steps 30 --warmup 2 --no-cpu-baseline --no-cifar --no-models ;;
        abstg) for r in 1 2; do for v in 123 10123 10023; do
                   run abstg_${v}_$r 300 env PO2Q_PAIR_VARIANT=$v python bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-cifar
               done; done ;;
        modeltests) run modeltests 600 python -u -m pytest tests/test_gpu_models.py -m gpu -x -q --timeout 300 --timeout-method thread
               if ! grep -q " passed" gpurun_out/modeltests.log || grep -q "failed\|error" gpurun_out/modeltests.log; then
                   echo "stopping: model GPU tests did not pass"; exit 1
               fi ;;
        dwb) run dwb 300 python tools/dw_bench.py ;;
        bwd) run bwd224 600 python tools/bwd_bench.py --batch 64
             run bwd32 600 python tools/bwd_bench.py --batch 256 --image 32
             run qatb 600 python tools/qat_bench.py resnet56 ;;
        layers) run layers 600 python tools/layer_bench.py --torch ;;
        layers32) run layers32 600 python tools/layer_bench.py --image 32 --tune --torch ;;
        bench32) run bench32 600 python bench.py --image 32 --steps 20 --warmup 3 --no-cpu-baseline ;;
        bench32g) run bench32g 600 python bench.py --image 32 --steps 50 --warmup 3 --graph --no-cpu-baseline ;;
        sweep) run sweep 900 python tools/tile_sweep.py ;;
        profc2) run profc2 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profc2 -o run \
                  -- python bench.py --image 32 --steps 50 --warmup 3 --graph --no-cpu-baseline --no-cifar --no-models ;;
        chainab) run chainab 300 python tools/chain_ab.py ;;
        sweepc) run sweepc 600 python tools/tile_sweep.py --shapes 7,8,9 --iters 21 ;;
        sweep036) run sweep036 600 python tools/tile_sweep.py --shapes 0,3,6 --iters 15 ;;
        sweep1) run sweep1 600 python tools/tile_sweep.py --shapes 1 --iters 21 ;;
        sweep4) run sweep4 600 python tools/tile_sweep.py --shapes 4 --iters 21 ;;
        sweep0) run sweep0 600 python tools/tile_sweep.py --shapes 0 --iters 21 ;;
        sweep3) run sweep3 600 python tools/tile_sweep.py --shapes 3 --iters 21 ;;
        sweep6) run sweep6 600 python tools/tile_sweep.py --shapes 6 --iters 21 ;;
        pmc1) run pmc1 900 bash tools/pmc.sh "--shape 16,224,16,3,1,1 --tile 7,4,112" s1 ;;
        pmcs3) run pmcs3 900 bash tools/pmc.sh "--shape 64,56,64,3,1,1" s3 "conv_rowsk" all
               python3 tools/pmc_summary.py gpurun_out/pmc_s3 177.6 > gpurun_out/pmc_s3_summary.txt 2>&1 ;;
        pmcch) for st in 1 3; do  # useful bf16 MFMA GFLOP per launch: 18 (17) layers x 3 x 1.208
                   gf=$([ $st = 1 ] && echo 65.2 || echo 61.6)
                   run pmcch$st 600 env PMC_DRIVER=tools/prof_chain.py bash tools/pmc.sh "--stage $st" ch$st "conv_chain" all
                   python3 tools/pmc_summary.py gpurun_out/pmc_ch$st $gf > gpurun_out/pmc_ch${st}_summary.txt 2>&1
               done ;;
        pmcs2) run pmcs2 900 bash tools/pmc.sh "--shape 32,112,32,3,1,1" s2 "conv_rowsf" all
               python3 tools/pmc_summary.py gpurun_out/pmc_s2 177.6 > gpurun_out/pmc_s2_summary.txt 2>&1 ;;
        pmc3) run pmc3 900 bash tools/pmc.sh "--shape 64,56,64,3,1,1 --tile 4,8,32" s3 ;;
        copyprobe) run copyprobe 300 tools/copy_probe 20 ;;
        ringprobe) run ringprobe 300 tools/copy_probe 20 1 ;;
        ringprobe2) run ringprobe2 300 tools/copy_probe 20 2 ;;
        ringprobe3) run ringprobe3 300 tools/copy_probe 20 3 ;;
        counters) run counters 120 rocprofv3 -L ;;
        traffic) run traffic 900 bash tools/pmc.sh "--shape 16,224,16,3,1,1" t1 "conv_x3p|conv_bf16x3" hbm
                 python3 tools/traffic.py gpurun_out/pmc_t1 --algorithmic 1644185600 >> gpurun_out/traffic.log 2>&1 ;;
        traffic_rows)  # HBM bytes of the row-streaming stage-1 plans (candidate indices 1..3)
                 cp profiles/traffic.json gpurun_out/traffic.json
                 for i in 1 2 3; do
                     run pmc_trows$i 300 bash tools/pmc.sh "--shape 16,224,16,3,1,1 --plan $i" trows$i "conv_rows" hbm
                     python3 tools/traffic.py gpurun_out/pmc_trows$i --algorithmic 1644185600 \
                         --out gpurun_out/traffic.json >> gpurun_out/traffic.log 2>&1
                 done ;;
        traffic_pair) run pmc_tpair 300 bash tools/pmc.sh "--pair --shape 16,224,16,3,1,1" tpair "conv_pair" hbm
                 cp profiles/traffic.json gpurun_out/traffic.json
                 python3 tools/traffic.py gpurun_out/pmc_tpair --algorithmic 1644274688 --out gpurun_out/traffic.json >> gpurun_out/traffic.log 2>&1
                 run pmc_pair 600 bash tools/pmc.sh "--pair --shape 16,224,16,3,1,1" pair "conv_pair" all
                 python3 tools/pmc_summary.py gpurun_out/pmc_pair 355.3 > gpurun_out/pmc_pair_summary.txt 2>&1 ;;
        pmc_pairw)  # the stage-2 role-split pair (conv_pairw): useful bf16 MFMA work 2 x 177.6 GFLOP
                 run pmc_pairw 600 bash tools/pmc.sh "--pair --shape 32,112,32,3,1,1" pairw "conv_pairw" all
                 python3 tools/pmc_summary.py gpurun_out/pmc_pairw 355.3 > gpurun_out/pmc_pairw_summary.txt 2>&1 ;;
        profhead) run profhead 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profhead -o run \
                  -- python bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-cifar --no-models ;;
        stamps) run stamps 600 python tools/stamps.py ;;
        pmcr1) run pmcr1 900 bash tools/pmc.sh "--shape 16,224,16,3,1,1" r1 "conv_bf16x3|conv_x3p" all ;;
        pmcr3) run pmcr3 900 bash tools/pmc.sh "--shape 64,56,64,3,1,1" r3 "conv_bf16x3|conv_x3p" all ;;
        pmcd1) run pmcd1 900 bash tools/pmc.sh "--shape 16,224,16,3,1,1" d1 ;;
        pmcd2) run pmcd2 900 bash tools/pmc.sh "--shape 32,112,32,3,1,1" d2 ;;
        ablate_rows1) run ablate_rows1 600 env PO2Q_LIB=$PWD/po2_quantization_amd/lib_rowsdiag/libpo2q.so python tools/ablate.py --shape 16,224,16,3,1,1 --plans 11,8 --var PO2Q_ROWS_DEBUG --values 0,3,32,35,8,4,16,19,51,48 --rounds 5 ;;
        ablate_rowsf) run ablate_rowsf 600 env PO2Q_LIB=$PWD/po2_quantization_amd/lib_rowsdiag/libpo2q.so python tools/ablate.py --shape 16,224,16,3,1,1 --plans 28 --var PO2Q_ROWSF_DEBUG --values 0,1,2,3,4,8,5,10,11 --rounds 5 ;;
        ablate_rowsf2) run ablate_rowsf2 600 env PO2Q_LIB=$PWD/po2_quantization_amd/lib_rowsdiag/libpo2q.so python tools/ablate.py --shape 32,112,32,3,1,1 --plans 0 --var PO2Q_ROWSF_DEBUG --values 0,1,4,8,5,9,12 --rounds 5 ;;
        ablate1) run ablate1 600 env PO2Q_LIB=$PWD/po2_quantization_amd/lib_stamps/libpo2q.so python tools/ablate.py --shape 16,224,16,3,1,1 --plans 2,3 ;;
        ablate) run ablate 600 env PO2Q_LIB=$PWD/po2_quantization_amd/lib_stamps/libpo2q.so bash -c 'python tools/ablate.py --shape 16,224,16,3,1,1 && python tools/ablate.py --shape 32,112,32,3,1,1 && python tools/ablate.py --shape 64,56,64,3,1,1' ;;
        prof) run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run \
                  -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-cifar --no-models ;;
        *) echo "unknown step $s" ;;
    esac
done

cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc" | tee -a gpurun_out/status13.txt
    tail -n 3 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping at $name"; exit $rc; fi
}
run t13 900 python -u -m pytest tests/test_gpu_ir.py tests/test_gpu_packs.py tests/test_gpu_models.py -m gpu -x -q --timeout 300 --timeout-method thread
run mb13_ir 300 python tools/model_bench.py --model mobilenet --image 32 --classes 10 --quantizer po2+ --only-fused --graph
run mb13_noir 300 python tools/model_bench.py --model mobilenet --image 32 --classes 10 --quantizer po2+ --only-fused --graph --no-ir
run prof13 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof13 -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-cifar --no-models
run pmc_pair13 600 bash tools/pmc.sh "--pair --shape 16,224,16,3,1,1" pair13 "conv_pair" all
python3 tools/pmc_summary.py gpurun_out/pmc_pair13 355.3 > gpurun_out/pmc_pair13_summary.txt 2>&1
python3 tools/traffic.py gpurun_out/pmc_pair13 --algorithmic 1644274688 --out gpurun_out/traffic13.json > gpurun_out/traffic13.log 2>&1
echo done

cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc" | tee -a gpurun_out/status14.txt
    tail -n 3 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping at $name"; exit $rc; fi
}
run t14 900 python -u -m pytest tests/test_gpu_ir.py tests/test_gpu_packs.py tests/test_gpu_models.py tests/test_capi.py -m gpu -x -q --timeout 300 --timeout-method thread
run mb14_ir 300 python tools/model_bench.py --model mobilenet --image 32 --classes 10 --quantizer po2+ --only-fused --graph
run mb14_noir 300 python tools/model_bench.py --model mobilenet --image 32 --classes 10 --quantizer po2+ --only-fused --graph --no-ir
run mb14_vit 300 python tools/model_bench.py --model mobilevit --image 256 --batch 64 --quantizer po2+ --bits 2 --only-fused --graph
run mb14_vit_noir 300 python tools/model_bench.py --model mobilevit --image 256 --batch 64 --quantizer po2+ --bits 2 --only-fused --graph --no-ir
run pairstamps14 300 python -u tools/pair_stamps.py

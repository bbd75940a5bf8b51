cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc" | tee -a gpurun_out/status12.txt
    tail -n 3 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping at $name"; exit $rc; fi
}
run t12_ir 600 python -u -m pytest tests/test_gpu_ir.py -m gpu -x -q --timeout 300 --timeout-method thread
run ir_ab12 300 python -u tools/ir_ab.py --rounds 3
run mb12_ir 300 python tools/model_bench.py --model mobilenet --image 32 --classes 10 --quantizer po2+ --only-fused --graph --ir
run mb12_noir 300 python tools/model_bench.py --model mobilenet --image 32 --classes 10 --quantizer po2+ --only-fused --graph
run chainstamps12 300 python -u tools/chain_stamps.py

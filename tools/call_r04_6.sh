cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name timeout cmd...   (a test failure, rc 1, does not stop the script; anything else does)
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc" | tee -a gpurun_out/status6.txt
    tail -n 3 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping at $name"; exit $rc; fi
}
run t6_ir 600 python -u -m pytest tests/test_gpu_ir.py -m gpu -x -q --timeout 300 --timeout-method thread
run mb6_ir 300 python tools/model_bench.py --model mobilenet --image 32 --classes 10 --quantizer po2+ --only-fused --graph
run mb6_noir 300 python tools/model_bench.py --model mobilenet --image 32 --classes 10 --quantizer po2+ --only-fused --graph --no-ir
run profmb6 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profmb6 -o run -- python tools/model_bench.py --model mobilenet --image 32 --classes 10 --quantizer po2+ --only-fused --graph
run t6_qatg 300 python -u -m pytest tests/test_qat.py -m gpu -x -q --timeout 200 --timeout-method thread -k graphed
run t6_chain 400 python -u -m pytest tests/test_gpu_chain.py -m gpu -x -q --timeout 300 --timeout-method thread
run t6_pairmw 600 python -u -m pytest tests/test_gpu_pair.py -m gpu -q --timeout 300 --timeout-method thread -k "memory_wave"

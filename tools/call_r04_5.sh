cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name timeout cmd...   (a test failure, rc 1, does not stop the script; anything else does)
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc" | tee -a gpurun_out/status5.txt
    tail -n 3 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping at $name"; exit $rc; fi
}
run t5_ir 600 python -u -m pytest tests/test_gpu_ir.py -m gpu -x -v --timeout 300 --timeout-method thread
run t5_qatg 300 python -u -m pytest tests/test_qat.py -m gpu -x -q --timeout 200 --timeout-method thread -k graphed
run mb_ir 300 python tools/model_bench.py --model mobilenet --image 32 --classes 10 --quantizer po2+ --only-fused --graph
run mb_noir 300 python tools/model_bench.py --model mobilenet --image 32 --classes 10 --quantizer po2+ --only-fused --graph --no-ir
run t5_pairmw 600 python -u -m pytest tests/test_gpu_pair.py -m gpu -x -q --timeout 300 --timeout-method thread -k "memory_wave or full_size or vs_oracle"
run pair_mw 300 python -u tools/pair_mw_bench.py
run t5_chain 400 python -u -m pytest tests/test_gpu_chain.py -m gpu -x -q --timeout 300 --timeout-method thread
run chain_ab 300 python -u tools/chain_ab.py

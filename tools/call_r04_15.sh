cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc" | tee -a gpurun_out/status15.txt
    tail -n 3 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping at $name"; exit $rc; fi
}
run t15 1200 python -u -m pytest tests/test_gpu_pair.py tests/test_gpu_conv.py tests/test_gpu_chain.py tests/test_gpu_depthwise.py tests/test_gpu_s2ds.py tests/test_gpu_ir.py -m gpu -x -q --timeout 300 --timeout-method thread
run pmw15 300 python -u tools/pair_mw_bench.py
run b15_1 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-cifar --no-models
run b15_2 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-cifar --no-models
run chainab15 300 python -u tools/chain_ab.py --variants 0,8 --rounds 3

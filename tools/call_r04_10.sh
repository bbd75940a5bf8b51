cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc" | tee -a gpurun_out/status10.txt
    tail -n 3 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping at $name"; exit $rc; fi
}
run t10_ir 600 python -u -m pytest tests/test_gpu_ir.py -m gpu -x -q --timeout 300 --timeout-method thread
run irstamps10 300 python -u tools/ir_stamps.py
run ir_ab10 300 python -u tools/ir_ab.py --rounds 3

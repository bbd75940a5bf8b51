cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name timeout cmd...   (a test failure, rc 1, does not stop the script; anything else does)
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc" | tee -a gpurun_out/status8.txt
    tail -n 3 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping at $name"; exit $rc; fi
}
run t8_ir 600 python -u -m pytest tests/test_gpu_ir.py -m gpu -x -q --timeout 300 --timeout-method thread
run ir_ab8 300 python -u tools/ir_ab.py --rounds 3
run ir_ab8_mb64 300 env PO2Q_IR_MINBLOCKS=64 python -u tools/ir_ab.py --rounds 3
run ir_ab8_mb16 300 env PO2Q_IR_MINBLOCKS=16 python -u tools/ir_ab.py --rounds 3

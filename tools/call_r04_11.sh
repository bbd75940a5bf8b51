cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc" | tee -a gpurun_out/status11.txt
    tail -n 3 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping at $name"; exit $rc; fi
}
run t11_pair 600 python -u -m pytest tests/test_gpu_pair.py -m gpu -x -q --timeout 300 --timeout-method thread
for r in 1 2; do
  run ab11_mw_$r 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-cifar --no-models
  run ab11_nomw_$r 300 env PO2Q_PAIR_MW=0 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-cifar --no-models
done
run ab11_c32ts 300 env PO2Q_PAIR_C32_TS=1 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-cifar --no-models
run qatb11 600 python -u tools/qat_bench.py resnet20

cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name timeout cmd...
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc" | tee -a gpurun_out/status3.txt
    tail -n 3 "gpurun_out/$name.log"
    if [ $rc -ne 0 ]; then echo "stopping at $name"; exit $rc; fi
}
run t3_tests 900 python -u -m pytest tests/test_gpu_packs.py tests/test_gpu_split.py tests/test_gpu_chain.py tests/test_gpu_models.py tests/test_qat.py -m gpu -x -q --timeout 300 --timeout-method thread
run t3_pairmw 600 python -u -m pytest tests/test_gpu_pair.py -m gpu -x -q --timeout 300 --timeout-method thread -k "memory_wave or full_size or vs_oracle"
run pair_mw 300 python -u tools/pair_mw_bench.py

cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
L=po2_quantization_amd/lib
cp $L/libpo2q.so /tmp/libpo2q_new.so
use() { cp "$1" $L/libpo2q.so; }
run() {
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc" | tee -a gpurun_out/status26.txt
    tail -n 2 "gpurun_out/$name.log" | cut -c1-300
    if [ $rc -ne 0 ]; then echo "stopping at $name"; exit $rc; fi
}
run t26 600 python -u -m pytest tests/test_gpu_pair.py -m gpu -x -q --timeout 300 --timeout-method thread
B="python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-cifar --no-models"
for r in 1 2; do
  use /tmp/libpo2q_new.so;                     PAIR_MW=0 ROUNDS=3 run pm26_w2r_$r 300 python -u tools/pair_mw_bench.py
  use po2_quantization_amd/lib_ab2/libpo2q.so; PAIR_MW=0 ROUNDS=3 run pm26_lds_$r 300 python -u tools/pair_mw_bench.py
  use /tmp/libpo2q_new.so;                     run b26_w2r_$r 300 $B
  use po2_quantization_amd/lib_ab2/libpo2q.so; run b26_lds_$r 300 $B
done
use /tmp/libpo2q_new.so

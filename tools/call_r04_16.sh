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
    echo "$name rc=$rc" | tee -a gpurun_out/status16.txt
    tail -n 2 "gpurun_out/$name.log"
    if [ $rc -ne 0 ]; then echo "stopping at $name"; exit $rc; fi
}
for r in 1 2 3; do
  use /tmp/libpo2q_new.so
  run b16_new_$r 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-cifar --no-models
  PAIR_MW=0,5 ROUNDS=3 run pmw16_new_$r 300 python -u tools/pair_mw_bench.py
  use po2_quantization_amd/lib_ab/libpo2q.so
  run b16_old_$r 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-cifar --no-models
  PAIR_MW=0,5 ROUNDS=3 run pmw16_old_$r 300 python -u tools/pair_mw_bench.py
done
use /tmp/libpo2q_new.so

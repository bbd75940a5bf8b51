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
    echo "$name rc=$rc" | tee -a gpurun_out/status17.txt
    tail -n 2 "gpurun_out/$name.log" | cut -c1-300
    if [ $rc -ne 0 ]; then echo "stopping at $name"; exit $rc; fi
}
B="python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-cifar --no-models"
for r in 1 2; do
  use /tmp/libpo2q_new.so;                      run b17_new_$r 300 $B
  use po2_quantization_amd/lib_ab2/libpo2q.so;  run b17_head_$r 300 $B
  use po2_quantization_amd/lib_ab/libpo2q.so;   run b17_old_$r 300 $B
done
for v in new head old; do
  case $v in new) use /tmp/libpo2q_new.so;; head) use po2_quantization_amd/lib_ab2/libpo2q.so;; old) use po2_quantization_amd/lib_ab/libpo2q.so;; esac
  PAIR_MW=5 ROUNDS=3 run pmw17_$v 300 python -u tools/pair_mw_bench.py
done
use /tmp/libpo2q_new.so
run p17_new 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p17_new -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-cifar --no-models
use po2_quantization_amd/lib_ab/libpo2q.so
run p17_old 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p17_old -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-cifar --no-models
use /tmp/libpo2q_new.so

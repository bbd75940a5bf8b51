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
    echo "$name rc=$rc" | tee -a gpurun_out/status21.txt
    tail -n 3 "gpurun_out/$name.log" | cut -c1-300
    if [ $rc -ne 0 ]; then echo "stopping at $name"; exit $rc; fi
}
run t21 600 python -u -m pytest tests/test_gpu_chain.py -m gpu -x -q --timeout 300 --timeout-method thread
for r in 1 2 3; do
  use /tmp/libpo2q_new.so;                     run cab21_scalar_$r 300 python -u tools/chain_ab.py --variants 0 --rounds 3
  use po2_quantization_amd/lib_ab2/libpo2q.so; run cab21_packed_$r 300 python -u tools/chain_ab.py --variants 0 --rounds 3
done
use /tmp/libpo2q_new.so

cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc" | tee -a gpurun_out/status19.txt
    tail -n 3 "gpurun_out/$name.log" | cut -c1-400
    if [ $rc -ne 0 ]; then echo "stopping at $name"; exit $rc; fi
}
run pipeab 300 python -u tools/rowsk_pipe_ab.py
B="python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-cifar --no-models"
for r in 1 2; do
  run b19_def_$r 300 $B
  PO2Q_ROWSK_PIPE=1 run b19_pipe_$r 300 $B
done

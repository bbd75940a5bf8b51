cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name timeout cmd...
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc" | tee -a gpurun_out/status4.txt
    tail -n 3 "gpurun_out/$name.log"
    if [ $rc -ne 0 ]; then echo "stopping at $name"; exit $rc; fi
}
run profmb 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profmb -o run -- python tools/model_bench.py --model mobilenet --image 32 --classes 10 --quantizer po2+ --only-fused --graph
run models_c3 300 python tools/model_bench.py --model mobilenet --image 32 --classes 10 --quantizer po2+ --graph
run models_c5 300 python tools/model_bench.py --model mobilevit --image 256 --batch 64 --quantizer po2+ --bits 2 --graph
run models_c4 300 python tools/model_bench.py --model resnet56 --image 224 --only-fused
run qatb 600 python -u tools/qat_bench.py resnet56

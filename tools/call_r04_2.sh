cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_quantizer.py tests/test_gpu_packs.py tests/test_gpu_split.py tests/test_gpu_chain.py tests/test_gpu_models.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t2.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/t2.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_check.sh profmb profr56 models

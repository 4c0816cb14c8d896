set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
run() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 gpurun_out/$name.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run pytest_new 600 python -u -m pytest tests/test_torch_ops.py tests/test_gpu_eval.py tests/test_sampler.py tests/test_gpu_dist.py tests/test_gpu_xgat.py -m gpu -v -rf --timeout 150 --timeout-method thread
run bench_eval 300 python -u tools/bench_eval.py
run bench2 300 python -u bench.py --steps 20 --warmup 5
run bench5 600 python -u bench.py --config 5 --steps 10 --warmup 3

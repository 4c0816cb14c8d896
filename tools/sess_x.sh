set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_xgat.py tests/test_gpu_dist.py tests/test_gpu_graph.py -m gpu -v -rf --timeout 150 --timeout-method thread > gpurun_out/pytest_x.log 2>&1; echo "rc=$?" >> gpurun_out/pytest_x.log
tail -3 gpurun_out/pytest_x.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -v -s -rf --durations=0 --timeout 170 --timeout-method thread > gpurun_out/pytest_fullsize.log 2>&1; echo "rc=$?" >> gpurun_out/pytest_fullsize.log
tail -3 gpurun_out/pytest_fullsize.log
timeout -k 10 600 python -u bench.py --config 5 --steps 10 --warmup 3 > gpurun_out/bench5.log 2>&1; echo "rc=$?" >> gpurun_out/bench5.log
tail -2 gpurun_out/bench5.log
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof5 -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --config 5 --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof5.log 2>&1; echo "rc=$?"

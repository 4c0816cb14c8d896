#!/bin/bash
# Session 10: split-K GEMM tests, FusionMLP tests and train-step bench.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/s10
run() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > gpurun_out/s10/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 gpurun_out/s10/$name.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run pytest 400 python -u -m pytest tests/test_gpu_xgat.py tests/test_gpu_fusion.py -m gpu -v -rf --timeout 170 --timeout-method thread
run fusion_bench 180 python -u tools/bench_fusion.py --train
echo done

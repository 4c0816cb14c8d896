#!/bin/bash
# Session 12: fused gt GEMM + D epilogue (config 5 backward): layer / full-size / halo tests, bench.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/s12
run() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > gpurun_out/s12/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 gpurun_out/s12/$name.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run pytest 600 python -u -m pytest tests/test_gpu_xgat.py tests/test_gpu_fullsize.py tests/test_gpu_dist.py -m gpu -x -v -rf --timeout 170 --timeout-method thread
run bench5 400 python -u bench.py --config 5 --steps 10 --warmup 3
echo done

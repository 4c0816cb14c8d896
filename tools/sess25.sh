#!/bin/bash
# Session 25: split NN / fusion kernels with LDS reads one step ahead.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/s25
run() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > gpurun_out/s25/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -1 gpurun_out/s25/$name.log | cut -c1-1500; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run cfg5 200 python -u tools/gemm_split_check.py --cfg5
run fusion 200 python -u tools/bench_fusion.py
run pytest 300 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_fusion.py tests/test_gpu_xgat.py -m gpu -q -rf --timeout 300 --timeout-method thread
echo done

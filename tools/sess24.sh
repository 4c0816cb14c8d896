#!/bin/bash
# Session 24: k_tnx with one wave per 128x128 partial (measure + GEMM tests).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/s24
run() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > gpurun_out/s24/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -1 gpurun_out/s24/$name.log | cut -c1-1500; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run gemm_split 120 python -u tools/gemm_split_check.py
run pytest 300 python -u -m pytest tests/test_gpu_gemm.py -m gpu -q -rf --timeout 300 --timeout-method thread
echo done

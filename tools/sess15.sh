#!/bin/bash
# Session 15: split-bf16 weight-gradient kernel k_tnx + dx prologue; GEMM tests, bench.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); mkdir -p gpurun_out/s15; export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > gpurun_out/s15/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 gpurun_out/s15/$name.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run gemm_split 120 python -u tools/gemm_split_check.py
PPGAT_GEMM=fp32 run gemm_fp32 120 python -u tools/gemm_split_check.py
run pytest 400 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_parity.py tests/test_gpu_train_ops.py -m gpu -q -rf --timeout 170 --timeout-method thread
run bench 300 python -u bench.py --cpu-baseline-seconds 0
echo done

#!/bin/bash
# Session 36: k_tnx at 8 waves by default -- GEMM/parity/train tests, bench.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/s36; mkdir -p $OUT
run() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -1 $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run pytest 600 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_parity.py tests/test_gpu_train_ops.py tests/test_gpu_fullsize.py tests/test_gpu_dist.py -m gpu -q -rf --timeout 300 --timeout-method thread
run bench 200 python -u bench.py --cpu-baseline-seconds 0
run bench2 200 python -u bench.py --cpu-baseline-seconds 0
echo done

#!/bin/bash
# Session 18: split NN variants (tile width x k chunk) and split TN at config-5 shapes; config-5 bench.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); mkdir -p gpurun_out/s18; export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > gpurun_out/s18/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -1 gpurun_out/s18/$name.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
for v in 4x32 4x64 8x32; do PPGAT_NNX=$v run cfg5_$v 200 python -u tools/gemm_split_check.py --cfg5; done
run pytest 300 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_xgat.py tests/test_gpu_fusion.py -m gpu -q -rf --timeout 170 --timeout-method thread
run bench5 300 python -u bench.py --config 5 --steps 10 --warmup 3 --cpu-baseline-seconds 0
echo done

#!/bin/bash
# Session 47: dist tests with the forward split opt-in (world-1 RCCL fsplit cases) + default bench.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/s47; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 240 --timeout-method thread > $OUT/dist.log 2>&1 || { echo "dist rc=$?"; tail -30 $OUT/dist.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $OUT/dist.log | tail -20
echo done

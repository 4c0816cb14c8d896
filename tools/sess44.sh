#!/bin/bash
# Session 44 (also the final check): forward split by destination class (replicated partition, item-row merge
# overlapped with the user destinations) -- dist tests first, then the full GPU suite + bench.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${SESS_OUT:-s44}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 240 --timeout-method thread > $OUT/dist.log 2>&1 || { echo "dist rc=$?"; tail -30 $OUT/dist.log; exit 1; }
tail -3 $OUT/dist.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/gpu.log 2>&1 || { echo "gpu rc=$?"; tail -30 $OUT/gpu.log; exit 1; }
tail -3 $OUT/gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python -u bench.py > $OUT/bench.log 2>&1 || { echo "bench rc=$?"; tail -20 $OUT/bench.log; exit 1; }
grep -E "^\{" $OUT/bench.log | cut -c1-400
echo done

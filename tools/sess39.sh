#!/bin/bash
# Session 39: vectorized multi-head destination sum (CSC-order dz) -- tests, config-5 bench.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/s39; mkdir -p $OUT
run() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -1 $OUT/$name.log | cut -c1-250; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run pytest 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_xgat.py tests/test_gpu_fullsize.py tests/test_gpu_dist.py -m gpu -q -rf --timeout 300 --timeout-method thread
run bench5 400 python -u bench.py --config 5 --steps 10 --warmup 3 --cpu-baseline-seconds 0
grep -E "^\{" $OUT/bench5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['kernel_ms_per_step'], d['roofline']['frac'])"
echo done

#!/bin/bash
# Session 37: dz in CSC order (pass B contiguous stores, destination sums through csr2csc).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/s37; mkdir -p $OUT
run() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -1 $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
b() { grep -E "^\{" $OUT/$1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_ms_per_step']; print('$1', round(d['ms_per_step'],4), {a: round(v,4) for a,v in k.items()}, 'frac', round(d['roofline']['frac'],3))"; }
run pytest_new 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -rf --timeout 300 --timeout-method thread -k "dz_csc or bitwise or pyg_gatconv"
run bench 200 python -u bench.py --cpu-baseline-seconds 0; b bench
run bench2 200 python -u bench.py --cpu-baseline-seconds 0; b bench2
run pytest 1000 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
echo done

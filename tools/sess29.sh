#!/bin/bash
# Session 29: + non-temporal streamed operands in the projection / weight-gradient GEMMs.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/s29
run() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > gpurun_out/s29/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
b() { grep -E "^\{" gpurun_out/s29/$1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_ms_per_step']; print('$1', round(d['ms_per_step'],4), {a: round(v,4) for a,v in k.items()}, 'frac', round(d['roofline']['frac'],3))"; }
run bench 200 python -u bench.py --cpu-baseline-seconds 0; b bench
run bench2 200 python -u bench.py --cpu-baseline-seconds 0; b bench2
run gemm 120 python -u tools/gemm_split_check.py; tail -1 gpurun_out/s29/gemm.log | cut -c1-200
run pytest 300 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_parity.py -m gpu -q -rf --timeout 300 --timeout-method thread; tail -1 gpurun_out/s29/pytest.log
echo done

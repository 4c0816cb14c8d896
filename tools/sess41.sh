#!/bin/bash
# Session 41: BPR backward zeroes only the untouched dZ rows (no whole-dZ memset).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/s41; mkdir -p $OUT
run() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -1 $OUT/$name.log | cut -c1-250; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
b() { grep -E "^\{" $OUT/$1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1', round(d['ms_per_step'],4), 'frac', round(d['roofline']['frac'],3))"; }
run pytest 900 python -u -m pytest tests/test_gpu_train_ops.py tests/test_gpu_fullsize.py tests/test_gpu_dist.py tests/test_gpu_graph.py tests/test_gpu_eval.py tests/test_sampler.py -m gpu -q -rf --timeout 300 --timeout-method thread
run bench 200 python -u bench.py --cpu-baseline-seconds 0; b bench
run bench2 200 python -u bench.py --cpu-baseline-seconds 0; b bench2
echo done

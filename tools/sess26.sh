#!/bin/bash
# Session 26: config-2 bench in order vs with the weight-gradient GEMMs on a side stream.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/s26
run() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > gpurun_out/s26/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; grep -E "^\{" gpurun_out/s26/$name.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'])"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run inorder 200 python -u bench.py --cpu-baseline-seconds 0
PPGAT_ASYNC_WGRAD=1 run async 200 python -u bench.py --cpu-baseline-seconds 0
run inorder2 200 python -u bench.py --cpu-baseline-seconds 0
PPGAT_ASYNC_WGRAD=1 run async2 200 python -u bench.py --cpu-baseline-seconds 0
echo done

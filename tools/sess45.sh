#!/bin/bash
# Session 45: replicated path at world 1 over RCCL (every collective forced), hipGraph capture:
# forward split by destination class on (default) vs off.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/s45; mkdir -p $OUT
run() { local name=$1; shift; timeout -k 10 240 "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; grep -E "^\{" $OUT/$name.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],4), d.get('hip_graph'))"; if [ $rc -ne 0 ]; then tail -20 $OUT/$name.log; exit $rc; fi; }
A="python -u bench.py --dist-at-1 --partition replicated --cpu-baseline-seconds 0"
run split $A
PPGAT_FWD_SPLIT=0 run nosplit $A
run split2 $A
PPGAT_FWD_SPLIT=0 run nosplit2 $A
echo done

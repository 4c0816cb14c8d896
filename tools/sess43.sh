#!/bin/bash
# Session 43: short-item unroll (rows in flight per 16-lane row) 4 (default) vs 8 vs 16.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/s43; mkdir -p $OUT
run() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; grep -E "^\{" $OUT/$name.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_ms_per_step']; print(round(d['ms_per_step'],4), 'fwd', round(k['fwd'],4), 'bwd_src', round(k['bwd_src'],4))"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run base 200 python -u bench.py --cpu-baseline-seconds 0
PPGAT_LIB=$PWD/libppgat_su8.so run su8 200 python -u bench.py --cpu-baseline-seconds 0
PPGAT_LIB=$PWD/libppgat_su16.so run su16 200 python -u bench.py --cpu-baseline-seconds 0
run base2 200 python -u bench.py --cpu-baseline-seconds 0
PPGAT_LIB=$PWD/libppgat_su8.so run su8b 200 python -u bench.py --cpu-baseline-seconds 0
echo done

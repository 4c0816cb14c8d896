#!/bin/bash
# Session 27: non-temporal streamed rows in the edge kernels (variant library) vs default.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/s27
run() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > gpurun_out/s27/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; grep -E "^\{" gpurun_out/s27/$name.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_ms_per_step']; print(round(d['ms_per_step'],4), 'fwd', round(k['fwd'],4), 'bwd_src', round(k['bwd_src'],4), 'frac', round(d['roofline']['frac'],3))"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run base 200 python -u bench.py --cpu-baseline-seconds 0
PPGAT_LIB=$PWD/libppgat_ntvariant.so run nt 200 python -u bench.py --cpu-baseline-seconds 0
run base2 200 python -u bench.py --cpu-baseline-seconds 0
PPGAT_LIB=$PWD/libppgat_ntvariant.so run nt2 200 python -u bench.py --cpu-baseline-seconds 0
PPGAT_LIB=$PWD/libppgat_ntvariant.so run nt5 300 python -u bench.py --config 5 --steps 5 --warmup 2 --cpu-baseline-seconds 0
echo done

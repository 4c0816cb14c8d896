#!/bin/bash
# Session 14: split-bf16 projection kernels (accuracy + time vs the fp32 MFMA kernels), then the
# whole -m gpu suite, smoke, default bench and its kernel profile.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); mkdir -p gpurun_out/s14; export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > gpurun_out/s14/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 gpurun_out/s14/$name.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run gemm_split 120 python -u tools/gemm_split_check.py
PPGAT_GEMM=fp32 run gemm_fp32 120 python -u tools/gemm_split_check.py
run pytest 1000 python -u -m pytest tests -m gpu -v -rf --durations=15 --timeout 170 --timeout-method thread
run smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
run bench 300 python -u bench.py
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/s14/prof" -o run --output-format csv -- python "$R/bench.py" --steps 10 --warmup 3 --cpu-baseline-seconds 0 > "$R/gpurun_out/s14/prof.log" 2>&1); echo "prof rc=$?"
echo done

#!/bin/bash
# Session 4: projection kernel A/B (k_proj32 vs k_proj16) + its parity, then FusionMLP
# training tests / bench / counters (tools/fusion_pmc.sh).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
run() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -4 gpurun_out/$name.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run proj_parity 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_train_ops.py -m gpu -x -v -rf --timeout 120 --timeout-method thread
run gemm32 120 python -u tools/bench_gemm.py --only proj_fwd_scores,proj_dx
PPGAT_LIB=build_variants/p16/libppgat.so run gemm16 120 python -u tools/bench_gemm.py --only proj_fwd_scores,proj_dx
run bench2 200 python -u bench.py --steps 20 --warmup 5
bash tools/fusion_pmc.sh

#!/bin/bash
# Session 21: k_projx 8 waves + register prefetch vs 16 waves without.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); mkdir -p gpurun_out/s21; export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > gpurun_out/s21/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -1 gpurun_out/s21/$name.log | cut -c1-1500; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run p8 120 python -u tools/gemm_split_check.py
PPGAT_PROJX=16 run p16 120 python -u tools/gemm_split_check.py
echo done

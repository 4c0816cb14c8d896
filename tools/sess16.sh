#!/bin/bash
# Session 16: per-kernel durations of the split-bf16 GEMMs (rocprofv3 kernel trace of the check)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); mkdir -p gpurun_out/s16; export TMPDIR=/tmp
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/s16/split" -o run --output-format csv -- python "$R/tools/gemm_split_check.py" > "$R/gpurun_out/s16/split.log" 2>&1; echo "split rc=$?"
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_INSTS_VMEM --kernel-trace -d "$R/gpurun_out/s16/pmc" -o p --output-format csv -- python "$R/tools/gemm_split_check.py" --iters 3 > "$R/gpurun_out/s16/pmc.log" 2>&1; echo "pmc rc=$?"
echo done

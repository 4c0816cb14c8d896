#!/bin/bash
# Session 20: split kernels -- projection counters, FusionMLP inference (split vs fp32), GEMM + fusion tests.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); mkdir -p gpurun_out/s20; export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > gpurun_out/s20/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -1 gpurun_out/s20/$name.log | cut -c1-1500; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run pytest 400 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_fusion.py -m gpu -q -rf --timeout 300 --timeout-method thread
run gemm_split 120 python -u tools/gemm_split_check.py
run fusion_split 200 python -u tools/bench_fusion.py
PPGAT_GEMM=fp32 run fusion_fp32 200 python -u tools/bench_fusion.py
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d "$R/gpurun_out/s20/pmc" -o p --output-format csv -- python "$R/tools/gemm_split_check.py" --iters 3 > "$R/gpurun_out/s20/pmc.log" 2>&1; echo "pmc rc=$?"
echo done

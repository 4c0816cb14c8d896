#!/bin/bash
# PMC passes over tools/bench_gemm.py (one rocprofv3 run per counter group).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ARGS="${GEMM_ARGS:-}"   # e.g. --cfg5 (the config-5 share shapes)
R=$(pwd); OUT=$R/gpurun_out/gemm_pmc${GEMM_TAG:-}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 120 python tools/bench_gemm.py $ARGS > "$OUT/bench.json" 2>&1 || exit $?
cat "$OUT/bench.json"
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM SQ_INSTS_LDS" "TA_BUSY_avr TA_TA_BUSY_sum GRBM_GUI_ACTIVE" "SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVES"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/p$i" -o p -- python "$R/tools/bench_gemm.py" $ARGS --iters 3 > "$OUT/p$i.log" 2>&1) || echo "pass $i rc=$?"
done
echo done

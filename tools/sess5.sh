#!/bin/bash
# Session 5: the whole -m gpu suite on the current tree, then the fusion bench + counters.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
run() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -4 gpurun_out/$name.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run pytest_all 900 python -u -m pytest tests -m gpu -v -rf --timeout 170 --timeout-method thread
run fusion_bench 180 python -u tools/bench_fusion.py --train
R=$(pwd); OUT=$R/gpurun_out/fusion5; mkdir -p "$OUT"; export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM SQ_INSTS_LDS" "GRBM_GUI_ACTIVE GRBM_COUNT" "SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVES SQ_INSTS_SALU"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/p$i" -o p -- python "$R/tools/bench_fusion.py" --iters 3 > "$OUT/p$i.log" 2>&1) || { echo "pass $i rc=$?"; exit 1; }
done
(cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o s -- python "$R/tools/bench_fusion.py" --train --iters 5 > "$OUT/stats.log" 2>&1) || echo "stats rc=$?"
echo done

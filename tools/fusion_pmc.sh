#!/bin/bash
# FusionMLP: GPU tests, inference + training bench, kernel stats and PMC passes over
# tools/bench_fusion.py (one rocprofv3 run per counter group).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); OUT=$R/gpurun_out/fusion${FUSION_TAG:-}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_fusion.py tests/test_gpu_eval.py -m gpu -v -rf --timeout 150 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -5 "$OUT/pytest.log"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 180 python -u tools/bench_fusion.py --train > "$OUT/bench.json" 2>&1 || exit $?
cat "$OUT/bench.json"
(cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o s -- python "$R/tools/bench_fusion.py" --train --iters 5 > "$OUT/stats.log" 2>&1) || { echo "stats rc=$?"; exit 1; }
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM SQ_INSTS_LDS" "GRBM_GUI_ACTIVE GRBM_COUNT" "SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVES SQ_INSTS_SALU"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/p$i" -o p -- python "$R/tools/bench_fusion.py" --iters 3 > "$OUT/p$i.log" 2>&1) || { echo "pass $i rc=$?"; exit 1; }
done
(cd /tmp && timeout -k 5 60 rocprofv3 -L > "$OUT/avail.txt" 2>&1) || echo "list rc=$?"
echo done

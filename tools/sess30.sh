#!/bin/bash
# Session 30: split FusionMLP kernel counters (MFMA busy), per-rank floors at W=8 (collectives stubbed).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); OUT=$R/gpurun_out/s30; mkdir -p "$OUT"; export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM SQ_INSTS_LDS" "GRBM_GUI_ACTIVE GRBM_COUNT" "SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVES SQ_INSTS_SALU"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/p$i" -o p -- python "$R/tools/bench_fusion.py" --iters 3 > "$OUT/p$i.log" 2>&1) || { echo "pass $i rc=$?"; exit 1; }
  echo "pass $i ok"
done
python tools/pmc_kernel.py k_fusion_fwdx $OUT/p1 $OUT/p2 $OUT/p3 > $OUT/fusion_fwdx_pmc.json
timeout -k 10 200 python -u tools/scale_probe.py --world 8 --rank 0 --partition replicated --graph > $OUT/probe_rep_r0.log 2>&1; echo "probe rep rc=$?"; tail -2 $OUT/probe_rep_r0.log
timeout -k 10 200 python -u tools/scale_probe.py --world 8 --rank 7 --partition replicated --graph > $OUT/probe_rep_r7.log 2>&1; echo "probe rep7 rc=$?"; tail -2 $OUT/probe_rep_r7.log
echo done

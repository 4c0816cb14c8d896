#!/bin/bash
# Session 46: per-rank cost of the forward split (collectives stubbed, comm-stream paths on),
# replicated partition, W=2 and W=8 rank 0, hipGraph.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/s46; mkdir -p $OUT
run() { local name=$1; shift; timeout -k 10 240 "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; grep -E "^\{" $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then tail -20 $OUT/$name.log; exit $rc; fi; }
for W in 2 8; do
  P="python -u tools/scale_probe.py --world $W --rank 0 --graph --streams"
  run w${W}_split $P
  PPGAT_FWD_SPLIT=0 run w${W}_nosplit $P
  run w${W}_split2 $P
  PPGAT_FWD_SPLIT=0 run w${W}_nosplit2 $P
done
echo done

#!/bin/bash
# Session 48: per-rank cost of the backward source-class split (the only comm-stream overlap on
# by default for the replicated partition): scale_probe with the stub reported as RCCL (--streams,
# bwd_split overlap on) vs not (one pass-B launch, all-reduce inline), W=2 and W=8 rank 0.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/s48; mkdir -p $OUT
run() { local name=$1; shift; timeout -k 10 240 "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; grep -E "^\{" $OUT/$name.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],4), round(d['host_enqueue_ms_per_step'],4))"; if [ $rc -ne 0 ]; then tail -20 $OUT/$name.log; exit $rc; fi; }
for W in 2 8; do
  P="python -u tools/scale_probe.py --world $W --rank 0 --graph"
  run w${W}_streams $P --streams
  run w${W}_inline $P
  run w${W}_streams2 $P --streams
  run w${W}_inline2 $P
done
echo done

#!/bin/bash
# Session 32: config-5 kernel profile on this round's kernels.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); OUT=$R/gpurun_out/s32; mkdir -p "$OUT"; export TMPDIR=/tmp
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof5" -o run --output-format csv -- python "$R/bench.py" --config 5 --steps 5 --warmup 2 --cpu-baseline-seconds 0 > "$OUT/prof5.log" 2>&1); echo "prof5 rc=$?"
tail -1 $OUT/prof5.log | cut -c1-300
echo done

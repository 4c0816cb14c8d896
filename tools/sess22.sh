#!/bin/bash
# Session 22: k_projx time vs rows (fixed cost vs per-tile slope).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/s22
for n in 8192 32768 65536 131072 255404 510808 1021616; do
  timeout -k 10 120 python -u tools/gemm_split_check.py --n $n > gpurun_out/s22/n$n.log 2>&1 || exit $?
  python - "$n" <<'PY'
import json,sys; n=sys.argv[1]; d=json.loads(open(f"gpurun_out/s22/n{n}.log").read().strip().splitlines()[-1]); print(n, round(d["us_fwd_scores"],1), round(d["us_dx"],1), round(d["us_tn_V"],1))
PY
done

#!/bin/bash
# Session 35: k_tnx with 8 waves (2 per SIMD, no batches in flight) vs 4 waves + ring.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/s35; mkdir -p $OUT
run() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -1 $OUT/$name.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: (round(v,1) if isinstance(v,float) and v>1 else v) for k,v in d.items() if 'us' in k or 'tn' in k})"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run w4 120 python -u tools/gemm_split_check.py
PPGAT_TNX_WAVES=8 run w8 120 python -u tools/gemm_split_check.py
run w4b 120 python -u tools/gemm_split_check.py
PPGAT_TNX_WAVES=8 run w8b 120 python -u tools/gemm_split_check.py
echo done

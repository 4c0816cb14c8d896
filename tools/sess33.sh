#!/bin/bash
# Session 33: split NN with double-buffered images (one barrier per chunk, staging interleaved).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/s33; mkdir -p $OUT
run() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -1 $OUT/$name.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: (round(v,1) if isinstance(v,float) and v>1 else v) for k,v in d.items() if 'us' in k or 'err' in k or 'equal' in k})"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run base 200 python -u tools/gemm_split_check.py --cfg5
PPGAT_NNX_DB=1 run db8 200 python -u tools/gemm_split_check.py --cfg5
PPGAT_NNX_DB=4 run db4 200 python -u tools/gemm_split_check.py --cfg5
echo done

#!/bin/bash
# Session 31: conflict-free staging writes of the split images (fusion, NN layout 1).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); OUT=$R/gpurun_out/s31; mkdir -p "$OUT"; export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -1 $OUT/$name.log | cut -c1-700; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run fusion 200 python -u tools/bench_fusion.py
run cfg5 200 python -u tools/gemm_split_check.py --cfg5
run pytest 300 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_fusion.py tests/test_gpu_xgat.py -m gpu -q -rf --timeout 300 --timeout-method thread
(cd /tmp && timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/p" -o p -- python "$R/tools/bench_fusion.py" --iters 3 > "$OUT/p.log" 2>&1) || { echo "pmc rc=$?"; exit 1; }
python tools/pmc_kernel.py k_fusion_fwdx $OUT/p
echo done

#!/bin/bash
# Session 11: config-2 PMC traffic on this round's tree (FETCH_SIZE and WRITE_SIZE in separate
# passes), the default bench line, and the tests touched since the last full run.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); mkdir -p gpurun_out/s11; export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > gpurun_out/s11/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 gpurun_out/s11/$name.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run pytest 400 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_fusion.py -m gpu -v -rf --timeout 170 --timeout-method thread
for c in FETCH_SIZE WRITE_SIZE; do
  (cd /tmp && timeout -s KILL 180 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$R/gpurun_out/s11/pmc_$c" -o p -- python "$R/bench.py" --steps 5 --warmup 2 --graph off --cpu-baseline-seconds 0 > "$R/gpurun_out/s11/pmc_$c.log" 2>&1) || { echo "pmc $c rc=$?"; exit 1; }
  echo "pmc $c ok"
done
python tools/pmc_summary.py gpurun_out/s11/pmc_FETCH_SIZE gpurun_out/s11/pmc_WRITE_SIZE gpurun_out/s11/cfg2_pmc_traffic.json 2 > gpurun_out/s11/pmc_summary.log 2>&1
run bench2 200 python -u bench.py
echo done

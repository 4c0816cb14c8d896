#!/bin/bash
# Session 9: whole -m gpu suite, smoke, N=1 bench (config 2, default flags) and its rocprofv3
# kernel summary, config 5 share bench.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); mkdir -p gpurun_out/s9; export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > gpurun_out/s9/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 gpurun_out/s9/$name.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run pytest_all 900 python -u -m pytest tests -m gpu -v -rf --timeout 170 --timeout-method thread
run smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
run bench2 200 python -u bench.py
(cd /tmp && timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/s9/prof2" -o s -- python "$R/bench.py" --steps 20 --warmup 5 --cpu-baseline-seconds 0 > "$R/gpurun_out/s9/prof2.log" 2>&1) || { echo "prof2 rc=$?"; exit 1; }
tail -1 gpurun_out/s9/prof2.log
run bench5 400 python -u bench.py --config 5 --steps 10 --warmup 3
echo done

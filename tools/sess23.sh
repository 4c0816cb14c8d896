#!/bin/bash
# Session 23: the whole -m gpu suite, smoke, config-2 bench + kernel profile, config-5 bench, fusion bench.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); mkdir -p gpurun_out/s23; export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > gpurun_out/s23/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -1 gpurun_out/s23/$name.log | cut -c1-600; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run pytest 1000 python -u -m pytest tests -m gpu -v -rf --durations=15 --timeout 300 --timeout-method thread
run smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
run bench 300 python -u bench.py
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/s23/prof" -o run --output-format csv -- python "$R/bench.py" --steps 10 --warmup 3 --cpu-baseline-seconds 0 > "$R/gpurun_out/s23/prof.log" 2>&1); echo "prof rc=$?"
run bench5 300 python -u bench.py --config 5 --steps 10 --warmup 3 --cpu-baseline-seconds 0
run fusion 200 python -u tools/bench_fusion.py
echo done

#!/bin/bash
# Session 41f (round-2 final tree, after the BPR gap zeroing): whole -m gpu suite, smoke, default bench + its kernel profile.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); OUT=$R/gpurun_out/s41f; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -1 $OUT/$name.log | cut -c1-250; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run pytest 1000 python -u -m pytest tests -m gpu -v -rf --durations=15 --timeout 300 --timeout-method thread
run smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
run bench 300 python -u bench.py
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python "$R/bench.py" --steps 10 --warmup 3 --cpu-baseline-seconds 0 > "$OUT/prof.log" 2>&1); echo "prof rc=$?"
echo done

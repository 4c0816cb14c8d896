#!/bin/bash
# Session 38: dz in CSC order -- bench line, kernel profile, config-2 PMC traffic, config-5 bench.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); OUT=$R/gpurun_out/s38; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -1 $OUT/$name.log | cut -c1-200; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python "$R/bench.py" --steps 10 --warmup 3 --cpu-baseline-seconds 0 > "$OUT/prof.log" 2>&1); echo "prof rc=$?"
for c in FETCH_SIZE WRITE_SIZE; do
  (cd /tmp && timeout -s KILL 180 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$OUT/pmc_$c" -o p -- python "$R/bench.py" --steps 5 --warmup 2 --graph off --cpu-baseline-seconds 0 > "$OUT/pmc_$c.log" 2>&1) || { echo "pmc $c rc=$?"; exit 1; }
  echo "pmc $c ok"
done
python tools/pmc_summary.py $OUT/pmc_FETCH_SIZE $OUT/pmc_WRITE_SIZE $OUT/cfg2_pmc_traffic.json 2 > $OUT/pmc_summary.log 2>&1; echo "summary rc=$?"
cp $OUT/cfg2_pmc_traffic.json profiles/r02/cfg2_pmc_traffic.json
run bench 300 python -u bench.py
run bench5 400 python -u bench.py --config 5 --steps 10 --warmup 3 --cpu-baseline-seconds 0
echo done

#!/bin/bash
# Session 8: per-rank kernel profiles of the two partitions at 8 ranks (scale_probe under
# rocprofv3 --stats), dropout/graph tests after folding the seed snapshot into k_fwd, N=1 bench.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); mkdir -p gpurun_out/s8; export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > gpurun_out/s8/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 gpurun_out/s8/$name.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run pytest_seed 400 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_parity.py tests/test_gpu_dist.py -m gpu -x -v -rf --timeout 170 --timeout-method thread
for part in halo replicated; do
  (cd /tmp && timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/s8/prof_$part" -o s -- python "$R/tools/scale_probe.py" --world 8 --rank 0 --partition $part --graph > "$R/gpurun_out/s8/prof_$part.log" 2>&1) || { echo "prof $part rc=$?"; exit 1; }
  tail -1 gpurun_out/s8/prof_$part.log
done
run probe_halo_r7 150 python -u tools/scale_probe.py --world 8 --rank 7 --partition halo --graph
run bench2 200 python -u bench.py --steps 20 --warmup 5
echo done

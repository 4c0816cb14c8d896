#!/bin/bash
# Session 7: fixed debug / trainer tests, halo per-rank floors, config-5 GEMM layout A/B,
# config-5 bench with the committed PMC traffic.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/s7
run() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > gpurun_out/s7/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 gpurun_out/s7/$name.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run pytest_fix 400 python -u -m pytest tests/test_gpu_debug.py "tests/test_gpu_eval.py::test_trainer_two_ranks_matches_single_gpu" -m gpu -v -rf --timeout 170 --timeout-method thread
for rk in 0 7; do
  run probe_halo_r$rk 150 python -u tools/scale_probe.py --world 8 --rank $rk --partition halo --graph
done
run gemm5 300 python -u tools/bench_gemm.py --cfg5 --iters 5
run gemm2 120 python -u tools/bench_gemm.py
run bench5 400 python -u bench.py --config 5 --steps 10 --warmup 3
echo done

#!/bin/bash
# Session 6: per-rank floors of the two partitions at 8 ranks (config 2 graph, collectives
# stubbed, graph replay), and the config-5 share's PMC traffic (separate passes per counter
# group) for the honest-HBM roofline.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); mkdir -p gpurun_out/s6; export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > gpurun_out/s6/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 gpurun_out/s6/$name.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run pytest_new 600 python -u -m pytest tests/test_gpu_debug.py tests/test_gpu_gemm.py tests/test_gpu_dist.py "tests/test_gpu_eval.py::test_trainer_two_ranks_matches_single_gpu" -m gpu -v -rf --timeout 170 --timeout-method thread || true
for part in replicated halo; do
  for rk in 0 7; do
    run probe_${part}_r$rk 150 python -u tools/scale_probe.py --world 8 --rank $rk --partition $part --graph
  done
done
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$R/gpurun_out/s6/c5p$i" -o p -- python "$R/bench.py" --config 5 --steps 2 --warmup 1 --graph off > "$R/gpurun_out/s6/c5p$i.log" 2>&1) || { echo "c5 pass $i rc=$?"; exit 1; }
  echo "c5 pass $i ok"
done
echo done

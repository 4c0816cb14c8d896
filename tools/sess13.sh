#!/bin/bash
# Session 13: replicated backward with the item-row all_reduce overlapped (RCCL at world 1 with
# every collective forced through it), incl. hipGraph capture of the overlapped step.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/s13
run() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > gpurun_out/s13/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 gpurun_out/s13/$name.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run pytest 500 python -u -m pytest tests/test_gpu_dist.py -m gpu -v -rf --timeout 170 --timeout-method thread
PPGAT_COMM_ALWAYS=1 run bench_d1 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29517 bench.py --dist-at-1 --graph on --steps 10 --warmup 3 --cpu-baseline-seconds 0
run probe_rep 200 python -u tools/scale_probe.py --world 8 --rank 0 --partition replicated --graph
echo done

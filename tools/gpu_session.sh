#!/bin/bash
# One gpurun session: GPU tests, smoke, bench, rocprofv3 kernel stats.
# Stops at the first step that does not end with 0 or 1 (a fault, abort, timeout...).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
export TMPDIR=/tmp
OUT=$R/gpurun_out
mkdir -p "$OUT"
STEPS="${STEPS:-tests smoke bench prof}"
TESTS="${TESTS:-tests}"   # the 'sel' step: the test files / node ids to run
BENCH_ARGS="${BENCH_ARGS:---steps 20 --warmup 5}"
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" | tee -a "$OUT/session.log"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a "$OUT/session.log"
  tail -5 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for s in $STEPS; do
  case $s in
    tests) run pytest_gpu 1100 python -u -m pytest tests -m gpu -v -rf --durations=15 --timeout 170 --timeout-method thread ;;
    fast) run pytest_gpu_fast 900 python -u -m pytest tests -m gpu -q -rf --durations=10 --timeout 120 --timeout-method thread --deselect tests/test_gpu_fullsize.py ;;
    fullsize) run pytest_fullsize 900 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -v -s -rf --durations=0 --timeout 170 --timeout-method thread ;;
    dist) run pytest_dist 600 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_graph.py -m gpu -v -rf --timeout 120 --timeout-method thread ;;
    gemm) run pytest_gemm 300 python -u -m pytest tests/test_gpu_gemm.py -m gpu -q -rf --timeout 120 --timeout-method thread ;;
    sampler) run pytest_sampler 300 python -u -m pytest tests/test_sampler.py "tests/test_gpu_eval.py::test_trainer_device_sampler" -m gpu -q -rf --timeout 120 --timeout-method thread ;;
    bsampler) run bench_sampler 300 python tools/bench_sampler.py ;;
    sel) run pytest_sel 1100 python -u -m pytest $TESTS -m gpu -v -s -rf --durations=15 --timeout 170 --timeout-method thread ;;
    traj) for v in default:PPGAT_NONE=1 fuseddxw0:PPGAT_FUSED_DXW=0 gemmfp32:PPGAT_GEMM=fp32; do
            run "traj_${v%%:*}" 900 env PPGAT_REPORT_TAG="${v%%:*}" "${v#*:}" python -u -m pytest tests/test_gpu_trajectory.py -m gpu -v -s -rf --timeout 800 --timeout-method thread
          done ;;
    probe5) for a in ${PROBES:-0:0 7:0 7:640}; do IFS=: read -r pr pg pe <<< "$a"
              run "probe5_r${pr}_a${pg}${pe:+_${pe//=/}}" 900 env ${pe:-PPGAT_NONE=1} python -u tools/scale_probe.py --config 5 --world 8 --rank $pr --streams --a2a-gbs $pg --steps 5 --warmup 2 ${PROBE_ARGS:-}
            done ;;
    gemm5) run gemm5_nnh 300 env PPGAT_LIB=lab_build/libppgat.so PPGAT_NNH2=0 python tools/bench_gemm.py --cfg5 --iters 10 && \
           run gemm5_nnh2 300 env PPGAT_LIB=lab_build/libppgat.so PPGAT_NNH2=2 python tools/bench_gemm.py --cfg5 --iters 10 && \
           for v in ${NNHVS:-3}; do run "gemm5_nnh$v" 300 env PPGAT_NNH2=$v python tools/bench_gemm.py --cfg5 --iters 10; done ;;
    pmcdst) (cd /tmp && run pmcdst_a 300 timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d "$OUT/pmcdst_a" -o a -- python "$R/bench.py" --steps 3 --warmup 1 --graph off --cpu-baseline-seconds 0) && \
            (cd /tmp && run pmcdst_b 300 timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_REQ_sum --kernel-trace --output-format csv -d "$OUT/pmcdst_b" -o b -- python "$R/bench.py" --steps 3 --warmup 1 --graph off --cpu-baseline-seconds 0) && \
            python "$R/tools/pmc_kernel.py" "k_dst_sum<true>" "$OUT/pmcdst_a" "$OUT/pmcdst_b" > "$OUT/pmc_dst_sum.json" && \
            python "$R/tools/pmc_kernel.py" "k_bwd_src<" "$OUT/pmcdst_a" "$OUT/pmcdst_b" > "$OUT/pmc_bwd_src_tcc.json" ;;
    dstlab) for a in ${DSTAUX:-0 2 17 19}; do
              (cd /tmp && run "dstlab2_aux$a" 300 env PPGAT_LIB=$R/lab_build/libppgat.so PPGAT_DST_AUX=$a timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RD_UNCACHED_32B_sum --kernel-trace --output-format csv -d "$OUT/dstlab2_$a" -o p -- python "$R/bench.py" --steps 3 --warmup 1 --graph off --cpu-baseline-seconds 0) || exit 1
              python "$R/tools/pmc_kernel.py" "k_dst_sum<true" "$OUT/dstlab2_$a" > "$OUT/dstlab2_aux$a.json"
              if [ -n "${DST5:-}" ]; then
                (cd /tmp && run "dstlab5_aux$a" 400 env PPGAT_LIB=$R/lab_build/libppgat.so PPGAT_DST_AUX=$a timeout -s KILL 360 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RD_UNCACHED_32B_sum --kernel-trace --output-format csv -d "$OUT/dstlab5_$a" -o p -- python -u "$R/bench.py" --config 5 --steps 2 --warmup 1 --graph off --cpu-baseline-seconds 0) || exit 1
                python "$R/tools/pmc_kernel.py" "k_dst_sum_vh<" "$OUT/dstlab5_$a" > "$OUT/dstlab5_long_aux$a.json"
                python "$R/tools/pmc_kernel.py" "k_dst_sum_vh_short" "$OUT/dstlab5_$a" > "$OUT/dstlab5_short_aux$a.json"
              fi
            done ;;
    e4lab) run gemm5_base 300 python tools/bench_gemm.py --cfg5 --iters 10 && \
           run gemm5_e4 300 env PPGAT_LIB=lab_build/libppgat.so PPGAT_NNH_E4=1 python tools/bench_gemm.py --cfg5 --iters 10 && \
           run bench5_e4 600 env PPGAT_LIB=lab_build/libppgat.so PPGAT_NNH_E4=1 python -u bench.py --config 5 --steps 10 --warmup 3 ;;
    occ2lab) run gemm5_base 300 python tools/bench_gemm.py --cfg5 --iters 10 && \
           run gemm5_occ2 300 env PPGAT_LIB=lab_build/libppgat.so PPGAT_NNH_OCC2=1 python tools/bench_gemm.py --cfg5 --iters 10 ;;
    tnpmc) run tn5_256 120 python tools/bench_gemm.py --tn5 --iters 10 && \
           run tn5_128 120 env PPGAT_LIB=lab_build/libppgat.so PPGAT_TNH256=0 python tools/bench_gemm.py --tn5 --iters 10 && \
           run tnpmc256 400 env GEMM_ARGS=--tn5 GEMM_TAG=_tn256 bash tools/gemm_pmc.sh && \
           python tools/pmc_kernel.py "k_gemm_tnh256" "$OUT/gemm_pmc_tn256/p1" "$OUT/gemm_pmc_tn256/p2" "$OUT/gemm_pmc_tn256/p3" > "$OUT/tn256_pmc.json" ;;
    nnhpmc) run "nnhpmc${NNHV:-3}" 500 env GEMM_ARGS=--cfg5 GEMM_TAG="_nnh${NNHV:-3}" PPGAT_NNH2="${NNHV:-3}" bash tools/gemm_pmc.sh ;;
    nnhlab) for l in ${LABS:-0 1 2 3}; do run "nnhlab$l" 300 env PPGAT_LIB=lab_build/libppgat.so PPGAT_NNH2_LAB=$l python tools/bench_gemm.py --cfg5 --iters 10; done ;;
    probec2) for a in ${C2PROBES:-2:300 4:300 8:300 8:0}; do set -- ${a%%:*} ${a#*:}
              run "probec2_w$1_a$2" 300 python -u tools/scale_probe.py --world $1 --rank 0 --graph --streams --a2a-gbs $2 --steps 20 --warmup 5
            done ;;
    profprobe640) (cd /tmp && run rocprof_probe5_640 900 rocprofv3 --kernel-trace --stats -d "$OUT/profprobe640" -o run --output-format csv -- python "$R/tools/scale_probe.py" --config 5 --world 8 --rank ${PROBE_RANK:-0} --streams --a2a-gbs 640 --steps 3 --warmup 1) ;;
    profprobe) (cd /tmp && run rocprof_probe5 900 rocprofv3 --kernel-trace --stats -d "$OUT/profprobe" -o run --output-format csv -- python "$R/tools/scale_probe.py" --config 5 --world 8 --rank ${PROBE_RANK:-7} --streams --steps 3 --warmup 1) ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py $BENCH_ARGS ;;
    bench3) run bench_cfg3 600 python bench.py --config 3 --cpu-baseline-seconds 0 ;;
    copylab) run copy_lab 120 tools/copy_lab ;;
    fwdxu) for u in ${FWDXU:-8 6 4}; do run "bench5_fwdx_u$u" 600 env PPGAT_LIB=lab_build/libppgat.so PPGAT_FWDX_U=$u python -u bench.py --config 5 --steps 5 --warmup 2 --graph off; done ;;
    bench5full) run bench_cfg5_full 1000 python -u bench.py --config 5 --scale 1 --steps ${FULL_STEPS:-3} --warmup 1 --graph ${FULL_GRAPH:-on} ;;
    prof5full) (cd /tmp && run rocprof_cfg5_full 1000 rocprofv3 --kernel-trace --stats -d "$OUT/prof5full" -o run --output-format csv -- python -u "$R/bench.py" --config 5 --scale 1 --steps 2 --warmup 1 --graph off) ;;
    bench5) run bench_cfg5 900 python -u bench.py --config 5 --steps 10 --warmup 3 ;;
    prof5)  (cd /tmp && run rocprof_cfg5 900 rocprofv3 --kernel-trace --stats -d "$OUT/prof5" -o run --output-format csv -- python "$R/bench.py" --config 5 --steps 5 --warmup 2) ;;
    pmc5)  (cd /tmp && run pmc5_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc5_fetch" -o fetch -- python "$R/bench.py" --config 5 --steps 2 --warmup 1 --graph off --cpu-baseline-seconds 0) && \
           (cd /tmp && run pmc5_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/pmc5_write" -o write -- python "$R/bench.py" --config 5 --steps 2 --warmup 1 --graph off --cpu-baseline-seconds 0) && \
           python "$R/tools/pmc_summary.py" "$OUT/pmc5_fetch" "$OUT/pmc5_write" "$OUT/cfg5_pmc_traffic.json" 5 scale=0.125 bwd_gather=gd > "$OUT/pmc5_summary.log" 2>&1 ;;
    fusion) run bench_fusion 300 python tools/bench_fusion.py && \
            run bench_fusion3 300 env PPGAT_NNH2=3 python tools/bench_fusion.py ;;
    fusionpmc) run "fusionpmc${NNHV:-3}" 500 env PPGAT_NNH2="${NNHV:-3}" FUSION_TAG="_nnh${NNHV:-3}" bash tools/fusion_pmc.sh ;;
    pmc6)  for pass in fetch:FETCH_SIZE write:WRITE_SIZE dram:"TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_DRAM_sum"; do
             (cd /tmp && run "pmc6_${pass%%:*}" 300 timeout -s KILL 240 rocprofv3 --pmc ${pass#*:} --kernel-trace --output-format csv -d "$OUT/pmc6_${pass%%:*}" -o p -- python "$R/bench.py" --steps 3 --warmup 1 --graph off --cpu-baseline-seconds 0) || exit 1
           done
           python "$R/tools/pmc_summary.py" "$OUT/pmc6_fetch" "$OUT/pmc6_write" "$OUT/cfg2_pmc_traffic.json" 2 dram_dir="$OUT/pmc6_dram" > "$OUT/pmc6_summary.log" 2>&1 ;;
    prof)  (cd /tmp && run rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python "$R/bench.py" --steps 10 --warmup 3 --cpu-baseline-seconds 0) ;;
    pmc)   (cd /tmp && run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_fetch" -o fetch -- python "$R/bench.py" --steps 3 --warmup 1 --cpu-baseline-seconds 0) && \
           (cd /tmp && run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_write" -o write -- python "$R/bench.py" --steps 3 --warmup 1 --cpu-baseline-seconds 0) && \
           python "$R/tools/pmc_summary.py" "$OUT/pmc_fetch" "$OUT/pmc_write" "$OUT/pmc_traffic.json" > "$OUT/pmc_summary.log" 2>&1 ;;
  esac
done
echo "session done"

#!/bin/bash
# Build experiment variants of libppgat.so that differ in one translation unit:
#   tools/build_variants.sh SRC NAME:"-DFLAG=1 ..." [NAME2:"..."] ...
# Each variant: $OUTDIR/NAME/libppgat.so (OUTDIR default build_variants; the other objects from
# csrc/build).  build_variants/ stays here (.gpurunignore); OUTDIR=lab_build travels to the box.
# Use with PPGAT_LIB=$OUTDIR/NAME/libppgat.so python tools/bench_gemm.py
set -e
cd "$(dirname "$0")/.."
C=plotpointe-gat-recommendation_amd/csrc
make -s -C $C >/dev/null
SRC=$1; shift
base=$(basename "$SRC" .hip)
others=$(ls $C/build/*.o | grep -v "/$base.o")
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  mkdir -p ${OUTDIR:-build_variants}/$name
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result $flags -I$C \
    -c "$SRC" -o ${OUTDIR:-build_variants}/$name/$base.o &
done
wait
for spec in "$@"; do
  name=${spec%%:*}
  O=${OUTDIR:-build_variants}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $O/$name/libppgat.so $O/$name/$base.o $others
  echo "built $O/$name/libppgat.so"
done

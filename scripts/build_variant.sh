#!/bin/bash
# Build an alternative libpoissbox_gpu.so with extra compile definitions into variants/<name>.so
# (load it with PB_LIB=variants/<name>.so). usage: scripts/build_variant.sh <name> -DFOO=1 ...
set -eu
name=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/poissbox_amd/csrc
B=/tmp/pb_variant_$name
mkdir -p $B $R/variants
objs=""
for f in pb_runtime.cpp pb_solver.cpp pb_stencil.hip pb_vecops.hip pb_compact.hip pb_compact_fast.hip pb_compact_lines.hip pb_cg_generic.hip pb_mg.hip pb_mg_sweep.hip pb_compact_dist.hip; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off "$@" -I$R/include -I/opt/rocm/include -x hip -c $C/$f -o $B/$f.o &
  objs="$objs $B/$f.o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $R/variants/$name.so $objs -L/opt/rocm/lib -lrccl -lrocprofiler-sdk-roctx -Wl,-rpath,/opt/rocm/lib
echo "built variants/$name.so"

#!/bin/bash
# Build an alternative libpoissbox_gpu.so with extra compile definitions into variants/<name>.so
# (load it with PB_LIB=variants/<name>.so). usage: scripts/build_variant.sh <name> -DFOO=1 ...
set -eu
name=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p $R/variants
make -s -j8 -C $R/poissbox_amd/csrc OUT=$R/variants/$name.so BUILD=/tmp/pb_variant_$name EXTRA="$*"
echo "built variants/$name.so"

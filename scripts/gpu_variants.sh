#!/bin/bash
# Kernel-variant experiment: bench timings per variant library (variants/<name>.so via PB_LIB,
# "-" = the product build), then PMC FETCH_SIZE / WRITE_SIZE passes per variant.
# usage: gpu_variants.sh OUTNAME REPS name... [-- bench args]
set -u
R=${GRAFT_REPO_ROOT:-.}
out=$1; reps=$2; shift 2
names=(); extra=()
while [ $# -gt 0 ]; do if [ "$1" == "--" ]; then shift; extra=("$@"); break; fi; names+=("$1"); shift; done
cfgs=()
for n in "${names[@]}"; do if [ "$n" == "-" ]; then cfgs+=("-"); else cfgs+=("PB_LIB=$R/variants/$n.so"); fi; done
bash $R/scripts/gpu_ab.sh $out $reps "${cfgs[@]}" -- "${extra[@]}" || exit $?
cd /tmp && export TMPDIR=/tmp
for n in "${names[@]}"; do
  for c in FETCH_SIZE WRITE_SIZE; do
    d=$R/gpurun_out/var_$out/$n/$c; mkdir -p $d
    if [ "$n" == "-" ]; then lib=""; else lib=$R/variants/$n.so; fi
    PB_LIB=$lib timeout -k 10 240 rocprofv3 --pmc $c -d $d -o pmc --output-format csv -- python3 $R/bench.py --steps 8 --warmup 2 --matvecs 8 --no-cpu-baseline "${extra[@]}" > $d/bench.json 2> $d/bench.err
    rc=$?; echo "pmc $n $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done

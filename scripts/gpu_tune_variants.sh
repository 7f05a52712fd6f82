#!/bin/bash
# A/B of kernel variants built by scripts/build_variant.sh: tune_stencil.py once per library
# (VARIANTS: space-separated names under variants/, "base" = the in-tree library).
set -u
mkdir -p gpurun_out
DEFCFG='[{}]'
[ -n "${CONFIGS:-}" ] || CONFIGS=$DEFCFG
for v in ${VARIANTS:-base}; do
  lib=""; [ "$v" != "base" ] && lib=$GRAFT_REPO_ROOT/variants/$v.so
  PB_LIB=$lib PB_TUNE_CONFIGS="$CONFIGS" PB_TUNE_ROUNDS=${ROUNDS:-4} timeout -k 10 600 python scripts/tune_stencil.py > gpurun_out/tune_$v.log 2>&1
  rc=$?; echo "variant $v rc=$rc"; cat gpurun_out/tune_$v.log | python3 -c "
import sys,json
for l in sys.stdin:
    l=l.strip()
    if not l.startswith('{'): print(l); continue
    d=json.loads(l); print('$v', d['cfg'], {k:round(x,4) for k,x in d.items() if k.endswith('med_ms')})"
  [ $rc -eq 0 ] || exit $rc
done

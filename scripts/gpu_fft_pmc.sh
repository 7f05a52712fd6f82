#!/bin/bash
# LDS / issue counters of the spectral-PC passes (bench_fft 512), default build and variants/zlds.so
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/fftpmc
cd /tmp && export TMPDIR=/tmp
for v in base zlds; do
  if [ $v = base ]; then unset PB_LIB; else export PB_LIB=$R/variants/$v.so; fi
  timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS -d $R/gpurun_out/fftpmc/$v -o pmc --output-format csv -- python3 $R/scripts/bench_fft.py 512 > $R/gpurun_out/fftpmc/$v.jsonl 2> $R/gpurun_out/fftpmc/$v.err
  rc=$?; echo "$v rc=$rc"; [ $rc -eq 0 ] || exit $rc
done

#!/bin/bash
# r03 CG fusions on the compact operator: compact / fft / mg parity subsets, then config-5
# solves (fused, and PB_CG_FUSE=0) and their kernel trace; then the Z-pass access probe
set -u
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/fuse
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "compact or fft" --timeout 300 --timeout-method thread > gpurun_out/fuse/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/fuse/pytest.log; [ $rc -eq 0 ] || exit $rc
OP=compact PCS=fft NO_CPU=1 timeout -k 10 300 python scripts/bench_solve.py 256 512 > gpurun_out/fuse/solve_fft_compact.jsonl 2> gpurun_out/fuse/s1.err
rc=$?; echo "cfg5 rc=$rc"; cat gpurun_out/fuse/solve_fft_compact.jsonl; [ $rc -eq 0 ] || exit $rc
PB_CG_FUSE=0 OP=compact PCS=fft NO_CPU=1 timeout -k 10 300 python scripts/bench_solve.py 256 512 > gpurun_out/fuse/solve_fft_compact_nofuse.jsonl 2> gpurun_out/fuse/s2.err
rc=$?; echo "cfg5 nofuse rc=$rc"; cat gpurun_out/fuse/solve_fft_compact_nofuse.jsonl; [ $rc -eq 0 ] || exit $rc
hipcc -O3 --offload-arch=gfx950 -o /tmp/zpass_probe scripts/zpass_probe.hip && timeout -k 10 120 /tmp/zpass_probe > gpurun_out/fuse/zpass_probe.jsonl
rc=$?; echo "probe rc=$rc"; cat gpurun_out/fuse/zpass_probe.jsonl; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
OP=compact PCS=fft NO_CPU=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/fuse/kt -o cfg5 --output-format csv \
  -- python3 $R/scripts/bench_solve.py 512 > $R/gpurun_out/fuse/kt.jsonl 2> $R/gpurun_out/fuse/kt.err
rc=$?; echo "kt rc=$rc"; exit $rc

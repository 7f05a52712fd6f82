#!/bin/bash
# r03 first GPU pass: tests + smoke + bench (gpu_check.sh), the self-launched 2-rank bench over
# the host transport, the Z-pass access-pattern probe, and PMC counters of the spectral PC's line
# passes at 512^3 and 1024^3 (one counter group per run). Stops at the first crash-class status.
set -u
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r3a
BENCH_ARGS="--steps 50 --warmup 5 --cpu-baseline none" bash scripts/gpu_check.sh
rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 2 --transport host --base 64 --steps 5 --warmup 2 \
  > gpurun_out/r3a/bench_self2.json 2> gpurun_out/r3a/bench_self2.err
rc=$?; echo "self-launch rc=$rc"; cat gpurun_out/r3a/bench_self2.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 scripts/zpass_probe > gpurun_out/r3a/zpass_probe.jsonl 2>&1
rc=$?; echo "probe rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  tag=$(echo $grp | tr ' ' '_')
  timeout -k 10 240 rocprofv3 --pmc $grp -d $R/gpurun_out/r3a/pmc_fft_$tag -o pmc --output-format csv \
    -- python3 $R/scripts/bench_fft.py 512 1024 > $R/gpurun_out/r3a/pmc_fft_$tag.jsonl 2> $R/gpurun_out/r3a/pmc_fft_$tag.err
  rc=$?; echo "$grp rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r3a/kt_fft -o fft --output-format csv \
  -- python3 $R/scripts/bench_fft.py 512 1024 > $R/gpurun_out/r3a/kt_fft.jsonl 2> $R/gpurun_out/r3a/kt_fft.err
rc=$?; echo "kt rc=$rc"; exit $rc

#!/bin/bash
# r03 closing profile set on one box: every GPU test, smoke, bench (gpu_check.sh); rocprofv3
# kernel-trace stats of the bench; PMC passes of the bench (gpu_pmc.sh) and of the spectral PC;
# per-row bench; MG / Jacobi / config-5 solves; SURVEY 8(d) protocol. Stops at the first failure.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/close
mkdir -p $O
cd $R && PYTEST_ARGS="--timeout 300 --timeout-method thread" bash scripts/gpu_check.sh || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 $R/bench.py --steps 50 --warmup 5 --no-cpu-baseline --secondary 0 > $O/bench_prof.json 2> $O/bench_prof.err
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd $R && bash scripts/gpu_pmc.sh || exit $?
cd /tmp
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  timeout -s KILL 120 rocprofv3 --pmc $grp -d $O/fftpmc_$grp -o pmc --output-format csv -- python3 $R/scripts/bench_fft.py 512 > $O/fftpmc_$grp.jsonl 2> $O/fftpmc_$grp.err
  rc=$?; echo "fft pmc $grp rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
cd $R && timeout -k 10 900 python scripts/bench_rows.py > $O/rows.jsonl 2> $O/rows.err
rc=$?; echo "rows rc=$rc"; [ $rc -eq 0 ] || exit $rc
PCS=mg,jacobi NO_CPU=1 timeout -k 10 600 python scripts/bench_solve.py 256 512 > $O/solve_star7.jsonl 2> $O/solve.err
rc=$?; echo "solve rc=$rc"; [ $rc -eq 0 ] || exit $rc
OP=compact PCS=fft NO_CPU=1 timeout -k 10 300 python scripts/bench_solve.py 256 512 > $O/solve_fft_compact.jsonl 2>> $O/solve.err
rc=$?; echo "cfg5 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/bench_fft.py 512 256 1024 > $O/fft.jsonl 2> $O/fft.err
rc=$?; echo "fft rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/bench_compact.py 512 256 > $O/compact.jsonl 2> $O/compact.err
rc=$?; echo "compact rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python scripts/bench_protocol.py 512 > $O/protocol_512.jsonl 2> $O/protocol.err
rc=$?; echo "protocol rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/bench_protocol.py 256 > $O/protocol_256.jsonl 2>> $O/protocol.err
rc=$?; echo "protocol256 rc=$rc"; exit $rc

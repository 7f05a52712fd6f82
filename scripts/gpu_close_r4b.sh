#!/bin/bash
# r04 closing set, part B (one box): per-row bench, solves, spectral-PC / compact passes, the
# SURVEY 8(d) protocol; stops at the first failure
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/close4b
mkdir -p $O
cd $R
timeout -k 10 900 python scripts/bench_rows.py > $O/rows.jsonl 2> $O/rows.err
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

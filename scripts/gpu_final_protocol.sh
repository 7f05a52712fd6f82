#!/bin/bash
# r06 final-tree measurement records: SURVEY 8(d) protocol at 512^3 and 256^3, full solves
# (Jacobi / MG at 256^3 and 512^3, config 5), per-row kernel bench. Outputs in gpurun_out/r6final.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6final
mkdir -p $O
cd $R
timeout -k 10 900 python scripts/bench_protocol.py 512 > $O/protocol_512.jsonl 2> $O/protocol.err || exit $?
echo "protocol 512 done"
timeout -k 10 600 python scripts/bench_protocol.py 256 > $O/protocol_256.jsonl 2>> $O/protocol.err || exit $?
echo "protocol 256 done"
PCS=mg,jacobi NO_CPU=1 timeout -k 10 600 python scripts/bench_solve.py 256 512 > $O/solve_star7.jsonl 2> $O/solve.err || exit $?
echo "solves done"
OP=compact PCS=fft NO_CPU=1 timeout -k 10 300 python scripts/bench_solve.py 256 512 > $O/solve_fft_compact.jsonl 2>> $O/solve.err || exit $?
echo "config5 solves done"

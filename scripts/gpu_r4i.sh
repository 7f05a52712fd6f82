# PMC traffic of the compact operator's line passes (512^3) and of the config-5 solve's kernels
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4i
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  timeout -s KILL 120 rocprofv3 --pmc $grp -d $O/compact_$grp -o pmc --output-format csv -- python3 $R/scripts/bench_compact.py 512 > $O/compact_$grp.jsonl 2> $O/compact_$grp.err
  rc=$?; echo "compact pmc $grp rc=$rc"; [ $rc -eq 0 ] || exit $rc
  timeout -s KILL 120 rocprofv3 --pmc $grp -d $O/cfft_$grp -o pmc --output-format csv -- python3 $R/bench.py --workload compact-fft --steps 5 --warmup 1 --no-cpu-baseline > $O/cfft_$grp.json 2> $O/cfft_$grp.err
  rc=$?; echo "cfft pmc $grp rc=$rc"; [ $rc -eq 0 ] || exit $rc
done

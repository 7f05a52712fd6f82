set -u
mkdir -p gpurun_out
timeout -k 10 300 python scripts/placement_pairs.py 512 6 15 > gpurun_out/pairs1.jsonl 2>&1
rc=$?; echo "pairs rc=$rc"; tail -1 gpurun_out/pairs1.jsonl
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/placement_pairs.py 512 6 15 > gpurun_out/pairs2.jsonl 2>&1
rc=$?; echo "pairs rc=$rc"; tail -1 gpurun_out/pairs2.jsonl
exit $rc

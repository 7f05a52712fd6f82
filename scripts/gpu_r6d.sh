set -u
mkdir -p gpurun_out
timeout -k 10 400 python scripts/placement_cfg.py 512 5 10 > gpurun_out/cfg1.jsonl 2>&1
rc=$?; echo "cfg rc=$rc"; cut -c1-200 gpurun_out/cfg1.jsonl
exit $rc

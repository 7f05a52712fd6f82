set -u
mkdir -p gpurun_out
timeout -k 10 800 python scripts/placement_cfg.py 512 6 8 '[{}, {"stencil_kc": 132}, {"stencil_kc": 134}, {"stencil_kc": 136}, {"stencil_kc": 138}, {"stencil_kc": 140}, {"stencil_kc": 144}]' > gpurun_out/cfg3.jsonl 2>&1
rc=$?; echo "cfg rc=$rc"; cut -c1-200 gpurun_out/cfg3.jsonl
exit $rc

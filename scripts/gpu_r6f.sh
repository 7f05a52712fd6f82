set -u
mkdir -p gpurun_out
timeout -k 10 800 python scripts/placement_cfg.py 512 6 8 '[{}, {"stencil_kc": 132}, {"stencil_kc": 136}, {"stencil_kc": 140}, {"stencil_kc": 144}, {"engine_kc_skew": 4}]' > gpurun_out/cfg3.jsonl 2>&1
rc=$?; echo "cfg rc=$rc"; grep config gpurun_out/cfg3.jsonl | cut -c1-200
[ $rc -eq 0 ] || exit $rc
timeout -k 10 800 python scripts/cg_cfg_probe.py 512 4 '[{}, {"engine_kc_skew": 4}, {"engine_kc_skew": 2}, {"engine_kc_skew": 8}]' > gpurun_out/cgcfg1.jsonl 2>&1
rc=$?; echo "cgcfg rc=$rc"; grep config gpurun_out/cgcfg1.jsonl
exit $rc

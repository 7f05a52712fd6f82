set -u
mkdir -p gpurun_out
timeout -k 10 900 python scripts/cg_cfg_probe.py 1024x1024x128 3 '[{}, {"engine_kc_skew": 2}]' > gpurun_out/cgcfg_cfg4.jsonl 2>&1
rc=$?; echo "rc=$rc"; grep config gpurun_out/cgcfg_cfg4.jsonl
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python scripts/cg_cfg_probe.py 512 3 '[{}]' > gpurun_out/cgcfg_512ref.jsonl 2>&1
rc=$?; echo "rc=$rc"; grep config gpurun_out/cgcfg_512ref.jsonl
exit $rc

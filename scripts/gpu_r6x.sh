set -u
mkdir -p gpurun_out
timeout -k 10 900 python scripts/cg_cfg_probe.py 256 4 '[{}, {"engine_kc_skew": 4}, {"engine_kc_skew": 8}, {"stencil_kc_skew": 0}]' > gpurun_out/cgcfg256.jsonl 2>&1
rc=$?; echo "rc=$rc"; grep config gpurun_out/cgcfg256.jsonl; exit $rc

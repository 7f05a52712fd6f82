set -u
mkdir -p gpurun_out
timeout -k 10 900 python scripts/cg_cfg_probe.py 256 3 '[{}, {"stencil_kc_skew": 0}]' > gpurun_out/cgcfg256b.jsonl 2>&1
rc=$?; echo "rc=$rc"; grep config gpurun_out/cgcfg256b.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python scripts/placement_cfg.py 512 4 8 '[{}, {"stencil_kc_skew": 0}]' > gpurun_out/cfg4.jsonl 2>&1
rc=$?; echo "rc=$rc"; grep config gpurun_out/cfg4.jsonl | cut -c1-220; exit $rc

set -u
mkdir -p gpurun_out
timeout -k 10 900 python scripts/cg_cfg_probe.py 512 3 '[{}, {"field_stagger_kib": 4}, {"field_stagger_kib": 68}, {"field_stagger_kib": 260}]' alloc > gpurun_out/cgcfg2.jsonl 2>&1
rc=$?; echo "cgcfg rc=$rc"; grep config gpurun_out/cgcfg2.jsonl
exit $rc

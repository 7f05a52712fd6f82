set -u
mkdir -p gpurun_out
timeout -k 10 900 python scripts/cg_cfg_probe.py 512 4 '[{}, {"cg_pass_a_ty": 2}, {}, {"cg_pass_a_ty": 2}]' > gpurun_out/cgcfg5.jsonl 2>&1
rc=$?; echo "cgcfg rc=$rc"; grep config gpurun_out/cgcfg5.jsonl
exit $rc

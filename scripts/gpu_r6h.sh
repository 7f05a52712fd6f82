set -u
mkdir -p gpurun_out
timeout -k 10 900 python scripts/cg_cfg_probe.py 512 2 '[{}, {"ksp_pool_pad_kib": 0}, {"ksp_pool_pad_kib": 4}, {"ksp_pool_pad_kib": 64}, {"ksp_pool_pad_kib": 1024}, {"ksp_pool_pad_kib": 2052}, {"ksp_pool_pad_kib": 0}, {"ksp_pool_pad_kib": 4}]' alloc > gpurun_out/cgcfg3.jsonl 2>&1
rc=$?; echo "cgcfg rc=$rc"; grep config gpurun_out/cgcfg3.jsonl
python - <<'PY'
import json
for l in open("gpurun_out/cgcfg3.jsonl"):
    r = json.loads(l)
    if "pass_b_samples" in r and r["rnd"] == 1:
        s = r["pass_b_samples"]
        pos = [round(sum(s[i::3]) / len(s[i::3]), 4) for i in range(3)]
        print(r["inst"], r["cfg"], round(r["ms_per_it"], 4), pos)
PY
exit $rc

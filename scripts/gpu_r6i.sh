set -u
mkdir -p gpurun_out
timeout -k 10 900 python scripts/cg_cfg_probe.py 512 4 '[{}, {"cg_tall": 1}, {"cg_tall": 1, "engine_kc_skew": 4}, {"engine_kc_skew": 2}]' > gpurun_out/cgcfg4.jsonl 2>&1
rc=$?; echo "cgcfg rc=$rc"; grep config gpurun_out/cgcfg4.jsonl
python - <<'PY'
import json
for l in open("gpurun_out/cgcfg4.jsonl"):
    r = json.loads(l)
    if "pass_b_samples" in r and r["rnd"] == 1:
        s = r["pass_b_samples"]
        pos = [round(sum(s[i::3]) / len(s[i::3]), 4) for i in range(3)]
        print(r["inst"], r["cfg"], round(r["ms_per_it"], 4), round(r.get("cg_pass_a", 0), 4), pos)
PY
exit $rc

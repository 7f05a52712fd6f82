"""Summarise gpurun_out/ab/<name>.jsonl files: per config, ms/step per rep and mean kernel times."""
import collections
import json
import sys

for f in sys.argv[1:]:
    d = collections.defaultdict(list)
    for line in open(f):
        j = json.loads(line)
        if "kernels" not in j:
            print(f, j)
            continue
        d[j["cfg"]].append(j)
    for c, v in d.items():
        ks = {k: round(sum(x["kernels"].get(k, 0) for x in v) / len(v), 4) for k in v[0]["kernels"]}
        print(f.split("/")[-1], c, [x["ms_per_step"] for x in v], ks)

"""Per-kernel means of rocprofv3 --pmc counters (one counter group per run directory).

usage: python scripts/pmc_kernel_means.py <dir with pmc_* run dirs> [kernel-name regex]
Prints one JSON object: {kernel: {counter: mean per launch, "launches": n}}.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

src = sys.argv[1]
pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(src, "pmc_*", "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            name = re.sub(r"\(.*$", "", row["Kernel_Name"])
            if pat and not pat.search(name):
                continue
            acc[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
out = {}
for k, ctr in acc.items():
    out[k] = {c: sum(v) / len(v) for c, v in sorted(ctr.items())}
    out[k]["launches"] = max(len(v) for v in ctr.values())
print(json.dumps(out, indent=1))

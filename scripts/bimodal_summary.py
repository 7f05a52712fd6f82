"""Summarise scripts/gpu_bimodal.sh: per profiled process, the x-update pass's (PassB<3, true, true>)
and the even pass B's (PassB<0, true, true>) mean duration and mean L2 counters per launch.
usage: python scripts/bimodal_summary.py gpurun_out/bimodal"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

PAT = {"x4": r"PassB<3, true, true>", "even": r"PassB<0, true, true>", "pass_a": r"PassAT<false>"}


def main(d):
    for run in sorted(glob.glob(os.path.join(d, "p*"))):
        cc = glob.glob(os.path.join(run, "**", "*counter_collection.csv"), recursive=True)
        kt = glob.glob(os.path.join(run, "**", "*kernel_trace.csv"), recursive=True)
        if not cc or not kt:
            continue
        dur = {}
        for row in csv.DictReader(open(kt[0])):
            dur[row["Dispatch_Id"]] = (row["Kernel_Name"],
                                       (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-6)
        ctr = defaultdict(dict)
        for row in csv.DictReader(open(cc[0])):
            ctr[row["Dispatch_Id"]][row["Counter_Name"]] = float(row["Counter_Value"])
        out = {}
        for role, pat in PAT.items():
            ids = [i for i, (nm, _) in dur.items() if re.search(pat, nm)]
            if not ids:
                continue
            ms = [dur[i][1] for i in ids]
            agg = defaultdict(float)
            for i in ids:
                for k, v in ctr.get(i, {}).items():
                    agg[k] += v / len(ids)
            out[role] = {"n": len(ids), "avg_ms": sum(ms) / len(ms), "min_ms": min(ms),
                         "max_ms": max(ms), **{k: round(v) for k, v in agg.items()}}
        print(json.dumps({"run": os.path.basename(run), **out}))


if __name__ == "__main__":
    main(sys.argv[1])

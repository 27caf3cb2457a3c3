#!/usr/bin/env python3
"""Instructions per wave per IPM iteration from a rocprofv3 SQ_* pass (tools/gpu/run10.sh).
usage: inst_summary.py PMC_DIR BENCH_JSON"""
import csv
import glob
import json
import sys
from collections import defaultdict

d, bj = sys.argv[1], sys.argv[2]
rows = []
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    rows += [r for r in csv.DictReader(open(f)) if "carmpc::ipm_" in r["Kernel_Name"]]
per = defaultdict(dict)
for r in rows:
    per[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    per[int(r["Dispatch_Id"])]["kernel"] = r["Kernel_Name"].split("(")[0]
b = json.load(open(bj))
launch = b["roofline"]["launches"]
iters = b["roofline"]["I_ref"]
for i, (k, v) in enumerate(sorted(per.items())[:3]):
    env = launch[i]["env"]; n = launch[i]["instances"]
    it = n * iters[env]
    print(f"{v['kernel'][-28:]:28s} {env:20s} VALU/iter {v['SQ_INSTS_VALU']/it*64/64:9.0f}  LDS/iter {v['SQ_INSTS_LDS']/it:7.0f}  "
          f"SALU/iter {v['SQ_INSTS_SALU']/it:7.0f}  busy/wavecyc {v['SQ_BUSY_CYCLES']/max(v['SQ_WAVE_CYCLES'],1):.3f}")

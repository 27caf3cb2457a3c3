#!/usr/bin/env python3
"""Per-kernel summary of tools/gpu/variant_pmc.sh output: mean duration from the kernel trace and the
SQ counters of one bench step, per library variant.  usage: variant_pmc_summary.py VARIANT..."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(k):
    m = re.search(r"ipm_riccati_kernel<(\d+), (\d+), .*?(Bicycle|Dense)Model, (true|false), (\d), (\d+)>", k)
    return f"ric N{m.group(1)} wpb{m.group(2)} mode{m.group(5)} lpq{m.group(6)}" if m else k.split("(")[0][-40:]


out = {}
for v in sys.argv[1:]:
    res = defaultdict(dict)
    for f in glob.glob(f"{REPO}/gpurun_out/vt_{v}/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "carmpc::" in r["Name"]:
                res[short(r["Name"])].update(calls=int(r["Calls"]), mean_us=float(r["AverageNs"]) / 1e3)
    for d in ("vsq1", "vsq2"):
        per = defaultdict(dict)
        for f in glob.glob(f"{REPO}/gpurun_out/{d}_{v}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if "ipm_riccati_kernel" not in r["Kernel_Name"]:
                    continue
                e = per[int(r["Dispatch_Id"])]
                e["k"] = short(r["Kernel_Name"])
                e["vgpr"], e["agpr"], e["scratch"], e["lds"] = r["VGPR_Count"], r["Accum_VGPR_Count"], r["Scratch_Size"], r["LDS_Block_Size"]
                e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        seen = set()
        for _, e in sorted(per.items()):      # first dispatch of each kernel = first bench step
            if e["k"] in seen:
                continue
            seen.add(e["k"])
            res[e["k"]].update({k: v_ for k, v_ in e.items() if k != "k"})
    out[v] = res
    print(f"== {v}")
    for k, e in res.items():
        wc = e.get("SQ_WAVE_CYCLES", 0) or 1
        print(f"  {k:32s} mean {e.get('mean_us', 0):8.1f} us  waves {e.get('SQ_WAVES', 0):6.0f} vgpr {e.get('vgpr')} agpr {e.get('agpr')} "
              f"scratch {e.get('scratch')} lds {e.get('lds')}")
        print(f"      VALU {e.get('SQ_INSTS_VALU', 0):.3e} LDS {e.get('SQ_INSTS_LDS', 0):.3e} SALU {e.get('SQ_INSTS_SALU', 0):.3e} "
              f"MFMA {e.get('SQ_INSTS_MFMA', 0):.3e} VMEM rd/wr {e.get('SQ_INSTS_VMEM_RD', 0):.2e}/{e.get('SQ_INSTS_VMEM_WR', 0):.2e}")
        print(f"      wave_cycles {wc:.3e} busy_cycles {e.get('SQ_BUSY_CYCLES', 0):.3e} active_valu/wc {e.get('SQ_ACTIVE_INST_VALU', 0) / wc:.3f} "
              f"wait_any/wc {e.get('SQ_WAIT_INST_ANY', 0) / wc:.3f} wait_lds/wc {e.get('SQ_WAIT_INST_LDS', 0) / wc:.3f} "
              f"active_lds/wc {e.get('SQ_ACTIVE_INST_LDS', 0) / wc:.3f} active_any/wc {e.get('SQ_ACTIVE_INST_ANY', 0) / wc:.3f} "
              f"bank_conflict/wc {e.get('SQ_LDS_BANK_CONFLICT', 0) / wc:.3f}")
json.dump(out, open(f"{REPO}/gpurun_out/variant_pmc_{'_'.join(sys.argv[1:])}.json", "w"), indent=1)

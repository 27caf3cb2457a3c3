#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes of a bench.py run into HBM bytes per step.

Usage (after separate `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` passes of
`bench.py --steps S --warmup 0 --no-cpu`, see tools/gpu/*.sh):

  python tools/pmc_summary.py --fetch DIR --write DIR [--counters DIR ...] \
      --key ipm_staged --per-gpu 131072 --out profiles/r01/staged_pmc_summary.json

Counting rules (/opt/skills/guides/MI355X_MICROARCH.md, HBM / rocprofv3 section):
  * FETCH_SIZE on gfx950 reports 1/2 of the bytes of wide coalesced reads -> doubled;
  * WRITE_SIZE taken as reported;
  * only the solve-kernel dispatches (name contains --match) are counted; one bench step
    is --segments consecutive dispatches; bytes/step = median over the steps of their sum.
Updates profiles/traffic.json[key] with hbm_bytes_per_step (what bench.py reports as
roofline.traffic)."""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def read_counters(d, match):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    rows = []
    for f in files:
        with open(f) as fh:
            rows += [r for r in csv.DictReader(fh) if match in r["Kernel_Name"]]
    per = defaultdict(dict)
    for r in rows:
        d_ = per[int(r["Dispatch_Id"])]
        d_["kernel"] = r["Kernel_Name"]
        d_["scratch"] = int(r["Scratch_Size"])
        d_["vgpr"] = int(r["VGPR_Count"])
        d_["agpr"] = int(r["Accum_VGPR_Count"])
        d_["lds"] = int(r["LDS_Block_Size"])
        d_[r["Counter_Name"]] = d_.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return dict(per)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--counters", nargs="*", default=[])
    ap.add_argument("--match", default="ipm_")
    ap.add_argument("--segments", type=int, default=3)
    ap.add_argument("--key", required=True)
    ap.add_argument("--per-gpu", type=int, default=131072)
    ap.add_argument("--out", required=True)
    ap.add_argument("--source", default="")
    a = ap.parse_args()
    fetch = read_counters(a.fetch, a.match)
    write = read_counters(a.write, a.match)
    nf, nw = len(fetch), len(write)
    if nf == 0 or nw == 0 or nf % a.segments or nw % a.segments:
        raise SystemExit(f"unexpected dispatch counts fetch={nf} write={nw}")
    # bytes per step = median over the steps of the sum over the step's dispatches (a single dispatch now
    # and then reports ten times its usual FETCH_SIZE; the median keeps such a glitch out, the per-dispatch
    # values stay in the output)
    def per_step(cnt, name):
        ids = sorted(cnt)
        steps = [sum(cnt[i][name] for i in ids[j:j + a.segments]) for j in range(0, len(ids), a.segments)]
        steps.sort()
        m = len(steps)
        return steps[m // 2] if m % 2 else 0.5 * (steps[m // 2 - 1] + steps[m // 2])
    fetch_kb = per_step(fetch, "FETCH_SIZE")
    write_kb = per_step(write, "WRITE_SIZE")
    hbm = 2.0 * fetch_kb * 1024 + write_kb * 1024
    per = {}
    for d in a.counters:
        for k, v in read_counters(d, a.match).items():
            per.setdefault(str(k), {}).update(v)
    out = {
        "source": a.source or "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) of bench.py",
        "kernel_key": a.key,
        "per_gpu_batch": a.per_gpu,
        "dispatches_per_step": a.segments,
        "FETCH_SIZE_KB_per_step": fetch_kb,
        "WRITE_SIZE_KB_per_step": write_kb,
        "gfx950_correction": "FETCH_SIZE doubled (MI355X_MICROARCH.md HBM section); WRITE_SIZE as reported",
        "hbm_bytes_per_step": hbm,
        "scratch_bytes_per_lane": sorted({v["scratch"] for v in fetch.values()}),
        "per_dispatch_fetch_write": {str(k): {"kernel": v["kernel"], "FETCH_SIZE_KB": v["FETCH_SIZE"],
                                              "WRITE_SIZE_KB": write.get(k, {}).get("WRITE_SIZE")}
                                     for k, v in fetch.items()},
        "per_dispatch_counters": per,
    }
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    tpath = os.path.join(REPO, "profiles", "traffic.json")
    tj = {}
    if os.path.exists(tpath):
        with open(tpath) as f:
            tj = json.load(f)
    if "hbm_bytes_per_step" in tj:          # old flat format (dense kernel only)
        tj = {"ipm_dense": dict(tj, per_gpu_batch=a.per_gpu)}
    tj[a.key] = {"hbm_bytes_per_step": hbm, "per_gpu_batch": a.per_gpu,
                 "from": os.path.relpath(os.path.abspath(a.out), REPO)}
    with open(tpath, "w") as f:
        json.dump(tj, f, indent=1)
    print(json.dumps({k: out[k] for k in ("kernel_key", "FETCH_SIZE_KB_per_step", "WRITE_SIZE_KB_per_step",
                                          "hbm_bytes_per_step", "scratch_bytes_per_lane")}))


if __name__ == "__main__":
    main()

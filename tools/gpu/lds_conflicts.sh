#!/bin/bash
# LDS bank-conflict share of the bench step's kernels: SQ_LDS_BANK_CONFLICT (extra LDS-array cycles) against
# SQ_LDS_IDX_ACTIVE (all LDS-array cycles) and the wave cycles, per kernel.  CARMPC_LIB selects a library variant.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=${TAG:-lds}
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ldsc_$T -o pmc -- python3 bench.py --steps 2 --warmup 0 --no-cpu --no-e2e > gpurun_out/ldsc_$T.log 2>&1 || exit $?
python3 - <<PY
import csv, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open("gpurun_out/ldsc_$T/pmc_counter_collection.csv")):
    if "ipm_riccati" in r["Kernel_Name"]:
        k = r["Kernel_Name"].split("BicycleModel, ")[-1][:16]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in acc.items():
    print("$T", k, {a: "%.3e" % b for a, b in v.items()}, "conflict/idx %.3f conflict/wave_cycles %.3f" % (v["SQ_LDS_BANK_CONFLICT"] / max(v["SQ_LDS_IDX_ACTIVE"], 1), v["SQ_LDS_BANK_CONFLICT"] / max(v["SQ_WAVE_CYCLES"], 1)))
PY

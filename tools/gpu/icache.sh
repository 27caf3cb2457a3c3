#!/bin/bash
# Instruction-cache and LDS-alignment counters of the bench step's kernels (two passes).  CARMPC_LIB selects a library.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=${TAG:-ic}
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ic1_$T -o pmc -- python3 bench.py --steps 2 --warmup 0 --no-cpu --no-e2e > gpurun_out/ic_$T.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQC_DCACHE_REQ SQC_DCACHE_MISSES SQ_INSTS_SMEM --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ic2_$T -o pmc -- python3 bench.py --steps 2 --warmup 0 --no-cpu --no-e2e >> gpurun_out/ic_$T.log 2>&1 || exit $?
python3 - <<PY
import csv, collections
for d in ("ic1_$T", "ic2_$T"):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open("gpurun_out/%s/pmc_counter_collection.csv" % d)):
        if "ipm_riccati" in r["Kernel_Name"]:
            k = r["Kernel_Name"].split("BicycleModel, ")[-1][:16]
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, v in acc.items():
        print(d, k, {a: "%.3e" % b for a, b in sorted(v.items())})
PY

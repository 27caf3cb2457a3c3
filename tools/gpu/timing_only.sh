#!/bin/bash
# phase split of the Riccati kernel from the profiling build (build/timing/libcarmpc.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/ric_timing.py 7 > gpurun_out/ric_timing.json 2> gpurun_out/ric_timing.err || { tail -3 gpurun_out/ric_timing.err; exit 1; }
python - <<'PY'
import json
d=json.load(open("gpurun_out/ric_timing.json"))
names=list(next(iter(d.values()))["share"].keys())
print("%-26s" % "phase" + "".join("%22s" % e for e in d))
for k in names:
    print("%-26s" % k + "".join("%12.4f %9.3e" % (b["share"][k], b["share"][k]*b["total_cycles_all_waves"]) for b in d.values()))
print("%-26s" % "total" + "".join("%22.3e" % b["total_cycles_all_waves"] for b in d.values()))
PY

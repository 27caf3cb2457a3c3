#!/bin/bash
# pipeline vs single kernel by batch size (CARMPC_RIC_PIPELINE_MIN: 0 = always pipeline, huge = never).
# Needs an experiment build that reads the variable:
#   bash tools/gpu/mkvar.sh pmin -DCARMPC_RIC_PIPELINE_MIN_ENV ; CARMPC_LIB=build/exp_pmin/libcarmpc.so
set -o pipefail
cd $GRAFT_REPO_ROOT
for B in 2048 8192 16384 32768 65536 131072; do
  for m in 0 1000000000; do
    CARMPC_RIC_PIPELINE_MIN=$m timeout -k 10 200 python bench.py --no-cpu --no-e2e --workload config3 --per-gpu $B --steps 20 > gpurun_out/pt.json 2>gpurun_out/pt.err || exit 1
    python -c "
import json; d=json.load(open('gpurun_out/pt.json')); print($B, 'pipeline' if $m==0 else 'single  ', round(d['value']/1e6,3), 'M QP/s', d['ms_per_step'], 'ms')"
  done
done

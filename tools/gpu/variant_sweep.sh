#!/bin/bash
# bench.py against library variants (CARMPC_LIB, built with tools/gpu/mkvar.sh): VARIANTS="base a b", WORKLOADS="config5 ..."
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
for v in ${VARIANTS:-base}; do
  if [ $v = base ]; then unset CARMPC_LIB; else export CARMPC_LIB=$GRAFT_REPO_ROOT/build/exp_$v/libcarmpc.so; fi
  for w in ${WORKLOADS:-config5}; do
    timeout -k 10 200 python -u bench.py --no-cpu --workload $w --steps ${STEPS:-20} > gpurun_out/vs_${v}_$w.txt 2>gpurun_out/vs_${v}_$w.err || exit $?
    python -c "import json;d=json.loads(open('gpurun_out/vs_${v}_$w.txt').read().strip().splitlines()[-1]);print('$v', '$w', d['value'], d['ms_per_step'], d['status_split'], d['iters_mean_optimal'])"
  done
done

#!/bin/bash
# bench lines of library variants (build/exp_<name>/libcarmpc.so, tools/gpu/mkvar.sh) on several workloads,
# plus the closed-loop rate (single kernel per step): VARIANTS="base a b" WORKLOADS="config5 config4" bash ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
for v in ${VARIANTS:-base}; do
  if [ $v = base ]; then unset CARMPC_LIB; else export CARMPC_LIB=$GRAFT_REPO_ROOT/build/exp_$v/libcarmpc.so; fi
  line="$v"
  for w in ${WORKLOADS:-config5 config4 config3 config2}; do
    timeout -k 10 200 python -u bench.py --no-cpu --workload $w > gpurun_out/vs_$v_$w.txt 2>&1 || exit $?
    line="$line $(python -c "import json;d=json.loads(open('gpurun_out/vs_$v_$w.txt').read().strip().splitlines()[-1]);print('$w %.2fM' % (d['value']/1e6))")"
  done
  if [ -n "$LOOP" ]; then
    timeout -k 10 300 python tools/gpu/loop_bench.py > gpurun_out/vs_loop.json 2> gpurun_out/vs_loop.err || exit 1
    line="$line $(python -c "import json;d=json.loads(open('gpurun_out/vs_loop.json').read().strip().splitlines()[-1]);print('loop %.2fM steps/s' % (d['mpc_steps_per_s']/1e6))")"
  fi
  echo "$line"
done

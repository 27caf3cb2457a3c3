#!/bin/bash
# waves per workgroup (= per CU) of the N = 10 kernels: library variants built with tools/gpu/mkvar.sh NAME -DCARMPC_RIC_WPB10=k
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
for v in ${VARIANTS:-base wpb6}; do
  if [ $v = base ]; then unset CARMPC_LIB; else export CARMPC_LIB=$GRAFT_REPO_ROOT/build/exp_$v/libcarmpc.so; fi
  timeout -k 10 200 python -u bench.py --no-cpu --workload config2 --per-gpu ${B:-131072} --steps 20 > gpurun_out/wpb_$v.txt 2>gpurun_out/wpb_$v.err || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/wpb_$v.txt').read().strip().splitlines()[-1]);print('$v', d['value'], d['ms_per_step'], d['status_split'], d['iters_mean_optimal'])"
done

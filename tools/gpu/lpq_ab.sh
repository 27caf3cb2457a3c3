#!/bin/bash
# lanes-per-QP variants of the Riccati launches (tools/gpu/mkvar.sh NAME -DCARMPC_RIC_LPQ_M1=32 ...): pipeline parity
# test on the variant library, then bench.py per variant
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
for v in ${VARIANTS:-base m1l32}; do
  if [ $v = base ]; then unset CARMPC_LIB; else export CARMPC_LIB=$GRAFT_REPO_ROOT/build/exp_$v/libcarmpc.so; fi
  if [ $v != base ]; then
    timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_segments.py tests/test_gpu_bench_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/lpq_test_$v.txt 2>&1
    rc=$?; tail -5 gpurun_out/lpq_test_$v.txt
    [ $rc -eq 0 ] || [ -n "$KEEP_GOING" ] || exit $rc
  fi
  for w in ${WORKLOADS:-config5}; do
    timeout -k 10 200 python -u bench.py --no-cpu --workload $w --steps 20 > gpurun_out/lpq_${v}_$w.txt 2>gpurun_out/lpq_${v}_$w.err || exit $?
    python -c "import json;d=json.loads(open('gpurun_out/lpq_${v}_$w.txt').read().strip().splitlines()[-1]);print('$v', '$w', d['value'], d['ms_per_step'], d['status_split'], d['iters_mean_optimal'])"
  done
done

# bench.py against library variants (CARMPC_LIB) built with different AMDGPU scheduling strategies
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
for v in ${VARIANTS:-base max-ilp iterative-ilp max-memory-clause}; do
  if [ $v = base ]; then unset CARMPC_LIB; else export CARMPC_LIB=$GRAFT_REPO_ROOT/build/exp_$v/libcarmpc.so; fi
  timeout -k 10 200 python -u bench.py --no-cpu > gpurun_out/sched_$v.txt 2>&1 || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/sched_$v.txt').read().strip().splitlines()[-1]);print('$v', d['value'], d['status_split'])"
done

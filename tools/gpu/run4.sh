# Staged kernel first GPU pass: parity (both kernels), then dense vs staged bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONDONTWRITEBYTECODE=1 MPLBACKEND=Agg
timeout -k 10 900 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu4.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu4.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu --kernel 2 > gpurun_out/bench4_staged.json 2> gpurun_out/bench4_staged.err || exit $?
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu --kernel 1 > gpurun_out/bench4_dense.json 2> gpurun_out/bench4_dense.err || exit $?
cat gpurun_out/bench4_staged.json gpurun_out/bench4_dense.json

# GPU parity (both kernels, equality pairs) + staged/dense bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONDONTWRITEBYTECODE=1 MPLBACKEND=Agg
timeout -k 10 900 python -m pytest tests -q -m gpu > gpurun_out/pytest_gpu5.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu5.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --kernel 2 > gpurun_out/bench5_staged.json 2> gpurun_out/bench5_staged.err || exit $?
cat gpurun_out/bench5_staged.json
tail -3 gpurun_out/pytest_gpu5.log

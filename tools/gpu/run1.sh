set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 MPLBACKEND=Agg
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/pytest_gpu1.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_gpu1.log
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-sample 6144 > gpurun_out/bench1.json 2> gpurun_out/bench1.err
echo "bench rc=$?"

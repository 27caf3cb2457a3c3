set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 MPLBACKEND=Agg
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu > gpurun_out/pytest_gpu2.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_gpu2.log
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-sample 6144 > gpurun_out/bench2_k0.json 2> gpurun_out/bench2_k0.err
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu --kernel 3 > gpurun_out/bench2_k3.json 2> gpurun_out/bench2_k3.err
echo done

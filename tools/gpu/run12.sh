set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONDONTWRITEBYTECODE=1 MPLBACKEND=Agg
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -x > gpurun_out/pytest_gpu${T:-12}.log 2>&1 || { tail -30 gpurun_out/pytest_gpu${T:-12}.log; exit 1; }
tail -1 gpurun_out/pytest_gpu${T:-12}.log
for k in ${KS:-2 4}; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --kernel $k > gpurun_out/bench${T:-12}_k$k.json 2> gpurun_out/bench${T:-12}_k$k.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/bench${T:-12}_k$k.json'));print($k, d['value'], d['status_split'], [ (l['env'], l['ms']) for l in d['roofline']['launches']])"
done

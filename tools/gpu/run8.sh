# DPP reductions: probe semantics, parity, bench, phase timing.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONDONTWRITEBYTECODE=1 MPLBACKEND=Agg
timeout -k 10 60 ./tools/probe/dpp_probe > gpurun_out/dpp_probe.txt || exit $?
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -x > gpurun_out/pytest_gpu8.log 2>&1 || { tail -30 gpurun_out/pytest_gpu8.log; exit 1; }
tail -1 gpurun_out/pytest_gpu8.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/bench8.json 2> gpurun_out/bench8.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench8.json'));print(d['value'], d['status_split'], [ (l['env'], l['ms']) for l in d['roofline']['launches']])"
timeout -k 10 300 python tools/phase_timing.py 2 > gpurun_out/phase8.json 2> gpurun_out/phase8.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/phase8.json'));[print(k, v['total_cycles_per_iteration'], v['cycles_per_iteration']) for k,v in d.items()]"

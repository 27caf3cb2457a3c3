# full GPU suite + bench (auto kernel) + rocprof kernel-trace stats of the bench
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONDONTWRITEBYTECODE=1 MPLBACKEND=Agg
T=${TAG:-14}
make -s -C oracle > /dev/null || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu$T.log 2>&1 || { tail -40 gpurun_out/pytest_gpu$T.log; exit 1; }
tail -2 gpurun_out/pytest_gpu$T.log
timeout -k 10 400 python bench.py > gpurun_out/bench$T.json 2> gpurun_out/bench$T.err || { tail gpurun_out/bench$T.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench$T.json'));print(d['value'], d['status_split'], d['roofline']['frac'], d.get('cpu_baseline'), [ (l['env'], l['ms']) for l in d['roofline']['launches']])"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof$T -o bench -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/bench${T}_prof.json 2> gpurun_out/bench${T}_prof.err || exit 1
ls gpurun_out/prof$T

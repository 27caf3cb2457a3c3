# parity + bench + phase timing + VALU/LDS instruction counts (own PMC pass)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONDONTWRITEBYTECODE=1 MPLBACKEND=Agg
T=${TAG:-10}
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -x > gpurun_out/pytest_gpu$T.log 2>&1 || { tail -30 gpurun_out/pytest_gpu$T.log; exit 1; }
tail -1 gpurun_out/pytest_gpu$T.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/bench$T.json 2> gpurun_out/bench$T.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench$T.json'));print(d['value'], d['status_split'], [ (l['env'], l['ms']) for l in d['roofline']['launches']])"
timeout -k 10 300 python tools/phase_timing.py 2 > gpurun_out/phase$T.json 2> gpurun_out/phase$T.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/phase$T.json'));[print(k, v['total_cycles_per_iteration'], v['cycles_per_iteration']) for k,v in d.items()]"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $R/gpurun_out/pmc$T -o pmc -- python $R/bench.py --steps 1 --warmup 0 --no-cpu > /dev/null 2> $R/gpurun_out/pmc$T.err || exit $?
cd $R
python tools/inst_summary.py gpurun_out/pmc$T gpurun_out/bench$T.json

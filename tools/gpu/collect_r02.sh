#!/bin/bash
# measurement set: bench lines of every configuration (with CPU baselines), per-instance and
# closed-loop rates, kernel trace + HBM counters of the default workload, kernel trace of config 4
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for w in config5 config4 config3 config2; do
  echo "== bench $w"
  timeout -k 10 500 python bench.py --workload $w > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || { tail -5 gpurun_out/bench_$w.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/bench_$w.json')); print(d['value'], d['ms_per_step'], d['status_split'], d['roofline']['frac'], d['roofline']['executed_frac'], d['roofline']['issued_frac'], d['cpu_baseline']['value'], d['cpu_baseline']['single_thread']['value'], d['cpu_baseline']['product_cpu_path']['value'])"
done
echo "== hetero"; timeout -k 10 300 python tools/gpu/hetero_bench.py --batch 131072 > gpurun_out/hetero.json 2> gpurun_out/hetero.err || exit 1; tail -1 gpurun_out/hetero.json
echo "== closed loop"; timeout -k 10 300 python tools/gpu/loop_bench.py > gpurun_out/loop.json 2> gpurun_out/loop.err || exit 1; tail -1 gpurun_out/loop.json
TAG=${TAG:-r02} bash tools/gpu/profile_bench.sh || exit 1
echo "== config4 trace"
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_c4_${TAG:-r02} -o run -- python3 bench.py --no-cpu --workload config4 > gpurun_out/trace_c4.json 2> gpurun_out/trace_c4.err || exit 1
echo done

#!/bin/bash
# measurement set: bench lines of every configuration (with CPU baselines), per-instance and closed-loop
# rates, full-shard parity, kernel trace + HBM / SQ counters of the default workload, kernel trace of config 4
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
T=${TAG:-r03}
mkdir -p gpurun_out
for w in config5 config4 config3 config2; do
  echo "== bench $w"
  timeout -k 10 500 python bench.py --workload $w > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || { tail -n 5 gpurun_out/bench_$w.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/bench_$w.json')); print(d['value'], d['ms_per_step'], d['status_split'], d['roofline']['frac'], d['roofline']['executed_frac'], d['roofline']['issued_frac'], d.get('e2e_qps_pcie_inclusive'), d['cpu_baseline']['value'], d['cpu_baseline']['single_thread']['value'], d['cpu_baseline']['product_cpu_path']['value'])"
done
echo "== hetero"; timeout -k 10 300 python tools/gpu/hetero_bench.py --batch 131072 > gpurun_out/hetero.json 2> gpurun_out/hetero.err || exit 1; tail -n 1 gpurun_out/hetero.json
echo "== closed loop"; timeout -k 10 300 python tools/gpu/loop_bench.py > gpurun_out/loop.json 2> gpurun_out/loop.err || exit 1; tail -n 1 gpurun_out/loop.json
echo "== full shard parity"; timeout -k 10 900 python tools/gpu/full_shard_check.py > gpurun_out/full_shard.json 2> gpurun_out/full_shard.err || { tail -n 5 gpurun_out/full_shard.err; exit 1; }; python -c "
import json; d=json.load(open('gpurun_out/full_shard.json')); print(json.dumps(d)[:1500])"
echo "== 1M instances in one call"; timeout -k 10 600 python tools/gpu/big_batch_check.py > gpurun_out/big_batch.txt 2> gpurun_out/big_batch.err || { tail -n 5 gpurun_out/big_batch.err; exit 1; }; tail -n 3 gpurun_out/big_batch.txt
TAG=$T bash tools/gpu/profile_bench.sh || exit 1
echo "== config4 trace"
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_c4_$T -o run -- python3 bench.py --no-cpu --workload config4 > gpurun_out/trace_c4.json 2> gpurun_out/trace_c4.err || exit 1
echo done

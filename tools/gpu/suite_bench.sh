#!/bin/bash
# GPU test suite, then the bench line of the default workload and of the other configurations
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | tail -12 | tee gpurun_out/gputests.txt || exit 1
for w in config5 config4 config3 config2; do
  echo "== bench $w"
  timeout -k 10 400 python bench.py --workload $w > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || { tail -5 gpurun_out/bench_$w.err; exit 1; }
  cat gpurun_out/bench_$w.json
done

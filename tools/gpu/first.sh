#!/bin/bash
# first GPU pass of the round: probe, GPU test suite, the not-yet-collected no-alloc test, bench
set -o pipefail
mkdir -p gpurun_out
echo "== mfma probe"; timeout -k 10 60 ./build/mfma_probe 2>&1 | tee gpurun_out/mfma_probe.txt || exit 1
echo "== gpu tests"; timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | tail -15 | tee gpurun_out/gputests.txt || exit 1
echo "== no-alloc"; timeout -k 10 300 python -u -m pytest tests/wip_no_alloc.py -x -v --timeout 120 --timeout-method thread 2>&1 | tail -15 | tee gpurun_out/noalloc.txt || exit 1
echo "== bench"; timeout -k 10 300 python bench.py > gpurun_out/bench_first.json 2> gpurun_out/bench_first.err || { tail -5 gpurun_out/bench_first.err; exit 1; }
cat gpurun_out/bench_first.json

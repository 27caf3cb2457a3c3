#!/bin/bash
# quick check of a Riccati-kernel change: solver parity tests, the default bench line, the phase split
set -o pipefail
mkdir -p gpurun_out
[ -x build/mfma_neg_probe ] && timeout -k 10 60 ./build/mfma_neg_probe
[ -x build/rcp_probe ] && timeout -k 10 60 ./build/rcp_probe | tail -6
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py tests/test_gpu_segments.py tests/test_gpu_closed_loop.py tests/test_gpu_disturbance.py tests/test_gpu_hetero.py tests/test_zz_no_alloc.py -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | tail -12 | tee gpurun_out/ric_quick_tests.txt || exit 1
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/ric_quick_bench.json 2> gpurun_out/ric_quick_bench.err || { tail -5 gpurun_out/ric_quick_bench.err; exit 1; }
python - <<'PY'
import json
d=json.load(open('gpurun_out/ric_quick_bench.json'))
print("QP/s %.3fM  ms/step %.3f  iters %.3f  status %s" % (d['value']/1e6, d['ms_per_step'], d['iters_mean_optimal'], d['status_split']))
PY
if [ -f build/timing/libcarmpc.so ]; then
  timeout -k 10 300 python tools/ric_timing.py 7 > gpurun_out/ric_timing.json 2> gpurun_out/ric_timing.err || { tail -3 gpurun_out/ric_timing.err; exit 1; }
  python - <<'PY'
import json
b=json.load(open('gpurun_out/ric_timing.json'))['RoadOneCarEnv']
tot=b['total_cycles_all_waves']
print("total cycles %.3e" % tot)
for k,v in b['share'].items(): print("  %-24s %.4f  %.3e" % (k, v, v*tot))
PY
fi

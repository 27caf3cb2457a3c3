# HBM traffic of the bench step's solve kernel: separate rocprofv3 --pmc passes (FETCH_SIZE,
# WRITE_SIZE), summarised by tools/pmc_summary.py into profiles/traffic.json.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=${TAG:-tr}
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/fetch_$T -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/traffic_$T.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/write_$T -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu >> gpurun_out/traffic_$T.log 2>&1 || exit $?
echo traffic passes ok

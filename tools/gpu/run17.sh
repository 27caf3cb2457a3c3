# Riccati kernel (auto default): HBM traffic PMC passes of one bench step (separate passes, kernel-trace only)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONDONTWRITEBYTECODE=1 MPLBACKEND=Agg TMPDIR=/tmp
T=${TAG:-17}
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc${T}a -o pmc -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu > /dev/null 2> $R/gpurun_out/pmc${T}a.err || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc${T}b -o pmc -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu > /dev/null 2> $R/gpurun_out/pmc${T}b.err || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $R/gpurun_out/pmc${T}c -o pmc -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu > /dev/null 2> $R/gpurun_out/pmc${T}c.err || exit $?
echo pmc ok

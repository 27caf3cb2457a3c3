#!/bin/bash
# Profile of the default bench step (config 5, one multi-problem launch per step):
#   1. rocprofv3 --kernel-trace --stats of `bench.py --no-cpu` (per-kernel durations),
#   2. separate --pmc passes: FETCH_SIZE, WRITE_SIZE (HBM traffic), two SQ passes (instruction mix).
# Raw output under gpurun_out/<kind>_$TAG; tools/pmc_summary.py turns it into profiles/.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=${TAG:-r02}
W=${WORKLOAD:-config5}
mkdir -p gpurun_out
echo "kernel trace $T $W"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/trace_$T -o run -- python3 bench.py --no-cpu --no-e2e --workload $W > gpurun_out/trace_$T.json 2> gpurun_out/trace_$T.err || exit $?
echo "fetch"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/fetch_$T -o pmc -- python3 bench.py --steps 2 --warmup 0 --no-cpu --no-e2e --workload $W > gpurun_out/pmc_$T.log 2>&1 || exit $?
echo "write"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/write_$T -o pmc -- python3 bench.py --steps 2 --warmup 0 --no-cpu --no-e2e --workload $W >> gpurun_out/pmc_$T.log 2>&1 || exit $?
echo "sq1"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $R/gpurun_out/sq1_$T -o pmc -- python3 bench.py --steps 2 --warmup 0 --no-cpu --no-e2e --workload $W >> gpurun_out/pmc_$T.log 2>&1 || exit $?
echo "sq2"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_F64 --output-format csv -d $R/gpurun_out/sq2_$T -o pmc -- python3 bench.py --steps 2 --warmup 0 --no-cpu --no-e2e --workload $W >> gpurun_out/pmc_$T.log 2>&1 || exit $?
echo profile passes ok

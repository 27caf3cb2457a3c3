# Staged kernel: bench + rocprof kernel trace + PMC passes (separate, kernel-trace only).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONDONTWRITEBYTECODE=1 MPLBACKEND=Agg
timeout -k 10 300 python bench.py > gpurun_out/bench6.json 2> gpurun_out/bench6.err || exit $?
cat gpurun_out/bench6.json
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof6 -o trace -- python $R/bench.py --steps 5 --warmup 1 --no-cpu > $R/gpurun_out/prof6_bench.json 2> $R/gpurun_out/prof6_bench.err || exit $?
echo "prof ok"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc6a -o pmc -- python $R/bench.py --steps 1 --warmup 0 --no-cpu > /dev/null 2> $R/gpurun_out/pmc6a.err || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc6b -o pmc -- python $R/bench.py --steps 1 --warmup 0 --no-cpu > /dev/null 2> $R/gpurun_out/pmc6b.err || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM --output-format csv -d $R/gpurun_out/pmc6c -o pmc -- python $R/bench.py --steps 1 --warmup 0 --no-cpu > /dev/null 2> $R/gpurun_out/pmc6c.err || exit $?
echo "pmc ok"

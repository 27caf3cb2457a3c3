set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONDONTWRITEBYTECODE=1 MPLBACKEND=Agg
timeout -k 10 900 python -m pytest tests -q -m gpu > gpurun_out/pytest_gpu3.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_gpu3.log
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof3 -o trace -- python $R/bench.py --steps 3 --warmup 1 --no-cpu > $R/gpurun_out/prof3_bench.json 2> $R/gpurun_out/prof3_bench.err
echo "prof rc=$?"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc3a -o pmc -- python $R/bench.py --steps 1 --warmup 0 --no-cpu > /dev/null 2> $R/gpurun_out/pmc3a.err
echo "pmc a rc=$?"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc3b -o pmc -- python $R/bench.py --steps 1 --warmup 0 --no-cpu > /dev/null 2> $R/gpurun_out/pmc3b.err
echo "pmc b rc=$?"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM --output-format csv -d $R/gpurun_out/pmc3c -o pmc -- python $R/bench.py --steps 1 --warmup 0 --no-cpu > /dev/null 2> $R/gpurun_out/pmc3c.err
echo "pmc c rc=$?"

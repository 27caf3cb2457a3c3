set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=${TAG:-p1}
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$T -o run -- python3 tools/gpu/ric_prof.py 2 7 > gpurun_out/prof_$T.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $R/gpurun_out/pmc_$T -o pmc -- python3 tools/gpu/ric_prof.py 2 7 >> gpurun_out/prof_$T.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_ANY --output-format csv -d $R/gpurun_out/pmc2_$T -o pmc -- python3 tools/gpu/ric_prof.py 2 7 >> gpurun_out/prof_$T.log 2>&1 || exit $?
find gpurun_out/prof_$T gpurun_out/pmc_$T gpurun_out/pmc2_$T -name "*.csv" | head -20

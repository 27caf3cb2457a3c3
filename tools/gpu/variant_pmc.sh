#!/bin/bash
# per-kernel durations and SQ counters of bench.py for library variants (CARMPC_LIB), one pass per run
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
mkdir -p gpurun_out
W=${WORKLOAD:-config5}
[ -f gpurun_out/counters_avail.txt ] || timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters_avail.txt 2>&1
for v in ${VARIANTS:-base m1l32}; do
  if [ $v = base ]; then unset CARMPC_LIB; else export CARMPC_LIB=$R/build/exp_$v/libcarmpc.so; fi
  echo "== $v trace"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/vt_$v -o run -- python3 bench.py --no-cpu --workload $W --steps 10 > gpurun_out/vt_$v.json 2> gpurun_out/vt_$v.err || exit $?
  echo "== $v sq1"
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $R/gpurun_out/vsq1_$v -o pmc -- python3 bench.py --steps 2 --warmup 0 --no-cpu --workload $W > gpurun_out/vpmc_$v.log 2>&1 || exit $?
  echo "== $v sq2"
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_LDS_BANK_CONFLICT --output-format csv -d $R/gpurun_out/vsq2_$v -o pmc -- python3 bench.py --steps 2 --warmup 0 --no-cpu --workload $W >> gpurun_out/vpmc_$v.log 2>&1 || exit $?
done
python3 tools/variant_pmc_summary.py ${VARIANTS:-base m1l32}

#!/bin/bash
# PMC passes + kernel trace for one bench workload (secondary kernels: k-means,
# irregular BP, cooperative BP).  Usage, on the GPU box:
#   bash tools/pmc_workload.sh NAME [bench.py args...]
# Outputs under gpurun_out/pmc_NAME/{a,b,t}; one counter group per rocprofv3 run,
# no trace domains beside --pmc; every step under its own time limit.
set -o pipefail
NAME=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc_$NAME
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P="--steps 2 --warmup 1 --no-cpu-baseline $*"
KML_COOP_LAUNCH=0 timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_INSTS_VALU_FLOPS_FP64 GRBM_GUI_ACTIVE -d $O/a -o run --output-format csv -- python3 $R/bench.py $P > $O/a.log 2>&1 || exit $?
KML_COOP_LAUNCH=0 timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES -d $O/b -o run --output-format csv -- python3 $R/bench.py $P > $O/b.log 2>&1 || exit $?
KML_COOP_LAUNCH=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/t -o run --output-format csv -- python3 $R/bench.py $P > $O/t.log 2>&1 || exit $?
KML_COOP_LAUNCH=0 timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/f -o run --output-format csv -- python3 $R/bench.py $P > $O/f.log 2>&1 || exit $?
KML_COOP_LAUNCH=0 timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/w -o run --output-format csv -- python3 $R/bench.py $P > $O/w.log 2>&1 || exit $?

#!/bin/bash
# Kernel trace + PMC passes of one bench workload, with the shipped launch
# configuration (cooperative launches included).  Usage, on the GPU box:
#   bash tools/pmc_workload.sh NAME [bench.py args...]
# Outputs under gpurun_out/pmc_NAME/{t,f,w,a,b}: t = rocprofv3 --kernel-trace
# --stats (bench line in t.json), f/w = FETCH_SIZE / WRITE_SIZE (separate
# passes, MI355X_MICROARCH.md), a/b = SQ counter groups (8 SQ + 1 GRBM at most
# per pass).  No trace domain beside --pmc; every step under its own limit.
set -o pipefail
NAME=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc_$NAME
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P="--steps 2 --warmup 1 --no-cpu-baseline --no-ber-match --full-loop-batches 0 $*"
step() { echo "== $NAME $1 $(date +%T)" >> $R/gpurun_out/pmc_steps.log; }
# PASSES selects passes (default all).  A process that made a cooperative launch
# under rocprofv3 crashes in the ROCm runtime's exit-time teardown after the
# profiler has written its output: run such a workload one pass
# per gpurun call, as the call's last step.
want() { case " ${PASSES:-t f w a b} " in *" $1 "*) return 0 ;; esac; return 1; }
if want t; then
  step t
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/t -o run --output-format csv -- python3 $R/bench.py $P > $O/t.json 2> $O/t.log || exit $?
fi
if want f; then
  step f
  timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d $O/f -o run --output-format csv -- python3 $R/bench.py $P > $O/f.log 2>&1 || exit $?
fi
if want w; then
  step w
  timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d $O/w -o run --output-format csv -- python3 $R/bench.py $P > $O/w.log 2>&1 || exit $?
fi
if want a; then
  step a
  timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_INSTS_VALU_FLOPS_FP64 GRBM_GUI_ACTIVE -d $O/a -o run --output-format csv -- python3 $R/bench.py $P > $O/a.log 2>&1 || exit $?
fi
if want b; then
  step b
  timeout -k 10 240 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES -d $O/b -o run --output-format csv -- python3 $R/bench.py $P > $O/b.log 2>&1 || exit $?
fi
step done

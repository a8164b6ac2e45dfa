#!/bin/bash
# k-means PMC passes (blind PEG2304 bench, 2 steps): issue / wait / instruction-
# cache counters of the k-means kernel, for the product kernel and an A/B
# environment setting ($2, e.g. KML_KMEANS=split).  Outputs gpurun_out/$1/<tag>_<pass>/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-kmpmc}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P="--blind --steps 2 --warmup 1 --no-cpu-baseline --no-ber-match --full-loop-batches 0"
for spec in main ${2:+alt:$2}; do
  tag=${spec%%:*}; E=""; case $spec in *:*) E=${spec#*:};; esac
  [ -n "$E" ] && export $E
  timeout -k 10 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES -d $O/${tag}_b -o run --output-format csv -- python3 $R/bench.py $P > $O/${tag}_b.log 2>&1 || exit $?
  timeout -k 10 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD -d $O/${tag}_i -o run --output-format csv -- python3 $R/bench.py $P > $O/${tag}_i.log 2>&1 || exit $?
  timeout -k 10 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_INSTS_SMEM SQ_INSTS_VALU_FLOPS_FP64 SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_INSTS_FLAT -d $O/${tag}_c -o run --output-format csv -- python3 $R/bench.py $P > $O/${tag}_c.log 2>&1 || exit $?
  [ -n "$E" ] && unset ${E%%=*}
done
echo done > $O/done

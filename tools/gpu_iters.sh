#!/bin/bash
# Headline kernel time against the iteration budget (prologue / per-iteration
# split), with the demap fused into the BP prologue and as a separate kernel.
set -o pipefail
O=gpurun_out/${1:-iters}; mkdir -p $O
A="--no-cpu-baseline --no-ber-match --full-loop-batches 0"
for it in 0 20; do
  timeout -k 10 120 python bench.py --max-iter $it $A > $O/it$it.json 2> $O/it$it.err || exit $?
  KML_FUSED_DEMAP=0 timeout -k 10 120 python bench.py --max-iter $it $A > $O/nf_it$it.json 2> $O/nf_it$it.err || exit $?
done

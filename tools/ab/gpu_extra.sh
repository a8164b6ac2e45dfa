#!/bin/bash
# Round-end extras on one GPU: the PCIe-inclusive host-buffer rate of the C ABI
# (tools/host_boundary_rate.py) and a 2-rank bench line (2 processes sharing the
# GPU, gloo counter reduction) to show the sharded launch path end to end.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/extra
mkdir -p $O
cd $R
timeout -k 10 300 python tools/host_boundary_rate.py > $O/host_boundary.json 2> $O/host_boundary.err || exit $?
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_2rank_gloo.json 2> $O/bench_2rank_gloo.err || exit $?

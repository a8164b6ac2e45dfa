#!/bin/bash
# The chunked host-buffer decode: its GPU parity tests, then the PCIe-inclusive
# rate with chunks (default) and in one piece (KML_HOST_CHUNK=0).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/chunk
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "chunked or fused_demap or decode_frames" > $O/gpu_tests.log 2>&1 || exit $?
timeout -k 10 200 python tools/host_boundary_rate.py > $O/host_chunked.json 2> $O/host_chunked.err || exit $?
KML_HOST_CHUNK=0 timeout -k 10 200 python tools/host_boundary_rate.py > $O/host_onepiece.json 2> $O/host_onepiece.err || exit $?
KML_HOST_CHUNK=4096 timeout -k 10 200 python tools/host_boundary_rate.py > $O/host_c4096.json 2> $O/host_c4096.err || exit $?
KML_HOST_CHUNK=16384 timeout -k 10 200 python tools/host_boundary_rate.py > $O/host_c16384.json 2> $O/host_c16384.err || exit $?

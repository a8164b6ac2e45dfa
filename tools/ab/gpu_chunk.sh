#!/bin/bash
# The chunked host-buffer decode: its GPU parity tests, then the PCIe-inclusive
# rate, chunked (default) and in one piece (KML_HOST_CHUNK=0), known channel and blind.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/chunk2
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "chunked or fused_demap or decode_frames" > $O/gpu_tests.log 2>&1 || exit $?
timeout -k 10 200 python tools/host_boundary_rate.py > $O/host_known_chunked.json 2> $O/a.err || exit $?
KML_HOST_CHUNK=0 timeout -k 10 200 python tools/host_boundary_rate.py > $O/host_known_onepiece.json 2> $O/b.err || exit $?
timeout -k 10 200 python tools/host_boundary_rate.py --blind > $O/host_blind_chunked.json 2> $O/c.err || exit $?
KML_HOST_CHUNK=0 timeout -k 10 200 python tools/host_boundary_rate.py --blind > $O/host_blind_onepiece.json 2> $O/d.err || exit $?

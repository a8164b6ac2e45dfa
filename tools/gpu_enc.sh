#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-enc}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "encoder or frames or monte or sim or cnterr or driver or sweep" > $O/gpu_tests.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline --no-ber-match > $O/bench.json 2> $O/bench.err || exit $?
KML_ENCODE_LANE=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-ber-match > $O/bench_lane.json 2> $O/bench_lane.err || exit $?
timeout -k 10 200 python bench.py --matrix PEG8064regular0.5.txt --modem 6bits_64QAM_Gray.txt --snr 6.77 --blind --batch 4096 --steps 3 --no-cpu-baseline --no-ber-match > $O/bench_peg8064.json 2> $O/bench_peg8064.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/${1:-enc}/t -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-ber-match > $GRAFT_REPO_ROOT/gpurun_out/${1:-enc}/t.log 2>&1 || exit $?

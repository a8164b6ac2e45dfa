#!/bin/bash
# Local build + CPU suite, then one gpurun call of tools/gpu_round.sh, then a
# one-line summary per bench.  Logs under /tmp/round_all/.
set -o pipefail
cd "$(dirname "$0")/.."
L=/tmp/round_all; mkdir -p $L
make -j8 all > $L/build.log 2>&1 || { echo BUILD_FAIL; grep -E "error" $L/build.log | head; exit 1; }
echo BUILD_OK
timeout 1500 python -m pytest tests -x -q -m "not gpu" -p no:cacheprovider > $L/cpu_tests.log 2>&1 || { echo CPU_TESTS_FAIL; tail -15 $L/cpu_tests.log; exit 1; }
tail -2 $L/cpu_tests.log
rm -rf gpurun_out/round
/usr/local/graft/bin/gpurun --timeout 1200 -- 'bash tools/gpu_round.sh' > $L/gpurun.log 2>&1; echo "gpurun rc=$?"
tail -8 $L/gpurun.log
cat gpurun_out/round/steps.log; tail -3 gpurun_out/round/gpu_tests.log
for b in bench bench_blind bench_bg2 bench_peg8064; do
  tail -1 gpurun_out/round/$b.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$b', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['stats'].get('stage_ms_per_step'))"
done

#!/bin/bash
# One GPU session: optionally the GPU tests ($TESTS=1, $TESTS_K a -k filter),
# then bench lines of several library builds for several workloads, two rounds
# each, interleaved (same box).  $LIBS: kmldpc_amd/libkmldpc_amd_<x>.so
# suffixes ("main" = the product build), each optionally with one environment
# setting as <lib>:VAR=VALUE (e.g. main:KML_KMEANS=split); $WORKLOADS: headline
# blind bg2 peg8064.
# Outputs under gpurun_out/$1/; every GPU step under its own time limit.
set -o pipefail
O=gpurun_out/${1:-ab}; mkdir -p $O
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${TESTS_K:+-k "$TESTS_K"} > $O/gpu_tests.log 2>&1
  rc=$?; echo "tests rc=$rc" >> $O/summary.txt
  [ $rc = 0 ] || [ $rc = 1 ] || exit $rc   # 1 = failed tests: benches still run; anything else stops the GPU
fi
for r in $(seq 1 ${ROUNDS:-2}); do
  for w in ${WORKLOADS:-headline}; do
    E=""
    case $w in
      headline) A="" ;;
      blind) A="--blind" ;;
      bg2) A="--matrix 5GLDPCBG2a3_R12_K960.txt --modem 4bit_16QAM_Gray.txt --is5g --snr 5.01 --max-iter 50 --batch 16384 --steps 5" ;;
      peg8064) A="--matrix PEG8064regular0.5.txt --modem 6bits_64QAM_Gray.txt --snr 6.77 --blind --batch 4096 --steps 3" ;;
      peg8064_512) A="--matrix PEG8064regular0.5.txt --modem 6bits_64QAM_Gray.txt --snr 6.77 --blind --batch 4096 --steps 3"; E="KML_PART=512" ;;
      peg8064_768) A="--matrix PEG8064regular0.5.txt --modem 6bits_64QAM_Gray.txt --snr 6.77 --blind --batch 4096 --steps 3"; E="KML_PART=768" ;;
      *) echo "unknown workload $w"; exit 2 ;;
    esac
    for spec in ${LIBS:-main}; do
      l=${spec%%:*}; LE=""; tag=$l
      case $spec in *:*) LE=${spec#*:}; tag=${l}_$(echo ${LE#KML_} | tr '=' '_');; esac
      if [ "$l" = main ]; then L=kmldpc_amd/libkmldpc_amd.so; else L=kmldpc_amd/libkmldpc_amd_$l.so; fi
      env $E $LE KML_LIB=$L timeout -k 10 200 python bench.py $A --no-cpu-baseline --no-ber-match --full-loop-batches 0 > $O/${w}_${tag}_$r.json 2> $O/${w}_${tag}_$r.err || exit $?
      python3 -c "import json,sys; d=json.loads(open('$O/${w}_${tag}_$r.json').read().strip().splitlines()[-1]); print('$w $tag $r', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['stats'].get('stage_ms_per_step'), 'redone', d['stats'].get('redone'))" >> $O/summary.txt
    done
  done
done
cat $O/summary.txt

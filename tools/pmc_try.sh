set -o pipefail
O=gpurun_out/pmc_try; mkdir -p $O; R=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "8064 or cooperative or partitioned" > $O/t.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVE_CYCLES -d $R/$O/a -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --matrix PEG8064regular0.5.txt --modem 6bits_64QAM_Gray.txt --snr 6.77 --batch 4096 --no-ber-match > $R/$O/a.log 2>&1; echo "rc=$?" >> $R/$O/a.log

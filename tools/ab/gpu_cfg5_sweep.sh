#!/bin/bash
# cfg5 on one GPU: the reference's run (kmldpc_amd.simulate = Simulator::Simulate) for
# PEG8064 + 64QAM-Gray, blind k-means receive, Eb/N0 0..4 dB (Es/N0 4.77..8.77 dB, rate 1/2,
# 6 bits per symbol), stop rule 1000 block errors / 40000 blocks per point.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/cfg5
mkdir -p $O
cd $R
for f in PEG8064regular0.5.txt 6bits_64QAM_Gray.txt; do gzip -dc tests/golden/data/$f.gz > $O/$f || exit $?; done
cat > $O/config.toml <<'TOML'
[range]
    minimum_snr = 4.77
    maximum_snr = 8.77
    step_snr = 1.0
    maximum_error_number = 1000
    maximum_block_number = 40000
    thread_block_number = 1000
[decoder]
    true_h_arg = false
[xcodec]
    5gldpc = false
    metric_type = false
    metric_iter = 5
[histogram]
    enable = false
[ldpc]
    max_iter = 20
    active = true
    matrix_file = "PEG8064regular0.5.txt"
[modem]
    modem_file = "6bits_64QAM_Gray.txt"
TOML
timeout -k 10 600 python -u -m kmldpc_amd.simulate $O/config.toml --batch 4096 > $O/sweep.log 2>&1 || exit $?

"""The reference-side shims on the GPU, against the reference's own CPU
classes in the same process (oracle/_ref/shim_check: the reference's sources
compiled in the build container + integration/kmldpc_gpu_codecs.hpp + the
product library).  Every codeword of the reference's seed-17 stream goes
through lab::BinaryLDPCCodec::Decoder and GpuBinaryLDPCCodec::Decoder,
KmCodec::Decoder and GpuKmCodec::Decoder, the reference KMeans and
gpu_kmeans_h_hats / GpuKMeans (clusters, idx, DumpToMat): no mismatch is
allowed in any output."""
import json
import os
import subprocess

import pytest

from conftest import REPO, write_config

pytestmark = pytest.mark.gpu
EXE = os.path.join(REPO, "oracle", "_ref", "shim_check")


@pytest.mark.skipif(not os.path.exists(EXE), reason="oracle/_ref/shim_check not built (needs /root/reference)")
@pytest.mark.parametrize("matrix,modem,is5g,known,max_iter,snr,n", [
    ("PEG2304regular0.5.txt", "2bits_QPSK.txt", False, True, 20, 2.0, 200),
    ("PEG2304regular0.5.txt", "2bits_QPSK.txt", False, False, 20, 2.0, 100),
    ("5GLDPCBG2a3_R12_K960.txt", "4bit_16QAM_Gray.txt", True, True, 50, 5.01, 40),
    ("5GLDPCBG2a3_R12_K960.txt", "4bit_16QAM_Gray.txt", True, False, 50, 5.01, 30),
    # PEG8064 (bp_part_kernel); the reference's two codec constructions take
    # about a minute each on one core (SystemMatrixH of 4032 x 8064)
    pytest.param("PEG8064regular0.5.txt", "6bits_64QAM_Gray.txt", False, True, 20, 6.77, 12,
                 marks=pytest.mark.timeout(420)),
    pytest.param("PEG8064regular0.5.txt", "6bits_64QAM_Gray.txt", False, False, 20, 6.77, 6,
                 marks=pytest.mark.timeout(420)),
])
def test_reference_side_shims_match_reference_classes(data_dir, tmp_path, matrix, modem, is5g, known, max_iter, snr, n):
    cfg = str(tmp_path / "config.toml")
    write_config(cfg, data_dir, matrix, modem, is5g=is5g, known=known, max_iter=max_iter, snr=snr)
    r = subprocess.run([EXE, cfg, repr(snr), str(n)], capture_output=True, text=True, timeout=400, cwd=tmp_path)
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    print(res)
    assert res["codewords"] == n
    for k in ("kmcodec_uu_mismatch", "candidate_mismatch", "bp_ret_mismatch", "bp_uu_mismatch", "bp_cc_hat_mismatch",
              "bp_syndrom_soft_mismatch", "kmeans_state_mismatch"):
        assert res[k] == 0, k
    assert res["err_bit_ref"] == res["err_bit_gpu"] and res["err_bit_ref"] > 0
    if not known:  # GpuKMeans::DumpToMat of the first codeword, read back
        import scipy.io
        m = scipy.io.loadmat(str(tmp_path / "kmeans0.mat"))
        S, Kc = m["data"].shape[0], m["cluster"].shape[0]
        assert m["idx"].dtype == "int32" and m["idx"].shape == (S, 1) and m["hHats"].shape == (4, 1)
        assert m["constellations"].shape == (Kc, 1) and m["realH"].shape == (1, 1)

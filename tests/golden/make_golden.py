"""Generate the committed golden fixtures from the reference itself.

TEST INFRASTRUCTURE ONLY.  Run in the build container (needs /root/reference and
oracle/_ref/ref_harness, built by ``make -C oracle ref``):

    python tests/golden/make_golden.py                 # data files, CASES, counters.json
    python tests/golden/make_golden.py --cases a,b     # regenerate the named CASES only
    python tests/golden/make_golden.py --check-direct  # re-run every CASE, check KmCodec == direct decode, write nothing
    python tests/golden/make_golden.py --sweep         # sweep/cfg5.npz (PEG8064 blind sweep counters)
    python tests/golden/make_golden.py --bench         # bench/*.npz (bench workload's reference counters)
    python tests/golden/make_golden.py --bench-cases a,b   # the named BENCH_CASES only
    python tests/golden/make_golden.py --bench-large   # bench/large_oracle.json (oracle, 8 streams)

What it writes (all small):
  tests/golden/data/*.txt.gz      the reference's H-matrix and constellation data
                                  files (config/*.txt), gzip'd, so the tests and
                                  the GPU box have the on-disk inputs without
                                  /root/reference.  Data, not source.
  tests/golden/<case>.npz         per case, seed 17 (CLCRandNum::SetSeed(-1)):
      * stream  : per-codeword chosen candidate, BP return value, error bits and
                  CRC32s of y / P0 / uu_hat / cc_hat / syndrom_soft
      * vectors : the first NVEC codewords in full (uu, cc, true_h, y, h_hat,
                  metrics, P0, cc_hat, syndrom_soft, uu_hat)
  tests/golden/counters.json      end-to-end SourceSink counters for 2000 cw

The record layout is written by oracle/ref_harness.cc.
"""
import gzip
import json
import os
import shutil
import struct
import subprocess
import sys
import tempfile
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_CFG = "/root/reference/config"
HARNESS = os.path.join(REPO, "oracle", "_ref", "ref_harness")
NVEC = 8

DATA_FILES = [
    "PEG2304regular0.5.txt", "PEG8064regular0.5.txt", "5GLDPCBG2a3_R12_K960.txt",
    "2bits_QPSK.txt", "2bits_4PSK.txt", "4bit_16QAM_Gray.txt", "4bit_16QAM_phi1.txt",
    "4bit_16QAM_phi2.txt", "6bits_64QAM_Gray.txt",
]

# name: (matrix, modem, 5g, known_h, max_iter, snr, n_cw, active)
CASES = {
    "peg2304_qpsk_known": ("PEG2304regular0.5.txt", "2bits_QPSK.txt", False, True, 20, 2.0, 600, True),
    "peg2304_qpsk_blind": ("PEG2304regular0.5.txt", "2bits_QPSK.txt", False, False, 20, 2.0, 600, True),
    "peg2304_16qam_blind": ("PEG2304regular0.5.txt", "4bit_16QAM_Gray.txt", False, False, 20, 5.01, 200, True),
    "peg2304_4psk_known_lowsnr": ("PEG2304regular0.5.txt", "2bits_4PSK.txt", False, True, 20, -1.0, 100, True),
    "bg2_16qam_known": ("5GLDPCBG2a3_R12_K960.txt", "4bit_16QAM_Gray.txt", True, True, 50, 5.01, 200, True),
    "bg2_16qam_blind": ("5GLDPCBG2a3_R12_K960.txt", "4bit_16QAM_Gray.txt", True, False, 50, 5.01, 100, True),
    "peg8064_64qam_blind": ("PEG8064regular0.5.txt", "6bits_64QAM_Gray.txt", False, False, 20, 6.77, 60, True),
    "peg8064_64qam_known": ("PEG8064regular0.5.txt", "6bits_64QAM_Gray.txt", False, True, 20, 6.77, 40, True),
    "peg2304_16qamphi1_blind": ("PEG2304regular0.5.txt", "4bit_16QAM_phi1.txt", False, False, 20, 8.0, 100, True),
    # the last shipped constellation (config/4bit_16QAM_phi2.txt), blind and known
    "peg2304_16qamphi2_blind": ("PEG2304regular0.5.txt", "4bit_16QAM_phi2.txt", False, False, 20, 14.0, 100, True),
    "peg2304_16qamphi2_known": ("PEG2304regular0.5.txt", "4bit_16QAM_phi2.txt", False, True, 20, 6.0, 100, True),
    # [ldpc] active = false: no SystemMatrixH, the file-order graph, all-zero
    # codewords (binaryldpccodec.cc:125-127, 148-161; binary5gldpccodec.cc:75-76, 92-108)
    "peg2304_qpsk_known_inactive": ("PEG2304regular0.5.txt", "2bits_QPSK.txt", False, True, 20, 1.0, 200, False),
    "peg2304_qpsk_blind_inactive": ("PEG2304regular0.5.txt", "2bits_QPSK.txt", False, False, 20, 2.0, 200, False),
    "bg2_16qam_known_inactive": ("5GLDPCBG2a3_R12_K960.txt", "4bit_16QAM_Gray.txt", True, True, 50, 4.0, 100, False),
    "bg2_16qam_blind_inactive": ("5GLDPCBG2a3_R12_K960.txt", "4bit_16QAM_Gray.txt", True, False, 50, 5.01, 60, False),
    # the (code x constellation) cross-product: [ldpc] matrix_file and [modem]
    # modem_file are independent keys (binaryldpccodec.cc:71-73, modem.cc:7)
    # PEG8064 + QPSK: S = 4032 symbols, 63 of km_wave_kernel's 64 lane-words
    "peg8064_qpsk_known": ("PEG8064regular0.5.txt", "2bits_QPSK.txt", False, True, 20, 1.6, 40, True),
    "peg8064_qpsk_blind": ("PEG8064regular0.5.txt", "2bits_QPSK.txt", False, False, 20, 2.3, 40, True),
    "peg8064_16qam_known": ("PEG8064regular0.5.txt", "4bit_16QAM_Gray.txt", False, True, 20, 6.0, 40, True),
    "peg8064_16qam_blind": ("PEG8064regular0.5.txt", "4bit_16QAM_Gray.txt", False, False, 20, 6.4, 40, True),
    # 5G BG2 + QPSK / 64QAM (S = 320: a partial k-means word) / 16QAM-phi1
    "bg2_qpsk_known": ("5GLDPCBG2a3_R12_K960.txt", "2bits_QPSK.txt", True, True, 50, 1.5, 100, True),
    "bg2_qpsk_blind": ("5GLDPCBG2a3_R12_K960.txt", "2bits_QPSK.txt", True, False, 50, 2.0, 100, True),
    "bg2_64qam_known": ("5GLDPCBG2a3_R12_K960.txt", "6bits_64QAM_Gray.txt", True, True, 50, 10.0, 60, True),
    "bg2_64qam_blind": ("5GLDPCBG2a3_R12_K960.txt", "6bits_64QAM_Gray.txt", True, False, 50, 11.0, 60, True),
    "bg2_16qamphi1_blind": ("5GLDPCBG2a3_R12_K960.txt", "4bit_16QAM_phi1.txt", True, False, 50, 11.0, 100, True),
    # PEG2304 + blind 4PSK (the axis-aligned QPSK: 2bits_4PSK.txt) and blind 64QAM
    "peg2304_4psk_blind": ("PEG2304regular0.5.txt", "2bits_4PSK.txt", False, False, 20, 2.0, 100, True),
    "peg2304_64qam_blind": ("PEG2304regular0.5.txt", "6bits_64QAM_Gray.txt", False, False, 20, 10.5, 60, True),
}

# soft syndrome metric ([xcodec] metric_type = true): name -> (matrix, modem, 5g,
# known_h, max_iter, snr, n_cw, metric_iter, harness mode); written to soft/<name>.npz
SOFT_CASES = {
    "peg2304_qpsk_soft": ("PEG2304regular0.5.txt", "2bits_QPSK.txt", False, False, 20, 2.0, 300, 5, "soft"),
    "peg2304_qpsk_soft_hisnr": ("PEG2304regular0.5.txt", "2bits_QPSK.txt", False, False, 20, 4.0, 300, 5, "soft"),
    "peg2304_qpsk_softhist": ("PEG2304regular0.5.txt", "2bits_QPSK.txt", False, False, 20, 3.0, 300, 5, "softhist"),
    "bg2_16qam_soft": ("5GLDPCBG2a3_R12_K960.txt", "4bit_16QAM_Gray.txt", True, False, 50, 5.01, 100, 5, "soft"),
    "peg2304_16qam_soft_it3": ("PEG2304regular0.5.txt", "4bit_16QAM_Gray.txt", False, False, 20, 7.0, 150, 3, "soft"),
}

# cfg5 (BASELINE.json configs[4]): the PEG8064 + 64QAM-Gray blind Eb/N0 0..4 dB
# sweep, snr = Eb/N0 + 10*log10(R*m) = Eb/N0 + 4.77 (6.77 is peg8064_64qam_blind).
SWEEP_SNRS = [4.77, 5.77, 6.77, 7.77, 8.77]
for _snr in SWEEP_SNRS:
    if _snr != 6.77:
        CASES[f"peg8064_64qam_blind_s{int(round(_snr * 100))}"] = (
            "PEG8064regular0.5.txt", "6bits_64QAM_Gray.txt", False, False, 20, _snr, 24, True)
NVEC_CASE = {k: 2 for k in CASES if k.startswith("peg8064_64qam_blind_s")}
NVEC_CASE.update({k: 4 for k in ("peg8064_qpsk_known", "peg8064_qpsk_blind", "peg8064_16qam_known",
                                 "peg8064_16qam_blind")})
SWEEP_N = 400

# the bench workload's reference counters: the first B codewords of the seed-17
# stream through the reference itself (SourceSink::CntErr), with per-codeword
# error bits for the BER standard error; tests/golden/bench/<name>.npz
BENCH_CASES = {
    "peg2304_qpsk_known_32768": ("PEG2304regular0.5.txt", "2bits_QPSK.txt", False, True, 20, 2.0, 32768, True),
    "peg2304_qpsk_blind_32768": ("PEG2304regular0.5.txt", "2bits_QPSK.txt", False, False, 20, 2.0, 32768, True),
    # cfg3: 5G BG2 + 16QAM-Gray, known channel, 50 iterations (bench_bg2 line)
    "bg2_16qam_known_16384": ("5GLDPCBG2a3_R12_K960.txt", "4bit_16QAM_Gray.txt", True, True, 50, 5.01, 16384, True),
    # cfg4: PEG8064 + 64QAM-Gray, blind k-means (bench_peg8064 line); the reference runs
    # this point at ~0.8 codewords/s on one core, so the stream is 2048 codewords
    "peg8064_64qam_blind_2048": ("PEG8064regular0.5.txt", "6bits_64QAM_Gray.txt", False, False, 20, 6.77, 2048, True),
}
# cfg5: the other four sweep points (Eb/N0 0, 1, 3, 4 dB), 1024 codewords each
for _snr in SWEEP_SNRS:
    if _snr != 6.77:
        BENCH_CASES[f"peg8064_64qam_blind_s{int(round(_snr * 100))}_1024"] = (
            "PEG8064regular0.5.txt", "6bits_64QAM_Gray.txt", False, False, 20, _snr, 1024, True)

COUNTER_CASES = {
    "peg2304_qpsk_known_2000": ("PEG2304regular0.5.txt", "2bits_QPSK.txt", False, True, 20, 2.0, 2000, True),
    "peg2304_qpsk_blind_2000": ("PEG2304regular0.5.txt", "2bits_QPSK.txt", False, False, 20, 2.0, 2000, True),
}


def write_toml(path, data_dir, matrix, modem, is5g, known, max_iter, active, metric_iter=5, soft=False):
    b = lambda v: "true" if v else "false"
    with open(path, "w") as f:
        f.write(f"""[range]
    minimum_snr = 2.0
    maximum_snr = 2.0
    step_snr = 1.0
    maximum_error_number = 1000000
    maximum_block_number = 1000
    thread_block_number = 1000
[decoder]
    true_h_arg = {b(known)}
[xcodec]
    5gldpc = {b(is5g)}
    metric_type = {b(soft)}
    metric_iter = {metric_iter}
[histogram]
    enable = false
[ldpc]
    max_iter = {max_iter}
    active = {b(active)}
    matrix_file = "{os.path.join(data_dir, matrix)}"
[modem]
    modem_file = "{os.path.join(data_dir, modem)}"
""")


class Reader:
    def __init__(self, buf):
        self.b = buf
        self.o = 0

    def i32(self):
        v = struct.unpack_from("<i", self.b, self.o)[0]
        self.o += 4
        return v

    def f64(self, n=None):
        if n is None:
            v = struct.unpack_from("<d", self.b, self.o)[0]
            self.o += 8
            return v
        v = np.frombuffer(self.b, dtype="<f8", count=n, offset=self.o).copy()
        self.o += 8 * n
        return v

    def u8(self, n):
        v = np.frombuffer(self.b, dtype=np.uint8, count=n, offset=self.o).copy()
        self.o += n
        return v


def crc(a):
    return zlib.crc32(np.ascontiguousarray(a).tobytes()) & 0xFFFFFFFF


def parse_frames(buf):
    r = Reader(buf)
    magic = r.i32()
    assert magic == 0x4B4D4C31
    K, N, S, M, Kc, known, is5g, max_iter, ncw = [r.i32() for _ in range(9)]
    snr = r.f64()
    cons = r.f64(2 * Kc).reshape(Kc, 2)
    recs = []
    for _ in range(ncw):
        d = {}
        d["uu"] = r.u8(K)
        d["cc"] = r.u8(N)
        d["true_h"] = r.f64(2)
        d["y"] = r.f64(2 * S).reshape(S, 2)
        d["h_hat"] = r.f64(2)
        d["metrics"] = r.f64(4)
        d["chosen"] = r.i32()
        d["p0"] = r.f64(N)
        d["ret"] = r.i32()
        ncol = r.i32()
        d["cc_hat"] = r.u8(ncol)
        d["syn"] = r.f64(M)
        d["uu_hat"] = r.u8(K)
        d["uu_hat_direct"] = r.u8(K)
        d["errs"] = r.i32()
        recs.append(d)
    assert r.o == len(buf)
    hdr = dict(K=K, N=N, S=S, M=M, Kc=Kc, known=known, is5g=is5g, max_iter=max_iter, ncw=ncw, snr=snr)
    return hdr, cons, recs


def parse_soft(buf):
    """Records of ref_harness modes soft / softhist."""
    r = Reader(buf)
    magic, K, N, S, M, Kc, known, is5g, max_iter, ncw = [r.i32() for _ in range(10)]
    snr = r.f64()
    r.f64(2 * Kc)
    recs = []
    for _ in range(ncw):
        d = {"uu": r.u8(K)}
        d["true_h"] = r.f64(2)
        d["y"] = r.f64(2 * S).reshape(S, 2)
        d["h_hat"] = r.f64(2)
        d["metrics"] = r.f64(4)
        d["chosen"] = r.i32()
        d["uu_hat"] = r.u8(K)
        d["errs"] = r.i32()
        recs.append(d)
    return dict(K=K, N=N, S=S, M=M, known=known, is5g=is5g, max_iter=max_iter, snr=snr), recs


def make_soft(tmp):
    os.makedirs(os.path.join(HERE, "soft"), exist_ok=True)
    for name, (mat, mod, is5g, known, it, snr, n, mit, mode) in SOFT_CASES.items():
        cfg = os.path.join(tmp, name + ".toml")
        write_toml(cfg, REF_CFG, mat, mod, is5g, known, it, True, metric_iter=mit, soft=True)
        out = os.path.join(tmp, name + ".bin")
        subprocess.run([HARNESS, cfg, repr(snr), str(n), out, mode], check=True)
        hdr, recs = parse_soft(open(out, "rb").read())
        hdr.update(matrix=mat, modem=mod, metric_iter=mit, mode=mode)
        # frames are regenerated by the oracle (same seed-17 stream as the
        # frames cases); only their CRCs are kept
        arrs = {"hdr_json": np.frombuffer(json.dumps(hdr).encode(), dtype=np.uint8)}
        arrs["crc_y"] = np.array([crc(d["y"]) for d in recs], np.uint32)
        arrs["crc_uu"] = np.array([crc(d["uu"]) for d in recs], np.uint32)
        for key in ["true_h", "h_hat", "metrics"]:
            arrs[key] = np.stack([d[key] for d in recs])
        arrs["uu_hat_bits"] = np.packbits(np.stack([d["uu_hat"] for d in recs]), axis=1)
        arrs["chosen"] = np.array([d["chosen"] for d in recs], np.int32)
        arrs["errs"] = np.array([d["errs"] for d in recs], np.int32)
        np.savez_compressed(os.path.join(HERE, "soft", name + ".npz"), **arrs)
        print(f"{name}: n={n} FER={np.mean(arrs['errs'] > 0):.4f} chosen={np.bincount(arrs['chosen'], minlength=4)} "
              f"inf_metrics={int(np.isinf(arrs['metrics']).sum())}")


# KMeans::clusters() / idx() fixtures: name -> (matrix, modem, snr, n)
KMSTATE_CASES = {
    "peg2304_qpsk_s2": ("PEG2304regular0.5.txt", "2bits_QPSK.txt", 2.0, 16),
    "peg2304_qpsk_sm1": ("PEG2304regular0.5.txt", "2bits_QPSK.txt", -1.0, 8),
    "peg2304_16qam_s5": ("PEG2304regular0.5.txt", "4bit_16QAM_Gray.txt", 5.01, 8),
    "peg8064_64qam_s677": ("PEG8064regular0.5.txt", "6bits_64QAM_Gray.txt", 6.77, 4),
}


def make_kmstate(tmp):
    """ref_harness mode kmstate -> golden/kmstate/<name>.npz (y, true_h, clusters, idx)."""
    os.makedirs(os.path.join(HERE, "kmstate"), exist_ok=True)
    for name, (mat, mod, snr, n) in KMSTATE_CASES.items():
        cfg = os.path.join(tmp, name + ".toml")
        write_toml(cfg, REF_CFG, mat, mod, False, False, 20, True)
        out = os.path.join(tmp, name + ".bin")
        subprocess.run([HARNESS, cfg, repr(snr), str(n), out, "kmstate"], check=True)
        buf = open(out, "rb").read()
        r = Reader(buf)
        K, N, S, M, Kc = (struct.unpack_from("<i", buf, 4 * i)[0] for i in range(1, 6))
        r.o = 4 * 10 + 8 + 16 * Kc
        th, ys, cls, idxs = [], [], [], []
        for _ in range(n):
            th.append(r.f64(2))
            ys.append(r.f64(2 * S).reshape(S, 2))
            cls.append(r.f64(2 * Kc).reshape(Kc, 2))
            idxs.append(np.frombuffer(buf, "<i4", S, r.o).copy())
            r.o += 4 * S
        assert r.o == len(buf)
        hdr = dict(matrix=mat, modem=mod, snr=snr, n=n, S=S, Kc=Kc, iters=20)
        np.savez_compressed(os.path.join(HERE, "kmstate", name + ".npz"),
                            hdr_json=np.frombuffer(json.dumps(hdr).encode(), dtype=np.uint8), true_h=np.stack(th),
                            y=np.stack(ys), clusters=np.stack(cls), idx=np.stack(idxs).astype(np.int32))
        print(f"{name}: n={n} S={S} Kc={Kc} idx counts {np.bincount(np.concatenate(idxs), minlength=Kc)[:8]}")


def make_rng(tmp, n=2000):
    """Reference RNG streams with SetSeed(-1) -> golden/host/rng.npz."""
    out = os.path.join(tmp, "rng.bin")
    subprocess.run([HARNESS, "unused.toml", "0", str(n), out, "rng"], check=True)
    b = open(out, "rb").read()
    o = 0
    arr = {}
    for key, cnt, dt in [("clc_u", n, "<f8"), ("wh_u", n, "<f8"), ("clc_n", n + 1, "<f8"), ("wh_n", n + 1, "<f8"),
                         ("sym16", n, "<i4"), ("sym3", n, "<i4"), ("bits", n, "<i4")]:
        arr[key] = np.frombuffer(b, dtype=dt, count=cnt, offset=o).copy()
        o += cnt * np.dtype(dt).itemsize
    os.makedirs(os.path.join(HERE, "host"), exist_ok=True)
    np.savez_compressed(os.path.join(HERE, "host", "rng.npz"), **arr)
    print("rng:", {k: v[:3] for k, v in arr.items()})


def run_simulate(tmp, name, mat, mod, is5g, known, it, snr, n, active=True):
    """Harness 'simulate' mode: the reference's counters plus per-codeword error bits."""
    cfg = os.path.join(tmp, name + ".toml")
    write_toml(cfg, REF_CFG, mat, mod, is5g, known, it, active)
    out = os.path.join(tmp, name + ".bin")
    subprocess.run([HARNESS, cfg, repr(snr), str(n), out, "simulate"], check=True)
    buf = open(out, "rb").read()
    K = struct.unpack_from("<i", buf, 4)[0]
    Kc = struct.unpack_from("<i", buf, 4 * 5)[0]
    r = Reader(buf)
    r.o = 4 * 10 + 8 + 16 * Kc
    tot_blk, err_blk = r.i32(), r.i32()
    ber, fer = r.f64(), r.f64()
    errs = np.frombuffer(buf, dtype="<i4", count=n, offset=r.o).copy()
    assert r.o + 4 * n == len(buf) and tot_blk == n
    assert int((errs > 0).sum()) == err_blk and abs(errs.sum() / (K * n) - ber) < 1e-15
    return dict(K=K, tot_blk=tot_blk, err_blk=err_blk, err_bit=int(errs.sum()), ber=ber, fer=fer), errs


def check_direct(name, recs):
    """The harness's cross-check: KmCodec::Decoder's uu_hat (kmcodec.cc:69-70, the
    chosen candidate's P0 through ldpc_codec_->Decoder at max_iter) equals a
    directly constructed codec's Decoder on the same P0 (ref_harness.cc).  BP is a
    pure function of P0, so this holds known and blind, PEG and 5G."""
    bad = [i for i, d in enumerate(recs) if not np.array_equal(d["uu_hat"], d["uu_hat_direct"])]
    assert not bad, f"{name}: KmCodec uu_hat != direct decode on codewords {bad[:10]}"


def frames_arrays(hdr, cons, recs, mat, mod, active, nv):
    arrs = {
        "hdr_json": np.frombuffer(json.dumps(dict(hdr, matrix=mat, modem=mod, active=active)).encode(), dtype=np.uint8),
        "cons": cons,
        "s_chosen": np.array([d["chosen"] for d in recs], np.int32),
        "s_ret": np.array([d["ret"] for d in recs], np.int32),
        "s_errs": np.array([d["errs"] for d in recs], np.int32),
        "s_crc_y": np.array([crc(d["y"]) for d in recs], np.uint32),
        "s_crc_p0": np.array([crc(d["p0"]) for d in recs], np.uint32),
        "s_crc_uuhat": np.array([crc(d["uu_hat"]) for d in recs], np.uint32),
        "s_crc_cchat": np.array([crc(d["cc_hat"]) for d in recs], np.uint32),
        "s_crc_syn": np.array([crc(d["syn"]) for d in recs], np.uint32),
        "s_crc_uu": np.array([crc(d["uu"]) for d in recs], np.uint32),
        "s_hhat": np.array([d["h_hat"] for d in recs]),
        "s_metrics": np.array([d["metrics"] for d in recs]),
        "s_true_h": np.array([d["true_h"] for d in recs]),
    }
    for key in ["uu", "cc", "y", "p0", "cc_hat", "syn", "uu_hat"]:
        arrs["v_" + key] = np.stack([recs[i][key] for i in range(nv)])
    return arrs


def make_frames_cases(tmp, names, check_only=False):
    from concurrent.futures import ThreadPoolExecutor

    def one(name):
        mat, mod, is5g, known, it, snr, n, active = CASES[name]
        cfg = os.path.join(tmp, name + ".toml")
        write_toml(cfg, REF_CFG, mat, mod, is5g, known, it, active)
        out = os.path.join(tmp, name + ".bin")
        subprocess.run([HARNESS, cfg, repr(snr), str(n), out], check=True)
        hdr, cons, recs = parse_frames(open(out, "rb").read())
        check_direct(name, recs)
        if check_only:
            return f"{name}: n={n} KmCodec::Decoder == direct BinaryLDPCCodec::Decoder on every codeword"
        arrs = frames_arrays(hdr, cons, recs, mat, mod, active, min(NVEC_CASE.get(name, NVEC), len(recs)))
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **arrs)
        return f"{name}: n={n} FER={np.mean(arrs['s_errs'] > 0):.4f} mean_ret={arrs['s_ret'].mean():.2f}"

    with ThreadPoolExecutor(4) as ex:
        for line in ex.map(one, names):
            print(line)


def make_sweep(tmp):
    """cfg5 sweep: the reference's counters over SWEEP_N codewords per point ->
    tests/golden/sweep/cfg5.npz (snr[P], counters[P][4], errs[P][SWEEP_N])."""
    from concurrent.futures import ThreadPoolExecutor

    def one(snr):
        return run_simulate(tmp, f"sweep_{snr}", "PEG8064regular0.5.txt", "6bits_64QAM_Gray.txt", False, False, 20,
                            snr, SWEEP_N)

    with ThreadPoolExecutor(5) as ex:
        res = list(ex.map(one, SWEEP_SNRS))
    cnt = np.array([[c["err_bit"], c["err_blk"], c["K"] * c["tot_blk"], c["tot_blk"]] for c, _ in res], np.int64)
    os.makedirs(os.path.join(HERE, "sweep"), exist_ok=True)
    np.savez_compressed(os.path.join(HERE, "sweep", "cfg5.npz"), snr=np.array(SWEEP_SNRS), counters=cnt,
                        errs=np.stack([e for _, e in res]).astype(np.int16))
    for snr, (c, _) in zip(SWEEP_SNRS, res):
        print(f"cfg5 snr {snr}: FER {c['fer']:.4f} BER {c['ber']:.6f}")


def make_bench(tmp, names=None):
    """names: a subset of BENCH_CASES (--bench-cases a,b); each stream is one
    sequential reference run, so the cases run in parallel processes."""
    from concurrent.futures import ThreadPoolExecutor

    os.makedirs(os.path.join(HERE, "bench"), exist_ok=True)
    names = names or list(BENCH_CASES)

    def one(name):
        mat, mod, is5g, known, it, snr, n, active = BENCH_CASES[name]
        c, errs = run_simulate(tmp, name, mat, mod, is5g, known, it, snr, n, active)
        hdr = dict(c, matrix=mat, modem=mod, is5g=is5g, known=known, max_iter=it, snr=snr, n=n, seed=17)
        np.savez_compressed(os.path.join(HERE, "bench", name + ".npz"),
                            hdr_json=np.frombuffer(json.dumps(hdr).encode(), dtype=np.uint8),
                            errs=errs.astype(np.int16))
        return f"{name}: FER {c['fer']:.5f} BER {c['ber']:.6f}"

    with ThreadPoolExecutor(min(len(names), 6)) as ex:
        for line in ex.map(one, names):
            print(line, flush=True)


# Larger reference samples of the bench points for the Monte-Carlo BER sigma:
# the oracle restatement (bit-exact vs the reference, tests/test_oracle.py) on
# 8 Park-Miller streams (seeds 17..24), n_per_stream codewords each.
BENCH_LARGE = {
    "peg2304_qpsk_known": ("PEG2304regular0.5.txt", "2bits_QPSK.txt", False, True, 20, 2.0, 32768),
    "peg2304_qpsk_blind": ("PEG2304regular0.5.txt", "2bits_QPSK.txt", False, False, 20, 2.0, 16384),
    # cfg3 (bench_bg2: 16384 GPU codewords per stats pass)
    "bg2_16qam_known": ("5GLDPCBG2a3_R12_K960.txt", "4bit_16QAM_Gray.txt", True, True, 50, 5.01, 4096),
}
# cfg4 / cfg5 (bench_peg8064 at 6.77 dB and the sweep points: 4096 GPU codewords per stats pass)
for _snr in SWEEP_SNRS:
    BENCH_LARGE["peg8064_64qam_blind" + ("" if _snr == 6.77 else f"_s{int(round(_snr * 100))}")] = (
        "PEG8064regular0.5.txt", "6bits_64QAM_Gray.txt", False, False, 20, _snr, 1024)


def make_bench_large(tmp):
    exe = os.path.join(REPO, "oracle", "cpu_baseline")
    for fn in DATA_FILES:
        with open(os.path.join(REF_CFG, fn), "rb") as f, open(os.path.join(tmp, fn), "wb") as g:
            g.write(f.read())
    out = {}
    fn = os.path.join(HERE, "bench", "large_oracle.json")
    names = list(BENCH_LARGE)
    if "--only" in sys.argv:  # regenerate the named entries, keep the others
        names = sys.argv[sys.argv.index("--only") + 1].split(",")
        out = json.load(open(fn))
    for name in names:
        mat, mod, is5g, known, it, snr, n = BENCH_LARGE[name]
        r = subprocess.run([exe, os.path.join(tmp, mat), os.path.join(tmp, mod), str(int(is5g)), repr(snr), str(it),
                            str(int(not known)), str(n), "8"], check=True, capture_output=True, text=True)
        d = json.loads(r.stdout.strip().splitlines()[-1])
        out[name] = dict(matrix=mat, modem=mod, is5g=is5g, known=known, max_iter=it, snr=snr, streams=8,
                         seeds="17..24", codewords=d["codewords"], err_bit=d["err_bit"], err_blk=d["err_blk"],
                         sum_e2=d["sum_e2"], K=d["K"], ber=d["ber"], fer=d["fer"],
                         source="oracle/cpu_baseline (oracle.c restatement, bit-exact vs the reference)")
        print(name, out[name], flush=True)
    os.makedirs(os.path.join(HERE, "bench"), exist_ok=True)
    with open(fn, "w") as f:
        json.dump(out, f, indent=1)


def main():
    for flag, fn in (("--bench", make_bench), ("--sweep", make_sweep), ("--bench-large", make_bench_large),
                     ("--kmstate", make_kmstate)):
        if flag in sys.argv:
            tmp = tempfile.mkdtemp()
            try:
                fn(tmp)
            finally:
                shutil.rmtree(tmp)
            return
    if "--bench-cases" in sys.argv:
        tmp = tempfile.mkdtemp()
        try:
            make_bench(tmp, sys.argv[sys.argv.index("--bench-cases") + 1].split(","))
        finally:
            shutil.rmtree(tmp)
        return
    if "--cases" in sys.argv or "--check-direct" in sys.argv:
        check = "--check-direct" in sys.argv
        names = list(CASES) if check else sys.argv[sys.argv.index("--cases") + 1].split(",")
        tmp = tempfile.mkdtemp()
        try:
            make_frames_cases(tmp, names, check_only=check)
        finally:
            shutil.rmtree(tmp)
        return
    if "--rng" in sys.argv:
        tmp = tempfile.mkdtemp()
        try:
            make_rng(tmp)
        finally:
            shutil.rmtree(tmp)
        return
    if "--soft" in sys.argv:
        tmp = tempfile.mkdtemp()
        try:
            make_soft(tmp)
        finally:
            shutil.rmtree(tmp)
        return
    if not os.path.exists(HARNESS):
        sys.exit("build oracle/_ref/ref_harness first (make -C oracle ref)")
    ddir = os.path.join(HERE, "data")
    os.makedirs(ddir, exist_ok=True)
    for fn in DATA_FILES:
        with open(os.path.join(REF_CFG, fn), "rb") as f:
            raw = f.read()
        with gzip.GzipFile(os.path.join(ddir, fn + ".gz"), "wb", mtime=0) as g:
            g.write(raw)
    tmp = tempfile.mkdtemp()
    try:
        make_frames_cases(tmp, list(CASES))
        counters = {}
        for name, (mat, mod, is5g, known, it, snr, n, active) in COUNTER_CASES.items():
            cfg = os.path.join(tmp, name + ".toml")
            write_toml(cfg, REF_CFG, mat, mod, is5g, known, it, active)
            out = os.path.join(tmp, name + ".bin")
            subprocess.run([HARNESS, cfg, repr(snr), str(n), out, "simulate"], check=True)
            buf = open(out, "rb").read()
            r = Reader(buf)
            r.o = 4 * 10 + 8
            Kc = struct.unpack_from("<i", buf, 4 * 5)[0]
            K = struct.unpack_from("<i", buf, 4)[0]
            r.o += 16 * Kc
            tot_blk, err_blk = r.i32(), r.i32()
            ber, fer = r.f64(), r.f64()
            err_bit = int(round(ber * K * tot_blk))
            counters[name] = dict(matrix=mat, modem=mod, is5g=is5g, known=known, max_iter=it, snr=snr,
                                  n=n, tot_blk=tot_blk, err_blk=err_blk, err_bit=err_bit, ber=ber, fer=fer)
            print(name, counters[name])
        with open(os.path.join(HERE, "counters.json"), "w") as f:
            json.dump(counters, f, indent=1)
    finally:
        shutil.rmtree(tmp)


if __name__ == "__main__":
    main()

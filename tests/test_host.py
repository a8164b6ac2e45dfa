"""CPU-side tests of the product library (no GPU): the C ABI loads and exports
every symbol include/kmldpc_amd.h declares, the host planner (config parsing,
H-matrix parsing, GF(2) elimination, graph order, encoder, constellation) is
bit-identical to the oracle, and the exact-math restatements used by the
device code equal glibc / libgcc on the host."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import REPO, load_case, write_config
from oracle import oracle as O

import kmldpc_amd as K

CODES = [
    ("PEG2304regular0.5.txt", False),
    ("5GLDPCBG2a3_R12_K960.txt", True),
    ("PEG8064regular0.5.txt", False),
]
MODEMS = ["2bits_QPSK.txt", "2bits_4PSK.txt", "4bit_16QAM_Gray.txt", "4bit_16QAM_phi1.txt", "4bit_16QAM_phi2.txt",
          "6bits_64QAM_Gray.txt"]


def test_library_exports_header_symbols():
    L = K.lib()
    syms = K.header_symbols()
    assert len(syms) >= 20
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    assert L.kml_abi_version() == 2


_oracle_codes = {}


def oracle_code(data_dir, matrix, is5g, active=True):
    key = (matrix, active)
    if key not in _oracle_codes:
        _oracle_codes[key] = O.Code(os.path.join(data_dir, matrix), is5g, active, False, 20)
    return _oracle_codes[key]


@pytest.mark.parametrize("matrix,is5g", CODES)
@pytest.mark.parametrize("active", [True, False])
def test_planner_matches_oracle(data_dir, matrix, is5g, active):
    if "8064" in matrix and not active:
        pytest.skip("covered by the active case")
    ctx = K.Context(matrix_file=os.path.join(data_dir, matrix), modem_file=os.path.join(data_dir, "2bits_QPSK.txt"),
                    is5g=is5g, active=active, device=-1)
    oc = oracle_code(data_dir, matrix, is5g, active)
    assert (ctx.M, ctx.Ncol, ctx.K, ctx.cc_len, ctx.Z, ctx.E, ctx.chk) == (oc.M, oc.N, oc.K, oc.cc_len, oc.Z, oc.E,
                                                                           oc.chk)
    assert np.array_equal(ctx.perm(), oc.perm())
    for a, b in zip(ctx.graph(), oc.graph()):
        assert np.array_equal(a, b)
    rng = np.random.default_rng(5)
    uu = rng.integers(0, 2, (6, ctx.K)).astype(np.uint8)
    cc = ctx.encode(uu)
    for i in range(uu.shape[0]):
        assert np.array_equal(cc[i], oc.encode(uu[i].astype(np.int32)).astype(np.uint8))
    if active:  # every codeword satisfies H (graph columns are the permuted ones)
        for i in range(uu.shape[0]):
            full = np.zeros(ctx.Ncol, np.uint8)
            full[ctx.Ncol - ctx.cc_len:] = cc[i]
            if is5g:  # punctured columns are the first 2Z info bits
                full[:2 * ctx.Z] = uu[i][:2 * ctx.Z]
            assert oc.parity_count(full) == 0


@pytest.mark.parametrize("modem", MODEMS)
def test_constellation_matches_oracle(data_dir, modem):
    ctx = K.Context(matrix_file=os.path.join(data_dir, "PEG2304regular0.5.txt"),
                    modem_file=os.path.join(data_dir, modem), device=-1)
    om = O.Modem(os.path.join(data_dir, modem))
    assert np.array_equal(ctx.constellation().reshape(-1), om.points)


def test_constellation_matches_reference_fixture(data_dir):
    hdr, z = load_case("peg8064_64qam_blind")
    ctx = K.Context(matrix_file=os.path.join(data_dir, "PEG2304regular0.5.txt"),
                    modem_file=os.path.join(data_dir, hdr["modem"]), device=-1)
    assert np.array_equal(ctx.constellation(), z["cons"])


def test_config_file_parsing(tmp_path, data_dir):
    cfg = tmp_path / "config.toml"
    write_config(str(cfg), data_dir, "5GLDPCBG2a3_R12_K960.txt", "4bit_16QAM_Gray.txt", is5g=True, max_iter=50,
                 metric_iter=7)
    ctx = K.Context(str(cfg), device=-1)
    assert ctx.K == 960 and ctx.cc_len == 1920 and ctx.Z == 96 and ctx.max_iter == 50 and ctx.bits == 4


def test_config_relative_paths_resolve_against_data_dir(tmp_path, data_dir):
    cfg = tmp_path / "config.toml"
    cfg.write_text("""# range
[range]
    minimum_snr = 15.0
    maximum_snr = 15.0
    step_snr = 5.0
    maximum_error_number = 1
    maximum_block_number = 1
    # maximum blocks for each threads under the snr
    thread_block_number = 1

[decoder]
    true_h_arg = false

[xcodec]
    # default, using normal ldcp.
    5gldpc = false
    # (false) hard metric, (true) soft metric
    metric_type = false
    # only use for 5g ldpc
    metric_iter = 5

[histogram]
    enable = false

[ldpc]
    max_iter = 50
    # (false) not encode, (true) encode
    active = true
    matrix_file = "PEG2304regular0.5.txt"

[modem]
    modem_file = "4bit_16QAM_Gray.txt"
""")
    ctx = K.Context(str(cfg), data_dir=data_dir, device=-1)
    assert ctx.K == 1152 and ctx.max_iter == 50 and ctx.Kc == 16


def test_errors_are_reported_not_fatal(tmp_path, data_dir):
    with pytest.raises(K.KmlError, match="Cannot open"):
        K.Context(matrix_file=str(tmp_path / "missing.txt"), modem_file=os.path.join(data_dir, "2bits_QPSK.txt"),
                  device=-1)
    bad = tmp_path / "bad.toml"
    bad.write_text("[ldpc]\nmax_iter = 20\n")
    with pytest.raises(K.KmlError, match="missing"):
        K.Context(str(bad), device=-1)
    lab = tmp_path / "badmodem.txt"
    lab.write_text("bits\n2\ndims\n2\nhdr\n0 0 0 1 0\n2 0 1 0 1\n")  # label mismatch (modem.cc:113-118)
    with pytest.raises(K.KmlError, match="binary expression"):
        K.Context(matrix_file=os.path.join(data_dir, "PEG2304regular0.5.txt"), modem_file=str(lab), device=-1)


def test_host_only_context_refuses_gpu_calls(data_dir):
    ctx = K.Context(matrix_file=os.path.join(data_dir, "PEG2304regular0.5.txt"),
                    modem_file=os.path.join(data_dir, "2bits_QPSK.txt"), device=-1)
    with pytest.raises(K.KmlError, match="host-only"):
        ctx.bp_decode(np.full((1, ctx.cc_len), 0.9))


def test_exact_math_host_restatement(tmp_path):
    """kml_hypot / kml_cdiv / kml_cmul (kmldpc_amd/csrc/exact_math.hpp) vs glibc
    hypot, libgcc __divdc3 and std::complex operator* (+ __muldc3, on every
    combination of zeros, infinities, NaNs and overflowing parts) — the routines
    std::abs / operator/ / operator* call in the reference."""
    exe = tmp_path / "emc"
    src = os.path.join(REPO, "tests", "native", "exact_math_check.cpp")
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-std=c++17", "-o", str(exe), src], check=True)
    out = subprocess.run([str(exe), "1000000"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout
    assert "hypot_mismatch=0 cdiv_mismatch=0 cmul_mismatch=0" in out.stdout


def test_exp_host_restatement(tmp_path):
    """kml_exp (glibc's table-driven exp, FMA-variant contraction pattern,
    table regenerated by tools/gen_exp_table.py) equals the host glibc exp."""
    exe = tmp_path / "expc"
    src = os.path.join(REPO, "tests", "native", "exp_check.cpp")
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-std=c++17", "-o", str(exe), src], check=True)
    out = subprocess.run([str(exe), "2000000"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout
    assert "exp_fma_mismatch=0" in out.stdout


def test_log_host_restatement(tmp_path):
    """kml_log (glibc's table-driven log, FMA-variant contraction pattern,
    constants from tools/gen_log_table.py) equals the host glibc log, including
    the close-to-1 branch, subnormals and special values."""
    exe = tmp_path / "logc"
    src = os.path.join(REPO, "tests", "native", "log_check.cpp")
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-std=c++17", "-o", str(exe), src], check=True)
    out = subprocess.run([str(exe), "2000000"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout
    assert "log_fma_mismatch=0" in out.stdout


def test_kernel_placement_plans(tmp_path, data_dir):
    """The lane / slot placement plans the kernels rely on (layout.cpp), on the
    reference's H files: bp_regular's interleaved row slots and c2v halves,
    bp_irregular's paired rounds (each column / row once, pairs of one degree
    within the limits, one degree per paired wave), bp_part's partition."""
    exe = tmp_path / "planc"
    csrc = os.path.join(REPO, "kmldpc_amd", "csrc")
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", "-I", csrc, "-o", str(exe),
                    os.path.join(REPO, "tests", "native", "plan_check.cpp"), os.path.join(csrc, "code.cpp"),
                    os.path.join(csrc, "layout.cpp")], check=True)
    out = subprocess.run([str(exe)] + [os.path.join(data_dir, f) for f in
                                       ("PEG2304regular0.5.txt", "5GLDPCBG2a3_R12_K960.txt", "PEG8064regular0.5.txt")],
                         capture_output=True, text=True)
    assert out.returncode == 0, out.stdout
    assert "plan_errors=0" in out.stdout


def test_host_code_under_sanitizers(tmp_path, data_dir):
    """The host side of the library (planner, GF(2) elimination + encoder,
    TOML reader, constellation loader, reference frame stream) built with
    AddressSanitizer + UndefinedBehaviorSanitizer: the placement-plan checks on
    the reference's H files, encoded codewords with a zero syndrome, and the
    error paths on truncated / garbage H and constellation files and broken
    TOML (tests/native/host_san_check.cpp).  Any sanitizer finding aborts."""
    csrc = os.path.join(REPO, "kmldpc_amd", "csrc")
    flags = ["g++", "-O1", "-g", "-std=c++17", "-pthread", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
             "-fno-omit-frame-pointer", "-I", csrc]
    host = [os.path.join(csrc, f) for f in ("code.cpp", "layout.cpp", "config.cpp", "modem.cpp", "refstream.cpp")]
    # the partition refinement's annealing at a short schedule (its full length
    # runs in test_kernel_placement_plans)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1",
               KML_PART_REFINE_ITERS="3000000")
    hsc, planc = tmp_path / "hsc", tmp_path / "planc"
    builds = [subprocess.Popen(flags + ["-o", str(hsc), os.path.join(REPO, "tests", "native", "host_san_check.cpp")]
                               + host),
              subprocess.Popen(flags + ["-o", str(planc), os.path.join(REPO, "tests", "native", "plan_check.cpp")]
                               + host[:2])]
    assert [b.wait() for b in builds] == [0, 0]
    scratch = tmp_path / "scratch"
    scratch.mkdir()
    out = subprocess.run([str(hsc), data_dir, str(scratch)], capture_output=True, text=True, env=env, timeout=600)
    assert out.returncode == 0, out.stdout + out.stderr[-4000:]
    assert "san_errors=0" in out.stdout
    out = subprocess.run([str(planc)] + [os.path.join(data_dir, f) for f in
                                         ("PEG2304regular0.5.txt", "5GLDPCBG2a3_R12_K960.txt", "PEG8064regular0.5.txt")],
                         capture_output=True, text=True, env=env, timeout=600)
    assert out.returncode == 0, out.stdout + out.stderr[-4000:]
    assert "plan_errors=0" in out.stdout


def test_cn_division_tail_exact_near_one():
    """The CN phases' division (near-one reciprocal RN(1/s), then the FAST
    tail) rounds n / s correctly on every significand where it could fail, for
    |s - 1| <= 64 ulp: exact rational evaluation (tools/verify_cn_division.py)."""
    out = subprocess.run([sys.executable, os.path.join(REPO, "tools", "verify_cn_division.py")],
                         capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout
    assert "near-one reciprocal misses: 0" in out.stdout


# ---------------------------------------------------------- host random sources
def test_reference_rngs_match_reference():
    """CLCRandNum / CWHRandNum / GetSymStr / GetBitStr with SetSeed(-1) equal the
    reference's streams (tests/golden/rng.npz, from the reference harness)."""
    z = np.load(os.path.join(REPO, "tests", "golden", "host", "rng.npz"))
    n = len(z["clc_u"])
    c = K.CLCRandNum()
    w = K.CWHRandNum()
    assert np.array_equal([c.Uniform() for _ in range(n)], z["clc_u"])
    assert np.array_equal([w.Uniform() for _ in range(n)], z["wh_u"])
    assert np.array_equal(c.Normal(n + 1), z["clc_n"])
    assert np.array_equal(w.Normal(n + 1), z["wh_n"])
    assert np.array_equal(c.GetSymStr(16, n), z["sym16"])
    assert np.array_equal(c.GetSymStr(3, n), z["sym3"])
    assert np.array_equal(c.GetBitStr(n), z["bits"].astype(np.uint8))


@pytest.mark.parametrize("case", ["peg2304_qpsk_known", "bg2_16qam_known", "peg8064_64qam_known"])
def test_ref_frames_reproduce_reference_stream(case, data_dir):
    """kml_ref_frames = the reference's frames for seed 17 (fixture CRCs): the
    product side of 'identical RNG seeds' parity runs."""
    import zlib
    from conftest import load_case
    hdr, z = load_case(case)
    ctx = K.Context(matrix_file=os.path.join(data_dir, hdr["matrix"]), modem_file=os.path.join(data_dir, hdr["modem"]),
                    is5g=bool(hdr["is5g"]), max_iter=hdr["max_iter"], device=-1)
    n = min(40, len(z["s_crc_y"]))
    uu, th, y = ctx.ref_frames(K.CLCRandNum(), hdr["snr"], n)
    for i in range(n):
        assert zlib.crc32(y[i].tobytes()) & 0xFFFFFFFF == z["s_crc_y"][i]
        assert zlib.crc32(uu[i].tobytes()) & 0xFFFFFFFF == z["s_crc_uu"][i]
    assert np.array_equal(th, z["s_true_h"][:n])


def test_first_backward_normalisation_is_identity():
    """bp_common.hpp: RN(c0 + RN(1 - c0)) == 1 for every c0 in [0, 1], so the
    FAST kernels skip the first backward normalisation of each column."""
    rng = np.random.default_rng(5)
    c0 = np.concatenate([
        rng.random(2_000_000),
        rng.random(500_000) * 1e-6,  # small messages, where 1 - c0 rounds
        1.0 - rng.random(500_000) * 1e-6,
        np.ldexp(rng.random(500_000) + 0.5, rng.integers(-40, 0, 500_000)),
        np.array([0.0, 1.0, 0.5, 1e-12, 1.0 - 1e-12, np.nextafter(0.5, 0.0), np.nextafter(0.5, 1.0),
                  np.nextafter(1.0, 0.0), 5e-324]),
    ])
    one_minus = 1.0 - c0
    assert np.all(c0 + one_minus == 1.0)
    assert np.all(c0 / (c0 + one_minus) == c0) and np.all(one_minus / (c0 + one_minus) == one_minus)


def test_kmeans_dump_mat_level5(tmp_path, data_dir):
    """KMeans::DumpToMat (src/kmeans.cc:99-109) through kml_kmeans_dump_mat:
    a MAT-file level 5 that scipy reads back with the reference's variable
    names, classes (complex double, int32) and n x 1 shapes (lib/lab/src/mat.cc
    WriteVector / WriteComplex), values bit-identical.  The data are the
    reference's own k-means state (golden/kmstate)."""
    import scipy.io

    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "kmstate", "peg2304_16qam_s5.npz"))
    hdr = json.loads(bytes(z["hdr_json"]).decode())
    om = O.Modem(os.path.join(data_dir, hdr["modem"]))
    y, cl, idx = z["y"][1], z["clusters"][1], z["idx"][1]
    cons = om.points.reshape(-1, 2)
    hh = cl[0, 0] + 1j * cl[0, 1]
    c0 = cons[0, 0] + 1j * cons[0, 1]
    append = np.array([hh / c0 * 1j ** j for j in range(4)] + [z["true_h"][1, 0] + 1j * z["true_h"][1, 1]])
    path = str(tmp_path / "km.mat")
    K.dump_kmeans_mat(path, y, cl, idx, cons, append)
    m = scipy.io.loadmat(path)
    assert m["__version__"] == "1.0"
    c = lambda a: a[:, 0] + 1j * a[:, 1]
    for name, want, dt in [("data", c(y), np.complex128), ("cluster", c(cl), np.complex128),
                           ("idx", idx, np.int32), ("constellations", c(cons), np.complex128),
                           ("hHats", append[:4], np.complex128), ("realH", append[4:], np.complex128)]:
        got = m[name]
        assert got.dtype == dt, name
        assert got.shape == (len(want), 1), name
        assert np.array_equal(got[:, 0], want), name
    with pytest.raises(K.KmlError):
        K.dump_kmeans_mat(str(tmp_path / "no" / "such" / "dir.mat"), y, cl, idx, cons, append)

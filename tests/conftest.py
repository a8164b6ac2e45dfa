import gzip
import json
import os
import sys

import numpy as np
import pytest

TESTS = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(TESTS)
GOLDEN = os.path.join(TESTS, "golden")
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def data_dir(tmp_path_factory):
    """The reference's config/*.txt data files (H matrices, constellations),
    decompressed from tests/golden/data into a temp dir."""
    d = tmp_path_factory.mktemp("kml_data")
    src = os.path.join(GOLDEN, "data")
    for fn in os.listdir(src):
        if fn.endswith(".gz"):
            with gzip.open(os.path.join(src, fn), "rb") as g:
                (d / fn[:-3]).write_bytes(g.read())
    return str(d)


def load_case(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    hdr = json.loads(bytes(z["hdr_json"]).decode())
    return hdr, z


def case_names():
    return sorted(f[:-4] for f in os.listdir(GOLDEN) if f.endswith(".npz"))


def write_config(path, data_dir, matrix, modem, is5g=False, known=True, max_iter=20, active=True, snr=2.0,
                 metric_type=False, metric_iter=5, max_blocks=1000, max_err=1000000, thread_blocks=1000,
                 snr_max=None, snr_step=1.0, histogram=False):
    b = lambda v: "true" if v else "false"
    snr_max = snr if snr_max is None else snr_max
    with open(path, "w") as f:
        f.write(f"""# written by tests
[range]
    minimum_snr = {float(snr)!r}
    maximum_snr = {float(snr_max)!r}
    step_snr = {float(snr_step)!r}
    maximum_error_number = {int(max_err)}
    maximum_block_number = {int(max_blocks)}
    thread_block_number = {int(thread_blocks)}

[decoder]
    true_h_arg = {b(known)}

[xcodec]
    5gldpc = {b(is5g)}
    metric_type = {b(metric_type)}
    metric_iter = {int(metric_iter)}

[histogram]
    enable = {b(histogram)}

[ldpc]
    max_iter = {int(max_iter)}
    active = {b(active)}
    matrix_file = "{os.path.join(data_dir, matrix)}"

[modem]
    modem_file = "{os.path.join(data_dir, modem)}"
""")
    return path


def soft_case_names():
    d = os.path.join(GOLDEN, "soft")
    return sorted(f[:-4] for f in os.listdir(d) if f.endswith(".npz")) if os.path.isdir(d) else []


def load_soft_case(name):
    z = np.load(os.path.join(GOLDEN, "soft", name + ".npz"))
    return json.loads(bytes(z["hdr_json"]).decode()), z

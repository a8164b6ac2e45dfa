"""The reference-side shims (integration/kmldpc_gpu_codecs.hpp, shown in
INTEGRATION.md) compile against the reference's own headers and link the
product library: GpuBinaryLDPCCodec overrides the virtual
lab::BinaryLDPCCodec::Decoder (lib/lab/include/binaryldpccodec.h:20) and
Binary5GLDPCCodec's (binary5gldpccodec.h:17); GpuKmCodec takes KmCodec::Decoder's
arguments (include/kmcodec.h:23-25).  Compile + link only (no GPU here); the
GPU run of the same program is tests/test_gpu_integration.py."""
import glob
import os
import subprocess
from concurrent.futures import ThreadPoolExecutor

import pytest

from conftest import REPO

REFK = "/root/reference/kmldpc"
INC = [f"-I{REFK}/include", f"-I{REFK}/lib/lab/include", f"-I{REFK}/lib/toml11", f"-I{REPO}/include",
       f"-I{REPO}/integration"]

pytestmark = pytest.mark.skipif(not os.path.isdir(REFK), reason="reference sources not present")


def _cc(args):
    src, obj = args
    r = subprocess.run(["g++", "-O0", "-std=c++17", "-w", *INC, '-D__FILENAME__="ref"', "-c", "-o", obj, src],
                       capture_output=True, text=True)
    return src, r.returncode, r.stderr


def test_shims_compile_and_link_against_reference(tmp_path):
    lib = os.path.join(REPO, "kmldpc_amd", "libkmldpc_amd.so")
    assert os.path.exists(lib), "make lib first"
    srcs = [os.path.join(REPO, "oracle", "shim_check.cc"), f"{REFK}/src/kmcodec.cc", f"{REFK}/src/kmeans.cc"]
    srcs += sorted(glob.glob(f"{REFK}/lib/lab/src/*.cc"))
    objs = [str(tmp_path / (os.path.basename(s) + ".o")) for s in srcs]
    with ThreadPoolExecutor(8) as ex:
        for src, rc, err in ex.map(_cc, zip(srcs, objs)):
            assert rc == 0, f"{src}: {err[-2000:]}"
    exe = str(tmp_path / "shim_check")
    r = subprocess.run(["g++", "-o", exe, *objs, f"-L{REPO}/kmldpc_amd", "-lkmldpc_amd", "-lpthread",
                        f"-Wl,-rpath,{REPO}/kmldpc_amd"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    # the overrides really are overrides (a signature drift would make `override` fail to compile above);
    # and the dynamic symbols the shims use resolve from the product library
    nm = subprocess.run(["nm", "-D", "--undefined-only", exe], capture_output=True, text=True).stdout
    for sym in ("kml_bp_decode", "kml_decode_candidates", "kml_kmeans", "kml_create", "kml_dims"):
        assert sym in nm, sym
    usage = subprocess.run([exe], capture_output=True, text=True)
    assert usage.returncode == 2 and "usage" in usage.stderr


def test_integration_doc_points_at_the_compiled_shims():
    doc = open(os.path.join(REPO, "INTEGRATION.md")).read()
    assert "integration/kmldpc_gpu_codecs.hpp" in doc
    hdr = open(os.path.join(REPO, "integration", "kmldpc_gpu_codecs.hpp")).read()
    for name in ("class GpuLdpcCodec", "using GpuBinaryLDPCCodec", "using GpuBinary5GLDPCCodec", "class GpuKmCodec"):
        assert name in hdr

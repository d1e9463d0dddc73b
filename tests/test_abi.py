"""C-ABI boundary checks that need no GPU: the library loads, exports every
function include/pbgpu.h declares, and fails loudly (no CPU fallback) when no
device is present."""
import ctypes as C
import os
import re
import subprocess

import pytest

from pacbio_amd import pbgpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "pbgpu.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pbgpu_[a-z_]+)\s*\(", src)))


def test_header_and_binding_agree():
    assert sorted(pbgpu.EXPORTS) == _declared()


def test_library_exports_every_declared_symbol():
    lib = C.CDLL(pbgpu.LIB_PATH)
    for name in _declared():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", pbgpu.LIB_PATH], capture_output=True, text=True).stdout
    for name in _declared():
        assert re.search(rf"\bT {name}\b", out), name


def test_abi_version():
    assert pbgpu.lib().pbgpu_abi_version() == 8


def test_record_layout_matches_header():
    assert pbgpu.RECORD_DTYPE.itemsize == 96
    assert pbgpu.GRAPH_NODE_DTYPE.itemsize == 24
    assert pbgpu.MEGA_DTYPE.itemsize == 72
    # pbgpu_coords_batch: 7 words + the graph and mega-read pointers (ABI 5)
    assert C.sizeof(pbgpu.CoordsBatch) == 96


def test_params_default_matches_yaggo_defaults():
    # jf_aligner_cmdline.yaggo: stretch-factor 1.3, stretch-constant 10, stretch-cap 10000, window 1, B 17, M 0, max-count 5000
    p = pbgpu.AlignParams()
    pbgpu.lib().pbgpu_align_params_default(C.byref(p))
    assert (p.k, p.stretch_factor, p.stretch_constant, p.stretch_cap, p.window_size, p.max_count,
            p.bases_matching, p.mers_matching) == (17, 1.3, 10.0, 10000.0, 1, 5000, 17.0, 0.0)


@pytest.mark.skipif(pbgpu.lib().pbgpu_device_count() > 0, reason="only meaningful without a GPU")
def test_no_gpu_fails_loudly():
    with pytest.raises(pbgpu.PbgpuError) as e:
        pbgpu.Index.from_records(["1F"], ["ACGT" * 20], 17)
    assert e.value.status == 4  # PBGPU_ERR_DEVICE


def test_invalid_params_rejected_before_device():
    with pytest.raises(pbgpu.PbgpuError) as e:
        pbgpu.Index.from_records(["1F"], ["ACGT" * 20], 40)
    assert e.value.status == 5
    with pytest.raises(pbgpu.PbgpuError) as e:
        pbgpu.Index.from_records(["1F"], ["ACGT" * 20], 13, psa_min=13)
    assert e.value.status == 5


def test_last_error_is_thread_local_message():
    with pytest.raises(pbgpu.PbgpuError):
        pbgpu.Index.from_records(["1F"], ["ACGT"], 40)
    assert b"k=40" in pbgpu.lib().pbgpu_last_error()


CLI = os.path.join(ROOT, "pacbio_amd", "bin", "jf_aligner")


@pytest.mark.parametrize("args,msg", [
    ([], "-s, --size is required"),
    (["-s", "1"], "-m, --mer is required"),
    (["-s", "1", "-m", "17"], "No output file given"),
    (["-s", "1", "-m", "17", "--coords", "/dev/null", "--max-count", "0"], "undefined behaviour"),
    (["-s", "1", "-m", "17", "-l", "x", "-u", "y"], "conflicts"),
    (["-s", "1", "-m", "17", "--coords", "/dev/null", "-l", "x"], "-k, --k-mer"),
])
def test_cli_argument_errors(args, msg):
    r = subprocess.run([CLI] + args, capture_output=True, text=True)
    assert r.returncode != 0 and msg in r.stderr, r.stderr


CMR = os.path.join(ROOT, "pacbio_amd", "bin", "create_mega_reads")


@pytest.mark.parametrize("args,msg", [
    ([], "-s, --size is required"),
    (["-s", "1"], "-m, --mer is required"),
    (["-s", "1", "-m", "17"], "-k, --k-mer is required"),
    (["-s", "1", "-m", "17", "-k", "31"], "unitig lengths (-l) or sequences (-u) are required"),
    (["-s", "1", "-m", "17", "-k", "31", "-l", "x", "-u", "y"], "conflicts"),
    (["-s", "1", "-m", "17", "-k", "31", "-l", "x", "--max-count", "0"], "undefined behaviour"),
    (["-s", "1", "-m", "17", "-k", "31", "-l", "x", "-T", "best"], "invalid --tiling"),
    (["-s", "1", "-m", "17", "-k", "31", "-l", "x", "--trim", "all"], "invalid --trim"),
    (["-s", "1", "-m", "17", "-k", "31", "-l", "/nonexistent/ul.txt"], "Failed to open unitig lengths"),
])
def test_create_mega_reads_argument_errors(args, msg):
    """create_mega_reads_cmdline.yaggo's required / conflicting options, checked before any GPU call"""
    r = subprocess.run([CMR] + args, capture_output=True, text=True)
    assert r.returncode != 0 and msg in r.stderr, r.stderr

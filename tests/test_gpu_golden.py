"""The GPU path (bin/jf_aligner -> libpbgpu.so) against the reference's own
CLI golden outputs, tests/aligner_output (copied under tests/golden/).  Those
files come from an older jf_aligner that printed an Rname column after Err;
the numeric fields and the super-read name are compared, exactly as
tests/test_oracle_cli.py does for the CPU restatement."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden", "aligner_output")
CLI = os.path.join(ROOT, "pacbio_amd", "bin", "jf_aligner")


def _norm_expected(path):
    rows = []
    for line in open(path).read().splitlines()[1:]:
        f = line.split()
        rows.append(f[:14] + [f[15]] + f[16:])  # drop the old Rname column
    return sorted(rows)


def _norm_ours(text):
    return sorted(line.split()[1:] for line in text.splitlines()[1:])


def _run(*extra):
    args = [CLI, "-s", "10k", "-m", "17", "-r", os.path.join(GOLD, "test_super_reads.fa"), "-p",
            os.path.join(GOLD, "test_pacbio.fa"), "--stretch-cap", "200", "--no-compact", "--coords", "/dev/stdout", *extra]
    r = subprocess.run(args, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    return r.stdout


def test_gpu_coords_normal_matches_reference_expected():
    got = _norm_ours(_run())
    assert len(got) > 0
    assert got == _norm_expected(os.path.join(GOLD, "coords_normal_expected"))


def test_gpu_coords_forward_matches_reference_expected():
    got = _norm_ours(_run("-l", os.path.join(GOLD, "test_unitigs_lengths"), "-k", "65", "-f"))
    assert got == _norm_expected(os.path.join(GOLD, "coords_forward_expected"))

"""End-to-end oracle vs the reference's own CLI golden files
(tests/aligner_output, produced by an older jf_aligner with the Rname column
after Err; the numeric fields are what is compared)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden", "aligner_output")
ORACLE = os.path.join(ROOT, "oracle", "pb_oracle")


def _norm_expected(path):
    rows = []
    for line in open(path).read().splitlines()[1:]:
        f = line.split()
        rows.append(f[:14] + [f[15]] + f[16:])  # drop the old Rname column
    return sorted(rows)


def _norm_ours(text):
    rows = []
    for line in text.splitlines()[1:]:
        f = line.split()
        rows.append(f[1:])  # drop the leading pb name (non-compact, current code)
    return sorted(rows)


def _run(*extra):
    args = [ORACLE, "-s", "10k", "-m", "17", "-r", os.path.join(GOLD, "test_super_reads.fa"), "-p",
            os.path.join(GOLD, "test_pacbio.fa"), "--stretch-cap", "200", "--no-compact", *extra]
    return subprocess.run(args, capture_output=True, text=True, check=True).stdout


def test_coords_normal_matches_reference_expected():
    assert _norm_ours(_run()) == _norm_expected(os.path.join(GOLD, "coords_normal_expected"))


def test_coords_forward_matches_reference_expected():
    got = _norm_ours(_run("-l", os.path.join(GOLD, "test_unitigs_lengths"), "-k", "65", "-f"))
    assert got == _norm_expected(os.path.join(GOLD, "coords_forward_expected"))


def test_cli_rejects_max_count_zero():
    r = subprocess.run([ORACLE, "-s", "1", "-m", "17", "--max-count", "0"], capture_output=True, text=True)
    assert r.returncode != 0

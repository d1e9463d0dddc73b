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
            os.path.join(GOLD, "test_pacbio.fa"), "--stretch-cap", "200", "--no-compact", "--coords", "/dev/stdout", *extra]
    return subprocess.run(args, capture_output=True, text=True, check=True).stdout


def test_coords_normal_matches_reference_expected():
    assert _norm_ours(_run()) == _norm_expected(os.path.join(GOLD, "coords_normal_expected"))


def test_coords_forward_matches_reference_expected():
    got = _norm_ours(_run("-l", os.path.join(GOLD, "test_unitigs_lengths"), "-k", "65", "-f"))
    assert got == _norm_expected(os.path.join(GOLD, "coords_forward_expected"))


def _details(*extra):
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "details")
        _run("--details", out, *extra)
        return sorted(open(out).read().splitlines())


def test_details_normal_matches_reference_expected():
    # print_details (jf_aligner.cc:72-108); lines of a read come from an unordered_map
    assert _details() == sorted(open(os.path.join(GOLD, "details_normal_expected")).read().splitlines())


def test_details_forward_matches_reference_expected():
    got = _details("-l", os.path.join(GOLD, "test_unitigs_lengths"), "-k", "65", "-f")
    assert got == sorted(open(os.path.join(GOLD, "details_forward_expected")).read().splitlines())


def fine_vs_coarse_properties(coarse_text, fine_text):
    """tests/aligner_output/compare_coarse_fine_alignments:1-61 restated: one fine
    record per coarse record (keyed by super-read name), same Rlen/Qlen/name, k-unitig
    sums consistent with Nmers/Qcover, fine coordinates contain the coarse ones and
    no match count decreases.  Lines are in the current non-compact format
    (pb name first)."""
    def read(text):
        res = {}
        for line in text.splitlines()[1:]:
            f = line.split()
            f = f[1:15] + [f[0]] + f[15:]  # to the old column layout the script indexes
            res[f[15]] = f
        return res

    def sum_up(a):
        mers = bases = 0
        for i in range(16, len(a)):
            m, b = (int(t) for t in a[i].split(":"))
            if i % 2 == 1:
                m, b = -m, -b
            mers += m; bases += b
        return mers, bases

    cl, fl = read(coarse_text), read(fine_text)
    assert len(cl) == len(fl), "Mismatching number of alignments"
    for q, cf in cl.items():
        ff = fl[q]
        assert ff[9] == cf[9] and ff[10] == cf[10] and ff[14] == cf[14] and ff[15] == cf[15], q
        assert (int(ff[4]), int(ff[8])) == sum_up(ff), q
        assert (int(cf[4]), int(cf[8])) == sum_up(cf), q
        assert int(ff[0]) <= int(cf[0]) and int(ff[1]) >= int(cf[1]) and int(ff[2]) <= int(cf[2]) \
            and int(ff[3]) >= int(cf[3]), q
        assert all(int(ff[i]) >= int(cf[i]) for i in range(4, 9)), q


def test_fine_aligner_reference_properties():
    # the reference's Tupfile runs -F 13 beside the forward run and checks it with
    # compare_coarse_fine_alignments (tests/aligner_output/Tupfile:8-9)
    fwd = ("-l", os.path.join(GOLD, "test_unitigs_lengths"), "-k", "65", "-f")
    coarse, fine = _run(*fwd), _run(*fwd, "-F", "13")
    assert coarse.count("\n") == 4
    fine_vs_coarse_properties(coarse, fine)


def test_cli_rejects_max_count_zero():
    r = subprocess.run([ORACLE, "-s", "1", "-m", "17", "--coords", "/dev/null", "--max-count", "0"], capture_output=True,
                       text=True)
    assert r.returncode != 0

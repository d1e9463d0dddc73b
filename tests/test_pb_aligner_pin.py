"""tests/test_pb_aligner.cc (PbAligner.FakeSequences) restated: a 1000-bp random
sequence, a 500-bp PacBio read from base 300 with a substitution at read base
100 and a 4-base insertion at 400, and ten 100-bp super-reads around those
features (odd forward, even reverse-complemented).  fetch_super_reads' lists
of every super-read -- their lengths and the first / last super-read offsets
(coarse_aligner.cc:128-140 order) -- are checked against the reference test's
expectations (test_pb_aligner.cc:108-167), with the one difference below.

The reference test predates the every-other toggle of the current
fetch_super_reads (coarse_aligner.cc:89,96-102): with k = 15 the 2nd k-mer
after a reset (len 16 <= 17) is skipped, so R1 and R2, the two super-reads
that cover the read's first k-mers, each have one hit fewer than the test
expects -- the one at read offset 2 -- and 8 of the 10 lists match it exactly.

The sequence comes from glibc random() without a seed, as in the reference
test; the lists are read from the --details output (print_details,
jf_aligner.cc:72-108: fwd hits carry positive super-read offsets, bwd hits
negative ones).  CPU: the oracle; GPU: the device path through the C ABI."""
import ctypes as C

import pytest

# test_pb_aligner.cc:108-167: read id -> (strand, list length, first sr offset, last sr offset)
EXPECTED = {
    1: ("fwd", 36, 51, 86), 2: ("bwd", 61, -61, -1), 3: ("fwd", 75, 12, 86), 4: ("bwd", 71, -86, -1),
    5: ("fwd", 70, 1, 86), 6: ("bwd", 70, -86, -1), 7: ("fwd", 16, 1, 16), 8: ("bwd", 6, -86, -81),
    9: ("fwd", 86, 1, 86), 10: ("bwd", 86, -86, -1),
}
K = 15


def _rev_comp(s):
    return s[::-1].translate(str.maketrans("ACGT", "TGCA"))


def fake_sequences():
    """generate_sequences (test_pb_aligner.cc:35-62) with glibc's unseeded random()"""
    libc = C.CDLL(None)
    libc.random.restype = C.c_long
    libc.srandom(1)  # the state random() starts from when never seeded
    base = "ACGT"
    seq = "".join(base[libc.random() % 4] for _ in range(1000))
    pb = list(seq[300:800])
    err = pb[100]
    while True:
        pb[100] = base[libc.random() % 4]
        if pb[100] != err:
            break
    pb[399] = "C"
    pb[400] = "G"
    pb = "".join(pb)
    pb = pb[:400] + "ACGT" + pb[400:]
    srs = [("R1", seq[250:350]), ("R2", _rev_comp(seq[275:375])), ("R3", seq[390:490]),
           ("R4", _rev_comp(seq[380:480])), ("R5", seq[660:760]), ("R6", _rev_comp(seq[670:770])),
           ("R7", seq[770:870]), ("R8", _rev_comp(seq[780:880])), ("R9", seq[500:600]),
           ("R10", _rev_comp(seq[550:650]))]
    return srs, pb


TOGGLED = {1, 2}  # lists that lose the read-offset-2 hit to the toggle


def lists_from_details(text):
    """{super-read name: (fwd hits, bwd hits)} in list order, hits = (pb offset, sr offset)"""
    out = {}
    for line in text.splitlines():
        f = line.split()
        if len(f) < 2:
            continue
        fwd, bwd = [], []
        for h in f[2:]:
            pb, so = (int(x) for x in h.strip("[]").split(":"))
            (fwd if so > 0 else bwd).append((pb, so))
        out[f[1]] = (fwd, bwd)
    return out


def check(lists):
    assert len(lists) == 10
    pbs = set()
    for rid, (strand, n, first, last) in EXPECTED.items():
        fwd, bwd = lists[f"R{rid}"]
        lst = fwd if strand == "fwd" else bwd
        assert not (bwd if strand == "fwd" else fwd)
        want = n - (1 if rid in TOGGLED else 0)
        assert (len(lst), lst[0][1], lst[-1][1]) == (want, first, last), (rid, len(lst), lst[:2], lst[-2:])
        pbs.update(p for p, _ in lst)
    assert 1 in pbs and 3 in pbs and 2 not in pbs  # the toggled k-mer, and only it


def test_oracle_fetch_super_reads_matches_reference_test():
    from oracle.oracle import OracleIndex, params
    srs, pb = fake_sequences()
    oix = OracleIndex.from_records([n for n, _ in srs], [s for _, s in srs], K)
    _, det = oix.align_format(params(k=K), ["pb"], [pb], details=True)
    oix.close()
    check(lists_from_details(det))


@pytest.mark.gpu
def test_gpu_fetch_super_reads_matches_reference_test():
    from pacbio_amd import pbgpu
    srs, pb = fake_sequences()
    gix = pbgpu.Index.from_records([n for n, _ in srs], [s for _, s in srs], K)
    al = pbgpu.Aligner(gix, k=K)
    al.set_details(True)
    al.align([pb])
    det = al.download_details().format(gix, ["pb"])
    al.close()
    gix.close()
    check(lists_from_details(det))

"""StreamAligner (one batch over S aligners on their own HIP streams and host
threads, sharing one index): the concatenated parts format byte-identically
to the CPU restatement (oracle/) for any S, including S larger than the
number of reads (empty ranges get no aligner)."""
import pytest

from tests._compare import assert_same_coords

pytestmark = pytest.mark.gpu

KW = dict(forward=True, unitigs_k=31, bases_matching=15.0)


@pytest.fixture(scope="module")
def case():
    from oracle.oracle import OracleIndex, params
    from pacbio_amd import pbgpu
    from tools.synth import Dataset
    ds = Dataset("small", seed=11)
    names, seqs = ds.sr_names(), ds.sr_seqs()
    pn, ps = ds.pb_names(), ds.pb_seqs()
    exp = OracleIndex.from_records(names, seqs, 17).align_format(
        params(k=17, unitig_lengths=ds.unitig_lengths, **KW), pn, ps, threads=4)
    gix = pbgpu.Index.from_records(names, seqs, 17)
    yield ds, gix, pn, ps, exp
    gix.close()


def _stream_align(gix, ds, pn, ps, S):
    from pacbio_amd import pbgpu
    sa = pbgpu.StreamAligner(gix, streams=S, k=17, unitig_lengths=ds.unitig_lengths, **KW)
    try:
        parts = sa.upload(seqs=ps)
        for _ in range(2):  # resident batches are re-aligned: outputs must not accumulate
            sa.align_resident(parts)
        got = sa.format(sa.download(parts), pn, [len(s) for s in ps])
        sa.free(parts)
        return got, sa.stats()
    finally:
        sa.close()


@pytest.mark.parametrize("S", [1, 2, 3])
def test_streams_parity(case, S):
    ds, gix, pn, ps, exp = case
    got, st = _stream_align(gix, ds, pn, ps, S)
    assert exp.count("\n") > 10
    assert_same_coords(got, exp, f"streams{S}")
    assert st["n_reads"] == 2 * len(ps)


def test_streams_more_than_reads(case):
    ds, gix, pn, ps, exp = case
    n = 2
    got, _ = _stream_align(gix, ds, pn[:n], ps[:n], 4)
    from oracle.oracle import OracleIndex, params
    e2 = OracleIndex.from_records(ds.sr_names(), ds.sr_seqs(), 17).align_format(
        params(k=17, unitig_lengths=ds.unitig_lengths, **KW), pn[:n], ps[:n], threads=2)
    assert_same_coords(got, e2, "streams>reads")

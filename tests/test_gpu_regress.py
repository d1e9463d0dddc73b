"""Regressions found at BASELINE scale (kept small enough to run in seconds)."""
import pytest

from tests._compare import assert_same_coords

pytestmark = pytest.mark.gpu


def test_lisw_chunk_boundary_read_11163():
    """C2 read 11163: a bwd strand of 75 hits whose element 64 (first of the
    second 64-lane chunk) fails the step test against element 63.  k_lis_w's
    register path read element 63 through a shuffle executed by lane 0 alone,
    got (0, 0) and took the whole strand for one clean run (3 extra lis
    points).  Found by bench.py's CPU-baseline parity check (r02)."""
    from oracle.oracle import OracleIndex, params
    from pacbio_amd import pbgpu
    from tools.synth import Dataset
    ds = Dataset("C2", seed=42, threads=16, n_pb=11164)
    kw = dict(k=17, forward=True, unitigs_k=31, unitig_lengths=ds.unitig_lengths, bases_matching=15.0,
              max_count=5000, stretch_cap=10000.0)
    names, seqs = ds.sr_names(), ds.sr_seqs()
    pn, ps = ds.pb_names()[11163:], ds.pb_seqs()[11163:]
    gix = pbgpu.Index.from_records(names, seqs, 17)
    got = pbgpu.Aligner(gix, **kw).align(ps).format(gix, pn, [len(s) for s in ps])
    exp = OracleIndex.from_records(names, seqs, 17, threads=16).align_format(params(**kw), pn, ps, threads=1)
    assert "15650R_15649R_15648R " in exp
    assert_same_coords(got, exp, "read 11163")

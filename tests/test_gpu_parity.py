"""GPU parity: libpbgpu.so (through the C ABI) vs the CPU restatement
(oracle/) on seeded synthetic workloads, byte-identical coords text."""
import pytest

from tests._compare import assert_same_coords

pytestmark = pytest.mark.gpu

CONFIGS = {
    "default": dict(),
    "forward_ul": dict(forward=True, unitigs_k=31, use_ul=True, bases_matching=15.0),
    "max_match": dict(forward=True, max_match=True, unitigs_k=31, use_ul=True, bases_matching=10.0),
    "window3": dict(window_size=3),
    "cap200": dict(stretch_cap=200.0),
    "M10": dict(mers_matching=10.0, bases_matching=0.0),
    "maxcount20": dict(max_count=20),
    "k21": dict(k=21),
    "k16_even": dict(k=16),
}


@pytest.fixture(scope="module")
def small():
    from tools.synth import Dataset
    return Dataset("small", seed=7)


def _run(ds, cfg):
    from oracle.oracle import OracleIndex, params
    from pacbio_amd import pbgpu
    cfg = dict(cfg)
    k = cfg.pop("k", 17)
    use_ul = cfg.pop("use_ul", False)
    ul = ds.unitig_lengths if use_ul else None
    names, seqs = ds.sr_names(), ds.sr_seqs()
    pnames, pseqs = ds.pb_names(), ds.pb_seqs()
    oix = OracleIndex.from_records(names, seqs, k)
    exp = oix.align_format(params(k=k, unitig_lengths=ul, **cfg), pnames, pseqs, threads=4)
    gix = pbgpu.Index.from_records(names, seqs, k)
    al = pbgpu.Aligner(gix, k=k, unitig_lengths=ul, **cfg)
    co = al.align(pseqs)
    got = co.format(gix, pnames, [len(s) for s in pseqs])
    return got, exp


@pytest.mark.parametrize("name", list(CONFIGS))
def test_parity_small(small, name):
    got, exp = _run(small, CONFIGS[name])
    assert exp.count("\n") > 10, "workload produced too few records to be meaningful"
    assert_same_coords(got, exp, name)


@pytest.fixture(scope="module")
def short_unitigs():
    """Unitigs from 31 bases (= unitigs_k) up: k-mers span several unitigs, the
    kmers_info paths beyond the next unitig run."""
    from tools.synth import Dataset
    return Dataset("small", seed=9, unitig_mean=40, unitig_min=31)


@pytest.mark.parametrize("name", ["forward_ul", "max_match"])
def test_parity_short_unitigs(short_unitigs, name):
    got, exp = _run(short_unitigs, CONFIGS[name])
    assert exp.count("\n") > 10, "workload produced too few records to be meaningful"
    assert_same_coords(got, exp, name)

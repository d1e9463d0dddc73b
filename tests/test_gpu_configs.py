"""Parity at BASELINE.json's own configurations (SURVEY 8(d) generator, seed 42),
GPU (through the C ABI, device-formatted text) vs the CPU restatement (oracle/):

  C1  exactly: 100 PB x 10 kb vs 1k SRs, k=17 -- defaults and the production flags;
  C2  the full 200k-SR index (k=17), the first 3000 reads of the 50k workload;
  C3  the full 1M-SR index (k=21), the first 1500 reads of the 300k workload.

Production flags: -m 17|21 --psa-min 13 -l ul.txt -k 31 -f -B 15
--max-count 5000 --stretch-cap 10000.  At C2/C3 scale the 99% threshold and the
max-count filter run on real repeat content (coarse_aligner.cc:81-141), which
the small presets barely reach."""
import pytest

from tests._compare import assert_same_coords

pytestmark = pytest.mark.gpu


def _prod(ds, k):
    return dict(k=k, forward=True, unitigs_k=31, unitig_lengths=ds.unitig_lengths, bases_matching=15.0,
                max_count=5000, stretch_cap=10000.0)


def _compare(ds, kw, ctx, threads=16):
    from oracle.oracle import OracleIndex, params
    from pacbio_amd import pbgpu
    k = kw["k"]
    names, seqs = ds.sr_names(), ds.sr_seqs()
    pnames, pseqs = ds.pb_names(), ds.pb_seqs()
    gix = pbgpu.Index.from_records(names, seqs, k)
    al = pbgpu.Aligner(gix, **kw)
    rd = al.upload(pseqs, names=pnames)
    al.align_resident(rd)
    got = al.format_device(rd)
    st = al.stats()
    rd.close()
    al.close()
    gix.close()
    oix = OracleIndex.from_records(names, seqs, k, threads=threads)
    exp = oix.align_format(params(**kw), pnames, pseqs, threads=threads)
    oix.close()
    assert exp.count("\n") > 10 * len(pseqs) // 100, f"{ctx}: too few records to be meaningful"
    assert_same_coords(got, exp, ctx)
    return st


@pytest.mark.parametrize("flags", ["defaults", "production", "max_match"])
def test_c1_exact(flags):
    from tools.synth import Dataset
    ds = Dataset("C1", seed=42)
    kw = {"defaults": dict(k=17), "production": _prod(ds, 17),
          "max_match": dict(_prod(ds, 17), max_match=True, bases_matching=10.0)}[flags]
    _compare(ds, kw, f"C1 {flags}")


def test_c2_full_index():
    from tools.synth import Dataset
    ds = Dataset("C2", seed=42, threads=16, n_pb=3000)
    st = _compare(ds, _prod(ds, 17), "C2 production")
    # the workload exercises the repeat filters: kept < looked-up k-mers, long hit lists
    assert st["n_kept"] < st["n_kmers"] and st["n_hits"] > 50 * st["n_kept"]


def test_c2_full_index_max_match():
    from tools.synth import Dataset
    ds = Dataset("C2", seed=42, threads=16, n_pb=500)
    _compare(ds, dict(_prod(ds, 17), max_match=True, bases_matching=10.0), "C2 max_match")


def test_c3_full_index():
    from tools.synth import Dataset
    ds = Dataset("C3", seed=42, threads=16, n_pb=1500)
    _compare(ds, _prod(ds, 21), "C3 production")


def test_c4_repeat_model_oracle():
    """C4's repeat model (2% of the genome in 5-50-copy repeats, 15-kb-N50 reads) at a size the
    oracle holds (tools/synth.py "C4r": 16 Mbp genome, 800k super-reads at C4's ~50x coverage,
    1000 reads), byte for byte against the oracle with the production flags and with
    --max-count 2000: the 99% threshold and the max-count filter (coarse_aligner.cc:104-125) on
    multi-copy repeats and long reads, beyond the property checks of the C4/C5 tests."""
    from oracle.oracle import OracleIndex, params
    from pacbio_amd import pbgpu
    from tools.synth import Dataset
    ds = Dataset("C4r", seed=42, threads=16)
    names, seqs = ds.sr_names(), ds.sr_seqs()
    pnames, pseqs = ds.pb_names(), ds.pb_seqs()
    gix = pbgpu.Index.from_records(names, seqs, 17)
    oix = OracleIndex.from_records(names, seqs, 17, threads=16)
    outs = {}
    for mc in (5000, 2000):
        kw = dict(_prod(ds, 17), max_count=mc)
        al = pbgpu.Aligner(gix, **kw)
        rd = al.upload(pseqs, names=pnames)
        al.align_resident(rd)
        got = al.format_device(rd)
        rd.close()
        al.close()
        exp = oix.align_format(params(**kw), pnames, pseqs, threads=16)
        assert exp.count("\n") > 100 * len(pseqs), f"C4r max_count {mc}: too few records"
        assert_same_coords(got, exp, f"C4r max_count {mc}")
        outs[mc] = exp
    oix.close()
    gix.close()
    # the repeats reach the limit: --max-count 2000 drops k-mers that 5000 keeps
    assert outs[2000] != outs[5000] and outs[2000].count("\n") < outs[5000].count("\n")

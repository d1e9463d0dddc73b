"""Index build at scale.

* The partitioned build (the path an index takes when its sort buffers do not
  fit the device beside it) gives the same index as the one-pass build: same
  counts, same coords, coarse and -F, on the small preset with P forced.
* C4 (BASELINE configs[3]): the full 10M-super-read index (~10 Gbp, built in
  partitions on one MI355X) with a read subsample.  The oracle cannot hold an
  index this size, so the checks are size-independent properties: per-read
  (rs, re, ql) order, record invariants against the inputs, and identical text
  from two aligners cutting the batch into different sub-batches."""
import os

import pytest

from tests._compare import assert_read_order, assert_same_coords

pytestmark = pytest.mark.gpu


def _with_parts(P, fn):
    old = os.environ.get("PBGPU_BUILD_PARTS")
    os.environ["PBGPU_BUILD_PARTS"] = str(P)
    try:
        return fn()
    finally:
        if old is None:
            del os.environ["PBGPU_BUILD_PARTS"]
        else:
            os.environ["PBGPU_BUILD_PARTS"] = old


@pytest.mark.parametrize("P", [3, 8])
def test_partitioned_build_same_index(P):
    from pacbio_amd import pbgpu
    from tools.synth import Dataset
    ds = Dataset("small", seed=7)
    names, seqs = ds.sr_names(), ds.sr_seqs()
    pn, ps = ds.pb_names(), ds.pb_seqs()
    one = pbgpu.Index.from_records(names, seqs, 17, fine_k=13)
    part = _with_parts(P, lambda: pbgpu.Index.from_records(names, seqs, 17, fine_k=13))
    a, b = one.info(), part.info()
    for f in ("n_kmers", "n_occurrences", "table_buckets"):
        assert a[f] == b[f], f
    for kw in (dict(forward=True, unitigs_k=31, unitig_lengths=ds.unitig_lengths, bases_matching=15.0),
               dict(fine_k=13, forward=True), dict(max_match=True)):
        outs = []
        for ix in (one, part):
            al = pbgpu.Aligner(ix, k=17, **kw)
            rd = al.upload(ps, names=pn)
            al.align_resident(rd)
            outs.append(al.format_device(rd))
            rd.close()
            al.close()
        assert outs[0].count("\n") > 100
        assert outs[0] == outs[1]
    one.close()
    part.close()


def _check_invariants(text, k, sr_len, read_len):
    n = 0
    for line in text.splitlines():
        if line.startswith(">"):
            _, name = line[1:].split(" ", 1)
            rl = read_len[name]
            continue
        t = line.split()
        rs, re, qs, qe, nb, pc, sc, pcov, scov, rlen, ql = map(int, t[:11])
        stretch = float(t[11])
        qname = t[14]
        assert rlen == rl
        assert ql == sr_len[qname], line
        assert 1 <= rs <= re <= rl, line
        assert 1 <= qs <= qe <= ql, line
        assert nb >= 1 and pc < nb and sc < nb, line
        assert k <= pcov <= re - rs + 1 and scov >= k, line
        assert stretch > 0, line
        info = t[15:]
        assert len(info) == 0 or len(info) == 2 * (qname.count("_") + 1) - 1, line
        n += 1
    return n


def test_c4_full_index_properties():
    from pacbio_amd import pbgpu
    from tools.synth import Dataset
    ds = Dataset("C4", seed=42, threads=16, n_pb=1500)
    gix = pbgpu.Index.from_pointers(*ds.sr_pointers(), k=17)
    info = gix.info()
    assert info["n_sr"] == 10_000_000 and info["text_len"] > 9e9
    pn, ps = ds.pb_names(), ds.pb_seqs()
    kw = dict(k=17, forward=True, unitigs_k=31, unitig_lengths=ds.unitig_lengths, bases_matching=15.0,
              max_count=5000, stretch_cap=10000.0)
    texts = []
    for budget in (None, 20_000_000):
        al = pbgpu.Aligner(gix, **kw)
        if budget:
            al.set_hit_budget(budget)
        rd = al.upload(ps, names=pn)
        al.align_resident(rd)
        texts.append(al.format_device(rd))
        st = al.stats()
        rd.close()
        al.close()
    assert texts[0] == texts[1]
    text = texts[0]
    assert_read_order(text, "C4")
    used = {line.split()[14] for line in text.splitlines() if not line.startswith(">")}
    sr_len = {}
    for i in range(info["n_sr"]):  # lengths of the super-reads the records name
        nm = gix.sr_name(i)
        if nm in used:
            sr_len[nm] = pbgpu.lib().pbgpu_index_sr_len(gix.h, i)
        nb = gix.sr_name(i, bwd=True)
        if nb in used:
            sr_len[nb] = pbgpu.lib().pbgpu_index_sr_len(gix.h, i)
    read_len = {(n.decode() if isinstance(n, bytes) else n): len(s) for n, s in zip(pn, ps)}
    n = _check_invariants(text, 17, sr_len, read_len)
    assert n > 100 * len(ps), "C4 subsample produced too few records"
    assert st["n_kept"] < st["n_kmers"]
    gix.close()

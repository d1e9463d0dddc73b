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


def _check_invariants(text, k, read_len):
    """Per-record invariants of the coords text against the read lengths."""
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
        assert 1 <= rs <= re <= rl, line
        assert 1 <= qs <= qe <= ql, line
        assert nb >= 1 and pc < nb and sc < nb, line
        assert k <= pcov <= re - rs + 1 and scov >= k, line
        assert stretch > 0, line
        info = t[15:]
        assert len(info) == 0 or len(info) == 2 * (qname.count("_") + 1) - 1, line
        n += 1
    return n


def check_records(co, sr_len, read_len):
    """Vectorised invariants of downloaded records: each record's ql is its
    super-read's length (by global sr_index) and its coordinates lie inside
    both sequences (the read being the one whose offset range holds it)."""
    import numpy as np
    r = co.records
    assert len(r) == int(co.read_offsets[-1])
    assert np.all(r["sr_index"] < len(sr_len))
    assert np.array_equal(r["ql"].astype(np.int64), sr_len[r["sr_index"]].astype(np.int64))
    rid = np.repeat(np.arange(co.n_reads), np.diff(co.read_offsets.astype(np.int64)))
    rl = np.asarray(read_len, np.int64)[rid]
    assert np.all((1 <= r["rs"]) & (r["rs"] <= r["re"]) & (r["re"] <= rl))
    assert np.all((1 <= r["qs"]) & (r["qs"] <= r["qe"]) & (r["qe"].astype(np.int64) <= r["ql"].astype(np.int64)))
    return len(r)


C4_KW = dict(k=17, forward=True, unitigs_k=31, bases_matching=15.0, max_count=5000, stretch_cap=10000.0)


@pytest.fixture(scope="module")
def c4():
    """C4 with a 1500-read sample; the whole index's text (one sub-batch and a
    20M-hit budget), its records, and the super-read lengths.  The whole index
    is freed before the sharded test runs."""
    import numpy as np
    from pacbio_amd import pbgpu
    from tools.synth import Dataset
    ds = Dataset("C4", seed=42, threads=16, n_pb=1500)
    gix = pbgpu.Index.from_pointers(*ds.sr_pointers(), k=17)
    info = gix.info()
    pn, ps = ds.pb_names(), ds.pb_seqs()
    texts, recs = [], None
    # --max-count 2000: below the repeats' whole-index counts (up to ~4400), so the
    # count filter and the 99% threshold act on k-mers no single C4 shard saturates
    al = pbgpu.Aligner(gix, unitig_lengths=ds.unitig_lengths, **dict(C4_KW, max_count=2000))
    rd = al.upload(ps, names=pn)
    al.align_resident(rd)
    text_mc = al.format_device(rd)
    rd.close()
    al.close()
    for budget in (None, 20_000_000):
        al = pbgpu.Aligner(gix, unitig_lengths=ds.unitig_lengths, **C4_KW)
        if budget:
            al.set_hit_budget(budget)
        rd = al.upload(ps, names=pn)
        al.align_resident(rd)
        texts.append(al.format_device(rd))
        if recs is None:
            recs = al.download()
        st = al.stats()
        rd.close()
        al.close()
    gix.close()
    sr_len = np.diff(np.ctypeslib.as_array(ds.sr.off, shape=(ds.sr.n + 1,)).astype(np.int64))
    yield dict(ds=ds, info=info, texts=texts, text_mc=text_mc, recs=recs, stats=st, pn=pn, ps=ps, sr_len=sr_len)
    ds.close()


def test_c4_full_index_properties(c4):
    info, texts = c4["info"], c4["texts"]
    assert info["n_sr"] == 10_000_000 and info["text_len"] > 9e9
    assert texts[0] == texts[1]
    text = texts[0]
    assert_read_order(text, "C4")
    pn, ps = c4["pn"], c4["ps"]
    read_len = {(n.decode() if isinstance(n, bytes) else n): len(s) for n, s in zip(pn, ps)}
    n = _check_invariants(text, 17, read_len)
    assert n > 100 * len(ps), "C4 subsample produced too few records"
    assert check_records(c4["recs"], c4["sr_len"], [len(s) for s in ps]) == n
    st = c4["stats"]
    assert st["n_kept"] < st["n_kmers"]


@pytest.mark.parametrize("max_count", [5000, 2000])
def test_c4_sharded_matches_whole_index(c4, max_count):
    """The sharded mode at real repeat content: the same 1500 C4
    reads through S = 4 shards of the C4 index -- per-shard saturated counts
    summed, shard-local chains, per-read merge -- give text byte-identical to
    the whole index on the same GPU (coarse_aligner.cc:108-125's count filter and
    99% threshold over the summed counts), with the production --max-count and
    with one the repeats exceed."""
    import numpy as np
    from pacbio_amd import pbgpu
    ds, pn, ps = c4["ds"], c4["pn"], c4["ps"]
    kw = dict(C4_KW, max_count=max_count)
    S = 4
    ptrs = ds.sr_pointers()
    nb = sum(len(s) for s in ps)
    shards = []
    for s in range(S):
        ix = pbgpu.Index.from_pointers(*ptrs, k=17, shard=s, n_shards=S)
        al = pbgpu.Aligner(ix, unitig_lengths=ds.unitig_lengths, **kw)
        rd = al.upload(ps, names=pn)
        al.shard_counts(rd)
        shards.append((ix, al, rd))
    info = [ix.info() for ix, _, _ in shards]
    assert info[0]["sr_begin"] == 0 and info[-1]["sr_end"] == 10_000_000
    assert all(info[i]["sr_end"] == info[i + 1]["sr_begin"] for i in range(S - 1))
    total = np.zeros(nb, np.uint64)
    per = []
    for _, al, _ in shards:
        c = al.counts_download(nb)
        per.append(c)
        total += c
    assert total.max() > 1000, "no repeat content in the sample"
    if max_count == 2000:
        # k-mers over the limit only once the shards' counts are summed
        over = total > max_count
        assert over.any() and (over & (np.max(per, axis=0) < max_count)).any()
    parts = []
    for _, al, rd in shards:
        al.counts_upload(total.astype(np.uint32))
        al.align_resident_shard(rd)
        parts.append(al.download())
    merged = pbgpu.merge_coords(parts)
    got = merged.format(shards[0][0], pn, [len(s) for s in ps])
    for ix, al, rd in shards:
        rd.close()
        al.close()
        ix.close()
    assert got == (c4["texts"][0] if max_count == 5000 else c4["text_mc"])
    assert got.count("\n") > 100 * len(ps)

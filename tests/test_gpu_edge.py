"""GPU edge cases, each checked byte-for-byte against the CPU restatement
(oracle/): degenerate reads, empty batches, determinism, the resident API,
sub-batching with a tiny hit budget, reads that touch more super-reads than
the LDS group tables hold (4096/8192-slot tiers and HBM tables), the
max-count threshold on a repetitive genome, k = 31, and -0 output."""
import pytest

from tests._compare import assert_same_coords

pytestmark = pytest.mark.gpu


def _oracle(ds_names, ds_seqs, pnames, pseqs, k=17, ul=None, zero_match=False, **cfg):
    from oracle.oracle import OracleIndex, params
    oix = OracleIndex.from_records(ds_names, ds_seqs, k)
    try:
        return oix.align_format(params(k=k, unitig_lengths=ul, **cfg), pnames, pseqs, threads=8,
                                zero_match=zero_match)
    finally:
        oix.close()


def _gpu(ds_names, ds_seqs, pnames, pseqs, k=17, ul=None, zero_match=False, budget=None, **cfg):
    from pacbio_amd import pbgpu
    gix = pbgpu.Index.from_records(ds_names, ds_seqs, k)
    al = pbgpu.Aligner(gix, k=k, unitig_lengths=ul, **cfg)
    if budget:
        al.set_hit_budget(budget)
    co = al.align(pseqs)
    txt = co.format(gix, pnames, [len(s) for s in pseqs], zero_match=zero_match)
    st = al.stats()
    return txt, st


@pytest.fixture(scope="module")
def small():
    from tools.synth import Dataset
    return Dataset("small", seed=11)


@pytest.fixture(scope="module")
def dense():
    # 60 kb genome under ~330x of 1 kb super-reads; 40 kb reads touch >10k super-reads each
    from tools.synth import Dataset
    return Dataset("small", seed=5, genome_len=60_000, n_sr=20_000, n_pb=3, pb_len_mean=40_000, pb_len_sigma=0.0,
                   err_ins=0.02, err_del=0.02, err_sub=0.01)


def test_degenerate_reads(small):
    real = small.pb_seqs()[:3]
    r0 = real[0]
    pseqs = [b"", b"ACG", b"N" * 5000, r0.lower(), r0[:3000] + b"N" * 40 + r0[3040:], r0.replace(b"A", b"R", 50),
             b"ACGT" * 2000, b"A" * 3000, r0[:16], r0[:17], real[1], real[2],
             # bytes that share a 2-bit code or a case bit with a base must still reset the k-mer
             r0.replace(b"C", b"\xc3", 30).replace(b"G", b"g", 40).replace(b"T", b"U", 25).replace(b"A", b"\x01", 25)]
    pnames = [f"edge{i}" for i in range(len(pseqs))]
    names, seqs = small.sr_names(), small.sr_seqs()
    for zm in (False, True):
        exp = _oracle(names, seqs, pnames, pseqs, zero_match=zm)
        got, _ = _gpu(names, seqs, pnames, pseqs, zero_match=zm)
        assert_same_coords(got, exp, f"degenerate zero_match={zm}")


def test_empty_batch(small):
    from pacbio_amd import pbgpu
    gix = pbgpu.Index.from_records(small.sr_names(), small.sr_seqs(), 17)
    al = pbgpu.Aligner(gix, k=17)
    co = al.align([])
    assert co.n_reads == 0 and co.n_records == 0
    co2 = al.align([b"", b"NNNN"])
    assert co2.n_records == 0


def test_determinism_and_resident_api(small):
    from pacbio_amd import pbgpu
    names, seqs = small.sr_names(), small.sr_seqs()
    pnames, pseqs = small.pb_names(), small.pb_seqs()
    gix = pbgpu.Index.from_records(names, seqs, 17)
    al = pbgpu.Aligner(gix, k=17, forward=True, unitigs_k=31, unitig_lengths=small.unitig_lengths,
                       bases_matching=15.0)
    lens = [len(s) for s in pseqs]
    a = al.align(pseqs).format(gix, pnames, lens)
    b = al.align(pseqs).format(gix, pnames, lens)
    assert a == b
    rr = al.upload(pseqs)
    for _ in range(2):
        al.align_resident(rr)
        c = al.download().format(gix, pnames, lens)
        assert c == a
    rr.close()


@pytest.mark.parametrize("budget", [1, 5000, 200_000])
def test_sub_batches(small, budget):
    names, seqs = small.sr_names(), small.sr_seqs()
    pnames, pseqs = small.pb_names(), small.pb_seqs()
    cfg = dict(forward=True, unitigs_k=31, bases_matching=15.0, max_match=True)
    exp = _oracle(names, seqs, pnames, pseqs, ul=small.unitig_lengths, **cfg)
    got, _ = _gpu(names, seqs, pnames, pseqs, ul=small.unitig_lengths, budget=budget, **cfg)
    assert_same_coords(got, exp, f"budget={budget}")


# ~330x coverage: max_count 400 filters part of the k-mers and moves the 99% threshold
@pytest.mark.parametrize("cfg", [dict(), dict(max_count=400), dict(forward=True, max_match=True)],
                         ids=["default", "maxcount400", "fwd_maxmatch"])
def test_dense_group_overflow(dense, cfg):
    names, seqs = dense.sr_names(), dense.sr_seqs()
    pnames, pseqs = dense.pb_names(), dense.pb_seqs()
    exp = _oracle(names, seqs, pnames, pseqs, **cfg)
    got, st = _gpu(names, seqs, pnames, pseqs, **cfg)
    if not cfg:
        assert st["n_chains"] > 3 * 8192, "reads must touch more super-reads than the largest LDS table"
        from tests._compare import split_reads
        # k_rec_sort stages keys in LDS up to 2048 records per read, in HBM above
        assert max(len(v) for v in split_reads(got)[1].values()) > 2048
    assert_same_coords(got, exp, f"dense {cfg}")


@pytest.mark.parametrize("refine", ["1", "0"], ids=["refine", "hbm"])
@pytest.mark.parametrize("data", ["dense", "small"])
def test_group_all_overflow(data, refine, dense, small, monkeypatch):
    """Every read predicted to fit the smallest (2048-slot) table: reads touching
    more super-reads abandon it mid k-mer group and go again in the 8192-slot
    LDS tier, split into hash partitions by their growth estimate (the default:
    an item that overflows again splits again, the partitions already placed
    keep their lists) or in HBM tables (PBGPU_GROUP_REFINE=0); a full table must
    never trap a thread."""
    ds = dense if data == "dense" else small
    monkeypatch.setenv("PBGPU_GROUP_PRED_SCALE", "0")
    monkeypatch.setenv("PBGPU_GROUP_REFINE", refine)
    names, seqs = ds.sr_names(), ds.sr_seqs()
    pnames, pseqs = ds.pb_names(), ds.pb_seqs()
    exp = _oracle(names, seqs, pnames, pseqs, ul=ds.unitig_lengths, forward=True, unitigs_k=31)
    got, st = _gpu(names, seqs, pnames, pseqs, ul=ds.unitig_lengths, forward=True, unitigs_k=31)
    assert_same_coords(got, exp, f"all-overflow {data} refine={refine}")
    if data == "dense":
        if refine == "1":
            assert st["group_refines"] > 0 and st["group_hbm_reads"] == 0, st
        else:
            assert st["group_refines"] == 0 and st["group_hbm_reads"] > 0, st


@pytest.mark.parametrize("first_p", ["2", "4"])
@pytest.mark.parametrize("data", ["dense", "small"])
def test_group_first_round_items_overflow(data, first_p, dense, small, monkeypatch):
    """Every read starts as P hash-partition items in the smallest table
    (PBGPU_GROUP_FIRST_P): on the dense reads every item overflows, so the first
    round's overflow list must hold one entry per item -- P per read -- not one per
    read (the list was sized by reads and k_group wrote past it).  One call
    per read too, so a one-read batch overflows P items at once."""
    ds = dense if data == "dense" else small
    monkeypatch.setenv("PBGPU_GROUP_FIRST_P", first_p)
    names, seqs = ds.sr_names(), ds.sr_seqs()
    pnames, pseqs = ds.pb_names(), ds.pb_seqs()
    exp = _oracle(names, seqs, pnames, pseqs, ul=ds.unitig_lengths, forward=True, unitigs_k=31)
    got, st = _gpu(names, seqs, pnames, pseqs, ul=ds.unitig_lengths, forward=True, unitigs_k=31)
    assert_same_coords(got, exp, f"first-round items {data} P={first_p}")
    if data == "dense":
        # more items overflowed than there are reads: the case the reads-sized list missed
        assert st["group_overflow_items"] > len(pseqs), st
        for i in range(len(pseqs)):
            one, st1 = _gpu(names, seqs, pnames[i:i + 1], pseqs[i:i + 1], ul=ds.unitig_lengths, forward=True,
                            unitigs_k=31)
            e1 = _oracle(names, seqs, pnames[i:i + 1], pseqs[i:i + 1], ul=ds.unitig_lengths, forward=True,
                         unitigs_k=31)
            assert_same_coords(one, e1, f"first-round items, read {i} alone, P={first_p}")
            assert st1["group_overflow_items"] >= 2, st1


@pytest.mark.parametrize("data,scale", [("dense", "8"), ("dense", "200"), ("small", "200"), ("small", "2000")])
def test_group_bucketed_reads(data, scale, dense, small, monkeypatch):
    """Reads predicted past the 8192-slot table in P >= 2 hash partitions are enumerated
    once into P buckets (a split item) whose partition items stream them (round 6).
    PBGPU_GROUP_PRED_SCALE inflates the prediction so that most reads take that path,
    with P up to hundreds (200): the same bytes as the oracle, and as the round-5 path
    where every partition item enumerates the read (PBGPU_GROUP_BUCKETS=0)."""
    ds = dense if data == "dense" else small
    monkeypatch.setenv("PBGPU_GROUP_PRED_SCALE", scale)
    names, seqs = ds.sr_names(), ds.sr_seqs()
    pnames, pseqs = ds.pb_names(), ds.pb_seqs()
    cfg = dict(ul=ds.unitig_lengths, forward=True, unitigs_k=31)
    exp = _oracle(names, seqs, pnames, pseqs, **cfg)
    got, st = _gpu(names, seqs, pnames, pseqs, **cfg)
    assert st["group_bucketed_reads"] >= len(pseqs) // 2, st
    assert_same_coords(got, exp, f"bucketed {data} scale={scale}")
    monkeypatch.setenv("PBGPU_GROUP_BUCKETS", "0")
    old, st0 = _gpu(names, seqs, pnames, pseqs, **cfg)
    assert st0["group_bucketed_reads"] == 0 and old == got


@pytest.mark.parametrize("extra", [dict(max_match=True, bases_matching=10.0), dict(forward=False, ul=None, unitigs_k=0),
                                   dict(window_size=3)])
def test_group_bucketed_reads_modes(extra, dense, monkeypatch):
    """The bucketed grouping under the modes that read the lists differently downstream:
    --max-match (discard rounds over the lists), both strands (-f off), a window of 3 (the
    generic LIS): oracle bytes, and those of the round-5 path (PBGPU_GROUP_BUCKETS=0)."""
    monkeypatch.setenv("PBGPU_GROUP_PRED_SCALE", "200")
    names, seqs = dense.sr_names(), dense.sr_seqs()
    pnames, pseqs = dense.pb_names(), dense.pb_seqs()
    cfg = dict(dict(ul=dense.unitig_lengths, forward=True, unitigs_k=31), **extra)
    exp = _oracle(names, seqs, pnames, pseqs, **cfg)
    got, st = _gpu(names, seqs, pnames, pseqs, **cfg)
    assert st["group_bucketed_reads"] >= len(pseqs) // 2, st
    assert_same_coords(got, exp, f"bucketed {extra}")
    monkeypatch.setenv("PBGPU_GROUP_BUCKETS", "0")
    old, st0 = _gpu(names, seqs, pnames, pseqs, **cfg)
    assert st0["group_bucketed_reads"] == 0 and old == got


def test_repeats_threshold():
    from tools.synth import Dataset
    ds = Dataset("small", seed=3, repeat_frac=0.2, n_pb=30)
    names, seqs = ds.sr_names(), ds.sr_seqs()
    pnames, pseqs = ds.pb_names(), ds.pb_seqs()
    for mc in (30, 5000):
        exp = _oracle(names, seqs, pnames, pseqs, max_count=mc)
        got, _ = _gpu(names, seqs, pnames, pseqs, max_count=mc)
        assert_same_coords(got, exp, f"repeats max_count={mc}")


def test_k31(small):
    names, seqs = small.sr_names(), small.sr_seqs()
    pnames, pseqs = small.pb_names(), small.pb_seqs()
    exp = _oracle(names, seqs, pnames, pseqs, k=31)
    got, _ = _gpu(names, seqs, pnames, pseqs, k=31)
    assert exp.count("\n") > 5
    assert_same_coords(got, exp, "k31")


@pytest.fixture(scope="module")
def long_strands():
    # 44 kb mean (up to 100 kb) super-reads, 90 kb low-error reads: strands of 4k-76k hits
    # exercise k_strand_order, the lane-per-strand k_lis and its 32-bit nodes (> 65535 hits)
    from tools.synth import Dataset
    return Dataset("small", seed=21, genome_len=400_000, n_sr=300, unitig_mean=4000, unitig_min=1000,
                   sr_max_unitigs=24, n_pb=6, pb_len_mean=90_000, pb_len_sigma=0.0, err_ins=0.003, err_del=0.003,
                   err_sub=0.002, n_run_rate=0.0)


@pytest.mark.parametrize("cfg", [dict(), dict(forward=True, max_match=True)], ids=["default", "fwd_maxmatch"])
def test_long_strands(long_strands, cfg):
    ds = long_strands
    names, seqs = ds.sr_names(), ds.sr_seqs()
    pnames, pseqs = ds.pb_names(), ds.pb_seqs()
    exp = _oracle(names, seqs, pnames, pseqs, **cfg)
    nb = [int(line.split()[4]) for line in exp.splitlines() if not line.startswith(">")]
    assert max(nb) > 65535 and sum(1 for x in nb if 4095 < x <= 65535) > 10
    got, _ = _gpu(names, seqs, pnames, pseqs, **cfg)
    assert_same_coords(got, exp, f"long strands {cfg}")


def test_fit_reciprocal_exact():
    """The fit divides by the point count n four times a point (least_square_2d.hpp:47-67);
    the device takes RN(1/n) with a shortened sequence (recip_int): it must equal the
    correctly rounded 1.0 / n for every n a strand can reach at C1-C5 scale (< 2^24)."""
    from pacbio_amd import pbgpu
    assert pbgpu.check_reciprocal(0, 1 << 24) == 0


@pytest.mark.parametrize("chunk", ["30000", "200000"])
def test_chunked_resident_batch(small, chunk, monkeypatch):
    """A resident batch larger than the device holds is aligned in chunks of reads
    (seeding and sub-batches per chunk, records appended; round 5, so that one
    pbgpu_align_resident call of C3's 3.6 Gbases no longer runs out of HBM).
    PBGPU_CHUNK_BASES forces small chunks: the same bytes as the oracle."""
    monkeypatch.setenv("PBGPU_CHUNK_BASES", chunk)
    names, seqs = small.sr_names(), small.sr_seqs()
    pnames, pseqs = small.pb_names(), small.pb_seqs()
    cfg = dict(forward=True, unitigs_k=31, bases_matching=15.0, max_match=True)
    exp = _oracle(names, seqs, pnames, pseqs, ul=small.unitig_lengths, **cfg)
    got, st = _gpu(names, seqs, pnames, pseqs, ul=small.unitig_lengths, budget=50_000, **cfg)
    assert st["kernel_launches"]["k_seed"] >= 2, st["kernel_launches"]  # one seeding per chunk
    assert_same_coords(got, exp, f"chunk={chunk}")

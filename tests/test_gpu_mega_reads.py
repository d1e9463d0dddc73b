"""create_mega_reads on the GPU (pacbio_amd/bin/create_mega_reads: pbgpu_run's
records consumer -> overlap_graph.cpp) against the CPU restatements: records
from oracle/pb_oracle.c, mega-reads from oracle/mega_reads.py.  Byte-identical
output for the reference's tests/mega_reads_output inputs with its Tupfile's
create_mega_reads flags, and for a synthetic dataset over the tiling / trim /
-b / -u options; multi-batch and two-index ("--devices 0,0") runs and gzip
input give the same bytes; --dot writes one graph per read with mega-reads.

Parity is pinned to the restatements only (see tests/test_mega_reads.py)."""
import gzip
import os
import shutil
import subprocess
import tempfile

import pytest

from oracle import mega_reads as MR
from oracle import oracle as O
from tests.test_mega_reads import MRO, read_fasta, read_ul, write_unitig_sequences

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CMR = os.path.join(ROOT, "pacbio_amd", "bin", "create_mega_reads")
BIG = str(1 << 30)  # --max-count: the Tupfile's 0 means INT_MAX upstream (undefined behaviour there)


def _run(args, timeout=120):
    r = subprocess.run([CMR, *args], capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr
    return r


def _expect(reads, ul, k, useqs=None, **opt):
    o = dict(play=1.3, errors=3.0, bases=False, density=0.029, min_len=100.0, tiling="greedy", trim="none")
    o.update(opt)
    return "".join(MR.mega_reads(n, recs, ul, k, useqs=useqs, **o) for n, recs in reads)


@pytest.fixture(scope="module")
def mro():
    names, seqs = read_fasta(os.path.join(MRO, "sr.fa"))
    ul = read_ul(os.path.join(MRO, "kUnitigLengths.txt"))
    oix = O.OracleIndex.from_records(names, seqs, 15)
    p = O.params(k=15, forward=True, max_count=1 << 30, bases_matching=10.0, stretch_cap=400.0, unitigs_k=70,
                 unitig_lengths=ul)
    pn, ps = read_fasta(os.path.join(MRO, "pb.fa"))
    reads = [(n, MR.records_of(oix, p, s)) for n, s in zip(pn, ps)]
    oix.close()
    return reads, ul


@pytest.mark.parametrize("threads", ["1", "4"])
def test_reference_inputs_tupfile_flags(mro, tmp_path, threads):
    """tests/mega_reads_output/Tupfile:16 (create_mega_reads -s 20k -m 15 -B 10 -L 0 -k 70
    --stretch-cap 400 --dot ...)"""
    reads, ul = mro
    out, dot = str(tmp_path / "crm_mega_reads"), str(tmp_path / "crm_mega_reads.dot")
    _run(["-s", "20k", "-m", "15", "-B", "10", "-L", "0", "--max-count", BIG, "-l",
          os.path.join(MRO, "kUnitigLengths.txt"), "-o", out, "-k", "70", "--stretch-cap", "400", "--dot", dot,
          "-t", threads, "-r", os.path.join(MRO, "sr.fa"), "-p", os.path.join(MRO, "pb.fa")])
    want = _expect(reads, ul, 70, min_len=0.0)
    assert want.count(">") == 2
    assert open(out).read() == want
    d = open(dot).read()
    assert d.count("digraph") == 2 and d.count("{") == d.count("}") and "[color=\"red\"]" in d


@pytest.fixture(scope="module")
def synth():
    from tools.synth import Dataset
    d = tempfile.mkdtemp(prefix="pbgpu_cmr_")
    ds = Dataset("small", seed=11)
    ds.write(d)
    ul = [int(x) for x in ds.unitig_lengths]
    names, seqs = [n.decode() for n in ds.sr_names()], ds.sr_seqs()
    pn, ps = [n.decode() for n in ds.pb_names()], ds.pb_seqs()
    ds.close()
    oix = O.OracleIndex.from_records(names, seqs, 17)
    cache = {}

    def reads_for(**pk):
        key = tuple((k, tuple(v) if isinstance(v, list) else v) for k, v in sorted(pk.items()))
        if pk.get("fine_k") and "fine" not in cache:
            oix.build_fine(pk["fine_k"])
            cache["fine"] = pk["fine_k"]
        if key not in cache:
            p = O.params(k=17, forward=True, unitigs_k=31, unitig_lengths=pk.pop("ul", ul), **pk)
            cache[key] = [(n, MR.records_of(oix, p, s)) for n, s in zip(pn, ps)]
        return cache[key]
    yield d, ul, reads_for
    oix.close()
    shutil.rmtree(d, ignore_errors=True)


CASES = [
    ([], {}, {}),
    (["-T", "maximal", "-L", "0"], {}, dict(tiling="maximal", min_len=0.0)),
    (["-T", "weighted", "--trim", "match"], {}, dict(tiling="weighted", trim="match")),
    (["-T", "none", "-b", "-d", "0.05"], {}, dict(tiling="none", bases=True, density=0.05)),
    # --trim branch trims nothing: create_mega_reads.cc:47-49 switches trimming on for "match" only
    (["-O", "1.5", "-e", "2", "--trim", "branch", "-L", "50"], {}, dict(play=1.5, errors=2.0, trim="none",
                                                                         min_len=50.0)),
    (["--max-match", "-B", "10", "--stretch-cap", "500"], dict(max_match=True, bases_matching=10.0, stretch_cap=500.0),
     {}),
    # -F: the records are the fine aligner's (create_mega_reads.cc:64-68)
    (["-F", "13", "-L", "0"], dict(fine_k=13), dict(min_len=0.0)),
]


@pytest.mark.parametrize("cli,aopt,gopt", CASES, ids=[" ".join(c[0]) or "defaults" for c in CASES])
def test_synthetic_options(synth, tmp_path, cli, aopt, gopt):
    d, ul, reads_for = synth
    out = str(tmp_path / "mr")
    _run(["-s", "1M", "-m", "17", "-k", "31", "-l", os.path.join(d, "ul.txt"), "-t", "4", "-o", out, *cli,
          "-r", os.path.join(d, "sr.fa"), "-p", os.path.join(d, "pb.fa")])
    want = _expect(reads_for(**aopt), ul, 31, **gopt)
    assert want.count(">") >= 10
    assert open(out).read() == want
    if "branch" in cli:  # the case must tell "branch" (no trim) from "match"
        assert _expect(reads_for(**aopt), ul, 31, **dict(gopt, trim="match")) != want


def test_synthetic_unitig_sequences(synth, tmp_path):
    """-u: unitig lengths from the sequences, each mega-read followed by its sequence"""
    d, ul, reads_for = synth
    up = str(tmp_path / "useqs.fa")
    useqs = write_unitig_sequences(up, ul)
    uls = [len(s) for s in useqs]
    out = str(tmp_path / "mr")
    _run(["-s", "1M", "-m", "17", "-k", "31", "-u", up, "-o", out, "-r", os.path.join(d, "sr.fa"), "-p",
          os.path.join(d, "pb.fa")])
    want = _expect(reads_for(ul=uls), uls, 31, useqs=useqs)
    assert open(out).read() == want


def test_batches_devices_gzip_identical(synth, tmp_path):
    """many small batches over two aligners on two indexes of device 0, gzip input: same bytes"""
    d, ul, _ = synth
    base = ["-s", "1M", "-m", "17", "-k", "31", "-l", os.path.join(d, "ul.txt"), "-T", "maximal",
            "-r", os.path.join(d, "sr.fa")]
    a, b = str(tmp_path / "a"), str(tmp_path / "b")
    _run([*base, "-o", a, "-p", os.path.join(d, "pb.fa")])
    gz = str(tmp_path / "pb.fa.gz")
    with open(os.path.join(d, "pb.fa"), "rb") as f, gzip.open(gz, "wb") as g:
        g.write(f.read())
    _run([*base, "-o", b, "-p", gz, "--devices", "0,0", "--streams", "2", "--batch-bases", "20k", "-t", "3"])
    ta = open(a).read()
    assert ta.count(">") >= 10 and open(b).read() == ta


def test_reads_without_records_and_empty_input(synth, tmp_path):
    """reads with no alignment print nothing (print_mega_reads prints only reads with
    mega-reads, overlap_graph.hpp:253-262); an empty PacBio file gives an empty output"""
    import random
    d, _, _ = synth
    rng = random.Random(3)
    pb = tmp_path / "pb.fa"
    pb.write_text(">empty\n\n>random\n" + "".join(rng.choice("ACGT") for _ in range(3000)) + "\n>short\nACGT\n")
    out = str(tmp_path / "mr")
    base = ["-s", "1M", "-m", "17", "-k", "31", "-l", os.path.join(d, "ul.txt"), "-r", os.path.join(d, "sr.fa")]
    _run([*base, "-o", out, "-p", str(pb)])
    assert open(out).read() == ""
    empty = tmp_path / "none.fa"
    empty.write_text("")
    _run([*base, "-o", out, "-p", str(empty)])
    assert open(out).read() == ""


def test_graph_error_exits_cleanly(synth, tmp_path):
    """a super-read naming a unitig past the -u sequences (super_read_name.cc:133, .at()
    throws upstream): the error of a graph thread ends the run with a message and exit
    status 1, not std::terminate"""
    d, _, _ = synth
    up = tmp_path / "few.fa"
    up.write_text(">0\n" + "ACGT" * 20 + "\n>1\n" + "TTGCA" * 20 + "\n")
    r = subprocess.run([CMR, "-s", "1M", "-m", "17", "-k", "31", "-u", str(up), "-t", "4", "-o",
                        str(tmp_path / "mr"), "-r", os.path.join(d, "sr.fa"), "-p", os.path.join(d, "pb.fa")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 1, (r.returncode, r.stderr[-500:])
    assert "unitig id beyond the unitig sequences" in r.stderr


@pytest.mark.parametrize("cli", [c[0] for c in CASES], ids=[" ".join(c[0]) or "defaults" for c in CASES])
def test_device_graph_equals_host_graph(synth, tmp_path, cli):
    """the traversal on the GPU (default) against the host's (--host-graph), and with
    PBGPU_GRAPH_NMAX=40 (reads of more than 40 records left to the host): same bytes"""
    d, _, _ = synth
    base = ["-s", "1M", "-m", "17", "-k", "31", "-l", os.path.join(d, "ul.txt"), "-t", "4", *cli,
            "-r", os.path.join(d, "sr.fa"), "-p", os.path.join(d, "pb.fa")]
    outs = []
    for extra, env in (([], None), (["--host-graph"], None), ([], {"PBGPU_GRAPH_NMAX": "40"})):
        o = str(tmp_path / f"mr{len(outs)}")
        r = subprocess.run([CMR, *base, *extra, "-o", o], capture_output=True, text=True, timeout=120,
                           env=dict(os.environ, **(env or {})))
        assert r.returncode == 0, r.stderr
        outs.append(open(o).read())
    assert outs[0].count(">") >= 10
    assert outs[0] == outs[1] == outs[2]


def test_device_graph_c2_reads(tmp_path):
    """C2 (200k super-reads, production aligner flags) on 1500 reads: the device
    traversal gives the host traversal's bytes (~560 records and ~12k edges a read)"""
    from tools.synth import Dataset
    ds = Dataset("C2", seed=42, threads=16, n_pb=1500)
    ds.write(str(tmp_path))
    ds.close()
    base = ["-s", "1M", "-m", "17", "--psa-min", "13", "-k", "31", "-l", str(tmp_path / "ul.txt"), "-B", "15",
            "--max-count", "5000", "--stretch-cap", "10000", "-t", "16",
            "-r", str(tmp_path / "sr.fa"), "-p", str(tmp_path / "pb.fa")]
    a, b = str(tmp_path / "dev"), str(tmp_path / "host")
    _run([*base, "-o", a], timeout=300)
    _run([*base, "--host-graph", "-o", b], timeout=300)
    ta = open(a).read()
    assert ta.count(">") > 1000 and ta == open(b).read()
    # many small batches on each of two aligners, with reads past a lowered device cap left to
    # the host in every batch: their descriptors hold an earlier batch's words, which the edge
    # scans must never read (round-4 review: stale descriptors of host reads)
    c = str(tmp_path / "mixed")
    r = subprocess.run([CMR, *base, "--batch-bases", "2M", "--streams", "2", "-o", c], capture_output=True, text=True,
                       timeout=300, env=dict(os.environ, PBGPU_GRAPH_NMAX="500"))
    assert r.returncode == 0, r.stderr[-2000:]
    assert open(c).read() == ta


def _format_device_mega(name, moff, recs, units, r):
    """print_mega_reads' text of read r from the device mega-reads (the C ABI batch)"""
    out = []
    for m in recs[int(moff[r]):int(moff[r + 1])]:
        u = units[int(m["unit_offset"]):int(m["unit_offset"]) + int(m["n_units"])]
        nm = "_".join(f"{int(x) >> 1}{'R' if int(x) & 1 else 'F'}" for x in u)
        out.append(f"{m['imp_s']:.2f} {m['imp_e']:.2f} {m['rs']} {m['re']} {m['qs']} {m['qend']} {m['lpath']} "
                   f"{m['density']:.4f} {nm} {m['sr_len']}\n")
    return (f">{name}\n" + "".join(out)) if out else ""


@pytest.mark.parametrize("tiling", ["greedy", "maximal"])
def test_abi_device_mega_reads_match_cli(synth, tmp_path, tiling):
    """the mega-reads through the C ABI (pbgpu_aligner_set_graph with mega_reads,
    pbgpu_download's mega arrays), formatted here, equal the CLI's file"""
    from pacbio_amd import pbgpu
    d, ul, _ = synth
    out = str(tmp_path / "mr")
    _run(["-s", "1M", "-m", "17", "-k", "31", "-l", os.path.join(d, "ul.txt"), "-T", tiling, "-L", "0", "-o", out,
          "-r", os.path.join(d, "sr.fa"), "-p", os.path.join(d, "pb.fa")])
    names, seqs = read_fasta(os.path.join(d, "sr.fa"))
    pn, ps = read_fasta(os.path.join(d, "pb.fa"))
    ix = pbgpu.Index.from_records(names, seqs, 17)
    al = pbgpu.Aligner(ix, k=17, forward=True, unitigs_k=31, unitig_lengths=ul)
    al.set_graph([pbgpu.parse_unitigs(n) for n in names], ul, 31, mega_reads=True, tiling=tiling, min_len=0.0)
    c = al.align(ps)
    moff, recs, units, host = c.mega
    assert not host.any() and len(recs) >= 10
    got = "".join(_format_device_mega(n.split()[0], moff, recs, units, r) for r, n in enumerate(pn))
    assert got == open(out).read()


def test_no_device_allocation_after_first_batch(tmp_path):
    """The run path allocates nothing after each aligner's first batch (round-3 review:
    a growing buffer's hipFree + hipMalloc blocked cold runs for seconds): 3000 C2
    reads in >= 12 ramped batches over two aligners, --timing's device_allocs_late and
    pinned_allocs_late are 0, and the mega-reads equal a one-batch run's."""
    import json
    from tools.synth import Dataset
    ds = Dataset("C2", seed=42, threads=16, n_pb=3000)
    ds.write(str(tmp_path))
    ds.close()
    base = ["-s", "1M", "-m", "17", "--psa-min", "13", "-k", "31", "-l", str(tmp_path / "ul.txt"), "-B", "15",
            "--max-count", "5000", "--stretch-cap", "10000", "-t", "16", "--timing",
            "-r", str(tmp_path / "sr.fa"), "-p", str(tmp_path / "pb.fa")]
    a, b = str(tmp_path / "many"), str(tmp_path / "one")
    r = _run([*base, "--batch-bases", "3200000", "-o", a], timeout=300)
    t = json.loads(r.stderr.strip().splitlines()[-1])
    assert t["batches"] >= 12, t
    assert t["device_allocs"] > 0, t  # counted at all: the first batches allocate
    assert t["device_allocs_late"] == 0 and t["pinned_allocs_late"] == 0, t
    _run([*base, "--batch-bases", "1000000000", "-o", b], timeout=300)
    ta = open(a).read()
    assert ta.count(">") > 2000 and ta == open(b).read()


@pytest.mark.parametrize("tiling", ["greedy", "weighted", "maximal"])
def test_read_with_many_components(tmp_path, tiling):
    """One read aligned by 320 super-reads of one unitig each (no name overlaps, so 320
    single-node components): more than k_mega's 256 in-LDS components, so the tiling keeps
    its intervals in HBM.  Device graph == host graph, and > 256 mega-reads."""
    import random
    rng = random.Random(5)
    n_sr, seg = 320, 400
    segs = ["".join(rng.choice("ACGT") for _ in range(seg)) for _ in range(n_sr)]
    (tmp_path / "sr.fa").write_text("".join(f">{i}F\n{s}\n" for i, s in enumerate(segs)))
    (tmp_path / "pb.fa").write_text(">read0\n" + "".join(segs) + "\n")
    (tmp_path / "ul.txt").write_text("".join(f"{seg}\n" for _ in range(n_sr)))
    base = ["-s", "1M", "-m", "17", "-k", "31", "-l", str(tmp_path / "ul.txt"), "-T", tiling,
            "-r", str(tmp_path / "sr.fa"), "-p", str(tmp_path / "pb.fa")]
    a, b = str(tmp_path / "dev"), str(tmp_path / "host")
    _run([*base, "-o", a])
    _run([*base, "--host-graph", "-o", b])
    ta = open(a).read()
    assert ta == open(b).read()
    assert ta.count("\n") > 257, ta[:500]  # a header line, then one line per mega-read


def test_device_graph_long_reads_c4r(tmp_path):
    """C4r (C4's repeat model and 15-kb-N50 reads, ~1300 records a read, ~9% of the reads
    over 4096 and ~2% over 8192): 300 reads.  Every read is traversed on the device -- up to
    8192 records in the LDS tiers, past that with its sort keys and node state in HBM
    (k_graph_sort_big / k_graph_relax_big, round 5) -- and the output equals the host
    graph's bytes, and those of a run that leaves the reads over 8192 records to the host
    (PBGPU_GRAPH_NMAX=8192, round 4's cap).  The C ABI flags no read for the host."""
    import numpy as np
    from pacbio_amd import pbgpu
    from tools.synth import Dataset
    ds = Dataset("C4r", seed=42, threads=16, n_pb=300)
    ds.write(str(tmp_path))
    names = [n.decode() for n in ds.sr_names()]
    ul = [int(x) for x in ds.unitig_lengths]
    blob, off = ds.pb_blob()  # (views into the dataset: closed at the end)
    base = ["-s", "1M", "-m", "17", "--psa-min", "13", "-k", "31", "-l", str(tmp_path / "ul.txt"), "-B", "15",
            "--max-count", "5000", "--stretch-cap", "10000", "-t", "16",
            "-r", str(tmp_path / "sr.fa"), "-p", str(tmp_path / "pb.fa")]
    outs = []
    for extra, env in (([], None), (["--host-graph"], None), ([], {"PBGPU_GRAPH_NMAX": "8192"})):
        o = str(tmp_path / f"mr{len(outs)}")
        r = subprocess.run([CMR, *base, *extra, "-o", o], capture_output=True, text=True, timeout=300,
                           env=dict(os.environ, **(env or {})))
        assert r.returncode == 0, r.stderr
        outs.append(open(o).read())
    assert outs[0].count(">") > 200 and outs[0] == outs[1] == outs[2]
    ix = pbgpu.Index.from_fasta([str(tmp_path / "sr.fa")], 17, psa_min=13)
    kw = dict(k=17, forward=True, unitigs_k=31, unitig_lengths=ul, bases_matching=15.0, max_count=5000,
              stretch_cap=10000.0)
    al0 = pbgpu.Aligner(ix, **kw)  # the records (graph nodes) a read
    al0.align_resident(al0.upload(blob=blob, offsets=off))
    nrec = np.diff(al0.download().read_offsets.astype(np.int64))
    al = pbgpu.Aligner(ix, **kw)
    al.set_graph([pbgpu.parse_unitigs(n) for n in names], ul, 31, mega_reads=True)
    al.align_resident(al.upload(blob=blob, offsets=off))
    host = al.download().mega[3].astype(bool)
    assert ((nrec > 4096) & (nrec <= 8192)).sum() >= 5, np.sort(nrec)[-40:]
    assert (nrec > 8192).sum() >= 2, np.sort(nrec)[-40:]
    assert not host.any() and al.stats()["graph_host_reads"] == 0
    ds.close()


def test_graph_ties_equal_implied_starts(tmp_path):
    """Ties the device relaxation resolves by rank keys: two super-reads of the
    same sequence under different names ("1F_2F_3F", "6F_2F_3F") align with identical
    implied spans, both overlap "2F_3F_4F", which overlaps "3F_4F_5F": node J is reached by
    two paths of equal length whose start nodes have equal imp_s, so the reference keeps
    the first (overlap_graph.cc:45, strictly greater).  A third copy ("8F_2F_3F") and a
    read of the reverse strand add more equal keys.  Device graph == host graph for every
    tiling, and with -b (path length in bases)."""
    import random
    rng = random.Random(11)
    ulen, step = 400, 370  # unitigs of 400 bases overlapping by k - 1 = 30
    g = "".join(rng.choice("ACGT") for _ in range(step * 6 + ulen))
    u = {i: g[(i - 1) * step:(i - 1) * step + ulen] for i in range(1, 7)}

    def sr(ids):
        s = u[ids[0]]
        for i in ids[1:]:
            s += u[i][30:]
        return s
    a = sr([1, 2, 3])
    srs = [("1F_2F_3F", a), ("6F_2F_3F", a), ("2F_3F_4F", sr([2, 3, 4])), ("3F_4F_5F", sr([3, 4, 5])),
           ("8F_2F_3F", a), ("4F_5F_6F", sr([4, 5, 6]))]
    (tmp_path / "sr.fa").write_text("".join(f">{n}\n{s}\n" for n, s in srs))
    read = sr([1, 2, 3, 4, 5, 6])
    rc = read[::-1].translate(str.maketrans("ACGT", "TGCA"))
    (tmp_path / "pb.fa").write_text(f">fwd\n{read}\n>rev\n{rc}\n>mid\n{read[200:2000]}\n")
    (tmp_path / "ul.txt").write_text("".join(f"u{i} {ulen}\n" for i in range(9)))
    for tiling in ("greedy", "maximal", "weighted", "none"):
        for extra in ([], ["-b"]):
            base = ["-s", "1M", "-m", "17", "-k", "31", "-l", str(tmp_path / "ul.txt"), "-T", tiling, "-L", "0",
                    *extra, "-r", str(tmp_path / "sr.fa"), "-p", str(tmp_path / "pb.fa")]
            a_out, b_out = str(tmp_path / "dev"), str(tmp_path / "host")
            _run([*base, "-o", a_out])
            _run([*base, "--host-graph", "-o", b_out])
            ta = open(a_out).read()
            assert ta == open(b_out).read(), (tiling, extra)
            assert ta.count(">") >= 2, ta


C4R_FLAGS = ["-s", "1M", "-m", "17", "--psa-min", "13", "-k", "31", "-B", "15", "--max-count", "5000",
             "--stretch-cap", "10000", "-t", "16"]


def test_device_graph_full_c4r_equals_host_graph(tmp_path):
    """All 20k C4r reads (the bench's C4r leg, 25.5 M records, ~2% of the reads past 8192
    records and none left to the host) through the CLI: the device graph -- the LDS tiers,
    the HBM sort / relaxation of the long reads, the edge scans' prefilter queue and k_mega --
    gives the bytes of --host-graph (round 5 checked this only as a profile,
    profiles/r05zy_cmr_full_device_vs_host.txt; the suite held 300 reads)."""
    import json
    from tools.synth import Dataset
    ds = Dataset("C4r", seed=42, threads=16, n_pb=20000)
    ds.write(str(tmp_path))
    ds.close()
    base = [*C4R_FLAGS, "-l", str(tmp_path / "ul.txt"), "--timing", "-r", str(tmp_path / "sr.fa"),
            "-p", str(tmp_path / "pb.fa")]
    dev, host = str(tmp_path / "dev"), str(tmp_path / "host")
    r = _run([*base, "-o", dev], timeout=600)
    t = json.loads(r.stderr.strip().splitlines()[-1])
    assert t["graph_host_reads"] == 0 and t["records"] > 20_000_000, t
    _run([*base, "--host-graph", "-o", host], timeout=600)
    td = open(dev).read()
    assert td.count(">") > 19_000 and td == open(host).read()


def test_read_past_8192_records_against_restatement(tmp_path):
    """A read of more than 8192 records -- C4r read 207 (9191 records: its sort keys and
    node state in HBM, k_graph_sort_big / k_graph_relax_big) -- checked against the
    independent Python restatement (oracle/mega_reads.py) on the CPU oracle's records of
    that read, not only against the product's own host graph (overlap_graph.cc:7-59,
    mega_reads_per_comp, tile_greedy)."""
    from tools.synth import Dataset
    big = Dataset("C4r", seed=42, threads=16, n_pb=1, pb_index_base=207)
    big.write(str(tmp_path))
    ul = [int(x) for x in big.unitig_lengths]
    oix = O.OracleIndex.from_records(big.sr_names(), big.sr_seqs(), 17, threads=16)
    p = O.params(k=17, forward=True, unitigs_k=31, unitig_lengths=ul, bases_matching=15.0, max_count=5000,
                 stretch_cap=10000.0)
    (name,), (seq,) = big.pb_names(), big.pb_seqs()
    recs = MR.records_of(oix, p, seq)
    oix.close()
    big.close()
    assert len(recs) > 8192, len(recs)
    out = str(tmp_path / "mr")
    _run([*C4R_FLAGS, "-l", str(tmp_path / "ul.txt"), "-o", out, "-r", str(tmp_path / "sr.fa"),
          "-p", str(tmp_path / "pb.fa")], timeout=300)
    want = _expect([(name.decode(), recs)], ul, 31)
    assert want.startswith(f">{name.decode()}") and want.count("\n") >= 2  # the header, then its mega-reads
    assert open(out).read() == want

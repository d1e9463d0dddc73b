"""Device coords text (pbgpu_format_device) and the file-to-file driver
(pbgpu_run, the jf_aligner CLI): byte-identical to the host formatter and,
per read, to the CPU restatement (oracle/), for every parity configuration,
multi-batch / multi-aligner / two-index ("--devices 0,0") runs, gzip input,
and the worker error path."""
import gzip
import os
import shutil
import subprocess
import tempfile

import pytest

from tests._compare import assert_same_coords
from tests.test_gpu_parity import CONFIGS

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "pacbio_amd", "bin", "jf_aligner")


@pytest.fixture(scope="module")
def small():
    from tools.synth import Dataset
    return Dataset("small", seed=7)


@pytest.fixture(scope="module")
def small_dir(small):
    d = tempfile.mkdtemp(prefix="pbgpu_fmt_")
    small.write(d)
    yield d
    shutil.rmtree(d, ignore_errors=True)


def _split(cfg):
    cfg = dict(cfg)
    k = cfg.pop("k", 17)
    use_ul = cfg.pop("use_ul", False)
    return k, use_ul, cfg


@pytest.mark.parametrize("name", list(CONFIGS))
def test_device_text_matches_host_and_oracle(small, name):
    from oracle.oracle import OracleIndex, params
    from pacbio_amd import pbgpu
    k, use_ul, cfg = _split(CONFIGS[name])
    ul = small.unitig_lengths if use_ul else None
    names, seqs = small.sr_names(), small.sr_seqs()
    pnames, pseqs = small.pb_names(), small.pb_seqs()
    gix = pbgpu.Index.from_records(names, seqs, k)
    al = pbgpu.Aligner(gix, k=k, unitig_lengths=ul, **cfg)
    rd = al.upload(pseqs, names=pnames)
    al.align_resident(rd)
    dev = al.format_device(rd)
    host = al.download().format(gix, pnames, [len(s) for s in pseqs])
    assert dev == host
    exp = OracleIndex.from_records(names, seqs, k).align_format(params(k=k, unitig_lengths=ul, **cfg), pnames, pseqs,
                                                                threads=8)
    assert_same_coords(dev, exp, name)
    # non-compact lines and -0 headers
    assert al.format_device(rd, compact=False, zero_match=True) == \
        al.download().format(gix, pnames, [len(s) for s in pseqs], compact=False, zero_match=True)
    rd.close()


def _oracle_file_text(ds, k=17, **cfg):
    from oracle.oracle import OracleIndex, params
    oix = OracleIndex.from_records(ds.sr_names(), ds.sr_seqs(), k)
    return oix.align_format(params(k=k, **cfg), ds.pb_names(), ds.pb_seqs(), threads=8, header=True)


def test_run_many_batches_two_indexes(small, small_dir):
    """pbgpu_run: tiny batches over 2 x 3 aligners on two index entries of
    device 0 (--devices 0,0) give the one-batch bytes, which match the oracle."""
    from pacbio_amd import pbgpu
    kw = dict(forward=True, unitigs_k=31, unitig_lengths=small.unitig_lengths, bases_matching=15.0)
    gix = pbgpu.Index.from_fasta([os.path.join(small_dir, "sr.fa")], 17)
    rep = gix.replicate(0)
    pb = [os.path.join(small_dir, "pb.fa")]
    out1, out2 = os.path.join(small_dir, "one.coords"), os.path.join(small_dir, "many.coords")
    st1 = pbgpu.run([gix], pb, out1, aligners_per_device=1, **kw)
    st2 = pbgpu.run([gix, rep], pb, out2, aligners_per_device=3, batch_bases=20_000, **kw)
    one, many = open(out1).read(), open(out2).read()
    assert st1["n_batches"] == 1 and st2["n_batches"] > 8
    assert st2["n_bases"] == st1["n_bases"] and st2["coords_bytes"] == len(many.encode())
    assert many == one
    assert_same_coords(one, _oracle_file_text(small, **kw), "run")
    rep.close()
    gix.close()


def test_run_more_than_64_batches(tmp_path):
    """Batch sizes past the ramp: the first batches hold batch_bases >> 3, >> 2,
    >> 1 bases, then every batch takes reads up to batch_bases (a shift by the
    batch id used to wrap to single-read batches from batch 41 on).  ~140
    batches of ~20 reads give the one-batch bytes."""
    from pacbio_amd import pbgpu
    from tools.synth import Dataset
    ds = Dataset("small", seed=5, n_pb=3000)
    d = str(tmp_path)
    ds.write(d)
    ds.close()
    gix = pbgpu.Index.from_fasta([os.path.join(d, "sr.fa")], 17)
    pb = [os.path.join(d, "pb.fa")]
    bb = 128_000
    a, b = os.path.join(d, "many.coords"), os.path.join(d, "one.coords")
    st = pbgpu.run([gix], pb, a, aligners_per_device=2, batch_bases=bb)
    st1 = pbgpu.run([gix], pb, b, aligners_per_device=1, batch_bases=1 << 30)  # ramp start 2^27 > the input
    gix.close()
    assert st1["n_batches"] == 1 and st["n_bases"] == st1["n_bases"]
    assert st["n_batches"] > 64
    # each full batch holds >= bb bases: 3 ramp batches + the full ones + one partial at most
    assert st["n_batches"] <= 3 + st["n_bases"] // bb + 1, (st["n_batches"], st["n_bases"])
    assert open(a).read() == open(b).read()


@pytest.fixture(scope="module")
def many_dir(tmp_path_factory):
    """3000 reads of the small preset, as one FASTA file and as the same reads split over two files"""
    from tools.synth import Dataset
    d = str(tmp_path_factory.mktemp("many"))
    ds = Dataset("small", seed=5, n_pb=3000)
    ds.write(d)
    ds.close()
    recs = open(os.path.join(d, "pb.fa")).read().split(">")[1:]
    with open(os.path.join(d, "pb_a.fa"), "w") as f:
        f.write("".join(">" + r for r in recs[:1234]))
    with open(os.path.join(d, "pb_b.fa"), "w") as f:
        f.write("".join(">" + r for r in recs[1234:]))
    return d


@pytest.mark.parametrize("n_parts,files", [(2, 1), (3, 2), (4, 1)])
def test_run_part_files_concatenate(many_dir, n_parts, files):
    """n_parts: part p holds the reads whose header starts in [p T / P, (p + 1) T / P)
    of the inputs, written by its own writer; the parts concatenated are the
    one-file bytes (header line in part 0 only), with one or two input files."""
    from pacbio_amd import pbgpu
    d = many_dir
    gix = pbgpu.Index.from_fasta([os.path.join(d, "sr.fa")], 17)
    rep = gix.replicate(0)
    pb = [os.path.join(d, "pb.fa")] if files == 1 else [os.path.join(d, "pb_a.fa"), os.path.join(d, "pb_b.fa")]
    one, part = os.path.join(d, f"one{n_parts}.coords"), os.path.join(d, f"part{n_parts}.coords")
    st1 = pbgpu.run([gix], pb, one, aligners_per_device=2, batch_bases=200_000)
    st = pbgpu.run([gix, rep], pb, part, aligners_per_device=2, batch_bases=200_000, n_parts=n_parts)
    rep.close()
    gix.close()
    texts = [open(f"{part}.{i}").read() for i in range(n_parts)]
    assert all(t.count("\n") > 100 for t in texts)
    assert "".join(texts) == open(one).read()
    assert st["n_reads"] == st1["n_reads"] == 3000 and st["coords_bytes"] == sum(len(t) for t in texts)


def test_run_part_files_refuse_gzip_and_fastq(many_dir, tmp_path):
    from pacbio_amd import pbgpu
    d = many_dir
    gix = pbgpu.Index.from_fasta([os.path.join(d, "sr.fa")], 17)
    gz = str(tmp_path / "pb.fa.gz")
    with open(os.path.join(d, "pb_a.fa"), "rb") as f, gzip.open(gz, "wb") as g:
        g.write(f.read())
    fq = str(tmp_path / "pb.fq")
    with open(fq, "w") as f:
        for i in range(50):
            f.write(f"@r{i}\n{'ACGT' * 300}\n+\n{'I' * 1200}\n")
    # a FIFO (or <(zcat ...)) reports size 0: split by byte range it would give every part
    # an empty range and write empty files without an error, so it is refused before it is opened
    fifo = str(tmp_path / "pb.fifo")
    os.mkfifo(fifo)
    for path in (gz, fq, fifo):
        with pytest.raises(pbgpu.PbgpuError) as e:
            pbgpu.run([gix], [path], str(tmp_path / "x.coords"), aligners_per_device=2, n_parts=2)
        assert e.value.status == 5, e.value  # PBGPU_ERR_UNSUPPORTED
    gix.close()


def test_cli_parts(many_dir, tmp_path):
    """jf_aligner --devices 0,0 --parts 2: the parts concatenated are the one-file output"""
    d = many_dir
    base = [CLI, "-s", "1", "-m", "17", "-r", os.path.join(d, "sr.fa"), "-l", os.path.join(d, "ul.txt"), "-k", "31",
            "-f", "-B", "15", "-p", os.path.join(d, "pb.fa")]
    one, part = str(tmp_path / "one.coords"), str(tmp_path / "part.coords")
    r1 = subprocess.run(base + ["--coords", one], capture_output=True, text=True, timeout=300)
    r2 = subprocess.run(base + ["--coords", part, "--devices", "0,0", "--parts", "2"], capture_output=True, text=True,
                        timeout=300)
    assert r1.returncode == 0, r1.stderr
    assert r2.returncode == 0, r2.stderr
    assert open(part + ".0").read() + open(part + ".1").read() == open(one).read()


def test_run_gzip_input(small, small_dir):
    from pacbio_amd import pbgpu
    pb = os.path.join(small_dir, "pb.fa")
    gz = os.path.join(small_dir, "pb.fa.gz")
    with open(pb, "rb") as f, gzip.open(gz, "wb") as g:
        g.write(f.read())
    gix = pbgpu.Index.from_fasta([os.path.join(small_dir, "sr.fa")], 17)
    a, b = os.path.join(small_dir, "plain.coords"), os.path.join(small_dir, "gz.coords")
    pbgpu.run([gix], [pb], a, batch_bases=50_000)
    pbgpu.run([gix], [gz], b, batch_bases=50_000)
    assert open(a).read() == open(b).read()
    assert open(a).read().count("\n") > 100
    gix.close()


def test_run_error_is_returned(small_dir):
    """a missing PacBio file fails the run with PBGPU_ERR_IO (reader thread error, no exit, no hang)"""
    from pacbio_amd import pbgpu
    gix = pbgpu.Index.from_fasta([os.path.join(small_dir, "sr.fa")], 17)
    with pytest.raises(pbgpu.PbgpuError) as e:
        pbgpu.run([gix], [os.path.join(small_dir, "pb.fa"), os.path.join(small_dir, "missing.fa")],
                  os.path.join(small_dir, "err.coords"), batch_bases=20_000)
    assert e.value.status == 2
    gix.close()


def test_cli_devices_and_gzip(small, small_dir):
    """jf_aligner --devices 0,0 and gzip input: the same bytes as one device and plain FASTA."""
    gz = os.path.join(small_dir, "pb2.fa.gz")
    with open(os.path.join(small_dir, "pb.fa"), "rb") as f, gzip.open(gz, "wb") as g:
        g.write(f.read())
    base = [CLI, "-s", "1", "-m", "17", "-r", os.path.join(small_dir, "sr.fa"), "-l", os.path.join(small_dir, "ul.txt"),
            "-k", "31", "-f", "-B", "15", "--coords", "/dev/stdout"]
    r1 = subprocess.run(base + ["-p", os.path.join(small_dir, "pb.fa")], capture_output=True, text=True, timeout=300)
    r2 = subprocess.run(base + ["-p", gz, "--devices", "0,0", "--batch-bases", "30k", "--timing"], capture_output=True,
                        text=True, timeout=300)
    assert r1.returncode == 0, r1.stderr
    assert r2.returncode == 0, r2.stderr
    assert r1.stdout == r2.stdout
    assert '"wall_s"' in r2.stderr
    assert_same_coords(r1.stdout, _oracle_file_text(small, forward=True, unitigs_k=31,
                                                     unitig_lengths=small.unitig_lengths, bases_matching=15.0), "cli")


def test_cli_bad_input_exits_1(small_dir):
    bad = os.path.join(small_dir, "bad.fa")
    with open(bad, "w") as f:
        f.write("not a fasta\nACGT\n")
    r = subprocess.run([CLI, "-s", "1", "-m", "17", "-r", os.path.join(small_dir, "sr.fa"), "-p", bad, "--coords",
                        "/dev/null"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 1
    assert "neither FASTA nor FASTQ" in r.stderr


def test_cli_records_counted_at_emission(small_dir):
    """The records stage's two paths give the same bytes: per-read counts and slots taken
    by k_coords as it emits (the default) and the count + scatter afterwards
    (PBGPU_REC_HIST=1, the path of --max-match and of record-overflow retries); many
    small batches over two aligners."""
    base = [CLI, "-s", "1", "-m", "17", "-r", os.path.join(small_dir, "sr.fa"), "-l", os.path.join(small_dir, "ul.txt"),
            "-k", "31", "-f", "-B", "15", "--batch-bases", "30k", "--coords", "/dev/stdout",
            "-p", os.path.join(small_dir, "pb.fa")]
    r1 = subprocess.run(base, capture_output=True, text=True, timeout=300)
    r2 = subprocess.run(base, capture_output=True, text=True, timeout=300, env=dict(os.environ, PBGPU_REC_HIST="1"))
    assert r1.returncode == 0, r1.stderr
    assert r2.returncode == 0, r2.stderr
    assert r1.stdout.count("\n") > 50 and r1.stdout == r2.stdout

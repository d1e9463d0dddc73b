"""On-disk index cache (optional): pbgpu_index_save /
pbgpu_index_load through the C ABI, and jf_aligner --index-cache.  A loaded
index must align byte for byte like the built one; a cache saved for other
inputs or parameters, or cut short, must be refused (PBGPU_ERR_IO), and the CLI
then rebuilds."""
import os
import shutil
import subprocess
import tempfile

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "pacbio_amd", "bin", "jf_aligner")
IO = 2  # PBGPU_ERR_IO


@pytest.fixture(scope="module")
def small():
    from tools.synth import Dataset
    return Dataset("small", seed=11)


@pytest.fixture(scope="module")
def work(small):
    d = tempfile.mkdtemp(prefix="pbgpu_ixc_")
    small.write(d)
    yield d
    shutil.rmtree(d, ignore_errors=True)


def _text(ix, ds, **kw):
    from pacbio_amd import pbgpu
    al = pbgpu.Aligner(ix, k=17, forward=True, unitigs_k=31, unitig_lengths=ds.unitig_lengths, bases_matching=15.0,
                       **kw)
    try:
        return al.align(ds.pb_seqs()).format(ix, ds.pb_names(), [len(s) for s in ds.pb_seqs()])
    finally:
        al.close()


@pytest.mark.parametrize("fine_k", [0, 13], ids=["coarse", "fine13"])
def test_save_load_same_alignment(small, work, fine_k):
    from pacbio_amd import pbgpu
    path = os.path.join(work, f"ix{fine_k}.pbix")
    ix = pbgpu.Index.from_records(small.sr_names(), small.sr_seqs(), 17, fine_k=fine_k)
    want = _text(ix, small, fine_k=fine_k)
    assert want.count("\n") > 10
    ix.save(path, tag="t1")
    a = ix.info()
    ix.close()
    ix2 = pbgpu.Index.load(path, tag="t1")
    b = ix2.info()
    for key in ("n_sr", "text_len", "n_kmers", "n_occurrences", "table_buckets", "device_bytes"):
        assert a[key] == b[key], key
    names = [n.decode() if isinstance(n, bytes) else n for n in small.sr_names()[:3]]
    assert [ix2.sr_name(i) for i in range(3)] == names
    assert _text(ix2, small, fine_k=fine_k) == want
    ix2.close()


def test_load_refuses_other_tag_and_truncation(small, work):
    from pacbio_amd import pbgpu
    path = os.path.join(work, "ixr.pbix")
    ix = pbgpu.Index.from_records(small.sr_names(), small.sr_seqs(), 17)
    ix.save(path, tag="k=17")
    ix.close()
    with pytest.raises(pbgpu.PbgpuError) as e:
        pbgpu.Index.load(path, tag="k=21")
    assert e.value.status == IO
    cut = os.path.join(work, "ixr_cut.pbix")
    with open(path, "rb") as f, open(cut, "wb") as g:
        g.write(f.read()[: os.path.getsize(path) // 2])
    with pytest.raises(pbgpu.PbgpuError) as e:
        pbgpu.Index.load(cut, tag="k=17")
    assert e.value.status == IO
    with pytest.raises(pbgpu.PbgpuError) as e:
        pbgpu.Index.load(os.path.join(work, "missing.pbix"))
    assert e.value.status == IO


def test_cli_index_cache(work):
    cache = os.path.join(work, "cli.pbix")
    sr = os.path.join(work, "sr.fa")
    cmd = [CLI, "-s", "1", "-m", "17", "-r", sr, "-p", os.path.join(work, "pb.fa"), "-l",
           os.path.join(work, "ul.txt"), "-k", "31", "-f", "-B", "15", "--coords", "/dev/stdout", "--timing",
           "--index-cache", cache]
    plain = subprocess.run(cmd[:-2], capture_output=True, text=True, timeout=300)
    first = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    second = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    for r in (plain, first, second):
        assert r.returncode == 0, r.stderr
    assert "saved to cache" in first.stderr and os.path.exists(cache)
    assert "loaded from cache" in second.stderr
    assert plain.stdout == first.stdout == second.stdout
    # other super-reads (a changed file): the cache is not used, the index is rebuilt
    os.utime(sr, ns=(os.stat(sr).st_atime_ns, os.stat(sr).st_mtime_ns + 1_000_000_000))
    third = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert third.returncode == 0, third.stderr
    assert "not used" in third.stderr and "saved to cache" in third.stderr
    assert third.stdout == plain.stdout


def test_save_load_shards(small, work):
    """Shards of a sharded index survive the cache: per-shard
    counts, the host sum and the per-shard alignment of loaded shards give the
    built shards' merged text (shard-local starts, global names)."""
    import numpy as np
    from pacbio_amd import pbgpu
    names, seqs, ps = small.sr_names(), small.sr_seqs(), small.pb_seqs()
    nb = sum(len(s) for s in ps)

    def merged_text(shards):
        als = [pbgpu.Aligner(ix, k=17) for ix in shards]
        rds = [al.upload(ps) for al in als]
        total = np.zeros(nb, np.uint64)
        for al, rd in zip(als, rds):
            al.shard_counts(rd)
            total += al.counts_download(nb)
        parts = []
        for al, rd in zip(als, rds):
            al.counts_upload(total.astype(np.uint32))
            al.align_resident_shard(rd)
            parts.append(al.download())
            rd.close()
            al.close()
        return pbgpu.merge_coords(parts).format(shards[0], small.pb_names(), [len(s) for s in ps])

    built = [pbgpu.Index.from_records(names, seqs, 17, shard=s, n_shards=3) for s in range(3)]
    want = merged_text(built)
    assert want.count("\n") > 10
    for s, ix in enumerate(built):
        ix.save(os.path.join(work, f"shard{s}.pbix"), tag=f"s{s}")
        ix.close()
    loaded = [pbgpu.Index.load(os.path.join(work, f"shard{s}.pbix"), tag=f"s{s}") for s in range(3)]
    assert [ix.info()["sr_begin"] for ix in loaded][0] == 0 and loaded[-1].info()["sr_end"] == len(names)
    assert merged_text(loaded) == want
    for ix in loaded:
        ix.close()

"""Multi-GPU paths on hardware, for a node with two or more
visible GPUs; every test skips on the one-GPU pool (each is a single run).

  * e1, reads sharded / index replicated: `jf_aligner --devices 0,1` builds the
    index once and copies it to device 1 with pbgpu_index_replicate (the
    hipMemcpyPeer branch), batches go to whichever GPU is free, and the output
    is the one-device bytes; the replica aligns on its own device like the
    original.
  * e2, index sharded: two ranks, one GPU each, shard s of 2 on device s, the
    saturated per-shard k-mer counts summed by the RCCL all-reduce over xGMI
    (pbgpu_shard_counts_allreduce, two 16-bit counts per ncclUint32), records
    merged per read -- equal to the oracle's whole-index text.
  * the bench's N = 2 launch (two spawned ranks, one per GPU).
"""
import json
import os
import shutil
import subprocess
import sys
import tempfile
import textwrap

import pytest

from tests._compare import assert_same_coords

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "pacbio_amd", "bin", "jf_aligner")


def _devices():
    from pacbio_amd import pbgpu
    return pbgpu.lib().pbgpu_device_count()


need2 = pytest.mark.skipif("_devices() < 2", reason="needs two visible GPUs (the pool's boxes have one)")


@pytest.fixture(scope="module")
def small():
    from tools.synth import Dataset
    return Dataset("small", seed=7)


@pytest.fixture(scope="module")
def small_dir(small):
    d = tempfile.mkdtemp(prefix="pbgpu_multi_")
    small.write(d)
    yield d
    shutil.rmtree(d, ignore_errors=True)


def _oracle(ds, header=False, **cfg):
    from oracle.oracle import OracleIndex, params
    oix = OracleIndex.from_records(ds.sr_names(), ds.sr_seqs(), 17)
    try:
        return oix.align_format(params(k=17, **cfg), ds.pb_names(), ds.pb_seqs(), threads=8, header=header)
    finally:
        oix.close()


@need2
def test_cli_devices_0_1_peer_replica(small, small_dir):
    """--devices 0,1: the index built on device 0 and replicated to device 1 (peer
    copy); small batches spread over both GPUs; the bytes of a one-device run."""
    base = [CLI, "-s", "1", "-m", "17", "-r", os.path.join(small_dir, "sr.fa"), "-l", os.path.join(small_dir, "ul.txt"),
            "-k", "31", "-f", "-B", "15", "-p", os.path.join(small_dir, "pb.fa"), "--coords", "/dev/stdout"]
    r1 = subprocess.run(base + ["--devices", "0"], capture_output=True, text=True, timeout=300)
    r2 = subprocess.run(base + ["--devices", "0,1", "--batch-bases", "30k", "--timing"], capture_output=True, text=True,
                        timeout=300)
    assert r1.returncode == 0, r1.stderr
    assert r2.returncode == 0, r2.stderr
    assert r1.stdout == r2.stdout
    t = json.loads(r2.stderr.strip().splitlines()[-1])
    assert t["batches"] >= 4, t
    assert_same_coords(r1.stdout, _oracle(small, header=True, forward=True, unitigs_k=31,
                                          unitig_lengths=small.unitig_lengths, bases_matching=15.0), "devices 0,1")


@need2
def test_index_replica_aligns_on_device_1(small):
    from pacbio_amd import pbgpu
    ix0 = pbgpu.Index.from_records(small.sr_names(), small.sr_seqs(), 17, device=0)
    ix1 = ix0.replicate(1)
    lens = [len(s) for s in small.pb_seqs()]
    txt = []
    for ix in (ix0, ix1):
        al = pbgpu.Aligner(ix, k=17, forward=True)
        txt.append(al.align(small.pb_seqs()).format(ix, small.pb_names(), lens))
        al.close()
    assert txt[0] == txt[1]
    assert_same_coords(txt[1], _oracle(small, forward=True), "replica on device 1")


@need2
def test_rccl_count_allreduce_two_gpus(small, tmp_path):
    """Two ranks, shard s of the index on GPU s: the count exchange is RCCL over
    xGMI (the communicator's id handed over through a file), the records gathered
    to rank 0 through files and merged; the oracle's whole-index bytes."""
    exp = _oracle(small)
    uid = tmp_path / "uid.bin"
    script = tmp_path / "rank.py"
    script.write_text(textwrap.dedent(f"""
        import os, sys, time, pickle
        sys.path.insert(0, {ROOT!r})
        import numpy as np
        from pacbio_amd import pbgpu
        from tools.synth import Dataset
        rank = int(sys.argv[1])
        ds = Dataset("small", seed=7)
        pseqs = ds.pb_seqs()
        if rank == 0:
            open({str(uid)!r} + ".tmp", "wb").write(pbgpu.rccl_unique_id())
            os.rename({str(uid)!r} + ".tmp", {str(uid)!r})
        t0 = time.time()
        while not os.path.exists({str(uid)!r}):
            assert time.time() - t0 < 60
            time.sleep(0.05)
        comm = pbgpu.RcclComm(rank, 2, rank, open({str(uid)!r}, "rb").read())
        ix = pbgpu.Index.from_records(ds.sr_names(), ds.sr_seqs(), 17, shard=rank, n_shards=2, device=rank)
        al = pbgpu.Aligner(ix, k=17)
        rr = al.upload(pseqs)
        al.shard_counts(rr)
        al.counts_allreduce(comm)
        n = sum(len(s) for s in pseqs)
        assert comm.last_bytes() == 4 * ((n + 1) // 2)
        al.align_resident_shard(rr)
        co = al.download()
        with open({str(tmp_path)!r} + f"/part{{rank}}.pkl", "wb") as f:
            pickle.dump((np.asarray(co.records), np.asarray(co.read_offsets), np.asarray(co.kmers_info),
                         np.asarray(co.bases_info)), f)
        comm.close()
    """))
    procs = [subprocess.Popen([sys.executable, str(script), str(r)], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                              text=True) for r in range(2)]
    outs = [p.communicate(timeout=300) for p in procs]
    assert all(p.returncode == 0 for p in procs), outs
    import ctypes as C
    import pickle
    import numpy as np
    from pacbio_amd import pbgpu
    keep, ptrs = [], []
    for r in range(2):
        with open(tmp_path / f"part{r}.pkl", "rb") as f:  # (written by this test's own ranks)
            recs, off, km, kb = pickle.load(f)
        recs = np.ascontiguousarray(recs)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        km = np.ascontiguousarray(km if len(km) else np.zeros(1, np.int32), dtype=np.int32)
        kb = np.ascontiguousarray(kb if len(kb) else np.zeros(1, np.int32), dtype=np.int32)
        keep += [recs, off, km, kb]
        b = pbgpu.CoordsBatch(len(off) - 1, len(recs), off.ctypes.data_as(C.POINTER(C.c_uint64)),
                              recs.ctypes.data if len(recs) else None, len(km),
                              km.ctypes.data_as(C.POINTER(C.c_int32)), kb.ctypes.data_as(C.POINTER(C.c_int32)))
        keep.append(b)
        ptrs.append(C.pointer(b))
    arr = (C.POINTER(pbgpu.CoordsBatch) * 2)(*ptrs)
    o = C.POINTER(pbgpu.CoordsBatch)()
    pbgpu._check(pbgpu.lib().pbgpu_coords_merge(arr, 2, C.byref(o)))
    ix = pbgpu.Index.from_records(small.sr_names(), small.sr_seqs(), 17)
    got = pbgpu.Coords(o).format(ix, small.pb_names(), [len(s) for s in small.pb_seqs()])
    assert_same_coords(got, exp, "rccl two GPUs")


@need2
def test_bench_two_ranks(tmp_path):
    """bench.py --gpus 2 without a launcher: two rank processes, one per GPU, one JSON
    line with n_gpus 2 and the device-side figures summed over the ranks."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--reads", "1500", "--steps", "1",
                        "--warmup", "1", "--device-steps", "1", "--cmr-steps", "0", "--parts", "0", "--c4r-reads", "0",
                        "--no-cpu-baseline", "--no-brand", "--workdir", str(tmp_path)],
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["value"] > 0 and line["value_device"] > 0, line

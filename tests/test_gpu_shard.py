"""GPU index-sharded mode (the C5 configuration): S shards of the
super-read index (here all on one GPU), per-shard saturated k-mer counts
summed across shards, shard-local hits -> chains -> records, per-read merge.
The merged coords must equal the oracle's whole-index output byte for byte."""
import os
import socket
import subprocess
import sys
import textwrap

import numpy as np
import pytest

from tests._compare import assert_same_coords

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def small():
    from tools.synth import Dataset
    return Dataset("small", seed=7)


def _oracle(ds, k, ul, cfg):
    from oracle.oracle import OracleIndex, params
    oix = OracleIndex.from_records(ds.sr_names(), ds.sr_seqs(), k)
    try:
        return oix.align_format(params(k=k, unitig_lengths=ul, **cfg), ds.pb_names(), ds.pb_seqs(), threads=8)
    finally:
        oix.close()


def _sharded(ds, S, k, ul, cfg):
    from pacbio_amd import pbgpu
    names, seqs = ds.sr_names(), ds.sr_seqs()
    pseqs = ds.pb_seqs()
    n_bases = sum(len(s) for s in pseqs)
    shards = []
    for s in range(S):
        ix = pbgpu.Index.from_records(names, seqs, k, shard=s, n_shards=S)
        al = pbgpu.Aligner(ix, k=k, unitig_lengths=ul, **cfg)
        shards.append((ix, al, al.upload(pseqs)))
    info = [ix.info() for ix, _, _ in shards]
    assert info[0]["sr_begin"] == 0 and info[-1]["sr_end"] == len(names)
    assert all(info[i]["sr_end"] == info[i + 1]["sr_begin"] for i in range(S - 1))
    total = np.zeros(n_bases, np.uint64)
    for ix, al, rr in shards:
        al.shard_counts(rr)
        total += al.counts_download(n_bases)  # the all-reduce, through host memory
    parts = []
    for ix, al, rr in shards:
        al.counts_upload(total.astype(np.uint32))
        al.align_resident_shard(rr)
        parts.append(al.download())
    merged = pbgpu.merge_coords(parts)
    return merged.format(shards[0][0], ds.pb_names(), [len(s) for s in pseqs])


CONFIGS = {
    "default_s2": (2, 17, False, dict()),
    "default_s3": (3, 17, False, dict()),
    "forward_ul_maxmatch_s2": (2, 17, True, dict(forward=True, max_match=True, unitigs_k=31, bases_matching=10.0)),
    "maxcount20_s5": (5, 17, False, dict(max_count=20)),
    "k16_even_s3": (3, 16, False, dict()),
    "k21_s4": (4, 21, True, dict(forward=True, unitigs_k=31, bases_matching=15.0)),
}


@pytest.mark.parametrize("name", list(CONFIGS))
def test_sharded_index_matches_whole_index(small, name):
    S, k, use_ul, cfg = CONFIGS[name]
    ul = small.unitig_lengths if use_ul else None
    exp = _oracle(small, k, ul, cfg)
    assert exp.count("\n") > 10
    got = _sharded(small, S, k, ul, cfg)
    assert_same_coords(got, exp, name)


def test_sharded_index_rejects_whole_index_calls(small):
    from pacbio_amd import pbgpu
    ix = pbgpu.Index.from_records(small.sr_names()[:50], small.sr_seqs()[:50], 17, shard=1, n_shards=2)
    al = pbgpu.Aligner(ix, k=17)
    with pytest.raises(pbgpu.PbgpuError) as e:
        al.align(small.pb_seqs()[:2])
    assert e.value.status == 1
    with pytest.raises(pbgpu.PbgpuError):
        al.set_details(True)


def test_rccl_single_rank_allreduce(small):
    """The RCCL exchange on this box's one GPU: a one-rank communicator's
    all-reduce leaves the counts unchanged, so the whole-index result follows."""
    from pacbio_amd import pbgpu
    exp = _oracle(small, 17, None, {})
    ix = pbgpu.Index.from_records(small.sr_names(), small.sr_seqs(), 17)
    al = pbgpu.Aligner(ix, k=17)
    rr = al.upload(small.pb_seqs())
    comm = pbgpu.RcclComm(0, 1, 0, pbgpu.rccl_unique_id())
    al.shard_counts(rr)
    before = al.counts_download(sum(len(s) for s in small.pb_seqs()))
    al.counts_allreduce(comm)
    assert np.array_equal(before, al.counts_download(len(before)))
    # one rank x (max_count + 1): two 16-bit counts per ncclUint32
    assert comm.last_bytes() == 4 * ((len(before) + 1) // 2)
    al.align_resident_shard(rr)
    got = al.download().format(ix, small.pb_names(), [len(s) for s in small.pb_seqs()])
    comm.close()
    assert_same_coords(got, exp, "rccl1")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_ranks_torch_distributed(small, tmp_path):
    """One process per shard with torch.distributed: the count all-reduce and the
    record gather cross ranks (gloo on host buffers here, both ranks on this
    box's one GPU; on separate GPUs the count exchange is the RCCL all-reduce of
    the test above)."""
    exp = _oracle(small, 17, None, {})
    out = tmp_path / "coords.txt"
    script = tmp_path / "rank.py"
    script.write_text(textwrap.dedent(f"""
        import os, sys, ctypes as C
        sys.path.insert(0, {ROOT!r})
        import numpy as np, torch, torch.distributed as dist
        from pacbio_amd import pbgpu
        from tools.synth import Dataset
        dist.init_process_group("gloo")
        rank, world = dist.get_rank(), dist.get_world_size()
        ds = Dataset("small", seed=7)
        pseqs = ds.pb_seqs()
        ix = pbgpu.Index.from_records(ds.sr_names(), ds.sr_seqs(), 17, shard=rank, n_shards=world)
        al = pbgpu.Aligner(ix, k=17)
        rr = al.upload(pseqs)
        n = sum(len(s) for s in pseqs)
        al.shard_counts(rr)
        h = torch.from_numpy(al.counts_download(n).astype(np.int64))
        dist.all_reduce(h)                       # SUM of the saturated per-shard counts
        al.counts_upload(h.numpy().astype(np.uint32))
        al.align_resident_shard(rr)
        co = al.download()
        mine = (co.records, co.read_offsets, co.kmers_info, co.bases_info)
        allp = [None] * world
        dist.all_gather_object(allp, mine)
        if rank == 0:
            keep, ptrs = [], []
            for recs, off, km, kb in allp:
                recs = np.ascontiguousarray(recs); off = np.ascontiguousarray(off, dtype=np.uint64)
                km = np.ascontiguousarray(km if len(km) else np.zeros(1, np.int32), dtype=np.int32)
                kb = np.ascontiguousarray(kb if len(kb) else np.zeros(1, np.int32), dtype=np.int32)
                keep += [recs, off, km, kb]
                b = pbgpu.CoordsBatch(len(off) - 1, len(recs), off.ctypes.data_as(C.POINTER(C.c_uint64)),
                                      recs.ctypes.data if len(recs) else None, len(km),
                                      km.ctypes.data_as(C.POINTER(C.c_int32)), kb.ctypes.data_as(C.POINTER(C.c_int32)))
                keep.append(b); ptrs.append(C.pointer(b))
            arr = (C.POINTER(pbgpu.CoordsBatch) * world)(*ptrs)
            o = C.POINTER(pbgpu.CoordsBatch)()
            pbgpu._check(pbgpu.lib().pbgpu_coords_merge(arr, world, C.byref(o)))
            txt = pbgpu.Coords(o).format(ix, ds.pb_names(), [len(s) for s in pseqs])
            open({str(out)!r}, "w").write(txt)
        dist.barrier()
    """))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE="2")
    procs = [subprocess.Popen([sys.executable, str(script)], env=dict(env, RANK=str(r), LOCAL_RANK="0"),
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(2)]
    outs = [p.communicate(timeout=200) for p in procs]
    assert all(p.returncode == 0 for p in procs), outs
    assert_same_coords(out.read_text(), exp, "two ranks")

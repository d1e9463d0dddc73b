"""C5 (BASELINE configs[4]): the whole-human workload on one
MI355X, index sharded by super-read range and the shards run one after another.

* 50M synthetic super-reads (~62 Gbp of text) over a 3.1 Gbp genome with the
  C4 repeat model; a sample of C5 PacBio reads (15 kb N50).  The super-reads
  are handed over as pointers into the generator's buffers (no FASTA).
* Pass 1, shard by shard: build the shard, its saturated k-mer counts of every
  read base (pbgpu_shard_counts), download, free.  The counts are summed on
  the host (the all-reduce of an S-GPU run).
* Pass 2, shard by shard (the last shard of pass 1 is still resident and goes
  first): build the shard again, upload the summed counts, align
  (pbgpu_align_resident_shard), download the records, free.
* pbgpu_coords_merge of the S batches, formatted with a shard's (global) names.

No whole index fits one GPU, so there is no byte comparison here (the C4
sharded-vs-whole test in test_gpu_scale.py is that pin); the checks are
size-independent: per-read (rs, re, ql) order, record invariants against the
super-read and read lengths, the shards tiling the super-reads, and the summed
counts within the saturation bound.

PBGPU_C5_SHARDS (default 16) and PBGPU_C5_READS (default 1000) size the run;
PBGPU_TEST_OUT names a directory for the per-phase timings (c5_timings.json)."""
import json
import os
import threading
import time

import numpy as np
import pytest

from tests._compare import assert_read_order
from tests.test_gpu_scale import _check_invariants, check_records

# the run takes ~370-400 s on one MI355X (31 shard builds): a per-test limit of its own,
# above that, so a runner's shorter --timeout does not kill it inside a shard's free
pytestmark = [pytest.mark.gpu, pytest.mark.timeout(1200)]

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

KW = dict(k=17, forward=True, unitigs_k=31, bases_matching=15.0, max_count=5000, stretch_cap=10000.0)


def test_c5_whole_human_sharded_one_gpu():
    S = int(os.environ.get("PBGPU_C5_SHARDS", "16"))
    n_reads = int(os.environ.get("PBGPU_C5_READS", "1000"))
    threads = int(os.environ.get("OMP_NUM_THREADS", "16"))
    T = {"shards": S, "reads": n_reads, "threads": threads}
    t0 = time.time()
    # progress and a heartbeat every 20 s into gpurun_out/ (or PBGPU_TEST_OUT): pytest
    # holds the test's own output, and a GPU run silent for minutes is taken to be hung
    out = os.environ.get("PBGPU_TEST_OUT") or os.path.join(ROOT, "gpurun_out")
    os.makedirs(out, exist_ok=True)
    plog = os.path.join(out, "c5_progress.log")
    last = ["start"]

    def progress(msg):
        last[0] = msg
        line = f"{time.time() - t0:8.1f}s {msg}"
        print(line, flush=True)
        with open(plog, "a") as f:
            f.write(line + "\n")
    done = threading.Event()

    def heartbeat():
        while not done.wait(20):
            with open(plog, "a") as f:
                f.write(f"{time.time() - t0:8.1f}s ... ({last[0]})\n")
    hb = threading.Thread(target=heartbeat, daemon=True)
    hb.start()
    try:
        _run(S, n_reads, threads, T, t0, out, progress)
    finally:
        done.set()
        hb.join()


def _run(S, n_reads, threads, T, t0, out, progress):
    from pacbio_amd import pbgpu
    from tools.synth import Dataset
    progress("generating C5")
    ds = Dataset("C5", seed=42, threads=threads, n_pb=n_reads)
    T["generate_s"] = time.time() - t0
    progress(f"generated: {ds.sr.n} super-reads")
    sr_off = np.ctypeslib.as_array(ds.sr.off, shape=(ds.sr.n + 1,))
    T["sr_text_bases"] = int(sr_off[-1])
    assert ds.sr.n == 50_000_000 and sr_off[-1] > 5e10
    ptrs = ds.sr_pointers()
    pn, ps = ds.pb_names(), ds.pb_seqs()
    lens = [len(s) for s in ps]
    nb = sum(lens)
    T["read_bases"] = nb

    def build(s):
        t = time.time()
        ix = pbgpu.Index.from_pointers(*ptrs, k=17, shard=s, n_shards=S)
        return ix, time.time() - t

    total = np.zeros(nb, np.uint64)
    infos, t_build1, t_count = [], [], []
    keep = None
    for s in range(S):
        ix, tb = build(s)
        t_build1.append(tb)
        infos.append(ix.info())
        t = time.time()
        al = pbgpu.Aligner(ix, unitig_lengths=ds.unitig_lengths, **KW)
        rd = al.upload(ps, names=pn)
        al.shard_counts(rd)
        total += al.counts_download(nb)
        rd.close()
        al.close()
        t_count.append(time.time() - t)
        t = time.time()
        if s == S - 1:
            keep = ix  # still resident: pass 2 starts with it
        else:
            ix.close()
        progress(f"pass 1 shard {s}: build {tb:.1f}s, counts {t_count[-1]:.1f}s, free {time.time() - t:.1f}s, "
                 f"{infos[-1]['device_bytes'] / 1e9:.1f} GB")
    T["pass1_build_s"], T["pass1_count_s"] = t_build1, t_count
    T["shard_info"] = [{k: v for k, v in i.items()} for i in infos]
    assert infos[0]["sr_begin"] == 0 and infos[-1]["sr_end"] == 50_000_000
    assert all(infos[i]["sr_end"] == infos[i + 1]["sr_begin"] for i in range(S - 1))
    assert sum(i["text_len"] for i in infos) >= sr_off[-1]  # + the k - 1-base seams
    # every shard's count is saturated at max_count + 1 before the sum
    assert total.max() <= S * (KW["max_count"] + 1)
    # repeat content: 5-50 copies at ~20x super-read coverage
    assert total.max() > 200, "no repeat content in the sample"
    T["max_summed_count"] = int(total.max())
    T["kmers_over_max_count"] = int((total > KW["max_count"]).sum())
    counts = total.astype(np.uint32)

    parts = [None] * S
    t_build2, t_align = [], []
    names_ix = None
    for s in reversed(range(S)):
        if s == S - 1:
            ix = keep
        else:
            ix, tb = build(s)
            t_build2.append(tb)
        t = time.time()
        al = pbgpu.Aligner(ix, unitig_lengths=ds.unitig_lengths, **KW)
        rd = al.upload(ps, names=pn)
        al.counts_upload(counts)
        al.align_resident_shard(rd)
        parts[s] = al.download()
        rd.close()
        al.close()
        t_align.append(time.time() - t)
        progress(f"pass 2 shard {s}: align {t_align[-1]:.1f}s, {parts[s].n_records} records")
        if s == 0:
            names_ix = ix  # names are global in every shard
        else:
            ix.close()
    T["pass2_build_s"], T["pass2_align_s"] = t_build2, t_align
    t = time.time()
    merged = pbgpu.merge_coords(parts)
    text = merged.format(names_ix, pn, lens)
    T["merge_format_s"] = time.time() - t
    names_ix.close()
    T["records"] = int(merged.n_records)
    T["total_s"] = time.time() - t0
    with open(os.path.join(out, "c5_timings.json"), "w") as f:
        json.dump(T, f, indent=1)
    print(json.dumps({k: v for k, v in T.items() if k != "shard_info"}))

    assert_read_order(text, "C5")
    read_len = {(n.decode() if isinstance(n, bytes) else n): len(s) for n, s in zip(pn, ps)}
    n = _check_invariants(text, 17, read_len)
    assert n == merged.n_records
    assert n > 100 * len(ps), "C5 sample produced too few records"
    assert check_records(merged, np.diff(sr_off.astype(np.int64)), lens) == n
    ds.close()

"""Find reads whose GPU coords differ from the oracle's (C2 workload, production flags)."""
import sys
sys.path.insert(0, ".")
from tools.synth import Dataset
from oracle.oracle import OracleIndex, params
from pacbio_amd import pbgpu
from tests._compare import split_reads

n = int(sys.argv[1]) if len(sys.argv) > 1 else 14433
ds = Dataset("C2", seed=42, threads=16, n_pb=n)
kw = dict(k=17, forward=True, unitigs_k=31, unitig_lengths=ds.unitig_lengths, bases_matching=15.0, max_count=5000,
          stretch_cap=10000.0)
names, seqs = ds.sr_names(), ds.sr_seqs()
pn, ps = ds.pb_names(), ds.pb_seqs()
gix = pbgpu.Index.from_records(names, seqs, 17)
al = pbgpu.Aligner(gix, **kw)
rd = al.upload(ps, names=pn)
al.align_resident(rd)
got = al.format_device(rd)
host = al.download().format(gix, pn, [len(s) for s in ps])
print("device == host text:", got == host)
oix = OracleIndex.from_records(names, seqs, 17, threads=16)
exp = oix.align_format(params(**kw), pn, ps, threads=16)
og, rg = split_reads(got)
oe, re_ = split_reads(exp)
print("reads gpu", len(og), "oracle", len(oe))
bad = [h for h in sorted(set(og) | set(oe)) if sorted(rg.get(h, [])) != sorted(re_.get(h, []))]
print("differing reads:", len(bad))
for h in bad[:5]:
    a, b = set(rg.get(h, [])), set(re_.get(h, []))
    print("READ", h, "gpu", len(rg.get(h, [])), "oracle", len(re_.get(h, [])))
    for x in sorted(a - b)[:6]:
        print("  only gpu   :", x)
    for x in sorted(b - a)[:6]:
        print("  only oracle:", x)
    # single-read re-run: does it reproduce alone?
    i = pn.index(h.split()[1].encode()) if isinstance(pn[0], bytes) else pn.index(h.split()[1])
    g1 = pbgpu.Aligner(gix, **kw).align([ps[i]]).format(gix, [pn[i]], [len(ps[i])])
    e1 = oix.align_format(params(**kw), [pn[i]], [ps[i]], threads=1)
    print("  alone: gpu==oracle", sorted(g1.splitlines()) == sorted(e1.splitlines()))

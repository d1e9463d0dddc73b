"""One C2 read through the GPU and the oracle with --details: compare the hit
lists and lis marks of the super-reads whose records differ."""
import sys
sys.path.insert(0, ".")
from tools.synth import Dataset
from oracle.oracle import OracleIndex, params
from pacbio_amd import pbgpu

ri = int(sys.argv[1])
ds = Dataset("C2", seed=42, threads=16, n_pb=ri + 1)
kw = dict(k=17, forward=True, unitigs_k=31, unitig_lengths=ds.unitig_lengths, bases_matching=15.0, max_count=5000,
          stretch_cap=10000.0)
names, seqs = ds.sr_names(), ds.sr_seqs()
pn, ps = ds.pb_names()[ri:ri + 1], ds.pb_seqs()[ri:ri + 1]
gix = pbgpu.Index.from_records(names, seqs, 17)
al = pbgpu.Aligner(gix, **kw)
al.set_details(True)
got = al.align(ps).format(gix, pn, [len(ps[0])])
gdet = al.download_details().format(gix, pn)
oix = OracleIndex.from_records(names, seqs, 17, threads=16)
exp, edet = oix.align_format(params(**kw), pn, ps, threads=1, details=True)
ga, ea = set(got.splitlines()), set(exp.splitlines())
srs = set()
for l in (ga ^ ea):
    t = l.split()
    if len(t) > 14:
        srs.add(t[14])
print("differing record SR names:", srs)
gd = {l.split()[1]: l for l in gdet.splitlines()}
ed = {l.split()[1]: l for l in edet.splitlines()}
print("details lists: gpu", len(gd), "oracle", len(ed), "same keys", set(gd) == set(ed))
ndiff = 0
for k in sorted(set(gd) | set(ed)):
    if gd.get(k) != ed.get(k):
        ndiff += 1
        if ndiff <= 4:
            a, b = gd.get(k, "").split()[2:], ed.get(k, "").split()[2:]
            print("LIST", k, "gpu", len(a), "oracle", len(b))
            strip = lambda x: x.strip("[]")
            print("  same hits:", [strip(x) for x in a] == [strip(x) for x in b])
            for i, (x, y) in enumerate(zip(a, b)):
                if x != y:
                    print("  first diff at", i, ":", a[max(0, i - 3):i + 6], "vs", b[max(0, i - 3):i + 6])
                    break
print("lists differing:", ndiff)

"""Find reads whose GPU coords differ from the oracle's (C2 workload, production flags)."""
import sys
sys.path.insert(0, ".")
from tools.synth import Dataset
from oracle.oracle import OracleIndex, params
from pacbio_amd import pbgpu
from tests._compare import split_reads

n = int(sys.argv[1]) if len(sys.argv) > 1 else 14433
chunk = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
ds = Dataset("C2", seed=42, threads=16, n_pb=n)
kw = dict(k=17, forward=True, unitigs_k=31, unitig_lengths=ds.unitig_lengths, bases_matching=15.0, max_count=5000,
          stretch_cap=10000.0)
names, seqs = ds.sr_names(), ds.sr_seqs()
PN, PS = ds.pb_names(), ds.pb_seqs()
gix = pbgpu.Index.from_records(names, seqs, 17)
oix = OracleIndex.from_records(names, seqs, 17, threads=16)
al = pbgpu.Aligner(gix, **kw)
tot_reads = tot_lines = 0
bad = []
for c0 in range(0, n, chunk):
    pn, ps = PN[c0:c0 + chunk], PS[c0:c0 + chunk]
    rd = al.upload(ps, names=pn)
    al.align_resident(rd)
    got = al.format_device(rd)
    rd.close()
    exp = oix.align_format(params(**kw), pn, ps, threads=16)
    og, rg = split_reads(got)
    oe, re_ = split_reads(exp)
    tot_reads += len(oe)
    tot_lines += exp.count("\n")
    bad += [(h, rg.get(h, []), re_.get(h, [])) for h in sorted(set(og) | set(oe))
            if sorted(rg.get(h, [])) != sorted(re_.get(h, []))]
    print(f"reads {c0}..{c0 + len(ps)}: {len(oe)} with records, {exp.count(chr(10))} lines, differing so far {len(bad)}",
          flush=True)
print(f"TOTAL reads {n}, reads with records {tot_reads}, text lines {tot_lines}, differing reads {len(bad)}")
for h, a, b in bad[:5]:
    a, b = set(a), set(b)
    print("READ", h)
    for x in sorted(a - b)[:6]:
        print("  only gpu   :", x)
    for x in sorted(b - a)[:6]:
        print("  only oracle:", x)

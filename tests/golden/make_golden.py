#!/usr/bin/env python3
"""Regenerate the golden fixtures under tests/golden/ (run in the build
container, where /root/reference exists and `make -C oracle ref` has built the
harnesses in oracle/_ref/).

Every expected value here comes from EXECUTING the reference's own sources
(via our harnesses in oracle/ref_harness/, compiled against /root/reference):
  lis_cases.json     lis_align::indices            (src_lis/lis_align.hpp)
  lsq_cases.json     least_square_2d               (src_jf_aligner/least_square_2d.hpp)
  encode_cases.json  compact_dna::copy_from_str    (src_psa/compact_dna.hpp)
  srname_cases.json  super_read_name parse/reverse (src_jf_aligner/super_read_name.cc)
  psa_cases.json     PSA::search hit sets + order  (src_psa/psa.hpp, mer_sa_imp.hpp)
  psa_fine_cases.json  the same for -F patterns shorter than max_size
The reference's own test data files (tests/aligner_output/*) are copied
verbatim as input/expected-output fixtures (aligner_output/).
"""
import json
import os
import random
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = os.path.join(ROOT, "oracle", "_ref")
REFSRC = "/root/reference"


def run(binary, stdin, *args):
    r = subprocess.run([os.path.join(REF, binary), *args], input=stdin, capture_output=True, text=True, check=True)
    return r.stdout


def lis_cases(rng):
    cases = []
    params = [(1, 0, 1.3, 10.0, 10000.0, 0, 1.3), (1, 0, 1.3, 10.0, 200.0, 0, 1.3), (2, 0, 1.3, 10.0, 10000.0, 0, 1.3),
              (3, 0, 1.3, 10.0, 10000.0, 0, 1.3), (5, 0, 5.0, 1.0, 1e9, 0, 5.0), (0, 0, 1.3, 10.0, 10000.0, 0, 1.3),
              (1, 1, 1.3, 10.0, 10000.0, 1, 1.3), (1, 0, 1.3, 10.0, 10000.0, 1, 1.3), (2, 1, 1.3, 10.0, 50.0, 0, 1.3)]
    for ci in range(400):
        W, mk, a, b, C, sk, sa = params[ci % len(params)]
        n = rng.choice([0, 1, 2, 3, 5, 8, 13, 30, 60, 120])
        X = []
        pb, sr = 1, rng.randint(-500, 500)
        style = ci % 4
        for _ in range(n):
            # chains with noise: diagonal steps, indels, repeats of the same pb, off-diagonal junk
            pb += rng.choice([0, 1, 1, 1, 2, 3, 7, 20])
            if style == 0:
                sr += rng.choice([1, 1, 1, 2, 0, -3, 15])
                X.append((pb, sr))
            elif style == 1:
                X.append((pb, rng.randint(-200, 200)))
            elif style == 2:
                sr += rng.choice([1, 1, 2, 3, 40, -1])
                X.append((pb, sr if rng.random() > 0.1 else sr - rng.randint(1, 100)))
            else:
                X.append((pb, pb * 2 + rng.randint(-3, 3)))
        cases.append({"W": W, "mer_all": mk, "a": a, "b": b, "C": C, "seq_all": sk, "seq_a": sa, "X": X})
    inp = "".join(f"{len(c['X'])} {c['W']} {c['mer_all']} {c['a']!r} {c['b']!r} {c['C']!r} {c['seq_all']} {c['seq_a']!r}\n"
                  + "".join(f"{x} {y}\n" for x, y in c["X"]) for c in cases)
    out = run("ref_lis", inp).splitlines()
    assert len(out) == len(cases)
    for c, line in zip(cases, out):
        v = [int(t) for t in line.split()]
        assert v[0] == len(v) - 1
        c["lis"] = v[1:]
    return cases


def lsq_cases(rng):
    cases = []
    for ci in range(200):
        n = rng.choice([1, 2, 3, 4, 10, 50, 200])
        a = rng.choice([1, 1, 1, -1]) * rng.uniform(0.9, 1.1)
        b = rng.randint(-3000, 3000)
        pts = []
        x = rng.randint(1, 2000)
        for _ in range(n):
            x += rng.randint(1, 20)
            pts.append((x, int(round(a * x + b)) + rng.randint(-5, 5)))
        cases.append({"pts": pts})
    inp = "".join(f"{len(c['pts'])}\n" + "".join(f"{x} {y}\n" for x, y in c["pts"]) for c in cases)
    out = run("ref_lsq", inp).splitlines()
    for c, line in zip(cases, out):
        c["hex"] = line.split()  # EX EY EXX EXY VX CXY NB a b
    return cases


def encode_cases(rng):
    alpha = "ACGTacgtNnRYKMSWBDHV-.*"
    lines = []
    for n in [0, 1, 3, 7, 8, 9, 15, 16, 17, 31, 32, 33, 40, 63, 64, 65, 70, 80, 100, 129]:
        for _ in range(3):
            lines.append("".join(rng.choice("ACGT" if rng.random() < 0.5 else alpha) for _ in range(n)))
    out = run("ref_encode", "".join(l + "\n" for l in lines)).splitlines()
    return [{"line": l, "codes": o} for l, o in zip(lines, out)]


def srname_cases(rng):
    names = ["", "1234F", "1234R", "1R_3F", "5F_4R_2F", "7R_2F", "17", "12F_7R some description", "abc",
             "12F_x", "_12F", "0F_1R_2F_3R_4F", "2147483647F_1R", "2147483648F", "99999999999F_1R", "12", "3R_",
             "42F_43F_44F_45F_46F_47F_48F_49F", "-5F_3R", "+7R"]
    for _ in range(30):
        k = rng.randint(1, 9)
        names.append("_".join(f"{rng.randint(0, 10**rng.randint(1, 7))}{rng.choice('FR')}" for _ in range(k)))
    out = run("ref_srname", "".join(n + "\n" for n in names)).split("\n")
    res = []
    for n, line in zip(names, out):
        cnt, rev, ids = line.split("\t")
        res.append({"name": n, "n": int(cnt), "bwd": rev, "ids": [int(t) for t in ids.split()] if ids else []})
    return res


def psa_cases(rng, k=17, min_size=13):
    genome = "".join(rng.choice("ACGT") for _ in range(3000))
    srs = []
    for i in range(40):
        s = rng.randint(0, len(genome) - 400)
        L = rng.randint(60, 400)
        seq = genome[s:s + L]
        if rng.random() < 0.5:
            seq = seq[::-1].translate(str.maketrans("ACGT", "TGCA"))
        srs.append((f"{i}F", seq))
    srs.append(("pal", "ACGTACGTACGTACGTACGTACGT"))  # palindromic k-mers for even k
    srs.append(("homo", "A" * 40 + "C" * 3 + "A" * 30))
    fa = os.path.join(HERE, "psa_sr.fa")
    with open(fa, "w") as f:
        for name, seq in srs:
            f.write(f">{name}\n")
            for p in range(0, len(seq), 60):
                f.write(seq[p:p + 60] + "\n")
    text = "".join(s for _, s in srs)
    queries = set()
    for _ in range(600):
        p = rng.randint(0, len(text) - k)
        q = text[p:p + k]
        queries.add(q)
        queries.add(q[::-1].translate(str.maketrans("ACGT", "TGCA")))
    for _ in range(100):
        queries.add("".join(rng.choice("ACGT") for _ in range(k)))
    queries.add("A" * k)
    queries = sorted(queries)
    out1 = run("ref_psa", "".join(q + "\n" for q in queries), fa, str(min_size), str(k), "1").splitlines()
    out4 = run("ref_psa", "".join(q + "\n" for q in queries), fa, str(min_size), str(k), "4").splitlines()
    assert out1 == out4, "hit order must not depend on the PSA build thread count for k > psa_min"
    res = []
    for q, line in zip(queries, out1):
        v = [int(t) for t in line.split()]
        res.append({"q": q, "count": v[0], "pos": v[1:]})
    return {"fasta": "psa_sr.fa", "k": k, "min_size": min_size, "cases": res}


def psa_fine_cases(rng, k=17, psa_min=13):
    """Short (-F) patterns: SA order of fine_k-mer matches in a PSA built the way
    jf_aligner.cc:202-203 builds it (min_size = min(fine_k, psa_min), max_size = k).
    Reuses psa_sr.fa (written by psa_cases) plus a text-end super-read so that
    matches whose k-base extension is truncated at the end of the text occur."""
    fa = os.path.join(HERE, "psa_fine_sr.fa")
    text = []
    with open(os.path.join(HERE, "psa_sr.fa")) as f, open(fa, "w") as o:
        for line in f:
            o.write(line)
            if not line.startswith(">"):
                text.append(line.strip())
        tail = "ACGTTGCAACGTAC" + "ACGTTGCAAC"  # the last 10 bases repeat 10 bases seen just before
        o.write(">tail\n" + tail + "\n")
        text.append(tail)
    text = "".join(text)
    out = {"fasta": "psa_fine_sr.fa", "k": k, "psa_min": psa_min, "sets": []}
    for fk in (11, 13, 15):
        queries = set()
        for _ in range(300):
            p = rng.randint(0, len(text) - fk)
            q = text[p:p + fk]
            queries.add(q)
            queries.add(q[::-1].translate(str.maketrans("ACGT", "TGCA")))
        for p in range(len(text) - fk - k, len(text) - fk + 1):
            queries.add(text[p:p + fk])
        queries.add("A" * fk)
        queries = sorted(queries)
        mn = min(fk, psa_min)
        o1 = run("ref_psa", "".join(q + "\n" for q in queries), fa, str(mn), str(k), "1").splitlines()
        o4 = run("ref_psa", "".join(q + "\n" for q in queries), fa, str(mn), str(k), "4").splitlines()
        assert o1 == o4, "fine hit order must not depend on the PSA build thread count"
        cases = []
        for q, line in zip(queries, o1):
            v = [int(t) for t in line.split()]
            cases.append({"q": q, "count": v[0], "pos": v[1:]})
        out["sets"].append({"fine_k": fk, "min_size": mn, "cases": cases})
    return out


def main():
    if not os.path.isdir(REF):
        sys.exit("oracle/_ref missing: run `make -C oracle ref` in the build container")
    rng = random.Random(20260101)
    for name, fn in [("lis_cases.json", lis_cases), ("lsq_cases.json", lsq_cases), ("encode_cases.json", encode_cases),
                     ("srname_cases.json", srname_cases), ("psa_cases.json", psa_cases)]:
        data = fn(rng)
        with open(os.path.join(HERE, name), "w") as f:
            json.dump(data, f, separators=(",", ":"))
        print(name, "ok")
    # added later with its own generator so the fixtures above stay byte-identical
    with open(os.path.join(HERE, "psa_fine_cases.json"), "w") as f:
        json.dump(psa_fine_cases(random.Random(20261016)), f, separators=(",", ":"))
    print("psa_fine_cases.json ok")
    dst = os.path.join(HERE, "aligner_output")
    os.makedirs(dst, exist_ok=True)
    for fn in ["test_super_reads.fa", "test_pacbio.fa", "test_unitigs_lengths", "coords_normal_expected",
               "coords_forward_expected", "details_normal_expected", "details_forward_expected"]:
        shutil.copyfile(os.path.join(REFSRC, "tests", "aligner_output", fn), os.path.join(dst, fn))
    print("aligner_output ok")
    copy_mega_reads_output()


def copy_mega_reads_output():
    """Inputs of the reference's tests/mega_reads_output (its Tupfile runs create_mega_reads on
    them; no expected mega-reads are held, and expect_coords is from an older aligner: the
    Tupfile's diff against it is commented out) -- data files, copied verbatim."""
    dst = os.path.join(HERE, "mega_reads_output")
    os.makedirs(dst, exist_ok=True)
    for fn in ["sr.fa", "pb.fa", "kUnitigLengths.txt"]:
        shutil.copyfile(os.path.join(REFSRC, "tests", "mega_reads_output", fn), os.path.join(dst, fn))
    print("mega_reads_output ok")


if __name__ == "__main__":
    main()

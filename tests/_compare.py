"""Coords text comparison with exactly the nondeterminism SURVEY A.10 allows:
records of one read may appear in any order (ties of (rs, re, ql) in the
reference); everything else byte-identical."""


def split_reads(text):
    reads, cur, order = {}, None, []
    for line in text.splitlines():
        if line.startswith(">"):
            cur = line
            order.append(cur)
            reads[cur] = []
        elif line.startswith("Rstart"):
            continue
        else:
            reads.setdefault(cur, []).append(line)
    return order, reads


def assert_read_order(text, ctx=""):
    """Records of each read must come out sorted by (rs, re, ql) (jf_aligner.cc:148-154)."""
    prev_name, prev_key = None, None
    for line in text.splitlines():
        if line.startswith(">"):
            prev_key = None
            continue
        if line.startswith("Rstart") or not line:
            continue
        t = line.split()
        off = sum(1 for x in t if ":" not in x) - 15  # 1 when the line starts with the read name
        if off:
            if t[0] != prev_name:
                prev_name, prev_key = t[0], None
        key = (int(t[off]), int(t[off + 1]), int(t[off + 10]))
        assert prev_key is None or key >= prev_key, f"{ctx}: records out of (rs, re, ql) order: {line}"
        prev_key = key


def assert_same_coords(got, exp, ctx=""):
    assert_read_order(got, ctx)
    if got == exp:
        return
    og, rg = split_reads(got)
    oe, re_ = split_reads(exp)
    assert og == oe, f"{ctx}: read header lines differ: {[x for x in og if x not in oe][:3]} vs {[x for x in oe if x not in og][:3]}"
    for h in oe:
        a, b = sorted(rg[h]), sorted(re_[h])
        if a != b:
            sa, sb = set(a), set(b)
            raise AssertionError(f"{ctx}: read {h}: {len(a)} vs {len(b)} records; only GPU: {sorted(sa - sb)[:3]}; "
                                 f"only oracle: {sorted(sb - sa)[:3]}")

"""The CPU restatement (oracle/) pinned against vectors produced by EXECUTING
the reference's own sources (tests/golden/make_golden.py) and against the
known-answer vectors of the reference's unit tests."""
import ctypes as C
import json
import os
import struct

import numpy as np
import pytest

from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


def test_lis_matches_reference_lis_align():
    # lis_align::indices executed on 400 seeded cases (window 0/1/2/3/5, caps, accept_all)
    for i, c in enumerate(_load("lis_cases.json")):
        got = O.lis(c["X"] if c["X"] else np.zeros((0, 2)), window=c["W"], a=c["a"], b=c["b"], cap=c["C"],
                    mer_all=c["mer_all"], seq_all=c["seq_all"], seq_a=c["seq_a"])
        assert got == c["lis"], f"case {i}: {got} != {c['lis']}"


@pytest.mark.parametrize("X,window,n,exp", [
    # tests/test_lis_align.cc:52-117 (affine_capped(5, 1, 1e9), linear(5))
    ([(1, 1), (3, 3), (4, 2), (5, 5), (7, 7)], 1, 5, [0, 1, 3, 4]),
    ([(1, 1), (2, 2), (3, 3), (10, 4)], 1, 4, None),
    ([(2, 2), (3, 3), (13, 4), (14, 5), (24, 6)], 2, 3, None),
    ([(2, 2), (3, 3), (13, 4), (14, 5), (24, 6)], 2, 4, None),
    ([(2, 2), (3, 3), (13, 4), (14, 5), (24, 6)], 2, 5, None),
    ([(1, 1), (2, 2), (3, 3), (14, 4), (16, 5)], 1, 5, None),
])
def test_lis_reference_unit_vectors(X, window, n, exp):
    got = O.lis(X[:n], window=window, a=5.0, b=1.0, cap=1e9, seq_a=5.0)
    sizes = {(1, 5, 0): 4, (1, 4, 1): 3, (2, 3, 2): 2, (2, 4, 3): 4, (2, 5, 4): 4, (1, 5, 5): 3}
    assert all(X[got[i]][1] < X[got[i + 1]][1] for i in range(len(got) - 1))
    if exp is not None:
        assert got == exp
    else:
        key = [k for k in sizes if k[0] == window and k[1] == n]
        assert len(got) in [sizes[k] for k in key]


def _hexd(h):
    return float.fromhex(h)


def test_least_square_matches_reference_bitwise():
    out = (C.c_double * 9)()
    for i, c in enumerate(_load("lsq_cases.json")):
        pts = np.array(c["pts"], dtype=np.float64)
        x = np.ascontiguousarray(pts[:, 0]); y = np.ascontiguousarray(pts[:, 1])
        O.lib().oracle_lsq(x.ctypes.data_as(C.POINTER(C.c_double)), y.ctypes.data_as(C.POINTER(C.c_double)),
                           len(pts), out)
        exp = [_hexd(h) for h in c["hex"]]
        for j in range(9):
            a, b = out[j], exp[j]
            assert struct.pack("<d", a) == struct.pack("<d", b) or (a != a and b != b), f"case {i} field {j}: {a} {b}"


def test_least_square_reference_unit_vectors():
    # tests/test_least_square_2d.cc:87 PerfectInt: y = x - 10
    x = np.arange(20, 120, dtype=np.float64); y = x - 10
    out = (C.c_double * 9)()
    O.lib().oracle_lsq(x.ctypes.data_as(C.POINTER(C.c_double)), y.ctypes.data_as(C.POINTER(C.c_double)), len(x), out)
    assert abs(out[7] - 1.0) < 1e-6 and abs(out[8] + 10.0) < 1e-6


def test_compact_dna_encoding_matches_reference():
    for c in _load("encode_cases.json"):
        line = c["line"].encode()
        codes = (C.c_uint8 * max(1, len(line)))()
        O.lib().oracle_encode_line(line, len(line), codes)
        assert "".join(str(codes[i]) for i in range(len(line))) == c["codes"], c["line"]


def test_super_read_names_match_reference():
    buf = C.create_string_buffer(1 << 16)
    for c in _load("srname_cases.json"):
        n = O.lib().oracle_sr_name_reverse(c["name"].encode(), buf, len(buf))
        assert n == c["n"], c
        assert buf.value.decode() == c["bwd"], c


def _code(s):
    m = 0
    for ch in s:
        m = (m << 2) | "ACGT".index(ch)
    return m


def test_index_lookup_matches_reference_psa():
    g = _load("psa_cases.json")
    ix = O.OracleIndex.from_fasta([os.path.join(GOLD, g["fasta"])], g["k"], threads=2)
    for c in g["cases"]:
        n, pos = ix.lookup(_code(c["q"]))
        assert n == c["count"], c["q"]
        assert pos == c["pos"], c["q"]  # descending text position == SA tie-break order


def test_fine_index_lookup_matches_reference_psa():
    """-F patterns shorter than max_size: the SA order within a match range is
    the order of the (k - fine_k)-base extension, a truncated extension first,
    then x descending (mer_sa_imp.hpp:351-364), executed from the reference."""
    g = _load("psa_fine_cases.json")
    for st in g["sets"]:
        ix = O.OracleIndex.from_fasta([os.path.join(GOLD, g["fasta"])], g["k"], threads=2).build_fine(st["fine_k"])
        for c in st["cases"]:
            n, pos = ix.lookup_fine(_code(c["q"]))
            assert n == c["count"], (st["fine_k"], c["q"])
            assert pos == c["pos"], (st["fine_k"], c["q"])
        ix.close()


# tests/test_kmers_info.cc:12-113 / 115-172 (known answers, unitigs_k=31, k=17)
KI_SIMPLE = [
    ("0F_1R_3F", [100, 100, 100], [20, 71, 85, 142, 170], [0, 0, 0, 0, 0], [0, 0, 0, 0, 0], "bad"),
]


def _kinfo(name, ul, pos):
    ul = np.array(ul, np.int32)
    pos = np.array(pos, np.int32)
    m = (C.c_int32 * 64)(); b = (C.c_int32 * 64)()
    n = O.lib().oracle_kmers_info(name.encode(), ul.ctypes.data_as(C.POINTER(C.c_int32)), len(ul), 31, 17,
                                  pos.ctypes.data_as(C.POINTER(C.c_int32)), len(pos), m, b, 64)
    return [m[i] for i in range(n)], [b[i] for i in range(n)]


@pytest.mark.parametrize("name,ul,steps", [
    ("0F_1R_3F", [100, 100, 100], [(20, [1, 0, 0, 0, 0], [17, 0, 0, 0, 0]), (71, [2, 1, 1, 0, 0], [34, 17, 17, 0, 0]),
                                   (85, [2, 1, 2, 0, 0], [47, 30, 31, 0, 0]), (142, [], []), (170, [], [])]),
    ("0F_1R_2F", [100, 100, 100], [(70, [1, 0, 0, 0, 0], [17, 16, 16, 0, 0]), (84, [2, 1, 1, 0, 0], [31, 30, 30, 0, 0]),
                                   (130, [2, 1, 2, 0, 0], [31, 30, 47, 6, 6]), (150, [2, 1, 3, 1, 1], [31, 30, 64, 23, 23]),
                                   (165, [2, 1, 3, 1, 2], [31, 30, 68, 27, 38])]),
    ("0F_1R_2F_3R_4F", [100, 31, 31, 40, 100], [
        (70, [1, 0, 0, 0, 0, 0, 0, 0, 0], [17, 16, 16, 15, 15, 14, 14, 4, 4]),
        (71, [2, 1, 1, 0, 0, 0, 0, 0, 0], [18, 17, 17, 16, 16, 15, 15, 5, 5]),
        (72, [3, 2, 2, 1, 1, 0, 0, 0, 0], [19, 18, 18, 17, 17, 16, 16, 6, 6]),
        (73, [4, 3, 3, 2, 2, 1, 1, 0, 0], [20, 19, 19, 18, 18, 17, 17, 7, 7]),
        (74, [5, 4, 4, 3, 3, 2, 2, 0, 0], [21, 20, 20, 19, 19, 18, 18, 8, 8]),
        (82, [6, 5, 5, 4, 4, 3, 3, 0, 0], [29, 28, 28, 27, 27, 26, 26, 16, 16]),
        (83, [7, 6, 6, 5, 5, 4, 4, 1, 1], [30, 29, 29, 28, 28, 27, 27, 17, 17]),
        (84, [8, 7, 7, 6, 6, 5, 5, 2, 2], [31, 30, 30, 29, 29, 28, 28, 18, 18]),
        (85, [8, 7, 8, 7, 7, 6, 6, 3, 3], [31, 30, 31, 30, 30, 29, 29, 19, 19]),
        (86, [8, 7, 8, 7, 8, 7, 7, 4, 4], [31, 30, 31, 30, 31, 30, 30, 20, 20]),
        (87, [8, 7, 8, 7, 8, 7, 8, 5, 5], [31, 30, 31, 30, 31, 30, 31, 21, 21]),
        (96, [8, 7, 8, 7, 8, 7, 9, 6, 6], [31, 30, 31, 30, 31, 30, 40, 30, 30]),
        (97, [8, 7, 8, 7, 8, 7, 9, 6, 7], [31, 30, 31, 30, 31, 30, 40, 30, 31]),
        (166, [8, 7, 8, 7, 8, 7, 9, 6, 8], [31, 30, 31, 30, 31, 30, 40, 30, 48]),
        (167, [], [])]),
])
def test_kmers_info_reference_vectors(name, ul, steps):
    pos = []
    for p, em, eb in steps:
        pos.append(p)
        m, b = _kinfo(name, ul, pos)
        assert (m, b) == (em, eb), (name, pos)


def test_compute_coords_info_reference_vectors():
    # tests/test_compute_coords_info.cc:6-30 (k=13, unitigs_k=70, forward)
    ul = np.array([50], np.int32)
    for fwd, lis, (st, off, err) in [([(10, 20)], [0], (1.0, -10.0, 0.0)),
                                     ([(10, 20), (11, 21), (12, 22), (13, 23)], [0, 1, 2, 3], (1.0, -10.0, 0.0))]:
        f = np.array(fwd, np.int32).reshape(-1); L = np.array(lis, np.uint32)
        rec = O.OracleRecord()
        O.lib().oracle_coords_info(b"1F", 50, f.ctypes.data_as(C.POINTER(C.c_int32)), len(fwd),
                                   L.ctypes.data_as(C.POINTER(C.c_uint32)), len(lis), None, 0, None, 0, 50, 13, 70,
                                   ul.ctypes.data_as(C.POINTER(C.c_int32)), 1, 1, C.byref(rec))
        assert abs(rec.stretch - st) < 1e-6 and abs(rec.offset - off) < 1e-6 and abs(rec.avg_err - err) < 1e-6

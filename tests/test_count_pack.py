"""The sharded-index count exchange packs two saturated per-shard counts into
one ncclUint32 (pacbio_amd/csrc/count_pack.h) when
n_ranks * (max_count + 1) < 65536.  CPU check of pack -> u32 sum -> unpack at
that boundary: exact below it, and a packed sum past it would carry between
the halves (which is why the all-reduce falls back to u32 there)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("cp") / "count_pack_test")
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", out, os.path.join(ROOT, "tests", "cpp", "count_pack_test.cpp")],
                   check=True)
    return out


def _run(exe, ranks, max_count, n, seed=1):
    return subprocess.run([exe, str(ranks), str(max_count), str(n), str(seed)], capture_output=True, text=True,
                          check=True).stdout.split()


@pytest.mark.parametrize("ranks,max_count,n", [
    (1, 5000, 1), (2, 5000, 7), (8, 5000, 10001),   # the production flags on 1-8 shards
    (13, 5040, 4096),                               # 13 * 5041 = 65533: the largest packed sum
    (16, 4094, 999),                                # 16 * 4095 = 65520
    (3, 21844, 12),                                 # 3 * 21845 = 65535: exactly at the limit
])
def test_packed_sum_exact_below_limit(exe, ranks, max_count, n):
    assert _run(exe, ranks, max_count, n) == ["ok", "1"]


@pytest.mark.parametrize("ranks,max_count", [(16, 4095), (2, 32767), (9, 8000)])
def test_limit_refuses_packing_where_a_half_can_carry(exe, ranks, max_count):
    # ranks * (max_count + 1) >= 65536: not packed; a packed sum of saturated counts would be wrong
    r = _run(exe, ranks, max_count, 5000)
    assert r[1] == "0"
    assert r[0] == "mismatch"

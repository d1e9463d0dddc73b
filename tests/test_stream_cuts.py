"""pbgpu.stream_cuts: how StreamAligner cuts a batch into contiguous read
ranges of about equal bases (host logic, no GPU)."""
import numpy as np
import pytest

from pacbio_amd.pbgpu import stream_cuts


def _off(lens):
    off = np.zeros(len(lens) + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    return off


@pytest.mark.parametrize("S", [1, 2, 3, 4, 7])
def test_cuts_cover_in_order(S):
    rng = np.random.default_rng(S)
    lens = rng.integers(1, 30000, size=1000)
    off = _off(lens)
    c = stream_cuts(off, S)
    assert c[0] == 0 and c[-1] == len(lens) and len(c) == S + 1
    assert all(a <= b for a, b in zip(c, c[1:]))
    parts = [int(off[b] - off[a]) for a, b in zip(c, c[1:])]
    assert sum(parts) == int(off[-1])
    assert max(parts) - min(parts) <= 2 * int(lens.max())  # about equal bases


def test_cuts_more_streams_than_reads():
    off = _off([100, 5])
    c = stream_cuts(off, 4)
    assert c[0] == 0 and c[-1] == 2 and all(a <= b for a, b in zip(c, c[1:]))
    assert sum(1 for a, b in zip(c, c[1:]) if b > a) <= 2


def test_cuts_empty_batch():
    assert stream_cuts(_off([]), 3) == [0, 0, 0, 0]

"""The C3 strong-scaling leg's read split (bench.py strong_split): for every rank
count the ranks' ranges tile the read set in order, and the reads each rank
generates for its range are exactly that slice of the one-rank read set, so the
ranks' outputs concatenated in rank order are the one-GPU output (the
reference's split-and-cat, mega_reads_assemble_cluster2.sh:325-354,447)."""
import pytest


@pytest.mark.parametrize("n_total", [1, 7, 300, 300_000])
@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_strong_split_tiles_the_reads(n_total, world):
    from bench import strong_split
    ranges = [strong_split(n_total, world, r) for r in range(world)]
    assert ranges[0][0] == 0 and ranges[-1][1] == n_total
    for (a0, a1), (b0, b1) in zip(ranges, ranges[1:]):
        assert a1 == b0
    sizes = [hi - lo for lo, hi in ranges]
    assert max(sizes) - min(sizes) <= 1


@pytest.mark.parametrize("world", [2, 3])
def test_rank_reads_are_the_slice(world):
    from bench import strong_split
    from tools.synth import Dataset
    n = 40
    whole = Dataset("small", seed=9, n_pb=n)
    seqs, names = whole.pb_seqs(), whole.pb_names()
    got_seqs, got_names = [], []
    for r in range(world):
        lo, hi = strong_split(n, world, r)
        d = Dataset("small", seed=9, n_pb=hi - lo, pb_index_base=lo)
        got_seqs += d.pb_seqs()
        got_names += d.pb_names()
        d.close()
    assert got_seqs == seqs and got_names == names
    # the super-reads do not depend on the read range
    d = Dataset("small", seed=9, n_pb=3, pb_index_base=17)
    assert d.sr_seqs() == whole.sr_seqs()

"""The order-free rules k_mega (pacbio_amd/csrc/pbgpu_kernels.hip) uses in place of
the reference's serial loops, checked against those loops on random inputs (CPU):

- per-root best: overlap_graph.cc:130-150 folds the candidates of a root in order,
  replacing the current one on a strictly larger (lpath, density); the kernel takes
  the first candidate with the largest pair, tested pairwise;
- tile_greedy's interval set (overlap_graph.cc:163-197, boost::icl::interval_set of
  right-open intervals): inserting [lo, hi) replaces exactly the stored intervals
  [s0, e) with s0 = #{y < lo}, e = #{x <= hi}, by l2 = min(lo, x[s0]),
  h2 = max(hi, y[e - 1]);
- the tiling order: the reference's stable insertion sort equals ranking each
  element by #{smaller key} + #{equal key, earlier}.
"""
import math
import random


def fold_best(cands):
    """The reference's fold per root: cands = [(root, lpath, density)] in order."""
    best = {}
    for c, (root, lp, d) in enumerate(cands):
        if root not in best:
            best[root] = c
        else:
            _, blp, bd = cands[best[root]]
            if lp > blp or (lp == blp and d > bd):
                best[root] = c
    return best


def pairwise_best(cands):
    """The kernel's winner test: no candidate of the root is larger, none earlier is equal."""
    best = {}
    for c, (root, lp, d) in enumerate(cands):
        win = True
        for e, (r2, lp2, d2) in enumerate(cands):
            better = lp2 > lp or (lp2 == lp and d2 > d)
            tie_before = lp2 == lp and d2 == d and e < c
            if r2 == root and (better or tie_before):
                win = False
        if win:
            assert root not in best
            best[root] = c
    return best


def test_per_root_best_matches_fold():
    rng = random.Random(7)
    dens = [0.0, -0.0, 0.5, 0.5, 1.0, math.inf, 2.0 / 3.0]
    for _ in range(3000):
        n = rng.randint(1, 40)
        cands = [(rng.randint(0, 6), rng.randint(0, 4), rng.choice(dens)) for _ in range(n)]
        assert pairwise_best(cands) == fold_best(cands)


def serial_add(cov, lo, hi):
    """IntervalSet::add as k_mega's serial restatement (and overlap_graph.cpp) does it."""
    s0 = 0
    while s0 < len(cov) and cov[s0][1] < lo:
        s0 += 1
    e = s0
    l2, h2 = lo, hi
    while e < len(cov) and cov[e][0] <= h2:
        l2 = min(l2, cov[e][0])
        h2 = max(h2, cov[e][1])
        e += 1
    return cov[:s0] + [(l2, h2)] + cov[e:]


def count_add(cov, lo, hi):
    s0 = sum(1 for x, y in cov if y < lo)
    e = sum(1 for x, y in cov if x <= hi)
    l2, h2 = lo, hi
    if e > s0:
        l2 = min(lo, cov[s0][0])
        h2 = max(hi, cov[e - 1][1])
    return cov[:s0] + [(l2, h2)] + cov[e:]


def test_interval_insert_by_counts_matches_serial():
    rng = random.Random(11)
    for _ in range(2000):
        cov_a, cov_b = [], []
        for _ in range(rng.randint(1, 30)):
            lo = float(rng.randint(0, 200))
            hi = lo + float(rng.randint(1, 40))
            cov_a = serial_add(cov_a, lo, hi)
            cov_b = count_add(cov_b, lo, hi)
            assert cov_a == cov_b
            # the invariant the counts rely on: sorted, non-empty, strict gaps
            for (x0, y0), (x1, y1) in zip(cov_a, cov_a[1:]):
                assert x0 < y0 < x1 < y1


def test_stable_rank_equals_insertion_sort():
    rng = random.Random(3)
    for _ in range(2000):
        keys = [rng.choice([-3.0, -1.0, 0.0, -0.0, 2.5, math.inf]) for _ in range(rng.randint(0, 25))]
        order = list(range(len(keys)))
        for x in range(1, len(order)):  # the reference's stable insertion sort by key
            v, y = order[x], x
            while y > 0 and keys[v] < keys[order[y - 1]]:
                order[y] = order[y - 1]
                y -= 1
            order[y] = v
        ranked = [None] * len(keys)
        for t, k in enumerate(keys):
            rank = sum(1 for u, k2 in enumerate(keys) if k2 < k or (k2 == k and u < t))
            ranked[rank] = t
        assert ranked == order

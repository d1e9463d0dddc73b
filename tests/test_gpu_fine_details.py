"""GPU --details and fine aligner (-F) against the reference's own golden
files and against the CPU restatement (oracle/) on synthetic workloads.

--details: print_details (jf_aligner.cc:72-108), lines compared sorted (the
reference iterates an unordered_map).
-F: fine_aligner (fine_aligner.cc:7-51): coords compared per read with the
oracle, plus the properties of the reference's compare_coarse_fine_alignments
script on its own test inputs (tests/aligner_output/Tupfile:8-9)."""
import os
import subprocess
import tempfile

import pytest

from tests._compare import assert_same_coords
from tests.test_oracle_cli import fine_vs_coarse_properties

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden", "aligner_output")
CLI = os.path.join(ROOT, "pacbio_amd", "bin", "jf_aligner")
ORACLE = os.path.join(ROOT, "oracle", "pb_oracle")
FWD = ("-l", os.path.join(GOLD, "test_unitigs_lengths"), "-k", "65", "-f")


def _cli(exe, *extra, details=False):
    with tempfile.TemporaryDirectory() as d:
        dpath = os.path.join(d, "details")
        args = [exe, "-s", "10k", "-m", "17", "-r", os.path.join(GOLD, "test_super_reads.fa"), "-p",
                os.path.join(GOLD, "test_pacbio.fa"), "--stretch-cap", "200", "--no-compact", "--coords", "/dev/stdout"]
        if details:
            args += ["--details", dpath]
        r = subprocess.run(args + list(extra), capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        return r.stdout, (open(dpath).read() if details else None)


@pytest.mark.parametrize("extra,expected", [((), "details_normal_expected"), (FWD, "details_forward_expected")])
def test_gpu_details_match_reference_expected(extra, expected):
    _, det = _cli(CLI, *extra, details=True)
    assert sorted(det.splitlines()) == sorted(open(os.path.join(GOLD, expected)).read().splitlines())


def test_gpu_fine_reference_inputs():
    coarse, _ = _cli(CLI, *FWD)
    fine, _ = _cli(CLI, *FWD, "-F", "13")
    exp, _ = _cli(ORACLE, *FWD, "-F", "13")
    assert sorted(fine.splitlines()) == sorted(exp.splitlines())
    fine_vs_coarse_properties(coarse, fine)


@pytest.fixture(scope="module")
def small():
    from tools.synth import Dataset
    return Dataset("small", seed=7)


def _both(ds, k=17, fine_k=0, use_ul=False, details=False, budget=None, **cfg):
    from oracle.oracle import OracleIndex, params
    from pacbio_amd import pbgpu
    ul = ds.unitig_lengths if use_ul else None
    names, seqs = ds.sr_names(), ds.sr_seqs()
    pnames, pseqs = ds.pb_names(), ds.pb_seqs()
    oix = OracleIndex.from_records(names, seqs, k)
    if fine_k:
        oix.build_fine(fine_k)
    exp = oix.align_format(params(k=k, unitig_lengths=ul, fine_k=fine_k, **cfg), pnames, pseqs, threads=8,
                           details=details)
    oix.close()
    gix = pbgpu.Index.from_records(names, seqs, k, fine_k=fine_k)
    al = pbgpu.Aligner(gix, k=k, unitig_lengths=ul, fine_k=fine_k, **cfg)
    if budget:
        al.set_hit_budget(budget)
    if details:
        al.set_details(True)
    co = al.align(pseqs)
    got = co.format(gix, pnames, [len(s) for s in pseqs])
    if details:
        got = (got, al.download_details().format(gix, pnames))
    return got, exp, al.stats()


DETAIL_CONFIGS = {
    "default": dict(),
    "forward_ul": dict(forward=True, unitigs_k=31, use_ul=True, bases_matching=15.0),
    "max_match": dict(forward=True, max_match=True, unitigs_k=31, use_ul=True, bases_matching=10.0),
    "budget": dict(budget=200_000),
}


@pytest.mark.parametrize("name", list(DETAIL_CONFIGS))
def test_gpu_details_parity(small, name):
    (got, gdet), (exp, edet), _ = _both(small, details=True, **DETAIL_CONFIGS[name])
    assert_same_coords(got, exp, name)
    assert edet.count("\n") > 100
    assert sorted(gdet.splitlines()) == sorted(edet.splitlines())


FINE_CONFIGS = {
    "f13_forward_ul": dict(fine_k=13, forward=True, unitigs_k=31, use_ul=True, bases_matching=15.0),
    "f15_forward": dict(fine_k=15, forward=True),
    "f11_forward_maxmatch": dict(fine_k=11, forward=True, max_match=True, bases_matching=10.0),
    "f17_same_k": dict(fine_k=17, forward=True),
    "f13_not_forward": dict(fine_k=13),  # reverse windows are empty: nb_mers = 0 records (UB fields as 0)
    "f13_budget": dict(fine_k=13, forward=True, budget=300_000),
    "f16_k21": dict(fine_k=16, k=21, forward=True),
}


@pytest.mark.parametrize("name", list(FINE_CONFIGS))
def test_gpu_fine_parity(small, name):
    got, exp, st = _both(small, **FINE_CONFIGS[name])
    assert exp.count("\n") > 10
    assert st["n_fine_windows"] > 0 and st["n_fine_hits"] > 0
    assert_same_coords(got, exp, name)


@pytest.mark.parametrize("streams", ["1", "3"])
def test_gpu_cli_stream_pipeline_in_order(streams):
    """Batches pipelined over several aligners (--streams) come out in input
    order: many small batches give the same coords and details files as one."""
    one, d_one = _cli(CLI, *FWD, details=True)
    many, d_many = _cli(CLI, *FWD, "--batch-bases", "2k", "--streams", streams, details=True)
    assert many == one
    assert sorted(d_many.splitlines()) == sorted(d_one.splitlines())

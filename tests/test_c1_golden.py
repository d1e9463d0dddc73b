"""The C1 configuration's frozen outputs (tests/golden/c1, made by
tests/golden/make_c1_golden.py from the CPU restatement): the oracle must keep
producing them byte for byte (CPU), and the GPU CLI must produce them too (GPU),
for the default flags, the production flags, window 3 / cap 200 / -M 10 /
--max-match and -F 13."""
import os
import subprocess
import tempfile

import pytest

from tests.golden.make_c1_golden import VARIANTS, run, write_inputs

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden", "c1")


@pytest.fixture(scope="module")
def c1_dir():
    with tempfile.TemporaryDirectory() as d:
        write_inputs(d)
        yield d


def _check(exe, d, tmp_path, variant):
    out = str(tmp_path / (variant + ".coords"))
    run(exe, d, variant, out)
    got, want = open(out).read(), open(os.path.join(GOLD, variant + ".coords")).read()
    assert want.count("\n") > 500
    assert got == want


@pytest.mark.parametrize("variant", list(VARIANTS))
def test_oracle_reproduces_c1_golden(c1_dir, tmp_path, variant):
    _check(os.path.join(ROOT, "oracle", "pb_oracle"), c1_dir, tmp_path, variant)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", list(VARIANTS))
def test_gpu_cli_reproduces_c1_golden(c1_dir, tmp_path, variant):
    _check(os.path.join(ROOT, "pacbio_amd", "bin", "jf_aligner"), c1_dir, tmp_path, variant)

import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libpbgpu.so on cuda:0)")


def _built():
    need = [os.path.join(ROOT, "oracle", "liboracle.so"), os.path.join(ROOT, "tools", "libpbsynth.so")]
    if not all(os.path.exists(p) for p in need):
        from pacbio_amd import build
        build.build_oracle()
        build.build_tools()


_built()

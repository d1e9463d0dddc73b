"""The device coords formatter's %.6g (pacbio_amd/csrc/pbgpu_fmt.h), run on
the host through pbgpu_format_double, against glibc's printf("%.6g") -- what
std::ostream << double prints at the default precision (jf_aligner.cc:53-58).
No GPU needed: the same __host__ __device__ code runs on the device."""
import ctypes as C
import math
import random
import struct

import numpy as np
import pytest

from pacbio_amd import pbgpu

_libc = C.CDLL(None)
_libc.snprintf.restype = C.c_int


def glibc_g6(v):
    buf = C.create_string_buffer(64)
    _libc.snprintf(buf, 64, b"%.6g", C.c_double(v))
    return buf.value.decode()


def ours(v):
    L = pbgpu.lib()
    L.pbgpu_format_double.argtypes = [C.c_double, C.c_char_p]
    L.pbgpu_format_double.restype = C.c_int
    buf = C.create_string_buffer(64)
    n = L.pbgpu_format_double(v, buf)
    assert n == len(buf.value)
    return buf.value.decode()


def _check(vals):
    bad = []
    for v in vals:
        a, b = ours(v), glibc_g6(v)
        if a != b:
            bad.append((v, a, b))
    assert not bad, bad[:10]


def test_g6_known():
    vals = [0.0, -0.0, 1.0, -1.0, 0.5, 1.015625, 1.0078125, 2.5, 1234565.0, 1234575.0, 999999.5, 999999.4999,
            99999.95, 999995.0, 0.0001, 0.00001, 1e-5, 9.999995e-5, 0.000099999949, 123456.0, 1234567.0, 1e6, 1e21,
            1e22, 1e-22, 1e-23, 5e-324, 2.2250738585072014e-308, 1.7976931348623157e308, float("inf"),
            float("-inf"), float("nan"), -float("nan"), 3.14159265358979, 1.3, 10.0, 100.0, 0.1, 0.2, 0.3,
            1234.5, 12345.5, 123456.5, 654321.5, 0.123456789, 2 ** 63, 2 ** 64, 2 ** 80, -2.5e-10, 7.0e-15]
    _check(vals)


def test_g6_random_bits():
    rng = random.Random(1)
    vals = []
    for _ in range(20000):
        (v,) = struct.unpack("<d", struct.pack("<Q", rng.getrandbits(64)))
        vals.append(v)
    _check(vals)


def test_g6_alignment_range():
    """values like the records' stretch / offset / avg_err, ties and near-ties"""
    rng = np.random.default_rng(7)
    vals = list(rng.normal(1.0, 0.05, 5000)) + list(rng.uniform(-2e5, 2e5, 5000)) + \
        list(rng.exponential(3.0, 5000)) + list(rng.uniform(-1e7, 1e7, 2000))
    # exact binary values with 7+ significant digits ending in 5 (ties at digit 7)
    vals += [k / 2 ** j for k in range(1, 3000, 7) for j in (1, 3, 6, 10)]
    vals += [k + 0.5 for k in range(99990, 100010)] + [k + 0.5 for k in range(999990, 1000010)]
    # just around powers of ten
    for e in range(-30, 30):
        p = 10.0 ** e
        vals += [p, math.nextafter(p, 0), math.nextafter(p, math.inf), p * 0.9999995, p * 0.99999949999]
    _check([float(v) for v in vals])

"""MI355X-native jf_aligner hot path (alekseyzimin/PacBio coarse aligner).

The product is libpbgpu.so (HIP kernels + the C ABI of include/pbgpu.h) and
the CLI bin/jf_aligner; `pacbio_amd.pbgpu` is the ctypes binding used by the
tests and bench.py."""

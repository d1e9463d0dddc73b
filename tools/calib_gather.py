"""Launches the two gather microbenchmarks (pbgpu_measure_gather_shape) for PMC
calibration runs: FETCH_SIZE of k_gather_sectors / k_gather_runs vs the bytes
they move (tools/rocprof_summary.py)."""
import sys
sys.path.insert(0, ".")
from pacbio_amd import pbgpu
for unit in (64, 512):
    print(unit, round(pbgpu.measure_gather(0, 16 << 30, unit), 1), "GB/s")

"""k_group's occurrence-read shape for PMC calibration (round 6): runs the three modes of
pbgpu_measure_group_shape (pass 0's 4-B ids, pass 1's 8-B words, both passes) and prints
the known per-launch byte counts, so a rocprofv3 FETCH_SIZE pass over this script reads
as a calibration factor for exactly k_group's access pattern (tools/r06/pmc_group.sh)."""
import json
import sys
sys.path.insert(0, ".")
from pacbio_amd import pbgpu

out = [pbgpu.measure_group_shape(0, 32 << 30, m) for m in (0, 1, 2)]
print(json.dumps(out))

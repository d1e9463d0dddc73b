"""Round-3 k_group experiment variants (never shipped): tier-0 ms by tools/exp/ab_group_ms.sh."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pacbio_amd.build import build_pbgpu_variant

G = ["-DPBGPU_EXP_GROUP_ONLY"]
V = {
    "gonly": G,
    "p0": G + ["-DPBGPU_EXP_SKIP_PASS1"],
    "p0notab": G + ["-DPBGPU_EXP_SKIP_PASS1", "-DPBGPU_EXP_P0_NOTABLE"],
    "nostore": G + ["-DPBGPU_EXP_GROUP_NOSTORE"],
}
for n in (sys.argv[1:] or V):
    print(build_pbgpu_variant(n, V[n]))

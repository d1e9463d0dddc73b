#!/bin/bash
# Round 6: the split serial on the aligner's stream unless the 16-wave tier runs: C2 tier 0 and
# group stage, C4 / C4r group stage
O=gpurun_out/r06sd; mkdir -p gpurun_out/r06sd
source tools/r06/lib.sh
for rep in 1 2; do
  step c2_$rep 300 python3 -u tools/prof_lis.py --workload C2 --reads 50000
  echo "c2 $rep: $(grep 'stages ms\|tier0' $O/c2_$rep.out | tr '\n' ' ' | cut -c1-260)"
  step c4_$rep 400 python3 -u tools/prof_c4.py --reads 50000
  echo "c4 $rep: $(grep -v '^W2026\|^E2026\|^generate\|^per base\|^group' $O/c4_$rep.out | head -2 | tr '\n' ' ' | cut -c1-230)"
done
step c4r 300 python3 -u tools/prof_c4.py --preset C4r --reads 20000
echo "c4r: $(grep -v '^W2026\|^E2026\|^generate\|^per base\|^group' $O/c4r.out | head -2 | tr '\n' ' ' | cut -c1-230)"

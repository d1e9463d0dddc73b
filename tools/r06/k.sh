#!/bin/bash
# Round 6: the default bench line end to end (C2 legs, C4r, C3 strong, C4), then the bucket
# threshold A/B on C2 and C4.
O=gpurun_out/r06k; mkdir -p gpurun_out/r06k
source tools/r06/lib.sh
step bench 1000 python3 -u bench.py
head -c 1500 $O/bench.out; echo
for mp in 2 3 4 999; do
  PBGPU_GROUP_BUCKET_MINP=$mp step c2_mp$mp 300 python3 -u tools/prof_lis.py --workload C2 --reads 50000
done
for f in c2_mp2 c2_mp3 c2_mp4 c2_mp999; do echo "$f: $(grep -v '^W\|^E' $O/$f.out | tr '\n' ' ')"; done
cat $O/steps.txt

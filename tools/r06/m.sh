#!/bin/bash
# Round 6: bucket items in 2048-slot 4-wave blocks (default now) -- the bucketing threshold
# again (P >= 2 / 3) on C2, C4r, C4; C4 phase profile of k_coords.
O=gpurun_out/r06m; mkdir -p gpurun_out/r06m
source tools/r06/lib.sh
for mp in 2 3; do
  PBGPU_GROUP_BUCKET_MINP=$mp step c2_mp$mp 300 python3 -u tools/prof_lis.py --workload C2 --reads 50000
  PBGPU_GROUP_BUCKET_MINP=$mp step c4r_mp$mp 300 python3 -u tools/prof_c4.py --preset C4r --reads 20000
  PBGPU_GROUP_BUCKET_MINP=$mp step c4_mp$mp 400 python3 -u tools/prof_c4.py --reads 50000
done
PBGPU_LIB=pacbio_amd/libpbgpu_prof.so step c4p 500 python3 -u tools/prof_c4.py --reads 50000
for f in c2_mp2 c2_mp3; do echo "$f: $(grep -v '^W\|^E' $O/$f.out | tr '\n' ' ')"; done
for f in c4r_mp2 c4r_mp3 c4_mp2 c4_mp3; do echo "== $f: $(grep -v "^W2026\|^E2026\|^generate\|^per base\|^group" $O/$f.out | tr '\n' ' ')"; done
grep -v "^W2026\|^E2026" $O/c4p.out
cat $O/steps.txt

#!/bin/bash
# Host-side I/O probe on the GPU box (round 2): filesystems, page-cache write
# bandwidth, pinned D2H bandwidth, and the jf_aligner CLI end to end on C2.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
O=gpurun_out/probe_io.txt
{
  echo "== cpu"; lscpu | grep -E 'Model name|^CPU\(s\)|Thread|Socket|NUMA node\(s\)'; nproc
  echo "== fs"; df -hT /tmp /dev/shm "$GRAFT_REPO_ROOT" 2>&1
  echo "== mem"; free -g
} > $O 2>&1
timeout -k 10 120 tools/probe_write /tmp/pw.bin 4 1 2 4 8 16 >> $O 2>&1
timeout -k 10 120 tools/probe_write /dev/shm/pw.bin 4 1 4 16 >> $O 2>&1
echo "== generate C2" >> $O
mkdir -p /tmp/c2
t0=$EPOCHREALTIME
timeout -k 10 300 tools/pbsynth C2 /tmp/c2 42 >> $O 2>&1 || exit 1
echo "gen $(python3 -c "print($EPOCHREALTIME-$t0)") s" >> $O
ls -la /tmp/c2 >> $O
echo "== CLI C2 -t 16" >> $O
t0=$EPOCHREALTIME
timeout -k 10 600 pacbio_amd/bin/jf_aligner -s 1 -m 17 --psa-min 13 -t 16 \
  --coords /tmp/c2/out.coords -l /tmp/c2/ul.txt -k 31 -f -B 15 --max-count 5000 --stretch-cap 10000 \
  -r /tmp/c2/sr.fa -p /tmp/c2/pb.fa >> $O 2>&1
echo "cli $(python3 -c "print($EPOCHREALTIME-$t0)") s" >> $O
ls -la /tmp/c2/out.coords >> $O
head -c 3000 /tmp/c2/out.coords > gpurun_out/c2_coords_head.txt
wc -l /tmp/c2/out.coords >> $O
cat $O

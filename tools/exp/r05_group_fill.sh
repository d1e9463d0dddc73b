# round 5: the 8192-slot group tier at lower fill limits (more hash partitions) on C4r / C2
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in "" fill4 fill3 fill2; do
  L=pacbio_amd/libpbgpu.so; [ -n "$v" ] && L=pacbio_amd/libpbgpu_$v.so
  for w in C4r:20000 C2:50000; do
    echo "== ${v:-base} $w" >> gpurun_out/r05j_group_fill.txt
    PBGPU_LIB=$L timeout -k 10 300 python -u tools/prof_lis.py --workload ${w%%:*} --reads ${w##*:} >> gpurun_out/r05j_group_fill.txt 2>&1 || exit 1
  done
done

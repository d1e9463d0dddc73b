# round 5: reads past 8192 records on the device graph -- tests, then create_mega_reads on 20k C4r reads;
# the group tier variants (libpbgpu_g*.so) on C4r / C2 reads; one C2 create_mega_reads with its working set
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_mega_reads.py > gpurun_out/r05d_tests.log 2>&1 || { tail -30 gpurun_out/r05d_tests.log; exit 1; }
tail -2 gpurun_out/r05d_tests.log
timeout -k 10 300 python -u tools/prof_graph_gpu.py --workload C4r --reads 20000 > gpurun_out/r05d_graph_c4r.txt 2>&1 || exit 1
bash tools/exp/cmr_c4r.sh 20000 > gpurun_out/r05d_cmr_c4r.txt 2>&1 || exit 1
for v in "" g12b512 g12b256 g13b512; do
  L=pacbio_amd/libpbgpu.so; [ -n "$v" ] && L=pacbio_amd/libpbgpu_$v.so
  for w in C4r:20000 C2:50000; do
    echo "== ${v:-base} $w" >> gpurun_out/r05d_group_variants.txt
    PBGPU_LIB=$L timeout -k 10 300 python -u tools/prof_lis.py --workload ${w%%:*} --reads ${w##*:} >> gpurun_out/r05d_group_variants.txt 2>&1 || exit 1
  done
done

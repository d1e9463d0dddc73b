# round 5: bucketed group tables (libpbgpu_bucket.so) -- parity and C4r / C2 times; edges' lazy name loads
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
O=gpurun_out/r05m
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_mega_reads.py > ${O}_tests.log 2>&1 || { tail -30 ${O}_tests.log; exit 1; }
tail -1 ${O}_tests.log
PBGPU_LIB=pacbio_amd/libpbgpu_bucket.so timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_edge.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_fine_details.py > ${O}_bucket_tests.log 2>&1 || { tail -30 ${O}_bucket_tests.log; exit 1; }
tail -1 ${O}_bucket_tests.log
timeout -k 10 300 python -u tools/prof_graph_gpu.py --workload C4r --reads 20000 > ${O}_graph.txt 2>&1 || exit 1
for v in "" bucket; do
  L=pacbio_amd/libpbgpu.so; [ -n "$v" ] && L=pacbio_amd/libpbgpu_$v.so
  for w in C4r:20000 C2:50000; do
    echo "== ${v:-base} $w" >> ${O}_group.txt
    PBGPU_LIB=$L timeout -k 10 300 python -u tools/prof_lis.py --workload ${w%%:*} --reads ${w##*:} >> ${O}_group.txt 2>&1 || exit 1
  done
done

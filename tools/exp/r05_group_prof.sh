# round 5: the 8192-slot group tier's table work by phase (prof build) on C4r; multi-GPU tests (skip on one GPU)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_multi.py -rs > gpurun_out/r05k_multi.log 2>&1 || { tail -20 gpurun_out/r05k_multi.log; exit 1; }
tail -3 gpurun_out/r05k_multi.log
PBGPU_LIB=pacbio_amd/libpbgpu_prof.so timeout -k 10 300 python -u tools/prof_lis.py --workload C4r --reads 20000 > gpurun_out/r05k_group_prof.txt 2>&1
PBGPU_LIB=pacbio_amd/libpbgpu_prof.so timeout -k 10 300 python -u tools/prof_graph_gpu.py --workload C4r --reads 20000 > gpurun_out/r05k_graph_prof.txt 2>&1
for v in "" lisw8; do
  L=pacbio_amd/libpbgpu.so; [ -n "$v" ] && L=pacbio_amd/libpbgpu_$v.so
  echo "== ${v:-base}" >> gpurun_out/r05k_lisw.txt
  PBGPU_LIB=$L timeout -k 10 300 python -u tools/prof_lis.py --workload C2 --reads 50000 >> gpurun_out/r05k_lisw.txt 2>&1
done

# round 5: k_graph_edges occupancy (waves-per-SIMD hint, staged window size) A/B on the graph stage
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
O=gpurun_out/r05ze
for rep in 1 2; do
  for lib in libpbgpu.so libpbgpu_ge6.so libpbgpu_ge6s256.so libpbgpu_ge8s192.so; do
    for wl in "C4r 20000" "C2 50000"; do
      set -- $wl
      echo "== $lib $1" >> ${O}_graph.txt
      PBGPU_LIB=pacbio_amd/$lib timeout -k 10 300 python -u tools/prof_graph_gpu.py --workload $1 --reads $2 >> ${O}_graph.txt 2>&1 || exit 1
    done
  done
done
PBGPU_LIB=pacbio_amd/libpbgpu_prof.so timeout -k 10 300 python -u tools/prof_lis.py --workload C4r --reads 20000 > ${O}_lis_prof.txt 2>&1 || exit 1

# round 5: A/B of the name-offset hoist and the LDS union-find limit (graph stage, resident calls)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
O=gpurun_out/r05zb
for rep in 1 2; do
  for lib in libpbgpu.so libpbgpu_nohoist.so libpbgpu_uf16k.so libpbgpu_uf0.so; do
    for wl in "C4r 20000" "C2 50000"; do
      set -- $wl
      echo "== $lib $1" >> ${O}_graph.txt
      PBGPU_LIB=pacbio_amd/$lib timeout -k 10 300 python -u tools/prof_graph_gpu.py --workload $1 --reads $2 >> ${O}_graph.txt 2>&1 || exit 1
    done
  done
done

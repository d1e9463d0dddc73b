# round 5: k_mega's LDS interval-set capacity (occupancy) and the HBM relaxation from 1024 records: graph stage A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
O=gpurun_out/r05zf
for rep in 1 2; do
  for v in "libpbgpu.so 2048" "libpbgpu.so 1024" "libpbgpu_gcap128.so 2048" "libpbgpu_gcap64.so 2048"; do
    set -- $v
    for wl in "C4r 20000" "C2 50000"; do
      echo "== $1 relax_big_min=$2 ${wl% *}" >> ${O}_graph.txt
      PBGPU_RELAX_BIG_MIN=$2 PBGPU_LIB=pacbio_amd/$1 timeout -k 10 300 python -u tools/prof_graph_gpu.py --workload ${wl% *} --reads ${wl#* } >> ${O}_graph.txt 2>&1 || exit 1
    done
  done
done

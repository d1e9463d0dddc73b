# round 5: k_graph_edges windows by XCD (and the prefilter queue) -- parity (device == host graph), A/B walls
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
O=gpurun_out/r05zq
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_mega_reads.py > ${O}_tests.log 2>&1 || { tail -30 ${O}_tests.log; exit 1; }
tail -1 ${O}_tests.log
for rep in 1 2; do
  for lib in libpbgpu.so libpbgpu_old.so libpbgpu_q.so; do
    for wl in "C4r 20000" "C2 50000"; do
      echo "== $lib ${wl% *}" >> ${O}_graph.txt
      PBGPU_LIB=pacbio_amd/$lib timeout -k 10 300 python -u tools/prof_graph_gpu.py --workload ${wl% *} --reads ${wl#* } >> ${O}_graph.txt 2>&1 || exit 1
    done
  done
done

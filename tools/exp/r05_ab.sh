# round 5: A/B -- k_coords occupancy hints (cw5 / cw6), edge-scan prefetch on / off (nopipe); parity subset
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
O=gpurun_out/r05x
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_edge.py > ${O}_tests.log 2>&1 || { tail -30 ${O}_tests.log; exit 1; }
tail -1 ${O}_tests.log
for lib in libpbgpu.so libpbgpu_cw5.so libpbgpu_cw6.so; do
  for wl in "C2 50000" "C4r 20000"; do
    set -- $wl
    echo "== $lib $1" >> ${O}_coords.txt
    PBGPU_LIB=pacbio_amd/$lib timeout -k 10 300 python -u tools/prof_lis.py --workload $1 --reads $2 >> ${O}_coords.txt 2>&1 || exit 1
  done
done
for lib in libpbgpu.so libpbgpu_nopipe.so libpbgpu.so libpbgpu_nopipe.so; do
  for wl in "C2 50000" "C4r 20000"; do
    set -- $wl
    echo "== $lib $1" >> ${O}_graph.txt
    PBGPU_LIB=pacbio_amd/$lib timeout -k 10 300 python -u tools/prof_graph_gpu.py --workload $1 --reads $2 >> ${O}_graph.txt 2>&1 || exit 1
  done
done

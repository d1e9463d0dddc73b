# round 5: k_graph_edges prefilter loads as global (libpbgpu.so) vs the compiler's flat loads (libpbgpu_flat.so)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
O=gpurun_out/r05zz
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_mega_reads.py > ${O}_tests.log 2>&1 || { tail -30 ${O}_tests.log; exit 1; }
tail -1 ${O}_tests.log
for rep in 1 2; do
for lib in libpbgpu.so libpbgpu_flat.so; do
  for wl in "C4r 20000" "C2 50000"; do
    D=${O}_${lib%.so}_${wl% *}
    PBGPU_LIB=pacbio_amd/$lib timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $D -- python3 -u tools/prof_graph_gpu.py --workload ${wl% *} --reads ${wl#* } > ${O}_run_${lib%.so}_${wl% *}.txt 2>&1 || { tail -20 ${O}_run_${lib%.so}_${wl% *}.txt; exit 1; }
    F=$(find $D -name "*kernel_stats.csv" | head -1)
    echo "== $lib ${wl% *}: $(grep "graph " ${O}_run_${lib%.so}_${wl% *}.txt)" >> ${O}_stats.txt
    grep -E "k_graph_edges<false>" "$F" | awk -F'",' '{print $2}' | cut -d, -f3 >> ${O}_stats.txt
    rm -rf $D
  done
done
done
cat ${O}_stats.txt

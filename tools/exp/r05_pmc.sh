# round 5: SQ counters of k_graph_edges / k_group / k_coords / k_graph_relax_big on C4r (resident call with the
# graph), and k_group's HBM bytes (FETCH_SIZE, WRITE_SIZE passes) on C2; relax threshold 1024 / 512 A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
O=gpurun_out/r05v
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_mega_reads.py > ${O}_tests.log 2>&1 || { tail -30 ${O}_tests.log; exit 1; }
tail -1 ${O}_tests.log
for m in 2048 1024 512; do
  echo "== PBGPU_RELAX_BIG_MIN=$m C4r" >> ${O}_graph.txt
  PBGPU_RELAX_BIG_MIN=$m timeout -k 10 300 python -u tools/prof_graph_gpu.py --workload C4r --reads 20000 >> ${O}_graph.txt 2>&1 || exit 1
  echo "== PBGPU_RELAX_BIG_MIN=$m C2" >> ${O}_graph.txt
  PBGPU_RELAX_BIG_MIN=$m timeout -k 10 300 python -u tools/prof_graph_gpu.py --workload C2 --reads 50000 >> ${O}_graph.txt 2>&1 || exit 1
done
bash tools/pmc_sq_any.sh "k_graph_edges|k_coords|k_group|k_graph_relax_big|k_lis_w" ${O}_sq -- python3 tools/prof_graph_gpu.py --workload C4r --reads 20000 > ${O}_sq.txt 2>&1 || exit 1
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-include-regex "k_group" --output-format csv -d ${O}_hbm/$C -o run -- python3 tools/prof_lis.py --workload C2 --reads 50000 > ${O}_hbm_$C.log 2>&1 || { tail -20 ${O}_hbm_$C.log; exit 1; }
done

# round 5: where the group stage's 16-wave tier spends its time on C4r reads (GROUP_ONLY variants)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in go go_p0 go_p0nt go_nostore go_noturn; do
  echo "== $v" >> gpurun_out/r05i_group_exp.txt
  PBGPU_LIB=pacbio_amd/libpbgpu_$v.so timeout -k 10 300 python -u tools/prof_lis.py --workload C4r --reads 20000 >> gpurun_out/r05i_group_exp.txt 2>&1 || exit 1
done

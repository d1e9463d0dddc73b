# round 5: __graft_entry__.smoke() on the GPU, and the C2 LIS / group phase profile (prof build)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_smoke.txt 2>&1 || { tail -20 gpurun_out/r05_smoke.txt; exit 1; }
tail -2 gpurun_out/r05_smoke.txt
PBGPU_LIB=pacbio_amd/libpbgpu_prof.so timeout -k 10 300 python -u tools/prof_lis.py --workload C2 --reads 50000 > gpurun_out/r05zm_c2_lis_prof.txt 2>&1 || exit 1
PBGPU_LIB=pacbio_amd/libpbgpu_prof.so timeout -k 10 300 python -u tools/prof_coords.py --reads 50000 > gpurun_out/r05zm_c2_coords_prof.txt 2>&1 || exit 1

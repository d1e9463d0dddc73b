# round 5: group partition refinement (A/B on C4r reads) + the overflow / C4r parity tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_edge.py tests/test_abi.py "tests/test_gpu_configs.py::test_c4_repeat_model_oracle" > gpurun_out/r05c_tests.log 2>&1 && \
timeout -k 10 240 python -u tools/prof_lis.py --workload C4r --reads 20000 > gpurun_out/r05c_c4r.txt 2>&1 && \
PBGPU_GROUP_REFINE=0 timeout -k 10 240 python -u tools/prof_lis.py --workload C4r --reads 20000 > gpurun_out/r05c_c4r_norefine.txt 2>&1

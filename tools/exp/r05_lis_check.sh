set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_regress.py tests/test_gpu_configs.py tests/test_gpu_fine_details.py tests/test_gpu_golden.py > gpurun_out/r05b_tests.log 2>&1 && \
timeout -k 10 240 python -u tools/prof_lis.py --workload C4r --reads 20000 > gpurun_out/r05b_c4r_lis.txt 2>&1 && \
timeout -k 10 240 python -u tools/prof_lis.py --workload C2 --reads 50000 > gpurun_out/r05b_c2_lis.txt 2>&1

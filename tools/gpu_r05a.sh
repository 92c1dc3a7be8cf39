set -o pipefail
mkdir -p gpurun_out
timeout -k 10 150 python tools/pivot_cycles.py gpurun_exp/libbos_pivcyc.so > gpurun_out/r05_pivcyc.txt 2>&1 &&
timeout -k 10 150 python tools/solver_stamps.py > gpurun_out/r05_stamps.txt 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_facade.py tests/test_gpu_parity.py tests/test_gpu_edge_cases.py tests/test_gpu_scenarios.py tests/test_gpu_plan_fallback.py -m gpu -x -v -s --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_parity.log 2>&1 &&
timeout -k 10 800 python -u -m pytest tests/test_gpu_c3_gn.py -m gpu -x -v -s --timeout 700 --timeout-method thread -p no:cacheprovider -k "matches_oracle" > gpurun_out/r05_c3acc.log 2>&1

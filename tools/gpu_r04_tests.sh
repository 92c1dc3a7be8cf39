# Round 4: A/B of library variants (tools/gn_ab.py), smoke, the full GPU test suite, shard timeline.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 420 python tools/gn_ab.py gpurun_exp/libbos_head.so gpurun_exp/libbos_nollrun.so gpurun_exp/libbos_llrun.so 2 > gpurun_out/t_ab.txt 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/t_smoke.log 2>&1 || { echo "smoke failed" >> gpurun_out/t_smoke.log; exit 1; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 700 --timeout-method thread -p no:cacheprovider > gpurun_out/t_pytest.log 2>&1 || { echo "pytest failed" >> gpurun_out/t_pytest.log; exit 1; }
timeout -k 10 400 python tools/shard_timeline.py 1 2 4 8 > gpurun_out/t_shard.txt 2>&1 || exit 1

# Round 4: backward-flow start A/B (kSolveWideLevel variants), two-rank direct-exchange bench rehearsal
# on one GPU.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 420 python tools/gn_ab.py gpurun_exp/libbos_base.so gpurun_exp/libbos_sw512.so gpurun_exp/libbos_sw1024.so gpurun_exp/libbos_sw2048.so 2 > gpurun_out/w_ab.txt 2>&1 || exit 1
timeout -k 10 400 python bench.py --gpus 2 --same-device --steps 20 --warmup 3 --no-cpu-baseline --no-gn-other --tri-steps 0 --replay-steps 0 --cold-steps 0 --no-partition-other > gpurun_out/w_bench2.json 2> gpurun_out/w_bench2.err || exit 1

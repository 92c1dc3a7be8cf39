# round 5: Schur leaf size re-swept with this round's kernels
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python tools/leaf_sweep.py 10 8 9 11 12 10 > gpurun_out/r05_leaf_sweep.txt 2>&1

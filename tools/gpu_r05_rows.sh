# round 5: the row loads' cycles split (diagnostic build)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python tools/pivot_cycles.py gpurun_exp/libbos_rowstamps.so --rows > gpurun_out/r05_rows_split.txt 2>&1

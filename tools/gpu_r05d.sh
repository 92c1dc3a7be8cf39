# round 5: the previous product (base), non-temporal L + LDS fixes (new), + tagged hand-offs (tag),
# + one-lane probes and the pinned rhs (probe = this build), and flow-threshold variants of it
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 150 python tools/pivot_cycles.py gpurun_exp/libbos_pivcyc.so > gpurun_out/r05_pivcyc_probe.txt 2>&1 &&
timeout -k 10 900 python tools/gn_ab.py gpurun_exp/libbos_base.so gpurun_exp/libbos_new.so gpurun_exp/libbos_tag.so gpurun_exp/libbos_probe.so gpurun_exp/libbos_sw1024.so gpurun_exp/libbos_sw8192.so gpurun_exp/libbos_fw4096.so 3 > gpurun_out/r05_ab_probe.txt 2>&1

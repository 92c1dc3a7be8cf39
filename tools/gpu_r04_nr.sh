# Round 4: v_rsq_f64 accuracy probe, one-Newton-step pivot variant A/B (diagnostics).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 ./tools/rsq_probe > gpurun_out/n_rsq.txt 2>&1 || exit 1
timeout -k 10 300 python tools/gn_ab.py gpurun_exp/libbos_chain.so gpurun_exp/libbos_nr1.so 3 > gpurun_out/n_ab.txt 2>&1 || exit 1

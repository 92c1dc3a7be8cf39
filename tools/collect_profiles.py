#!/usr/bin/env python3
"""Copy the summaries of tools/gpu_profile.sh (gpurun_out/prof_<tag>/) into profiles/<tag>_*: bench
lines, rocprofv3 kernel stats, J+H PMC summaries (in-step and warm replay)."""
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1] if len(sys.argv) > 1 else "r03"
src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
dst = os.path.join(ROOT, "profiles")


def bench_line(path):
    lines = [ln for ln in open(path).read().splitlines() if ln.startswith("{")]
    return json.loads(lines[-1])


for prec in ("fp32", "fp64"):
    json.dump(bench_line(os.path.join(src, f"bench_{prec}_instep.json")),
              open(os.path.join(dst, f"{tag}_bench_{prec}_instep.json"), "w"), indent=1)
    shutil.copy(os.path.join(src, f"trace_{prec}_instep", "run_kernel_stats.csv"),
                os.path.join(dst, f"{tag}_kernel_stats_{prec}_instep.csv"))
    for mode in ("instep", "warm"):
        shutil.copy(os.path.join(src, f"pmc_linearize_{prec}_{mode}.json"),
                    os.path.join(dst, f"{tag}_pmc_linearize_{prec}_{mode}.json"))
    print(prec, "ok")
json.dump(bench_line(os.path.join(src, "bench_fp32_default.json")),
          open(os.path.join(dst, f"{tag}_bench_fp32_default.json"), "w"), indent=1)
shutil.copy(os.path.join(src, "trace_fp32_default", "run_kernel_stats.csv"),
            os.path.join(dst, f"{tag}_kernel_stats_fp32_default.csv"))
for name in ("gn_step_timeline.txt", "solver_stamps.txt"):
    shutil.copy(os.path.join(src, name), os.path.join(dst, f"{tag}_{name}"))
print("default ok")

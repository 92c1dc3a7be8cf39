#!/usr/bin/env python3
"""Copy the summaries of tools/gpu_profile.sh (gpurun_out/prof_<tag>/) into profiles/<tag>_*."""
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1] if len(sys.argv) > 1 else "r02"
src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
dst = os.path.join(ROOT, "profiles")
for prec in ("fp32", "fp64"):
    for suf in ("", "_cold"):
        lines = [ln for ln in open(os.path.join(src, f"bench_{prec}{suf}.json")).read().splitlines() if ln.startswith("{")]
        json.dump(json.loads(lines[-1]), open(os.path.join(dst, f"{tag}_bench_{prec}{suf}.json"), "w"), indent=1)
        shutil.copy(os.path.join(src, f"trace_{prec}{suf}", "run_kernel_stats.csv"),
                    os.path.join(dst, f"{tag}_kernel_stats_{prec}{suf}.csv"))
        shutil.copy(os.path.join(src, f"pmc_linearize_{prec}{suf}.json"),
                    os.path.join(dst, f"{tag}_pmc_linearize_{prec}{suf}.json"))
    print(prec, "ok")

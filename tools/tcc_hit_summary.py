#!/usr/bin/env python3
"""L2 (TCC) hit rate of the J+H kernel in the GN step against back-to-back builds (diagnostics;
VERDICT r04 item 4: where the in-step build's extra time comes from). Reads two rocprofv3 --pmc
passes of TCC_HIT_sum TCC_MISS_sum (tools/gpu_run.sh l2hit) and prints per-launch hits, misses and the
hit rate, median over the profiled launches.

    python tools/tcc_hit_summary.py DIR_INSTEP DIR_WARM
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import load  # noqa: E402

for label, d in (("in-step", sys.argv[1]), ("back to back", sys.argv[2])):
    rows, _ = load(d)
    hits = [v.get("TCC_HIT_sum", 0.0) for v in rows]
    miss = [v.get("TCC_MISS_sum", 0.0) for v in rows]
    h, m = statistics.median(hits), statistics.median(miss)
    print(f"{label:13s}: {len(hits)} launches, TCC hits {h:.4g}, misses {m:.4g} per launch, hit rate {h / max(h + m, 1):.3f}")

#!/usr/bin/env python3
"""Synchronous GN steps of the one-rank sharded path (config 3, fp32 J+H, Schur), for a rocprofv3
kernel trace of its launches (diagnostics; read the trace with tools/step_timeline.py):

    rocprofv3 --kernel-trace -d gpurun_out/tr -- python3 tools/shard_step_trace.py rccl|p2p|plain [steps]

rccl: a one-rank communicator; p2p: the direct exchange to its own mailbox; plain: the one-GPU step.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prb-project-bearing-only-slam_amd"))
import bos  # noqa: E402

if os.environ.get("BOS_LIB"):   # a library build variant (diagnostics)
    bos.LIB_PATH = os.path.abspath(os.environ["BOS_LIB"])
    bos.ALLOW_MISSING_SYMBOLS = True

mode = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
P = bos.synthetic(100000, 200000, 10, seed=0xB05EED01 + 3)
kw = dict(precision=bos.BOS_FP32, solver=bos.BOS_SOLVER_SCHUR)
if mode == "rccl":
    S = bos.Solver(P, rank=0, world_size=1, nccl_id=bos.nccl_unique_id(), **kw)
elif mode == "p2p":
    S = bos.Solver(P, rank=0, world_size=1, nccl_id=bos.nccl_unique_id(), **kw)   # sharded at world 1
    S.p2p_connect([S.p2p_handle()])
else:
    S = bos.Solver(P, **kw)
st = [S.step() for _ in range(steps)]
med = sorted(g["t_solve_ms"] for g in st)[steps // 2]
print(f"{mode}: {steps} steps, chi2 {st[-1]['chi2']:.6f}, median t_solve {med * 1e3:.1f} us, "
      f"t_exchange {sorted(g['t_exchange_ms'] for g in st)[steps // 2] * 1e3:.1f} us", flush=True)
S.close()

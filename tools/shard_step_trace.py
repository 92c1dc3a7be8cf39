#!/usr/bin/env python3
"""Synchronous GN steps of the one-rank sharded path (config 3, fp32 J+H, Schur), for a rocprofv3
kernel trace of its launches (diagnostics; read the trace with tools/step_timeline.py):

    rocprofv3 --kernel-trace -d gpurun_out/tr -- python3 tools/shard_step_trace.py rccl|p2p|plain [steps]

rccl: a one-rank communicator; p2p: the direct exchange to its own mailbox; plain: the one-GPU step;
ranks W: the W ranks of a W-way subtree partition on this one GPU, one after another per phase with host
exchanges (as tools/shard_timeline.py; read with tools/burst_timeline.py DIR W).
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
if mode == "ranks":
    import numpy as np
    W = int(sys.argv[2])
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    P = bos.synthetic(100000, 200000, 10, seed=0xB05EED01 + 3)
    S = [bos.Solver(P, precision=bos.BOS_FP32, solver=bos.BOS_SOLVER_SCHUR, rank=r, world_size=W) for r in range(W)]
    for it in range(steps):
        for h in S:
            h.step_phase(0)
            h.synchronize()
        recv = np.concatenate([h.exchange_download(1) for h in S])
        for h in S:
            h.exchange_upload(1, recv)
            h.step_phase(1)
            h.synchronize()
        recv = np.concatenate([h.exchange_download(2) for h in S])
        for h in S:
            h.exchange_upload(2, recv)
        st = [h.step_phase(2) for h in S]
        for h in S:
            h.synchronize()
    print(f"ranks {W}: {steps} steps, chi2 {st[0]['chi2']:.6f}", flush=True)
    for h in S:
        h.close()
    sys.exit(0)
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

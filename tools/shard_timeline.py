#!/usr/bin/env python3
"""Per-rank phase times of the sharded GN step on ONE GPU (ranks run one after another, each alone
on the device, exchanges by host copies): what each rank's GPU would spend per iteration on an
N-GPU node, minus the two RCCL all-gathers. The phase times are the device stamps the phases'
kernels write (StepStatus stamp slots), so the host's exchange copies between phases are not in
them. W = 1 runs the RCCL path with a one-rank communicator (the whole iteration, collectives
included, one graph) and is also timed on the host clock beside the plain one-GPU step.
Config 3, fp32 J+H, Schur solver.

    python tools/shard_timeline.py [worlds...]      (default 1 2 4 8)
    BOS_LPP=2|4: J+H lanes per pose (bos_options.lanes_per_pose; default: the plan's choice)
    BOS_LIB=path: a library build variant
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prb-project-bearing-only-slam_amd"))
import numpy as np  # noqa: E402

import bos  # noqa: E402

if os.environ.get("BOS_LIB"):   # a library build variant (diagnostics)
    bos.LIB_PATH = os.path.abspath(os.environ["BOS_LIB"])
    bos.ALLOW_MISSING_SYMBOLS = True

worlds = [int(a) for a in sys.argv[1:]] or [1, 2, 4, 8]
LPP = int(os.environ.get("BOS_LPP", "0"))
P = bos.synthetic(100000, 200000, 10, seed=0xB05EED01 + 3)
out = {}
for W in worlds:
    t0 = time.perf_counter()
    if W == 1:
        S = [bos.Solver(P, precision=bos.BOS_FP32, solver=bos.BOS_SOLVER_SCHUR, rank=0, world_size=1,
                        nccl_id=bos.nccl_unique_id(), lanes_per_pose=LPP)]
    else:
        S = [bos.Solver(P, precision=bos.BOS_FP32, solver=bos.BOS_SOLVER_SCHUR, rank=r, world_size=W,
                        lanes_per_pose=LPP) for r in range(W)]
    t_create = time.perf_counter() - t0
    rows, split = [], []
    for it in range(6):
        if W == 1:
            st = [S[0].step()]
        else:
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
        if it >= 1:
            rows.append([[s["t_linearize_ms"], s["t_solve_ms"], s["t_update_ms"], s["t_exchange_ms"]] for s in st])
            if W > 1:   # own subtrees (J+H end -> phase 0 done) and top + backward (exchange 1 in -> phase 1 done)
                stp = [h.last_step_stamps().astype(np.int64) for h in S]
                split.append([[(t[4] - t[1]) * 1e-5, (t[6] - t[5]) * 1e-5] for t in stp])
    a = np.median(np.array(rows), axis=0)   # [rank][phase]
    sp = np.median(np.array(split), axis=0) if split else None   # [rank][own, top + backward]
    per_rank = a[:, :3].sum(axis=1)
    wall = {}
    if W == 1:   # host-clock rate of the one-rank RCCL path against the plain one-GPU step
        S1 = bos.Solver(P, precision=bos.BOS_FP32, solver=bos.BOS_SOLVER_SCHUR, lanes_per_pose=LPP)
        S2 = bos.Solver(P, precision=bos.BOS_FP32, solver=bos.BOS_SOLVER_SCHUR, rank=0, world_size=1,
                        nccl_id=bos.nccl_unique_id(), lanes_per_pose=LPP)
        S2.p2p_connect([S2.p2p_handle()])
        for name, h in (("rccl_one_rank", S[0]), ("p2p_one_rank", S2), ("one_gpu", S1)):
            init = h.get_state()
            h.step()
            h.synchronize()
            t0 = time.perf_counter()
            for _ in range(20):
                h.step()
            h.synchronize()
            wall[name] = (time.perf_counter() - t0) / 20 * 1e3
            h.set_state(*init)
        st2 = [S2.step() for _ in range(5)]
        wall["p2p_one_rank_exchange_ms"] = float(np.median([g["t_exchange_ms"] for g in st2]))
        S1.close()
        S2.close()
        print(f"W=1 wall ms/step: RCCL one-rank path {wall['rccl_one_rank']:.3f}, direct-exchange one-rank path "
              f"{wall['p2p_one_rank']:.3f} (exchanges {wall['p2p_one_rank_exchange_ms']:.3f}), one GPU "
              f"{wall['one_gpu']:.3f}", flush=True)
    info = [h.system_info() for h in S]
    out[W] = {"create_s": t_create, "jh_ms": a[:, 0].tolist(), "solve_ms": a[:, 1].tolist(), "update_ms": a[:, 2].tolist(),
              "exchange_ms": a[:, 3].tolist(),
              "max_rank_ms": float(per_rank.max()), "own_fronts": [i["own_fronts"] for i in info],
              "top_fronts": info[0]["top_fronts"], "pose_lane_groups": [i["pose_lane_groups"] for i in info],
              "wall_ms_per_step": wall,
              "own_subtrees_ms": sp[:, 0].tolist() if sp is not None else None,
              "top_and_backward_ms": sp[:, 1].tolist() if sp is not None else None}
    print(f"W={W}: per-rank compute (J+H + solve + update) max {per_rank.max():.3f} ms "
          f"(J+H {a[:, 0].max():.3f}, solve {a[:, 1].max():.3f}, update {a[:, 2].max():.3f}; between the phases "
          f"{a[:, 3].max():.3f}); top fronts "
          f"{info[0]['top_fronts']}; create {t_create:.1f} s" +
          (f"; slowest rank: own subtrees {sp[:, 0].max():.3f}, top + backward {sp[:, 1].max():.3f} ms"
           if sp is not None else ""), flush=True)
    for h in S:
        h.close()
print(json.dumps(out))

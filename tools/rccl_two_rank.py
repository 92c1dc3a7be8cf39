#!/usr/bin/env python3
"""Two ranks on one GPU through the RCCL exchange path (diagnostics): each rank builds its shard of
the J+H build of config 2, the grouped ncclBroadcast exchange reassembles H and b, and both ranks
take 3 GN steps; rank 0 compares with a one-rank solver. RCCL may refuse two ranks on one device;
that is reported, not hidden."""
import multiprocessing as mp
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prb-project-bearing-only-slam_amd"))


def worker(rank, world, idq, q):
    try:
        import bos
        if rank == 0:   # the id is made in a rank, never in the parent (which must not touch the GPU first)
            nid = bos.nccl_unique_id()
            for _ in range(world - 1):
                idq.put(nid)
        else:
            nid = idq.get(timeout=60)
        P = bos.synthetic(1000, 2000, 20)
        S = bos.Solver(P, device=0, rank=rank, world_size=world, nccl_id=nid)
        st = S.linearize()
        r, c, v, b = S.export_system()
        for _ in range(3):
            S.step()
        pose, lm = S.get_state()
        S.close()
        q.put((rank, st["chi2"], v, b, pose, lm, None))
    except Exception as e:  # reported to the parent
        q.put((rank, None, None, None, None, None, repr(e)))


def main():
    import numpy as np
    import bos
    world = 2
    ctx = mp.get_context("spawn")
    q, idq = ctx.Queue(), ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, world, idq, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=150) for _ in range(world)], key=lambda x: x[0])
    for p in ps:
        p.join(timeout=30)
    errs = [x[6] for x in res if x[6]]
    if errs:
        print("RANK ERRORS:", errs)
        sys.exit(2)
    P = bos.synthetic(1000, 2000, 20)
    S = bos.Solver(P, device=0)
    st = S.linearize()
    r, c, v, b = S.export_system()
    for _ in range(3):
        S.step()
    pose, lm = S.get_state()
    for rank, chi, v1, b1, p1, l1, _ in res:
        print(f"rank {rank}: chi2 {chi!r} vs {st['chi2']!r}; H equal {np.array_equal(v1, v)}; b equal "
              f"{np.array_equal(b1, b)}; state after 3 steps max diff "
              f"{max(np.abs(p1 - pose).max(), np.abs(l1 - lm).max()):.3g}")


if __name__ == "__main__":
    main()

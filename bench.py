#!/usr/bin/env python3
"""Benchmark of the GN hot path (J+H build) on MI355X — BASELINE.json metric:
"GN iterations/sec + observations/sec (J+H build) at 1/2/4/8 GPUs vs CPU".

A *step* is one J+H build (reference slam/solver.cpp:28-69) over the whole synthetic
config-3 world (100k poses / 200k landmarks / 1M bearings / 99 999 odometry edges), inputs
resident in HBM. ``value`` = observations (bearings + odometry edges) processed per second by
the whole job. With ``--gpus N > 1`` the same world is sharded across N ranks (strong scaling):
each rank builds the part of H its subtrees and the replicated top read, so the
J+H needs no exchange; a GN iteration has two RCCL all-gathers.

Also reported: GN iterations/s (full steps: J+H + sparse Cholesky + exchanges + box-plus), the
J+H kernel's HBM roofline fraction from cold caches (in-step) and back to back (algorithmic
bytes), and the CPU baselines (the oracle, oracle/bos_oracle.cpp, timed on this
host's usable cores).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--precision fp32|fp64]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "prb-project-bearing-only-slam_amd"))

import numpy as np  # noqa: E402

import bos  # noqa: E402

# libbos.so (and the system ROCm 7.2 libraries it links: HIP runtime, rocBLAS/rocSOLVER, RCCL) is
# loaded before torch, exactly as in the test suite (tests/conftest.py): whichever copy of those
# sonames loads first serves the process, so the benchmarked binary runs on the runtime the parity
# tests validated, not on torch's bundled copies.
bos.lib()

METRIC = "GN iterations/sec + observations/sec (J+H build) at 1/2/4/8 GPUs vs CPU"
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md, HBM3E peak (spec)
CONFIG3 = dict(num_poses=100000, num_landmarks=200000, bearings_per_pose=10, seed=0xB05EED01 + 3)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def host_cpus():
    """CPUs this process may use (affinity mask, capped by a cgroup CPU quota when one is set), the
    machine's logical CPU count and the CPU model (lscpu), for the CPU baselines' record."""
    n_aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
            if q != "max":
                quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    usable = min(n_aff, quota) if quota else n_aff
    model = ""
    try:
        import subprocess
        for ln in subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout.splitlines():
            if ln.startswith("Model name:"):
                model = ln.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    return {"usable": usable, "nproc": os.cpu_count(), "affinity": n_aff, "cgroup_quota_cpus": quota,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"), "model": model}


def cpu_baseline(P, precision, cpus, budget_s=12.0):
    """The oracle's J+H build on this host (bounded sample): the reference-order accumulation on one
    thread and the owner-computes parallel form (oracle linearize(owner=True)) on every usable CPU;
    the faster one is the baseline."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle as O
    from helpers import to_oracle
    Q = to_oracle(P)
    prec = 32 if precision == bos.BOS_FP32 else 64
    nobs = len(P.b_z) + len(P.o_z)
    best = None
    threads_all = cpus["usable"]
    O.owner_index(Q)   # built once, like the GPU plan
    forms = {}
    for th, owner in sorted({(1, False), (threads_all, True)}):
        O.linearize(Q, precision=prec, threads=th, owner=owner)   # warm-up
        t0 = time.perf_counter()
        n = 0
        while time.perf_counter() - t0 < budget_s / 2:
            O.linearize(Q, precision=prec, threads=th, owner=owner)
            n += 1
        dt = (time.perf_counter() - t0) / n
        rate = nobs / dt
        form = "owner-computes" if owner else "reference order"
        forms[f"{form}, {th} threads"] = rate
        log(f"cpu oracle J+H {form} threads={th}: {dt * 1e3:.1f} ms/step, {rate / 1e6:.2f} Mobs/s ({n} steps)")
        if best is None or rate > best[0]:
            best = (rate, th, n, form)
    return {"value": best[0], "unit": "obs/s", "cores": best[1], "kind": "port",
            "sample": f"{best[2]} full J+H builds of config 3 ({nobs} obs each, {prec}-bit) by the C++ oracle "
                      f"({best[3]}), ~{budget_s / 2:.0f} s per form; best of 1 thread (reference order) and "
                      f"{threads_all} threads (owner-computes)",
            "forms_obs_per_s": forms, "host": cpus}


def cpu_gn_baseline(P, cpus, budget_s=8.0):
    """Full CPU GN iterations of config 3 by the build's own C++ CPU backend (include/bos_host.h
    bos_cpu_gn_*: the plan's J+H lanes, the host multifrontal Cholesky with each tree level's fronts
    in parallel, box-plus; fp64), bounded sample, on 1 thread and on every usable CPU; the faster one
    is the baseline."""
    forms = {}
    best = None
    for th in sorted({1, cpus["usable"]}):
        c = bos.CpuGN(P, th)
        c.step()   # warm-up (first-touch of the factor buffers)
        t0 = time.perf_counter()
        n = 0
        while time.perf_counter() - t0 < budget_s / 2 or n < 2:
            c.step()
            n += 1
        dt = (time.perf_counter() - t0) / n
        c.close()
        forms[f"{th} threads"] = 1.0 / dt
        log(f"cpu GN (host multifrontal) threads={th}: {dt * 1e3:.0f} ms/iteration ({n} iterations)")
        if best is None or 1.0 / dt > best[0]:
            best = (1.0 / dt, th, n)
    return {"value": best[0], "unit": "it/s", "cores": best[1], "kind": "port",
            "sample": f"{best[2]} GN iterations of config 3 by the build's C++ CPU backend (fp64 J+H, host "
                      f"multifrontal Cholesky, box-plus) on {best[1]} threads; best of 1 and {cpus['usable']} threads",
            "forms_it_per_s": forms, "host": cpus}


FP64_PEAK_TFLOPS = 78.6    # MI355X fp64 (vector and matrix), spec
HANDOFF_US = 1.5           # one cross-CU flag + payload hand-off under load (MI355X_MICROARCH.md,
                           # handoff rows: 0.8-1.0 idle, 1.5-3 with streaming neighbours)


def solver_model(P, phase, world):
    """What bounds the sparse solve (solver.cpp:75-85 replaced by the multifrontal Cholesky):
    its flops at the fp64 peak, its compulsory bytes at the achievable HBM rate, and the dependency
    chain of the elimination tree (levels x two hand-offs, factor and backward) — the measured
    t_solve_ms against each."""
    if world != 1:
        return None
    info = bos.plan_inspect(P, solver=bos.BOS_SOLVER_SCHUR)
    flops = float(info["mf_flops"])
    nnz_l = float(info["nnz_factor"])
    nnz_h = float(info["nnz_lower"])
    levels = int(info["mf_levels"])
    # L written once (factor) and read once (backward), H read once in fp64
    byts = 8.0 * (2.0 * nnz_l + nnz_h)
    t_solve_us = phase["t_solve_ms"] * 1e3
    t_flops = flops / (FP64_PEAK_TFLOPS * 1e12) * 1e6
    t_bytes = byts / (6.3e12) * 1e6
    t_chain = levels * 2 * 2 * HANDOFF_US
    return {"flops": flops, "nnz_factor": nnz_l, "tree_levels": levels, "supernodes": int(info["mf_supernodes"]),
            "bytes": byts, "t_flops_us": t_flops, "t_bytes_us": t_bytes, "t_chain_us": t_chain,
            "t_solve_us": t_solve_us, "bound": "dependency chain (latency)",
            "frac_of_chain_bound": t_chain / t_solve_us, "frac_of_bytes_bound": t_bytes / t_solve_us}


PROFILE_TAG = "r02"   # profiles/<tag>_pmc_linearize_<prec>.json, written by tools/pmc_summary.py


def traffic_from_profile(precision):
    """Fabric bytes per launch of the J+H kernel from the committed rocprofv3 PMC summaries
    (L2 <-> fabric requests by size, tools/gpu_profile.sh): {"warm": ..., "cold": ...}."""
    out = {}
    for label in ("warm", "cold"):
        name = f"{PROFILE_TAG}_pmc_linearize_" + ("fp32" if precision == bos.BOS_FP32 else "fp64") + \
            ("_cold" if label == "cold" else "") + ".json"
        path = os.path.join(ROOT, "profiles", name)
        try:
            with open(path) as f:
                out[label] = float(json.load(f)["hbm_bytes_per_launch"])
        except (OSError, ValueError, KeyError):
            out[label] = None
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--precision", choices=["fp32", "fp64"], default="fp32")
    ap.add_argument("--gn-steps", type=int, default=50,
                    help="GN iterations timed (sync and as one bos_step_n batch: the reference UI steps 50 at a time)")
    ap.add_argument("--cold-steps", type=int, default=20, help="J+H builds timed from cold caches (in-step roofline)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-gn-other", action="store_true", help="skip timing the other solver ordering")
    ap.add_argument("--tri-steps", type=int, default=20, help="device triangulations timed (0: skip)")
    ap.add_argument("--exchange", choices=["rccl", "gloo"], default="rccl",
                    help="N > 1: the sharded step's two all-gathers on RCCL (default), or through host memory "
                         "and gloo (rehearsal of the N-rank path on fewer GPUs, with --same-device)")
    ap.add_argument("--same-device", action="store_true", help="every rank on GPU 0 (rehearsal only)")
    ap.add_argument("--solver", choices=["supernodal", "schur"], default="schur",
                    help="GN linear solver: landmarks-first Schur multifrontal (config 5, default) or "
                         "nested-dissection multifrontal; the other one is timed too (gn_other)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    # torch only for the rendezvous (gloo, host memory): the GPU work and its timing go through
    # libbos.so (HIP events on the handle's stream), and the exchange runs on RCCL inside it
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo")
    precision = bos.BOS_FP32 if args.precision == "fp32" else bos.BOS_FP64

    t_gen = time.perf_counter()
    P = bos.synthetic(**CONFIG3)
    nobs = len(P.b_z) + len(P.o_z)
    log(f"rank {rank}: config 3 world NP={P.NP} NL={P.NL} Mb={len(P.b_z)} Mo={len(P.o_z)} "
        f"({time.perf_counter() - t_gen:.1f} s)")

    nccl_id = None
    if world > 1 and args.exchange == "rccl":
        obj = [bos.nccl_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        nccl_id = obj[0]
    device = 0 if args.same_device else local_rank
    t_create = time.perf_counter()
    solver = bos.BOS_SOLVER_SCHUR if args.solver == "schur" else bos.BOS_SOLVER_SUPERNODAL
    S = bos.Solver(P, precision=precision, solver=solver, device=device, rank=rank, world_size=world,
                   nccl_id=nccl_id)
    info = S.system_info()
    log(f"rank {rank}: bos_create {time.perf_counter() - t_create:.1f} s, n={info['n']} "
        f"nnz(H lower)={info['nnz_lower']} nnz(L)={info['nnz_factor']}")

    def barrier():
        if world > 1:
            dist.barrier()

    def max_over_ranks(v):
        if world == 1:
            return v
        t = torch.tensor([v], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    # ---- J+H build throughput: K builds back to back (the timed region), warm caches
    if args.warmup > 0:
        S.time_linearize(args.warmup)
    S.synchronize()
    barrier()
    S.synchronize()
    t0 = time.perf_counter()
    kernel_ms = S.time_linearize(args.steps)   # synchronises the handle's stream
    barrier()
    wall = max_over_ranks(time.perf_counter() - t0)
    ms_per_step = wall / args.steps * 1e3
    value = nobs * args.steps / wall
    # ---- the same build from cold caches (512 MiB read before each): what it costs inside a GN
    # iteration, where the solver's factor streams between two builds
    cold_ms = S.time_linearize(args.cold_steps, flush_caches=True) if args.cold_steps > 0 else None

    # ---- full GN iterations (J+H + exchanges + solve + update)
    def gloo_allgather(h, which):
        mine = torch.from_numpy(h.exchange_download(which))
        parts = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(parts, mine)
        h.exchange_upload(which, torch.cat(parts).numpy())

    def gn_step(h):
        if world == 1 or args.exchange == "rccl":
            return h.step()
        h.step_phase(0)
        gloo_allgather(h, 1)
        h.step_phase(1)
        gloo_allgather(h, 2)
        return h.step_phase(2)

    def time_gn(solver_handle):
        """GN iterations/s three ways: synchronous bos_step calls in a C loop (bos_time_steps: each
        call returns with the state updated and the status read, as Solver::step() in the reference's
        C++ driver; the host round trip is inside every iteration), the same calls one by one from
        Python through ctypes (the binding's per-call overhead included), and bos_step_n batches (the
        reference driver's loop of steps, executables/bearing_only_slam.cpp:95-98: every iteration
        runs in full, the host synchronises once per batch). Every timed run starts from the initial
        guess (bos_set_state), so each times the same iterations 1..gn_steps of the solve; run on past
        convergence, the fp32 J+H build of this world loses positive definiteness after ~150
        iterations (tools/gn_trajectory.py)."""
        init = solver_handle.get_state()

        def restart():
            solver_handle.set_state(*init)
            barrier()

        gn_step(solver_handle)   # first iteration includes the one-time factorization analysis
        restart()
        tg = time.perf_counter()
        stats = [gn_step(solver_handle) for _ in range(args.gn_steps)]
        barrier()
        gn_wall = max_over_ranks(time.perf_counter() - tg)
        assert all(g["solver_info"] == 0 for g in stats), "non-positive pivot in a benchmarked GN step"
        ph = {k: float(np.median([g[k] for g in stats])) for k in
              ("t_linearize_ms", "t_exchange_ms", "t_solve_ms", "t_update_ms")}
        batched, c_loop = None, None
        if world == 1 or args.exchange == "rccl":
            restart()
            c_loop = 1e3 / max_over_ranks(solver_handle.time_steps(args.gn_steps))
            restart()
            tg = time.perf_counter()
            last = solver_handle.step_n(args.gn_steps)
            barrier()
            batched = args.gn_steps / max_over_ranks(time.perf_counter() - tg)
            assert last["solver_info"] == 0, "non-positive pivot in a benchmarked GN step"
        restart()
        return c_loop if c_loop else args.gn_steps / gn_wall, ph, batched, args.gn_steps / gn_wall

    gn_it_s, phase, gn_other, gn_batched, gn_python = None, None, None, None, None
    if args.gn_steps > 0:
        gn_it_s, phase, gn_batched, gn_python = time_gn(S)
        if world == 1 and not args.no_gn_other:   # the other multifrontal ordering, for comparison
            other = "supernodal" if args.solver == "schur" else "schur"
            S2 = bos.Solver(P, precision=precision, device=local_rank,
                            solver=bos.BOS_SOLVER_SUPERNODAL if other == "supernodal" else bos.BOS_SOLVER_SCHUR)
            it2, ph2, b2, _ = time_gn(S2)
            gn_other = {"solver": other, "gn_iters_per_s": it2, "gn_iters_per_s_batched": b2,
                        "t_solve_ms": ph2["t_solve_ms"]}
            S2.close()

    # ---- landmark triangulation on the device (slam/triangulation.cpp:65-74), config 3 (run last:
    # it re-estimates the landmarks of S)
    tri = None
    if world == 1 and args.tri_steps > 0:
        S.triangulate()
        tri_ms = S.time_triangulate(args.tri_steps)
        tri = {"landmarks": P.NL, "bearings": int(len(P.b_z)), "ms": tri_ms, "landmarks_per_s": P.NL / (tri_ms * 1e-3)}
        if not args.no_cpu_baseline:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle as O
            pose, _ = S.get_state()
            t0 = time.perf_counter()
            O.triangulate(pose, P.b_pose, P.b_lm, P.b_z)
            cpu_ms = (time.perf_counter() - t0) * 1e3
            tri["cpu_baseline"] = {"ms": cpu_ms, "landmarks_per_s": P.NL / (cpu_ms * 1e-3), "cores": 1,
                                   "kind": "port", "sample": "one triangulation of config 3 by the C++ oracle"}

    if rank == 0:
        algo = info["algorithmic_bytes"]
        traffic = traffic_from_profile(precision) if world == 1 else None

        def roof(ms, label, timing):
            a = algo / (ms * 1e-3) / 1e9
            return {"bound": "hbm", "achieved": a, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": a / HBM_PEAK_GBS,
                    "traffic": traffic.get("warm" if label == "warm" else "cold") if traffic else None,
                    "algorithmic_bytes_per_launch": algo, "kernel_ms": ms, "caches": label, "timing": timing}
        instep = phase["t_linearize_ms"] if phase else None
        r_instep = roof(instep, "in-step", "median over the timed GN steps of the device realtime clock from the "
                        "J+H launch's start to the next launch's start (stamped by the step's kernels)") if instep else None
        r_cold = roof(cold_ms, "cold", "HIP events around each build, 512 MiB read before it (event cost included)") \
            if cold_ms else None
        r_warm = roof(kernel_ms, "warm", "HIP events around the back-to-back builds")
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "obs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32" if precision == bos.BOS_FP32 else "f64",
            "data": "synthetic",
            "config": {
                "workload": "config 3: synthetic 100k poses / 200k landmarks / 1M bearings / 99999 odometry "
                            "edges; J+H build " + ("fp32" if precision == bos.BOS_FP32 else "fp64") +
                            " (solve fp64, " + args.solver + ")",
                "poses": P.NP, "landmarks": P.NL, "bearings": int(len(P.b_z)), "odometry": int(len(P.o_z)),
                "parallelism": (f"subtree-sharded x{world} ({'RCCL' if args.exchange == 'rccl' else 'gloo rehearsal'} "
                                f"all-gathers; top fronts replicated: {info['top_fronts']})") if world > 1 else "single GPU",
            },
            "gn_iters_per_s": gn_it_s,
            "gn_iters_per_s_batched": gn_batched,
            "gn_iters_per_s_python": gn_python,
            "gn_phase_ms": phase,
            "solver_model": solver_model(P, phase, world) if phase else None,
            "gn_solver": args.solver,
            "gn_other": gn_other,
            "triangulation": tri,
            # the J+H as it runs inside the GN iteration (inputs from HBM after the solver's stream)
            # first; the same from cold caches by events, and the back-to-back replay (working set
            # partly served by the Infinity Cache), beside it
            "roofline": r_instep or r_cold or r_warm,
            "roofline_cold_events": r_cold,
            "roofline_warm_replay": r_warm,
        }
        if world == 1 and not args.no_cpu_baseline:
            cpus = host_cpus()
            line["cpu_baseline"] = cpu_baseline(P, precision, cpus)
            line["cpu_baseline_gn"] = cpu_gn_baseline(P, cpus)
            line["speedup_vs_cpu"] = value / line["cpu_baseline"]["value"]
            if gn_it_s:
                line["gn_speedup_vs_cpu"] = gn_it_s / line["cpu_baseline_gn"]["value"]
        print(json.dumps(line), flush=True)
    S.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

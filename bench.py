"""Benchmark of the GN hot path (J+H build) on MI355X — BASELINE.json metric:
"GN iterations/sec + observations/sec (J+H build) at 1/2/4/8 GPUs vs CPU".

A *step* is one Gauss-Newton iteration of the reference's Solver::step (slam/solver.cpp:27-97) over
the whole synthetic config-3 world (100k poses / 200k landmarks / 1M bearings / 99 999 odometry
edges), inputs resident in HBM. The timed region is K such steps (synchronous bos_step calls) from the
initial guess, iterations 1..K of the solve (default 50, the reference UI's batch; the world converges,
so any K runs positive definite). ``value`` = observations (bearings + odometry edges)
per second of the J+H build *as it runs inside those steps* (device realtime stamps written by the
step's own kernels, median over the K steps, the slowest rank); ``ms_per_step`` is that J+H time
(= roofline.kernel_ms). The steps' wall rate is ``gn_iters_per_s``.

With ``--gpus N > 1`` the same world is split over N ranks (strong scaling), one process per GPU:
under torch.distributed.run (RANK / WORLD_SIZE set), or — without a launcher — this script starts the N
rank processes itself before anything touches the GPU. The exchanges go through a ladder (DESIGN.md
§7): the direct peer exchange (p2p), else RCCL all-gathers, else the gloo host exchange — a mode that
fails on any rank (set-up, the three-step chi^2 check or the timed steps) is dropped on every rank
together and the next one runs; the line records each attempt with every failing rank's reason
(``exchange_decision``), every rank's device and rank 0's peer-access matrix (``topology``), and if no
mode completes rank 0 still prints a line (``value`` null, ``error``). The exchange must span N ranks
(``ranks_seen``: the RCCL communicator's count or the process group's). The default partition
(BOS_PARTITION_SUBTREE) gives each rank the subtrees of the Schur assembly tree below a
replicated top: its J+H builds only the H its fronts read, two all-gathers per iteration. The north
star's partition (BOS_PARTITION_OBSERVATIONS: the J+H lanes split by measurement order, one
all-reduce of (H, b), the solve replicated) is timed beside it (``partition_observations``).

Also reported: the J+H kernel's HBM roofline fraction (in-step; from cold caches by events; back to
back), GN iterations/s, and the CPU baselines (the oracle, oracle/bos_oracle.cpp, and the build's
C++ CPU backend, timed on this host's usable cores).

``--config c2`` times BASELINE config 2 instead (synthetic 1k / 2k / 20k, fp64, one GPU): microseconds
per GN iteration and per J+H build beside the CPU backend's (the size is launch-bound: no roofline).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--precision fp32|fp64] [--config c3|c2]
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "prb-project-bearing-only-slam_amd"))

import numpy as np  # noqa: E402

bos = None   # the product binding, imported in main() after the rank launcher (no HIP in a launcher)

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
    if world != 1 or not phase:
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


PROFILE_TAG = "r06"   # profiles/<tag>_pmc_linearize_<prec>_<mode>.json, written by tools/pmc_summary.py


def lib_sha256():
    import hashlib
    with open(bos.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def traffic_from_profile(precision, profiles_dir=None):
    """Fabric bytes per launch of the J+H kernel from the committed rocprofv3 PMC summaries
    (L2 <-> fabric requests by size, tools/gpu_profile.sh): the in-step launches of the timed GN steps
    ("instep") and back-to-back builds ("warm"). A summary counts only if it was taken with the very
    libbos.so this process loaded (its libbos_sha256): counters of another build are not this line's
    traffic, so the value is then None and the reason is returned beside it."""
    out, why = {}, {}
    mine = lib_sha256()
    for label in ("instep", "warm"):
        name = f"{PROFILE_TAG}_pmc_linearize_" + ("fp32" if precision == bos.BOS_FP32 else "fp64") + f"_{label}.json"
        path = os.path.join(profiles_dir or os.path.join(ROOT, "profiles"), name)
        out[label] = None
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            why[label] = f"no profiles/{name}"
            continue
        if d.get("libbos_sha256") != mine:
            why[label] = f"profiles/{name} was taken with another libbos.so build"
            continue
        out[label] = float(d["hbm_bytes_per_launch"])
        why[label] = f"profiles/{name} (rocprofv3 --pmc of this libbos.so build)"
    return out, why


def free_port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(n, deadline_s=1800.0):
    """No launcher but --gpus N > 1: start N rank processes of this script (one per GPU, env as
    torch.distributed.run sets it), relay rank 0's JSON line, exit with the worst exit code. Runs
    before anything in this process touches HIP. Every rank is polled against one deadline: as soon
    as any rank exits non-zero (or the deadline passes) the others are killed, so a rank that dies
    before the rendezvous cannot leave the rest waiting forever."""
    import threading
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))
    out = []
    reader = threading.Thread(target=lambda: out.append(procs[0].stdout.read()), daemon=True)
    reader.start()
    t_end = time.monotonic() + deadline_s
    failed = False
    while True:
        rcs = [p.poll() for p in procs]
        if all(rc is not None for rc in rcs):
            break
        if any(rc not in (None, 0) for rc in rcs) or time.monotonic() > t_end:
            failed = True
            break
        time.sleep(0.2)
    own = [rc for rc in rcs if rc not in (None, 0)]   # ranks that failed by themselves
    if failed:
        for p in procs:
            if p.poll() is None:
                p.kill()
    rcs = [p.wait() for p in procs]
    reader.join(timeout=10)
    for ln in (out[0] if out else b"").decode(errors="replace").splitlines():
        # the JSON line to stdout; anything else rank 0's libraries printed there (gloo's connection
        # notice) to stderr
        (sys.stdout if ln.startswith("{") else sys.stderr).write(ln + "\n")
    sys.stdout.flush()
    bad = own + [rc for rc in rcs if rc != 0]
    if bad:
        log(f"launcher: rank exit codes {rcs}" + (" (killed after a failure or the deadline)" if failed else ""))
    return bad[0] if bad else 0


LADDER = {"p2p": ("p2p", "rccl", "gloo"), "rccl": ("rccl", "gloo"), "gloo": ("gloo",)}


def agree_all(dist, torch, ok, why=None):
    """Every rank's verdict on one step of the exchange ladder: (True only if every rank is ok, every
    rank's reason in rank order). Without a process group: (ok, [why])."""
    if dist is None:
        return ok, [why]
    t = torch.tensor([1 if ok else 0], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    whys = [None] * dist.get_world_size()
    dist.all_gather_object(whys, why)
    return bool(int(t.item()) == 1), whys


def run_ladder(modes, setup, run, agree, close, log):
    """The N > 1 exchange ladder: try each mode in order — set it up on every rank
    (setup(mode), local apart from its own collective calls), agree, run it (run(mode, handle): the
    consistency check and the timed steps, collective-safe), agree — and keep the first mode every
    rank completed. A mode that fails on any rank is closed on every rank and the next one is tried,
    so all ranks always take the same decision. Returns (mode or None, handle, run's result, attempts:
    one record per mode tried, with each failing rank's reason)."""
    attempts = []
    for mode in modes:
        h, why = None, None
        try:
            h = setup(mode)
        except Exception as e:
            why = f"setup: {type(e).__name__}: {e}"
        ok, whys = agree(why is None, why)
        if not ok:
            attempts.append({"mode": mode, "ok": False, "stage": "setup",
                             "why": {r: w for r, w in enumerate(whys) if w}})
            log(f"exchange {mode}: setup failed {attempts[-1]['why']}")
            close(h)
            continue
        res, why = None, None
        try:
            res = run(mode, h)
        except Exception as e:
            why = f"{type(e).__name__}: {e}"
        ok, whys = agree(why is None, why)
        if ok:
            attempts.append({"mode": mode, "ok": True})
            return mode, h, res, attempts
        attempts.append({"mode": mode, "ok": False, "stage": "run", "why": {r: w for r, w in enumerate(whys) if w}})
        log(f"exchange {mode}: run failed {attempts[-1]['why']}")
        close(h)
    return None, None, None, attempts


def topology(rank, world, local_rank, device, ndev, dist):
    """Where the ranks run: every rank's (rank, local rank, device, visible devices, visibility
    variables), and rank 0's peer-access matrix of the visible devices (hipDeviceCanAccessPeer)."""
    mine = {"rank": rank, "local_rank": local_rank, "device": device, "visible_devices": ndev,
            "host": socket.gethostname(),
            "HIP_VISIBLE_DEVICES": os.environ.get("HIP_VISIBLE_DEVICES"),
            "ROCR_VISIBLE_DEVICES": os.environ.get("ROCR_VISIBLE_DEVICES")}
    peer = None
    if rank == 0:
        try:
            peer = bos.device_peer_access()
        except Exception as e:
            peer = f"unavailable: {e}"
    ranks = [mine]
    if dist is not None and world > 1:
        ranks = [None] * world
        dist.all_gather_object(ranks, mine)
    return {"ranks": ranks, "peer_access": peer}


def fail_line(args, world, attempts, topo=None):
    """No exchange mode (or the one-GPU run) completed: rank 0 still prints one line saying so."""
    if int(os.environ.get("RANK", "0")) != 0:
        return
    print(json.dumps({"metric": METRIC, "value": None, "unit": "obs/s", "n_gpus": world, "steps": args.steps,
                      "warmup": args.warmup, "ms_per_step": None, "higher_is_better": True, "scaling": "strong",
                      "vs_baseline": None, "dtype": args.precision.replace("fp", "f"), "data": "synthetic",
                      "config": {"workload": "config 3 (no run completed)"},
                      "error": "no exchange mode completed" if world > 1 else "the GN run failed",
                      "exchange_decision": {"mode": None, "attempts": attempts}, "topology": topo}), flush=True)


def check_ladder(args, rank, dist, torch):
    """--check-launch --check-ladder: the exchange ladder of main() with stand-in modes (no GPU) that
    fail where the spec says; each stand-in run makes the real run's kinds of collective calls after
    its failure point too (a barrier, a chi^2 reduction), as check_and_time does."""
    fails = set()
    for item in filter(None, (args.check_ladder or "").split(",")):
        mode_stage, _, r = item.partition("@")
        fails.add((mode_stage, r or "*"))

    def failing(mode, stage):
        return (f"{mode}:{stage}", "*") in fails or (f"{mode}:{stage}", str(rank)) in fails

    def setup(mode):
        if failing(mode, "setup"):
            raise RuntimeError(f"stand-in {mode} setup failure")
        return mode

    def run(mode, h):
        err = "stand-in run failure" if failing(mode, "run") else None
        dist.barrier()
        t = torch.tensor([float("nan") if err else 1.0], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        if err:
            raise RuntimeError(err)
        return mode

    mode, _, _, attempts = run_ladder(LADDER[args.exchange], setup, run,
                                      lambda ok, why: agree_all(dist, torch, ok, why), lambda h: None,
                                      lambda *a: None)
    return {"mode": mode, "attempts": attempts}


def bench_c2(args):
    """BASELINE config 2 on one GPU: the synthetic 1k-pose / 2k-landmark / 20k-bearing
    world the GPU parity tests check (bos.synthetic(1000, 2000, 20)), fp64 J+H and solve. At this size the
    step is launch- and latency-bound (1.7 MB of J+H traffic), so the line reports microseconds: per GN
    iteration (synchronous bos_step, the Python loop and the C loop; bos_step_n batches), the in-step
    phases (device stamps) and the J+H build back to back, beside the build's C++ CPU backend (full GN
    iterations on 1 thread and on every usable CPU) and the oracle's J+H on the same host."""
    global bos
    import bos as _bos
    bos = _bos
    bos.lib()
    precision = bos.BOS_FP64 if args.precision == "fp64" else bos.BOS_FP32
    P = bos.synthetic(1000, 2000, 20)
    nobs = len(P.b_z) + len(P.o_z)
    S = bos.Solver(P, precision=precision, solver=bos.BOS_SOLVER_SCHUR, device=0)
    init = S.get_state()
    for _ in range(max(args.warmup, 20)):
        S.step()
    S.set_state(*init)
    S.synchronize()
    k = args.steps
    t0 = time.perf_counter()
    stats = [S.step() for _ in range(k)]
    S.synchronize()
    wall = time.perf_counter() - t0
    assert all(g["solver_info"] == 0 for g in stats), "non-positive pivot in a timed C2 step"
    S.set_state(*init)
    ph = {key: float(np.median([g[key] for g in stats])) for key in ("t_linearize_ms", "t_solve_ms", "t_update_ms")}
    c_loop_ms = S.time_steps(k)
    S.set_state(*init)
    tb = time.perf_counter()
    last = S.step_n(args.batch)
    S.synchronize()
    batched_ms = (time.perf_counter() - tb) * 1e3 / args.batch
    assert last["solver_info"] == 0
    S.set_state(*init)
    warm_ms = S.time_linearize(max(args.replay_steps, 200))
    S.close()
    # the other multifrontal ordering (nested dissection, landmarks not folded) on the same world
    S2 = bos.Solver(P, precision=precision, solver=bos.BOS_SOLVER_SUPERNODAL, device=0)
    for _ in range(5):
        S2.step()
    t2 = time.perf_counter()
    st2 = [S2.step() for _ in range(k)]
    S2.synchronize()
    other = {"solver": "supernodal", "gn_us_per_iteration": (time.perf_counter() - t2) * 1e6 / k,
             "t_solve_us": float(np.median([g["t_solve_ms"] for g in st2])) * 1e3}
    S2.close()
    cpus = host_cpus()
    cpu = {}
    for th in sorted({1, cpus["usable"]}):
        c = bos.CpuGN(P, th)
        c.step()
        n, tc = 0, time.perf_counter()
        while time.perf_counter() - tc < 3.0 or n < 5:
            c.step()
            n += 1
        cpu[f"{th} threads"] = (time.perf_counter() - tc) * 1e6 / n
        c.close()
    cpu_best = min(cpu.values())
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle as O
    from helpers import to_oracle
    Q = to_oracle(P)
    O.linearize(Q, precision=64 if precision == bos.BOS_FP64 else 32)
    n, tc = 0, time.perf_counter()
    while time.perf_counter() - tc < 2.0 or n < 5:
        O.linearize(Q, precision=64 if precision == bos.BOS_FP64 else 32)
        n += 1
    oracle_jh_us = (time.perf_counter() - tc) * 1e6 / n
    gn_us = wall * 1e6 / k
    line = {
        "metric": METRIC, "value": nobs / (ph["t_linearize_ms"] * 1e-3), "unit": "obs/s", "n_gpus": 1, "steps": k,
        "warmup": max(args.warmup, 20), "ms_per_step": ph["t_linearize_ms"], "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f64" if precision == bos.BOS_FP64 else "f32",
        "data": "synthetic",
        "config": {"workload": "config 2: synthetic 1k poses / 2k landmarks / 20k bearings / 999 odometry edges "
                               "(bos.synthetic(1000, 2000, 20), the GPU parity tests' world); J+H and solve "
                               + args.precision + ", schur", "poses": P.NP, "landmarks": P.NL,
                   "bearings": int(len(P.b_z)), "odometry": int(len(P.o_z)), "parallelism": "single GPU"},
        "note": "launch-bound size (SURVEY.md §8(d)): microseconds per iteration, no roofline",
        "gn_us_per_iteration": gn_us, "gn_iters_per_s": 1e6 / gn_us,
        "gn_us_per_iteration_c_loop": c_loop_ms * 1e3, "gn_us_per_iteration_batched": batched_ms * 1e3,
        "gn_phase_us": {key.replace("_ms", "_us"): v * 1e3 for key, v in ph.items()}, "gn_other": other,
        "jh_us_in_step": ph["t_linearize_ms"] * 1e3, "jh_us_back_to_back": warm_ms * 1e3,
        "cpu_baseline_gn": {"us_per_iteration": cpu_best, "forms_us_per_iteration": cpu, "kind": "port",
                            "sample": "full GN iterations of config 2 by the build's C++ CPU backend (fp64 J+H, host "
                                      "multifrontal Cholesky, box-plus), >= 3 s per thread count", "host": cpus},
        "cpu_baseline_jh": {"us_per_build": oracle_jh_us, "cores": 1, "kind": "port",
                            "sample": "the C++ oracle's J+H of config 2 in reference order, >= 2 s"},
        "gn_speedup_vs_cpu": cpu_best / gn_us, "jh_speedup_vs_cpu": oracle_jh_us / (ph["t_linearize_ms"] * 1e3),
        "libbos_sha256": lib_sha256(),
    }
    print(json.dumps(line), flush=True)
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50, help="GN iterations timed (from the initial guess)")
    ap.add_argument("--warmup", type=int, default=5, help="untimed GN iterations before the timed ones")
    ap.add_argument("--device-warmup", type=int, default=1000,
                    help="untimed GN iterations (bos_step_n batches of 100, about 0.5 s on one GPU) before the "
                         "headline's warmup: brings the GPU to its steady clocks (tools/jh_placement_probe.py); "
                         "0 = off")
    ap.add_argument("--precision", choices=["fp32", "fp64"], default=None,
                    help="J+H precision (default fp32 for config 3, fp64 for config 2)")
    ap.add_argument("--config", choices=["c3", "c2"], default="c3",
                    help="c3: the headline (100k / 200k / 1M, fp32 J+H); c2: BASELINE config 2 (synthetic 1k poses / "
                         "2k landmarks / 20k bearings, fp64, one GPU), launch-bound: microseconds per GN iteration "
                         "and per J+H build beside the CPU backend's (SURVEY.md §8(d))")
    ap.add_argument("--replay-steps", type=int, default=200, help="J+H builds back to back (warm-replay roofline)")
    ap.add_argument("--cold-steps", type=int, default=20, help="J+H builds timed from cold caches by events")
    ap.add_argument("--batch", type=int, default=50, help="GN iterations per bos_step_n batch (the reference UI's 50)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-gn-other", action="store_true", help="skip timing the other solver ordering")
    ap.add_argument("--no-partition-other", action="store_true", help="N > 1: skip the observations partition")
    ap.add_argument("--tri-steps", type=int, default=20, help="device triangulations timed (0: skip)")
    ap.add_argument("--exchange", choices=["p2p", "rccl", "gloo"], default="p2p",
                    help="N > 1, subtree partition: the two exchanges per iteration written directly into the other "
                         "ranks' mailboxes over xGMI (p2p, default; falls back to RCCL if a rank cannot map the "
                         "others'), RCCL all-gathers, or host memory and gloo (rehearsal of the N-rank path on fewer "
                         "GPUs, with --same-device)")
    ap.add_argument("--same-device", action="store_true", help="every rank on GPU 0 (rehearsal only)")
    ap.add_argument("--check-launch", action="store_true",
                    help="launch / rendezvous check only (no GPU): every rank joins the gloo group, rank 0 prints "
                         "the ranks seen")
    ap.add_argument("--check-launch-fail-rank", type=int, default=-1,
                    help="with --check-launch: this rank exits 5 before the rendezvous (tests the launcher)")
    ap.add_argument("--check-ladder", default=None,
                    help="with --check-launch: run the exchange ladder with stand-in modes that fail as listed "
                         "(comma-separated MODE:STAGE@RANK, STAGE setup|run, RANK a rank or *), print the decision "
                         "(tests/test_bench.py; no GPU)")
    ap.add_argument("--solver", choices=["supernodal", "schur"], default="schur",
                    help="GN linear solver: landmarks-first Schur multifrontal (config 5, default) or "
                         "nested-dissection multifrontal; the other one is timed too (gn_other)")
    ap.add_argument("--lanes-per-pose", type=int, default=0, choices=[0, 1, 2, 4],
                    help="J+H lanes per pose (bos_options.lanes_per_pose); 0 = the plan's rule (1 at config 3), "
                         "the same at every N so that the scaling curve compares the same arithmetic")
    args = ap.parse_args()

    if args.precision is None:
        args.precision = "fp64" if args.config == "c2" else "fp32"
    if args.config == "c2":
        if args.gpus != 1:
            log("error: --config c2 runs on one GPU")
            sys.exit(2)
        sys.exit(bench_c2(args))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"error: --gpus {args.gpus} but WORLD_SIZE={world}")
        sys.exit(2)

    if args.check_launch:   # the rank processes and their rendezvous, nothing else (tests/test_bench.py)
        seen = 1
        if rank == args.check_launch_fail_rank:
            sys.exit(5)
        if world > 1:
            import torch
            import torch.distributed as dist
            dist.init_process_group("gloo")
            t = torch.tensor([rank], dtype=torch.int64)
            parts = [torch.zeros_like(t) for _ in range(world)]
            dist.all_gather(parts, t)
            seen = len({int(x) for x in parts})
            decision = None
            if args.check_ladder is not None:
                decision = check_ladder(args, rank, dist, torch)
            dist.destroy_process_group()
        else:
            decision = None
        if rank == 0:
            out = {"check_launch": True, "ranks_seen": seen, "world": world}
            if decision is not None:
                out["exchange_decision"] = decision
            print(json.dumps(out), flush=True)
        if decision is not None and decision["mode"] is None:
            sys.exit(4)
        sys.exit(0 if seen == args.gpus else 3)

    global bos
    import bos as _bos
    bos = _bos
    # libbos.so (and the system ROCm 7.2 libraries it links: HIP runtime, rocBLAS/rocSOLVER, RCCL) is
    # loaded before torch, exactly as in the test suite (tests/conftest.py): whichever copy of those
    # sonames loads first serves the process, so the benchmarked binary runs on the runtime the parity
    # tests validated, not on torch's bundled copies.
    bos.lib()

    # torch only for the rendezvous and the gloo rehearsal (host memory): the GPU work and its timing
    # go through libbos.so, and the exchanges run on RCCL inside it
    dist, torch = None, None
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

    def barrier():
        if world > 1:
            dist.barrier()

    def max_over_ranks(v):
        if world == 1:
            return v
        t = torch.tensor([v], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    # the rank's device: LOCAL_RANK among the visible devices; a launcher that shows each rank only
    # its own GPU (one visible device) gets device 0
    ndev = bos.device_count()
    device = 0 if (args.same_device or (ndev == 1 and local_rank > 0)) else local_rank
    topo = topology(rank, world, local_rank, device, ndev, dist)
    solver = bos.BOS_SOLVER_SCHUR if args.solver == "schur" else bos.BOS_SOLVER_SUPERNODAL

    lpp = args.lanes_per_pose

    def make_handle(partition, mode):
        """A handle for `mode` (world 1: "single"; N > 1: "p2p", "rccl" or "gloo"). Collective-safe:
        every rank makes the same collective calls whatever fails locally (the RCCL id broadcast),
        then creates its handle locally; raises on a local failure."""
        nccl_id = None
        if mode == "rccl":
            uid = None
            if rank == 0:
                try:
                    uid = bos.nccl_unique_id()
                except Exception as e:   # broadcast None: every rank then fails this mode alike
                    log(f"rank 0: ncclGetUniqueId failed: {e}")
            obj = [uid]
            dist.broadcast_object_list(obj, src=0)
            nccl_id = obj[0]
            if nccl_id is None:
                raise RuntimeError("no RCCL unique id (ncclGetUniqueId failed on rank 0)")
        t0 = time.perf_counter()
        h = bos.Solver(P, precision=precision, solver=solver, device=device, rank=rank, world_size=world,
                       nccl_id=nccl_id, partition=partition, lanes_per_pose=lpp)
        try:
            inf = h.system_info()
            # the ranks the exchange actually spans: the communicator's count (RCCL), or the process group's
            seen = inf["comm_ranks"] if nccl_id is not None else (dist.get_world_size() if world > 1 else 1)
            log(f"rank {rank}: bos_create ({'observations' if partition else 'subtree'} partition, {mode}) "
                f"{time.perf_counter() - t0:.1f} s, n={inf['n']} nnz(H lower)={inf['nnz_lower']} "
                f"nnz(L)={inf['nnz_factor']}, ranks seen {seen}")
            if seen != args.gpus:
                raise RuntimeError(f"the exchange spans {seen} ranks, --gpus {args.gpus}")
        except Exception:
            h.close()
            raise
        return h, inf, seen

    # ---- one GN iteration, per exchange mode
    def gloo_allgather(h, which):
        mine = torch.from_numpy(h.exchange_download(which))
        parts = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(parts, mine)
        h.exchange_upload(which, torch.cat(parts).numpy())

    def gloo_allreduce(h):
        t = torch.from_numpy(h.exchange_download(1))
        dist.all_reduce(t)
        h.exchange_upload(1, t.numpy())

    def gn_step(h, partition, mode):
        if mode != "gloo":
            return h.step()
        if partition == bos.BOS_PARTITION_OBSERVATIONS:
            h.step_phase(0)
            gloo_allreduce(h)
            return h.step_phase(1)
        h.step_phase(0)
        gloo_allgather(h, 1)
        h.step_phase(1)
        gloo_allgather(h, 2)
        return h.step_phase(2)

    def quiet(fn, *a):
        try:
            fn(*a)
        except Exception as e:
            log(f"rank {rank}: {getattr(fn, '__name__', fn)}: {e}")

    def timed_steps(h, partition, k, warmup, mode, device_warmup=0):
        """`device_warmup` untimed GN iterations as one batch (not with the gloo exchange), `warmup`
        untimed GN iterations, then the state reset to the initial guess (outside the
        timed region) and k GN iterations from it, timed as one region: iterations 1..k of the solve
        (the world converges; tests/test_gpu_c3_gn.py checks 200 fp32 iterations positive definite).
        Collective-safe (N > 1): a local failure stops this rank's stepping but not its barriers and
        reductions, so every rank leaves together. Returns (wall seconds of the timed steps, max over
        ranks; per-step stats; the local error or None)."""
        err, init, stats = None, None, []
        try:
            init = h.get_state()
            if device_warmup > 0 and mode != "gloo":
                for b in range(0, device_warmup, 100):   # batches of <= 100 from the initial guess (the
                    h.step_n(min(100, device_warmup - b))  # trajectory tests/test_gpu_c3_gn.py checks)
                    h.set_state(*init)
            for _ in range(warmup):
                gn_step(h, partition, mode)
            h.set_state(*init)
            h.synchronize()
        except Exception as e:
            err = f"warm-up: {type(e).__name__}: {e}"
        barrier()
        quiet(h.synchronize)
        t0 = time.perf_counter()
        if err is None:
            try:
                for _ in range(k):
                    stats.append(gn_step(h, partition, mode))
                h.synchronize()
            except Exception as e:
                err = f"timed GN step {len(stats) + 1}: {type(e).__name__}: {e}"
        barrier()
        quiet(h.synchronize)
        wall = max_over_ranks(time.perf_counter() - t0)
        if init is not None:
            quiet(h.set_state, *init)
        bad = [i + 1 for i, g in enumerate(stats) if g["solver_info"] != 0]
        if err is None and bad:
            err = f"non-positive pivot or stall in benchmarked GN iterations {bad[:5]}"
        return wall, stats, err

    def chi2_agree(vals):
        """Every rank's chi^2 sequence equal bit for bit (NaN, a failed rank's placeholder, never is)."""
        if world == 1:
            return True
        mine = torch.tensor(vals, dtype=torch.float64)
        lo, hi = mine.clone(), mine.clone()
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        return bool(torch.equal(lo, hi))

    def check_and_time(mode, hinf, partition, k, warmup, device_warmup):
        """One exchange mode's run (collective-safe; raises at the end on a local or global failure):
        the direct exchange connected (every rank maps every other rank's mailbox), three GN steps from
        the initial guess giving every rank the same chi^2 (each rank combines all ranks' headers, so a
        payload that did not arrive intact shows as a difference), then the timed steps, whose per-step
        chi^2 must agree on every rank too."""
        h = hinf[0]
        err = None
        if mode == "p2p":
            mine = None
            try:
                mine = h.p2p_handle()
            except Exception as e:
                err = f"p2p handle: {e}"
            handles = [None] * world
            dist.all_gather_object(handles, mine)
            if err is None:
                try:
                    if any(x is None for x in handles):
                        raise RuntimeError("another rank has no mailbox handle")
                    h.p2p_connect(handles)
                except Exception as e:
                    err = f"p2p connect: {e}"
        if not agree_all(dist, torch, err is None)[0]:
            raise RuntimeError(err or "the direct exchange failed on another rank")
        chk = [float("nan")] * 3
        if world > 1:
            try:
                init = h.get_state()
                chk = [gn_step(h, partition, mode)["chi2"] for _ in range(3)]
                h.set_state(*init)
            except Exception as e:
                err = f"check steps: {type(e).__name__}: {e}"
                chk = [float("nan")] * 3
        same = chi2_agree(chk)
        if err is None and not same:
            err = "the ranks' chi^2 differ over three GN steps"
        if not agree_all(dist, torch, err is None)[0]:
            raise RuntimeError(err or "the check failed on another rank")
        wall, stats, err = timed_steps(h, partition, k, warmup, mode, device_warmup)
        vals = [g["chi2"] for g in stats] if err is None and len(stats) == k else [float("nan")] * k
        same = chi2_agree(vals)
        if err is None and not same:
            err = f"the ranks' per-step chi^2 differ (exchange {mode})"
        if err is not None:
            raise RuntimeError(err)
        return wall, stats

    def close_handle(hinf):
        if hinf is not None:
            quiet(hinf[0].close)

    # ---- the timed region: K GN iterations; the J+H inside them is the headline (K = 0: no GN steps,
    # the J+H builds alone, for profiling runs). N > 1: the exchange ladder (p2p -> RCCL -> gloo host
    # exchange, from --exchange on) — every rank takes the same decision, the line records why.
    modes = ("single",) if world == 1 else LADDER[args.exchange]
    mode, hinf, res, attempts = run_ladder(
        modes,
        setup=lambda m: make_handle(bos.BOS_PARTITION_SUBTREE, m),
        run=lambda m, hi: check_and_time(m, hi, bos.BOS_PARTITION_SUBTREE, args.steps, args.warmup,
                                         args.device_warmup) if args.steps > 0 or world > 1 else (0.0, []),
        agree=lambda ok, why: agree_all(dist, torch, ok, why),
        close=close_handle, log=log)
    if mode is None:
        fail_line(args, world, attempts, topo)
        sys.exit(4)
    S, info, ranks_seen = hinf
    exchange = {"single": "single GPU", "p2p": "p2p", "rccl": "rccl", "gloo": "gloo"}[mode]
    exchange_reason = None
    if world > 1:
        exchange_reason = {"p2p": "every rank mapped every other rank's mailbox (HIP IPC, peer access) and three GN "
                                  "steps gave every rank the same chi^2",
                           "rccl": "RCCL all-gathers; three GN steps gave every rank the same chi^2",
                           "gloo": "host exchange over the gloo process group (no device-to-device path)"}[mode]
        if args.exchange != mode:
            exchange_reason += f" (--exchange {args.exchange} failed, see attempts)"
    wall, stats = res
    phase, jh_ms, gn_it_s = None, None, None
    ranks_consistent = True if world > 1 and args.steps > 0 else None
    per_rank = None

    def phases(stats):
        return {k: float(np.median([g[k] for g in stats])) for k in
                ("t_linearize_ms", "t_exchange_ms", "t_solve_ms", "t_update_ms")}

    def rank_breakdown(h, partition, steps=20):
        """Per-rank phase times (device stamps of the step's own kernels, bos_last_step_stamps), the
        median over `steps` untimed GN iterations after the timed region, gathered to every rank:
        J+H, own subtrees (solver inputs, factorization and forward of this rank's subtrees, exchange-1
        pack), exchange-1 wait, replicated top (its factorization and solves) + own backward + pack,
        exchange-2 wait, box-plus + status. Lists in rank order; None on any rank's failure."""
        med = None
        try:
            init = h.get_state()
            rows = []
            for _ in range(steps):
                gn_step(h, partition, mode)
                t = h.last_step_stamps().astype(np.int64)
                d = lambda a, b: max(0.0, float(t[b] - t[a]) * 1e-5)   # ms (100 MHz ticks)
                rows.append([d(0, 1), d(1, 4), d(4, 5), d(5, 6), d(6, 7), d(7, 3), d(0, 3)])
            h.set_state(*init)
            med = [float(x) for x in np.median(np.array(rows), axis=0)]
        except Exception as e:
            log(f"rank {rank}: per-rank breakdown: {e}")
        allr = [None] * world
        dist.all_gather_object(allr, med)
        if any(r is None for r in allr):
            return None
        keys = ("jh_ms", "own_subtrees_ms", "exchange1_wait_ms", "top_and_backward_ms", "exchange2_wait_ms",
                "update_ms", "step_device_ms")
        return {k: [r[i] for r in allr] for i, k in enumerate(keys)}

    if args.steps > 0:
        phase = phases(stats)
        jh_ms = max_over_ranks(phase["t_linearize_ms"])      # the slowest rank's in-step J+H
        if world > 1:
            per_rank = rank_breakdown(S, partition=bos.BOS_PARTITION_SUBTREE)
        gn_it_s = args.steps / wall
        log(f"rank {rank}: {args.steps} GN steps in {wall * 1e3:.1f} ms ({gn_it_s:.0f} it/s); phases {phase}")

    def local(fn, what):
        """A secondary measurement on this rank: its value, or None (logged) if it raised."""
        try:
            return fn()
        except Exception as e:
            log(f"rank {rank}: {what}: {type(e).__name__}: {e}")
            return None

    def max_or_none(v):
        """Max over ranks of a secondary measurement; None if any rank has none (collective-safe)."""
        m = max_over_ranks(float("nan") if v is None else float(v))
        return None if m != m else m

    # ---- other GN loops (the headline's timed region above is the reference for value)
    gn_c_loop, gn_batched = None, None
    init = S.get_state()
    if args.steps > 0 and mode != "gloo":
        c_ms = max_or_none(local(lambda: S.time_steps(min(args.steps, 50)), "C-loop steps"))   # bos_step in a C loop
        gn_c_loop = 1e3 / c_ms if c_ms else None
        local(lambda: S.set_state(*init), "state reset")
        barrier()
        tg = time.perf_counter()

        def batch():
            last = S.step_n(args.batch)                       # executables/bearing_only_slam.cpp:95-98
            S.synchronize()
            if last["solver_info"] != 0:
                raise RuntimeError("non-positive pivot in a benchmarked GN step")
            return True
        ok = local(batch, "batched steps")
        barrier()
        dt = max_or_none(time.perf_counter() - tg if ok else None)
        gn_batched = args.batch / dt if dt else None
        local(lambda: S.set_state(*init), "state reset")

    # ---- the drop-in caller's loop: proj02::Solver::step() through the C++ façade, as the reference's
    # executable calls it (executables/bearing_only_slam.cpp:93-99), then one read of solver.state
    facade = None
    if world == 1 and args.steps > 0:
        nf = min(args.steps, 50)
        f = bos.time_facade_steps(P, nf, bos.options(solver=solver, precision=precision, lanes_per_pose=lpp))
        facade = {"steps": nf, "ms_per_step": f["ms_per_step"], "ms_state_read": f["ms_state_read"],
                  "gn_iters_per_s_incl_state_read": nf / ((nf * f["ms_per_step"] + f["ms_state_read"]) * 1e-3),
                  "gn_iters_per_s_c_loop_same_handle": 1e3 / f["ms_per_step_capi"],
                  "state_mismatches_vs_device": f["state_mismatches"]}
        assert f["state_mismatches"] == 0, "solver.state differs from the device state"
        log(f"facade: {1e3 / f['ms_per_step']:.0f} it/s, state read {f['ms_state_read']:.2f} ms, C loop on the same "
            f"handle {1e3 / f['ms_per_step_capi']:.0f} it/s")

    # ---- the J+H alone: back to back (warm replay) and from cold caches (events)
    barrier()
    replay_ms = max_or_none(local(lambda: S.time_linearize(args.replay_steps), "warm J+H")) \
        if args.replay_steps > 0 else None
    cold_ms = max_or_none(local(lambda: S.time_linearize(args.cold_steps, flush_caches=True), "cold J+H")) \
        if args.cold_steps > 0 else None

    gn_other = None
    if world == 1 and not args.no_gn_other and args.steps > 0:   # the other multifrontal ordering
        other = "supernodal" if args.solver == "schur" else "schur"
        S2 = bos.Solver(P, precision=precision, device=device,
                        solver=bos.BOS_SOLVER_SUPERNODAL if other == "supernodal" else bos.BOS_SOLVER_SCHUR)
        w2, st2, err2 = timed_steps(S2, bos.BOS_PARTITION_SUBTREE, min(args.steps, 50), 1, "single")
        gn_other = {"solver": other, "gn_iters_per_s": min(args.steps, 50) / w2,
                    "t_solve_ms": phases(st2)["t_solve_ms"]} if err2 is None else {"solver": other, "error": err2}
        S2.close()

    # ---- N > 1: the north star's partition (observations by measurement order, all-reduce of (H, b)),
    # a secondary leg through its own ladder (RCCL all-reduce, else gloo on the host with fewer steps;
    # a failure is reported in the line, never fatal to it)
    part_obs = None
    if world > 1 and not args.no_partition_other and args.steps > 0:
        obs_modes = tuple(m for m in ("rccl", "gloo") if not any(t["mode"] == m and not t["ok"] for t in attempts))
        obs_steps = lambda m: args.steps if m == "rccl" else min(args.steps, 5)
        mode3, h3, res3, att3 = run_ladder(
            obs_modes,
            setup=lambda m: make_handle(bos.BOS_PARTITION_OBSERVATIONS, m),
            run=lambda m, hi: check_and_time(m, hi, bos.BOS_PARTITION_OBSERVATIONS, obs_steps(m),
                                             min(args.warmup, 2), 0),
            agree=lambda ok, why: agree_all(dist, torch, ok, why),
            close=close_handle, log=log)
        if mode3 is None:
            part_obs = {"error": "no exchange mode worked", "attempts": att3}
        else:
            w3, st3 = res3
            ph3 = phases(st3)
            jh3 = max_over_ranks(ph3["t_linearize_ms"])
            ex3 = max_over_ranks(ph3["t_exchange_ms"])
            part_obs = {"partition": "observations (measurement-order lane ranges, one all-reduce of (H, b) per "
                                     "iteration, solve replicated)",
                        "exchange": mode3, "attempts": att3, "steps": obs_steps(mode3),
                        "ranks_seen": h3[2], "gn_iters_per_s": obs_steps(mode3) / w3, "gn_phase_ms": ph3,
                        "jh_ms_max_rank": jh3, "jh_obs_per_s": nobs / (jh3 * 1e-3) if jh3 > 0 else None,
                        "jh_plus_allreduce_obs_per_s": nobs / ((jh3 + ex3) * 1e-3) if jh3 + ex3 > 0 else None,
                        "allreduce_bytes": int(info["num_block_values"] + 3 * P.NP + 2 * P.NL) *
                        (4 if precision == bos.BOS_FP32 else 8)}
            close_handle(h3)

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
        layout = info["layout_bytes"]
        traffic, traffic_src = traffic_from_profile(precision) if world == 1 else (None, None)

        def roof(ms, label, timing):
            a = algo / (ms * 1e-3) / 1e9
            return {"bound": "hbm", "achieved": a, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": a / HBM_PEAK_GBS,
                    "traffic": traffic.get("warm" if label == "warm" else "instep") if traffic else None,
                    "traffic_source": traffic_src.get("warm" if label == "warm" else "instep") if traffic_src else
                    "not collected for N > 1",
                    "algorithmic_bytes_per_launch": algo, "kernel_ms": ms, "caches": label, "timing": timing,
                    # the bytes this layout moves at minimum (pose-landmark blocks stored as 3 factors
                    # when pl_factored) and the fraction of the roofline on those
                    "layout_bytes_per_launch": layout, "frac_layout": layout / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS}
        r_instep = roof(jh_ms, "in-step", "median over the timed GN steps of the device realtime clock from the "
                        "J+H launch's start to the next launch's start (stamped by the step's kernels); max over ranks") \
            if jh_ms else None
        r_cold = roof(cold_ms, "cold", "HIP events around each build, 512 MiB read before it (event cost included)") \
            if cold_ms else None
        r_warm = roof(replay_ms, "warm", "HIP events around the back-to-back builds") if replay_ms else None
        head_ms = jh_ms if jh_ms else replay_ms   # K = 0 (profiling runs): the back-to-back builds
        value = nobs / (head_ms * 1e-3)
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "obs/s",
            "n_gpus": ranks_seen,
            "steps": args.steps,
            "warmup": args.warmup,
            "device_warmup": args.device_warmup if args.steps > 0 else 0,
            "ms_per_step": head_ms,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32" if precision == bos.BOS_FP32 else "f64",
            "data": "synthetic",
            "config": {
                "workload": "config 3: synthetic 100k poses / 200k landmarks / 1M bearings / 99999 odometry "
                            "edges; J+H build " + ("fp32" if precision == bos.BOS_FP32 else "fp64") +
                            " inside full GN iterations (solve fp64, " + args.solver + ")",
                "poses": P.NP, "landmarks": P.NL, "bearings": int(len(P.b_z)), "odometry": int(len(P.o_z)),
                "parallelism": (f"subtree-sharded x{world} ({exchange} exchanges; top fronts replicated: "
                                f"{info['top_fronts']})") if world > 1 else "single GPU",
                "exchange": exchange,
                "lanes_per_pose": info["lanes_per_pose"],
            },
            "ranks_seen": ranks_seen,
            "ranks_consistent": ranks_consistent,
            "exchange_decision": {"mode": exchange, "reason": exchange_reason, "attempts": attempts}
            if world > 1 else None,
            # every rank's device and visibility, rank 0's peer-access matrix (hipDeviceCanAccessPeer)
            "topology": topo if world > 1 else None,
            # N > 1: per-rank phase medians (device stamps), rank order (rank_breakdown)
            "per_rank": per_rank,
            "devices": 1 if (args.same_device or world == 1) else world,
            "timed_region_ms": wall * 1e3,
            "gn_iters_per_s": gn_it_s,
            "gn_iters_per_s_c_loop": gn_c_loop,
            "gn_iters_per_s_batched": gn_batched,
            # proj02::Solver::step() through the C++ façade (solver.state lazily downloaded on read)
            "gn_iters_per_s_facade": 1e3 / facade["ms_per_step"] if facade else None,
            "facade": facade,
            "gn_phase_ms": phase,
            "solver_model": solver_model(P, phase, world),
            "gn_solver": args.solver,
            "gn_other": gn_other,
            "partition_observations": part_obs,
            "triangulation": tri,
            # the J+H as it runs inside the GN iteration (inputs from HBM after the solver's stream);
            # the same from cold caches by events, and the back-to-back replay (working set partly
            # cache resident), beside it
            "roofline": r_instep or r_warm,
            "roofline_cold_events": r_cold,
            "roofline_warm_replay": r_warm,
            "libbos_sha256": lib_sha256(),
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

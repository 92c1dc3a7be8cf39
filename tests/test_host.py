"""CPU tests of the product's host code (libbos.so) — loader, triangulation, synthetic worlds,
the static plan and the C ABI — without a GPU. No compute call reaches the HIP path here."""
import os
import re
import subprocess

import numpy as np
import pytest
import scipy.sparse as sp
import scipy.sparse.linalg as spla

import bos
import oracle as O
from conftest import C1, MINI, ROOT
from helpers import oracle_lower_nf, to_oracle


def _header_functions():
    names = set()
    for h in ("bos.h", "bos_host.h"):
        txt = open(os.path.join(ROOT, "include", h)).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        for m in re.finditer(r"\b(bos_[a-z0-9_]+)\s*\(", txt):
            names.add(m.group(1))
    return names


def test_library_exports_every_header_symbol():
    L = bos.lib()
    names = _header_functions()
    assert names, "no declarations parsed"
    missing = [n for n in sorted(names) if not hasattr(L, n)]
    assert not missing, missing
    assert set(bos.EXPORTED_SYMBOLS) == names
    assert L.bos_abi_version() == bos.ABI_VERSION == 3


@pytest.mark.skipif(bos.device_count() > 0, reason="a HIP device is visible")
def test_create_fails_loudly_without_gpu():
    P = bos.load_g2o(MINI)
    with pytest.raises(bos.BosError, match="no HIP device"):
        bos.Solver(P)


def test_headless_driver_without_gpu_exits_nonzero():
    exe = os.path.join(ROOT, "prb-project-bearing-only-slam_amd", "lib", "bearing_only_slam")
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 1 and "usage" in r.stdout
    if bos.device_count() == 0:
        r = subprocess.run([exe, MINI, "--iters", "1", "--quiet"], capture_output=True, text=True)
        assert r.returncode == 2 and "no HIP device" in r.stderr


@pytest.mark.parametrize("path", [MINI, C1])
def test_loader_and_triangulation_match_oracle(path):
    P = bos.load_g2o(path)
    Q = O.load(path)
    assert np.array_equal(P.pose_ids, Q.pose_ids) and np.array_equal(P.lm_ids, Q.lm_ids)
    assert np.array_equal(P.pose_xyt, Q.pose_xyt)
    assert np.array_equal(P.b_pose, Q.b_pose) and np.array_equal(P.b_lm, Q.b_lm)
    assert np.array_equal(P.b_z, Q.b_z)
    assert np.array_equal(P.o_src, Q.o_src) and np.array_equal(P.o_dst, Q.o_dst)
    assert np.array_equal(P.o_z, Q.o_z) and np.array_equal(P.o_omega, Q.o_omega)
    assert P.fixed == Q.fixed
    # independent implementations of the column-pivoted least squares (MGS vs Householder)
    assert np.abs(P.lm_xy - Q.lm_xy).max() <= 1e-9 * max(1.0, np.abs(Q.lm_xy).max())
    cnt = np.bincount(P.b_lm, minlength=P.NL)
    for j in np.nonzero(cnt == 1)[0]:
        assert np.array_equal(P.lm_xy[j] == 0.0, Q.lm_xy[j] == 0.0)


def test_loader_edge_cases(tmp_path):
    f = tmp_path / "x.g2o"
    # no FIX (default = first pose), empty lines, unknown tokens, info column ignored
    f.write_text("VERTEX_SE2 7 0 0 0\n\nVERTEX_SE2 8 1 0 0\nFOO 1 2\n"
                 "EDGE_SE2 7 8 1 0 0 500 0 0 500 0 5000\n"
                 "EDGE_BEARING_SE2_XY 7 3 0.5 1234\nEDGE_BEARING_SE2_XY 8 3 1.2 99\n")
    P = bos.load_g2o(str(f))
    assert P.fixed == 0 and P.fixed_pose_id == 7
    assert P.NP == 2 and P.NL == 1 and len(P.b_z) == 2 and len(P.o_z) == 1
    with pytest.raises(bos.BosError):
        bos.load_g2o(str(tmp_path / "missing.g2o"))
    g = tmp_path / "bad.g2o"
    g.write_text("VERTEX_SE2 1 abc 0 0\n")
    with pytest.raises(bos.BosError):
        bos.load_g2o(str(g))
    h = tmp_path / "unknown_id.g2o"
    h.write_text("VERTEX_SE2 1 0 0 0\nEDGE_SE2 1 2 1 0 0 1 0 0 1 0 1\nEDGE_BEARING_SE2_XY 1 5 0.1 1\n")
    with pytest.raises(bos.BosError, match="unknown id"):
        bos.load_g2o(str(h))


def test_g2o_writer_roundtrip(tmp_path):
    P = bos.load_g2o(C1)
    out = str(tmp_path / "dump.g2o")
    bos.write_g2o(P, out, source=C1)
    g = O.parse_g2o(out)
    assert len(g.pose_ids) == P.NP and len(g.lm_vertex_ids) == P.NL
    assert np.allclose(np.array(g.pose_xyt)[:, :2], P.pose_xyt[:, :2], atol=1e-12)
    assert np.allclose(np.array(g.lm_vertex_xy), P.lm_xy, atol=1e-12)
    assert g.fixed_pose_id == 1498
    assert len(g.bearing_raw) == len(P.b_z) and len(g.odom_z) == len(P.o_z)


def test_synthetic_world_properties():
    P = bos.synthetic(600, 1200, 14, seed=7)
    assert (P.NP, P.NL, len(P.b_z), len(P.o_z)) == (600, 1200, 600 * 14, 599)
    assert np.all(np.bincount(P.b_pose, minlength=P.NP) == 14)
    assert np.bincount(P.b_lm, minlength=P.NL).min() >= 2
    pairs = P.b_pose.astype(np.int64) * P.NL + P.b_lm
    assert len(np.unique(pairs)) == len(pairs)
    assert P.fixed == 0 and np.array_equal(P.pose_xyt[0], P.gt_pose_xyt[0])
    # the initial guess is the dead-reckoned odometry chain
    Q = to_oracle(P)
    for k in range(len(P.o_z)):
        pred = O.predict_odometry(Q.pose_xyt[P.o_src[k]], Q.pose_xyt[P.o_dst[k]])
        d = pred - P.o_z[k]
        d[2] = (d[2] + np.pi) % (2 * np.pi) - np.pi
        assert np.abs(d).max() < 1e-9
    # visible (|bearing| < pi/2) from ground truth
    for k in range(0, len(P.b_z), 97):
        b = O.predict_bearing(P.gt_pose_xyt[P.b_pose[k]], P.gt_lm_xy[P.b_lm[k]])
        assert abs(b) < np.pi / 2
    Q2 = bos.synthetic(600, 1200, 14, seed=7)
    assert np.array_equal(P.b_z, Q2.b_z) and np.array_equal(P.lm_xy, Q2.lm_xy)
    Q3 = bos.synthetic(600, 1200, 14, seed=8)
    assert not np.array_equal(P.b_z, Q3.b_z)
    with pytest.raises(bos.BosError):
        bos.synthetic(10, 100, 2)


def ray_parallax(P):
    """Per landmark: the spread (rad) of the world-frame ray angles from its observing poses, at
    ground truth."""
    gp, gl = P.gt_pose_xyt, P.gt_lm_xy
    bp, bl = P.b_pose, P.b_lm
    ang = np.arctan2(gl[bl, 1] - gp[bp, 1], gl[bl, 0] - gp[bp, 0])
    ref = np.zeros(P.NL)
    ref[bl[::-1]] = ang[::-1]   # the first observation's ray
    d = (ang - ref[bl] + np.pi) % (2 * np.pi) - np.pi
    lo = np.zeros(P.NL)
    hi = np.zeros(P.NL)
    np.minimum.at(lo, bl, d)
    np.maximum.at(hi, bl, d)
    return hi - lo


@pytest.mark.parametrize("size", [(1000, 2000, 20, 0xB05EED01 + 2), (100000, 200000, 10, 0xB05EED01 + 3)])
def test_synthetic_world_parallax(size):
    """every landmark observed >= 2 times with parallax. The generator guarantees a
    ray spread >= 20 deg (csrc/host/synthetic.cpp), and every bearing is in front of its pose
    (|bearing| < 85 deg) — the property that makes GN converge on the benchmark world (the old
    generator's 0.8 deg tail never did)."""
    P = bos.synthetic(*size)
    par = ray_parallax(P)
    assert np.bincount(P.b_lm, minlength=P.NL).min() >= 2
    assert par.min() >= np.radians(20.0) * (1 - 1e-12), np.degrees(par.min())
    g = P.gt_pose_xyt[P.b_pose]
    l = P.gt_lm_xy[P.b_lm]
    c, s = np.cos(g[:, 2]), np.sin(g[:, 2])
    dx, dy = l[:, 0] - g[:, 0], l[:, 1] - g[:, 1]
    bearing = np.arctan2(-s * dx + c * dy, c * dx + s * dy)
    assert np.abs(bearing).max() < np.radians(85.0)
    assert np.hypot(dx, dy).min() > 0.5


@pytest.mark.parametrize("which", ["mini", "c1", "c2"])
def test_plan_pattern_matches_oracle(which):
    P = {"mini": lambda: bos.load_g2o(MINI), "c1": lambda: bos.load_g2o(C1),
         "c2": lambda: bos.synthetic(1000, 2000, 20)}[which]()
    Q = to_oracle(P)
    info = bos.plan_inspect(P, entries=True)
    H = oracle_lower_nf(Q, O.linearize(Q)).tocoo()
    S = set(zip(H.row.tolist(), H.col.tolist()))
    T = set(zip(info["rows"].tolist(), info["cols"].tolist()))
    assert S == T and len(T) == info["nnz_lower"]
    assert info["ordering"] == "nested-dissection"
    perm = info["perm_to_ref"]
    assert sorted(perm.tolist()) == list(range(P.N))
    assert set(perm[info["n"]:].tolist()) == {3 * P.fixed, 3 * P.fixed + 1, 3 * P.fixed + 2}


@pytest.mark.parametrize("which", ["mini", "c1", "c2"])
def test_consecutive_pose_landmark_lanes(which):
    """A landmark lane whose poses are consecutive (p0, p0 + 1, ..., no repeat) reads no pose
    records (LinParams::ll_run); the plan's count equals a direct count over the bearings."""
    P = {"mini": lambda: bos.load_g2o(MINI), "c1": lambda: bos.load_g2o(C1),
         "c2": lambda: bos.synthetic(1000, 2000, 20)}[which]()
    want = 0
    for lm in range(P.lm_xy.shape[0]):
        poses = np.sort(P.b_pose[P.b_lm == lm])
        want += poses.size > 0 and bool(np.all(poses == poses[0] + np.arange(poses.size)))
    info = bos.plan_inspect(P, solver=bos.BOS_SOLVER_SCHUR)
    assert info["lm_lanes_consecutive"] == want
    if which == "c2":   # the synthetic generator's windows are consecutive poses
        assert want == P.lm_xy.shape[0]
    # odometry chain poses (BlockLayout::po_chain): exactly edges p - 1 = (p - 1, p), p = (p, p + 1)
    NP, Mo = P.pose_xyt.shape[0], len(P.o_src)
    chain = 0
    for p in range(1, NP - 1):
        mine = np.nonzero(((P.o_src == p) | (P.o_dst == p)) & (P.o_src != P.o_dst))[0]
        chain += (p < Mo and sorted(mine.tolist()) == [p - 1, p] and P.o_src[p - 1] == p - 1 and P.o_dst[p - 1] == p
                  and P.o_src[p] == p and P.o_dst[p] == p + 1)
    assert info["pose_odometry_chain"] == chain
    if which == "c2":   # the synthetic trajectory is one chain
        assert chain == NP - 2


@pytest.mark.parametrize("solver", ["supernodal", "schur"])
@pytest.mark.parametrize("which", ["c1", "c2"])
def test_multifrontal_structure_solves_like_scipy(which, solver):
    """The supernodal tree and its maps (host/plan.cpp build_multifrontal) re-run on the host
    reproduce a SciPy solve of H_nf x = b."""
    P = bos.load_g2o(C1) if which == "c1" else bos.synthetic(1000, 2000, 20)
    kind = bos.BOS_SOLVER_SCHUR if solver == "schur" else bos.BOS_SOLVER_SUPERNODAL
    Q = to_oracle(P)
    lin = O.linearize(Q)
    Hl = oracle_lower_nf(Q, lin).tocsr()
    info = bos.plan_inspect(P, entries=True, solver=kind)
    vals = np.asarray(Hl[info["rows"], info["cols"]]).ravel()
    n = info["n"]
    perm = info["perm_to_ref"][:n]
    x = bos.plan_mf_selftest(P, vals, lin.b[perm], solver=kind)
    Hf = (Hl + sp.tril(Hl, -1).T).tocsc()
    keep = np.ones(P.N, dtype=bool)
    keep[3 * P.fixed:3 * P.fixed + 3] = False
    idx = np.nonzero(keep)[0]
    xr = np.zeros(P.N)
    xr[idx] = spla.spsolve(Hf[idx][:, idx], lin.b[idx])
    assert np.abs(x - xr[perm]).max() <= 1e-8 * np.abs(xr).max()
    assert info["mf_levels"] >= 1 and info["mf_max_front"] >= 3
    if solver == "schur":   # every landmark is its own 2-column supernode, eliminated before any pose
        assert info["ordering"] == "schur-landmarks-first"
        assert info["mf_supernodes"] > P.NL and set(perm[:2 * P.NL].tolist()) == set(range(3 * P.NP, P.N))


def _system(P, solver):
    """Stored entries of H_nf (one-rank plan order) and the right-hand side in the permuted order."""
    Q = to_oracle(P)
    lin = O.linearize(Q)
    Hl = oracle_lower_nf(Q, lin).tocsr()
    info = bos.plan_inspect(P, entries=True, solver=solver)
    vals = np.asarray(Hl[info["rows"], info["cols"]]).ravel()
    perm = info["perm_to_ref"][:info["n"]]
    return vals, lin.b[perm], Hl, lin, perm


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("which", ["c1", "synthetic"])
@pytest.mark.parametrize("solver", ["schur", "supernodal"])
def test_sharded_solve_equals_one_rank(world, which, solver):
    """The multi-GPU algorithm (subtree shards + replicated top, two exchanges; host/shard.cpp) run on
    the host for every rank: each rank holds only the H its own J+H lanes compute, the merged
    solution equals the one-rank solution bit for bit, the ranks agree on the top, every observation's
    chi^2 is counted by exactly one rank, and every node a rank's J+H reads stays current (the
    selftest raises otherwise). The N>1 data path checked without N GPUs."""
    P = bos.load_g2o(C1) if which == "c1" else bos.synthetic(3000, 6000, 10, seed=5)
    kind = bos.BOS_SOLVER_SCHUR if solver == "schur" else bos.BOS_SOLVER_SUPERNODAL
    vals, rhs, Hl, lin, perm = _system(P, kind)
    x = bos.plan_shard_selftest(P, world, vals, rhs, solver=kind)
    x1 = bos.plan_mf_selftest(P, vals, rhs, solver=kind)
    assert np.array_equal(x, x1)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_shard_partition(world):
    """Every node but the fixed pose has one owner (a rank or the replicated top); every rank has
    subtrees; each rank's plan computes exactly the stored entries of H its fronts read (validated
    per rank) and together the ranks compute every entry; the J+H lanes of all ranks cover every
    pose and landmark; the top is small next to the subtrees."""
    P = bos.synthetic(10000, 20000, 10, seed=3)
    own = bos.plan_node_owner(P, world)
    assert own[P.fixed] == -2 and np.all(own[np.arange(P.NP + P.NL) != P.fixed] >= -1)
    counts = np.bincount(own[own >= 0], minlength=world)
    assert np.all(counts > 0)
    assert (own == -1).sum() < 0.05 * len(own)
    assert counts.max() <= 1.25 * counts.mean()
    computed = None
    b_cov = np.zeros(P.N, dtype=int)
    for r in range(world):
        info = bos.plan_inspect(P, r, world, entries=True, solver=bos.BOS_SOLVER_SCHUR)
        computed = info["owned"].astype(int) if computed is None else computed + info["owned"]
        b_cov += info["b_owned"]
        assert info["shard_top_fronts"] > 0 and info["shard_own_fronts"] > 0
    assert np.all(computed >= 1)
    keep = np.ones(P.N, dtype=bool)
    keep[3 * P.fixed:3 * P.fixed + 3] = False
    assert np.all(b_cov[keep] >= 1)


def test_lanes_per_pose_rule():
    """plan_lanes_per_pose: one lane per pose on one GPU, two on sharded ranks when no (pose,
    landmark) or odometry pair repeats (interleaved groups, bit-identical to one lane), one with a
    repeated pair (a split would change the summation order); an explicit option wins."""
    P = bos.synthetic(2000, 4000, 10, seed=5)
    lpp = lambda Q, world, opt=0: bos.plan_inspect(Q, 0, world, solver=bos.BOS_SOLVER_SCHUR,
                                                    lanes_per_pose=opt)["lanes_per_pose"]
    assert lpp(P, 1) == 1 and lpp(P, 2) == 2 and lpp(P, 8) == 2 and lpp(P, 2, 1) == 1 and lpp(P, 1, 4) == 4
    D = bos.Problem(P.pose_xyt, P.lm_xy, np.append(P.b_pose, P.b_pose[0]), np.append(P.b_lm, P.b_lm[0]),
                    np.append(P.b_z, P.b_z[0]), P.o_src, P.o_dst, P.o_z, P.o_omega, P.fixed)
    assert lpp(D, 1) == 1 and lpp(D, 2) == 1


def test_shard_world1_is_the_unsharded_plan():
    P = bos.load_g2o(C1)
    a = bos.plan_inspect(P, 0, 1, solver=bos.BOS_SOLVER_SCHUR)
    assert a["shard_top_fronts"] == 0 and a["shard_pose_lanes"] == P.NP and a["shard_lm_lanes"] == P.NL
    own = bos.plan_node_owner(P, 1)
    assert np.all(own[np.arange(P.NP + P.NL) != P.fixed] == 0)


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_schur_plan_fronts_fit_the_wave_kernels(seed):
    """The Schur plan retries other separator balances until every front fits the fast kernels:
    m <= 64 (one wavefront) everywhere and m <= 48 (the dataflow launch) from level 2 up; the
    default 40 % leaves a 66-row front on some of these worlds."""
    P = bos.synthetic(30000, 60000, 10, seed=seed)
    info = bos.plan_inspect(P, 0, 1, solver=bos.BOS_SOLVER_SCHUR)
    assert info["mf_fits"]
    assert info["mf_max_front"] <= 64 and info["mf_max_front_upper"] <= 48
    assert info["mf_balance_pct"] in (40, 35, 45, 30, 20)


@pytest.mark.parametrize("seed", [1, 2])
def test_schur_folds_alone_read_the_landmark_region(seed):
    """With the Schur ordering every landmark is folded into a pose front, so only the folds read the
    pose-landmark and landmark-diagonal entries of H (bos::mf_fold_reads_fp32): an fp32 build's folds
    then read them from the fp32 block array and its fp64 copy skips the region. The
    nested-dissection ordering factors landmark fronts itself, so it must not qualify."""
    P = bos.synthetic(3000, 6000, 10, seed=seed)
    assert bos.plan_inspect(P, 0, 1, solver=bos.BOS_SOLVER_SCHUR)["mf_fold_fp32"]
    assert not bos.plan_inspect(P, 0, 1, solver=bos.BOS_SOLVER_SUPERNODAL)["mf_fold_fp32"]


def test_schur_plan_fallback_keeps_a_valid_plan():
    """When no separator balance fits (forced here with 40-pose leaves: every leaf front has more
    than 64 rows), the first (40 %) plan is kept; it still validates and solves like SciPy."""
    P = bos.load_g2o(C1)
    info = bos.plan_inspect(P, 0, 1, entries=True, solver=bos.BOS_SOLVER_SCHUR, schur_leaf=40)
    assert not info["mf_fits"] and info["mf_balance_pct"] == 40 and info["mf_max_front"] > 64
    Q = to_oracle(P)
    lin = O.linearize(Q)
    Hl = oracle_lower_nf(Q, lin).tocsr()
    vals = np.asarray(Hl[info["rows"], info["cols"]]).ravel()
    perm = info["perm_to_ref"][:info["n"]]
    x = bos.plan_mf_selftest(P, vals, lin.b[perm], solver=bos.BOS_SOLVER_SCHUR, schur_leaf=40)
    Hf = (Hl + sp.tril(Hl, -1).T).tocsc()
    keep = np.ones(P.N, dtype=bool)
    keep[3 * P.fixed:3 * P.fixed + 3] = False
    idx = np.nonzero(keep)[0]
    xr = np.zeros(P.N)
    xr[idx] = spla.spsolve(Hf[idx][:, idx], lin.b[idx])
    assert np.abs(x - xr[perm]).max() <= 1e-8 * np.abs(xr).max()


def _with_odometry(P, src, dst, z, om):
    return bos.Problem(P.pose_xyt, P.lm_xy, P.b_pose, P.b_lm, P.b_z, np.concatenate([P.o_src, src]),
                       np.concatenate([P.o_dst, dst]), np.concatenate([P.o_z, z]), np.concatenate([P.o_omega, om]),
                       P.fixed, pose_ids=P.pose_ids, lm_ids=P.lm_ids)


@pytest.mark.parametrize("solver", [bos.BOS_SOLVER_SCHUR, bos.BOS_SOLVER_SUPERNODAL, bos.BOS_SOLVER_ROCSOLVER_RF])
def test_plan_accepts_reversed_edges_and_self_loops(solver):
    """Inputs the reference handles (slam/solver.cpp:48-62): odometry edges in both directions
    between two poses, and self-loops. The plan validates (every block written once), the reversed
    pair shares one pose-pose block, and the multifrontal tree still solves like SciPy."""
    P = bos.load_g2o(C1)
    k = np.arange(0, 40, 4)
    src = np.concatenate([P.o_dst[k], [5, 77]]).astype(np.int32)
    dst = np.concatenate([P.o_src[k], [5, 77]]).astype(np.int32)
    z = np.zeros((len(src), 3))
    z[:len(k)] = -P.o_z[k]
    om = np.concatenate([P.o_omega[k], P.o_omega[:2]])
    V = _with_odometry(P, src, dst, z, om)
    info = bos.plan_inspect(V, 0, 1, entries=True, solver=solver)
    base = bos.plan_inspect(P, 0, 1, solver=solver)
    assert info["nnz_lower"] == base["nnz_lower"]   # no new structure: same pairs, loops add nothing
    if solver == bos.BOS_SOLVER_ROCSOLVER_RF:
        return
    Q = to_oracle(V)
    lin = O.linearize(Q)
    Hl = oracle_lower_nf(Q, lin).tocsr()
    vals = np.asarray(Hl[info["rows"], info["cols"]]).ravel()
    perm = info["perm_to_ref"][:info["n"]]
    x = bos.plan_mf_selftest(V, vals, lin.b[perm], solver=solver)
    Hf = (Hl + sp.tril(Hl, -1).T).tocsc()
    keep = np.ones(V.N, dtype=bool)
    keep[3 * V.fixed:3 * V.fixed + 3] = False
    idx = np.nonzero(keep)[0]
    xr = np.zeros(V.N)
    xr[idx] = spla.spsolve(Hf[idx][:, idx], lin.b[idx])
    assert np.abs(x - xr[perm]).max() <= 1e-8 * np.abs(xr).max()


def test_oracle_self_loop_adds_chi2_only():
    """The oracle's self-loop semantics (J_s + J_d = 0 exactly): H and b are those of the problem
    without the loop; chi^2 grows by the loop's rho = z^T Omega z (theta wrapped)."""
    P = bos.load_g2o(C1)
    z = np.array([[0.3, -0.2, 0.1]])
    om = P.o_omega[:1]
    V = _with_odometry(P, np.array([9], np.int32), np.array([9], np.int32), z, om)
    a, b = O.linearize(to_oracle(P)), O.linearize(to_oracle(V))
    assert np.array_equal(a.pose_diag, b.pose_diag) and np.array_equal(a.b, b.b)
    assert np.all(b.hoff[-1] == 0.0)
    e = -z[0]
    assert abs(b.chi2 - a.chi2 - e @ om[0] @ e) < 1e-12


def test_parallel_g2o_parser_equals_line_parser(tmp_path, monkeypatch):
    """The chunked parallel g2o parser (default) and the line-by-line one give identical problems,
    on the reference dataset and on a written synthetic world large enough to use several chunks."""
    import ctypes
    L = bos.lib()
    h = ctypes.c_void_p()
    assert L.bos_dataset_synthetic(3000, 6000, 10, 7, ctypes.byref(h)) == 0
    path = str(tmp_path / "w.g2o")
    assert L.bos_dataset_write_g2o(h, path.encode(), None, None, 1) == 0
    L.bos_dataset_free(h)
    with open(path, "a") as f:   # pad past 1 MiB so the parser cuts several chunks
        f.write("\n" * (3 << 20))
    keys = ("pose_xyt", "lm_xy", "b_pose", "b_lm", "b_z", "o_src", "o_dst", "o_z", "o_omega", "pose_ids", "lm_ids")
    for p in (C1, path):
        bos.lib().bos_debug_set_g2o_parser(1)
        try:
            A = bos.load_g2o(p)
        finally:
            bos.lib().bos_debug_set_g2o_parser(0)
        B = bos.load_g2o(p)
        assert A.fixed == B.fixed
        for k in keys:
            assert np.array_equal(getattr(A, k), getattr(B, k)), k


def test_headless_driver_renders_initial_state(tmp_path):
    """--ppm writes the initial state (before the solver exists, so on the CPU too) as a binary
    PPM: odometry, landmarks and poses of the reference's draw_state, without OpenCV."""
    exe = os.path.join(ROOT, "prb-project-bearing-only-slam_amd", "lib", "bearing_only_slam")
    out = tmp_path / "c1.ppm"
    subprocess.run([exe, C1, "--iters", "0", "--quiet", "--ppm", str(out)], capture_output=True, text=True)
    init = tmp_path / "c1_initial.ppm"
    data = init.read_bytes()
    assert data.startswith(b"P6\n800 800\n255\n")
    px = np.frombuffer(data[len(b"P6\n800 800\n255\n"):], dtype=np.uint8).reshape(800, 800, 3)
    colors = {tuple(c) for c in px.reshape(-1, 3)[::7]}
    assert (255, 0, 0) in colors and (0, 0, 255) in colors      # poses and landmarks drawn


def _harness(eps):
    exe = os.path.join(ROOT, "prb-project-bearing-only-slam_amd", "lib", "jacobian_harness")
    from conftest import C1_GT
    out = subprocess.run([exe, C1, C1_GT, "--eps", repr(eps)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    return {k: float(v) for k, v in (ln.split() for ln in out.stdout.splitlines())}


def test_facade_reference_harness():
    """The reference's own numeric harness (tests/solver_stuff.cpp:17-163) through the C++ façade
    proj02::Solver (no GPU: the handle is created only by step()): predict_bearing known answers,
    predict_odometry(initial guess) == measurement on every edge, and analytic-vs-numerical Jacobians.
    With the reference's epsilon (1e-3) the statistics stay under the figures the reference records
    in fp32 (:82-88, :156-162); with 1e-6 in fp64 they are far tighter."""
    pi = np.pi
    r = _harness(1e-3)
    kat = [r[f"kat{i}"] for i in range(7)]
    assert abs(kat[0]) < 1e-15 and abs(kat[1] - pi / 2) < 1e-15 and abs(abs(kat[2]) - pi) < 1e-15
    assert abs(kat[3] + pi / 2) < 1e-15 and abs(kat[4] - pi / 4) < 1e-15 and abs(kat[5] + pi / 4) < 1e-15
    assert abs(abs(kat[6]) - pi) < 1e-12
    assert r["odometry_count"] == 300 and r["bearing_count"] == 2132
    assert r["odometry_predict_max_diff"] < 1e-4          # file values carry 6 significant digits
    assert r["bearing_highest_max"] <= 0.0131645 and r["bearing_average_max"] <= 0.000166852
    assert r["bearing_highest_sum"] <= 0.0135395 and r["bearing_average_sum"] <= 0.000372358
    assert r["odometry_highest_max"] <= 0.000556946 and r["odometry_average_max"] <= 0.000354741
    t = _harness(1e-6)
    assert t["bearing_highest_max"] < 1e-6 and t["odometry_highest_max"] < 1e-6


@pytest.mark.parametrize("threads", [1, 4])
def test_cpu_baseline_matches_oracle(threads):
    """The CPU baseline bench.py times (bos_cpu_gn_*: the same GN iteration on host threads with the
    build's host multifrontal Cholesky) follows the oracle: chi^2 per iteration and the state after
    5 iterations on C1 (the C1 bounds of the GPU tests)."""
    P = bos.load_g2o(C1)
    c = bos.CpuGN(P, threads)
    chis = [c.step() for _ in range(5)]
    pg, lg = c.get_state()
    c.close()
    po, lo, chio = O.run(to_oracle(P), 5)
    assert np.allclose(chis, chio, rtol=1e-9, atol=1e-12)
    from helpers import close_state
    ok, ep, el = close_state(pg, lg, po, lo)
    assert ok, (ep, el)

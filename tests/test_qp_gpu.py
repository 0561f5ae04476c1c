"""GPU tests of the dense standard-form QP batch (cmpc_solve_qp_batch): quadprog
semantics (Matlab-tests/yalmip/.../solvers/callquadprog.m:63-69) and the
osqp_solve_qp adapter (distributedPlanner/LPV_Planner.py:192-249), checked against
analytic optima, the KKT-certified oracle IPM (oracle/qp_ipm.py) and the optimum of
a QP captured from the reference's own PlannerLPV (tests/golden)."""
import numpy as np
import pytest

from conftest import LPV_CASES, assert_matches_optimum, lpv_qps

pytestmark = pytest.mark.gpu

X_TOL = 1e-6


def _rand_qp(rng, n, mi, me):
    M = rng.standard_normal((n, n))
    H = M @ M.T + 0.5 * np.eye(n)
    f = rng.standard_normal(n)
    x_feas = rng.uniform(-0.5, 0.5, n)
    A = rng.standard_normal((mi, n))
    b = A @ x_feas + rng.uniform(0.0, 1.0, mi)
    Aeq = rng.standard_normal((me, n))
    beq = Aeq @ x_feas
    lb = np.full(n, -2.0)
    ub = np.full(n, 2.0)
    lb[::3] = -np.inf
    return H, f, A, b, Aeq, beq, lb, ub


def _oracle(H, f, A, b, Aeq, beq, lb, ub):
    from oracle import qp_ipm

    n = H.shape[0]
    rows = [A, Aeq, np.eye(n)]
    lo = np.hstack([np.full(len(b), -np.inf), beq, lb])
    hi = np.hstack([b, beq, ub])
    return qp_ipm.solve_qp(H, f, np.vstack(rows), lo, hi)


def test_unconstrained_and_box_known_answers(gpu_ctx):
    import cmpc

    c = np.array([1.5, -3.0, 0.25, 7.0])
    r = cmpc.quadprog(np.eye(4), -c, ctx=gpu_ctx)
    assert r["exitflag"] == 1 and np.abs(r["x"] - c).max() < X_TOL
    lb, ub = np.array([-1.0, -1.0, -1.0, -1.0]), np.array([1.0, 1.0, 1.0, np.inf])
    r = cmpc.quadprog(np.eye(4), -c, lb=lb, ub=ub, ctx=gpu_ctx)
    assert r["exitflag"] == 1 and np.abs(r["x"] - np.clip(c, lb, ub)).max() < X_TOL
    # equality sum(x) = 1: x = c + (1 - sum c)/n, multiplier -(1 - sum c)/n
    r = cmpc.quadprog(np.eye(4), -c, Aeq=np.ones((1, 4)), beq=np.array([1.0]), ctx=gpu_ctx)
    assert r["exitflag"] == 1
    assert np.abs(r["x"] - (c + (1.0 - c.sum()) / 4)).max() < X_TOL
    assert abs(r["lambda"]["eqlin"][0] + (1.0 - c.sum()) / 4) < X_TOL
    assert abs(r["fval"] - (0.5 * r["x"] @ r["x"] - c @ r["x"])) < 1e-9


@pytest.mark.parametrize("seed,n,mi,me", [(0, 8, 6, 2), (1, 20, 15, 5), (2, 40, 30, 0), (3, 30, 0, 10)])
def test_random_qps_match_certified_oracle(gpu_ctx, seed, n, mi, me):
    import cmpc

    rng = np.random.default_rng(seed)
    probs = [_rand_qp(rng, n, mi, me) for _ in range(6)]
    stack = [np.stack([p[i] for p in probs]) for i in range(8)]
    r = cmpc.quadprog(*stack, ctx=gpu_ctx)
    assert (r["exitflag"] == 1).all(), r["exitflag"]
    for k, p in enumerate(probs):
        ref = _oracle(*p)
        assert ref.status == "solved"
        assert np.abs(r["x"][k] - ref.x).max() < X_TOL


def _osqp_args(c):
    """(P, q, G, h, A, b) exactly as PlannerLPV.solve passes them (LPV_Planner.py:156-157): csr
    matrices, G = F, h = b, A = G_eq, b = E x0 + Eu uOld (recovered from OSQP's stacked form)."""
    import scipy.sparse as sp

    Aall, l, u = c["A"], c["l"], c["u"]
    eq = np.isfinite(l) & (l == u)
    return (sp.csr_matrix(c["P"]), c["q"], sp.csr_matrix(Aall[~eq]), u[~eq], sp.csr_matrix(Aall[eq]), u[eq])


@pytest.mark.parametrize("name", LPV_CASES)
def test_osqp_adapter_on_reference_captured_qp(gpu_ctx, name):
    """Every captured reference QP of every golden file through osqp_solve_qp, called exactly as
    PlannerLPV.solve calls it.  The adapter recognises the agent-QP structure (an exact
    rebuild, cmpc.structure) and solves it on the structured kernels: z within 1e-6 of the
    KKT-certified optimum, the solver's KKT residual and the reference-form primal residual
    both <= 1e-6, OSQP status 'solved'."""
    import cmpc

    for j, c in lpv_qps(name):
        res, feasible = cmpc.osqp_solve_qp(*_osqp_args(c), ctx=gpu_ctx)
        assert res.info.solver == "structured"
        assert feasible == 1 and res.info.status_val == 1, (j, res.info.status)
        assert res.info.kkt <= 1e-6 and res.info.pri_res <= 1e-6, (res.info.kkt, res.info.pri_res)
        assert_matches_optimum(res.x, c, 1e-6)
        fz = 0.5 * c["z"] @ c["P"] @ c["z"] + c["q"] @ c["z"]
        assert abs(res.info.obj_val - fz) <= 1e-9 * max(1.0, abs(fz))


def test_osqp_adapter_batch_groups_reference_qps(gpu_ctx):
    """All captured QPs of the 3-agent N=30 case in one osqp_solve_qp_batch call (one
    structured launch) give the same answers as one call per QP."""
    import cmpc

    cs = [c for _, c in lpv_qps("lpv_n30_a3")]
    out = cmpc.osqp_solve_qp_batch([_osqp_args(c) for c in cs], ctx=gpu_ctx)
    for c, (res, feasible) in zip(cs, out):
        one, _ = cmpc.osqp_solve_qp(*_osqp_args(c), ctx=gpu_ctx)
        assert feasible == 1 and res.info.solver == "structured"
        assert np.array_equal(res.x, one.x)
        assert np.abs(res.x - c["z"]).max() < 1e-6


@pytest.mark.parametrize("name", ["lpv_n10_a2", "lpv_n30_a3"])
def test_dense_path_on_reference_captured_qp(gpu_ctx, name):
    """The generic dense kernel (structure recognition off) on the reference's own QPs.  It does
    not see the stage structure and works on the reduced Hessian, whose condition number is ~1e8
    (Qs = 1e7): the bar on z is 1e-4 (OSQP's own default eps is 1e-3) and the
    optimal value agrees to 1e-7 relative; the structured path above holds 1e-6."""
    import cmpc

    for j, c in lpv_qps(name):
        if c["step"] > 1:
            continue
        res, feasible = cmpc.osqp_solve_qp_batch([_osqp_args(c)], ctx=gpu_ctx, structured=False)[0]
        assert res.info.solver == "dense"
        assert feasible == 1 and res.info.status_val == 1
        fz = 0.5 * c["z"] @ c["P"] @ c["z"] + c["q"] @ c["z"]
        assert abs(res.info.obj_val - fz) <= 1e-7 * max(1.0, abs(fz))
        assert np.abs(res.x - c["z"]).max() < 1e-4


def test_infeasible_and_nonconvex_flags(gpu_ctx):
    import cmpc

    # x <= -1 and x >= 1
    r = cmpc.quadprog(np.eye(1), np.zeros(1), A=np.array([[1.0], [-1.0]]), b=np.array([-1.0, -1.0]), ctx=gpu_ctx,
                      max_iter=60)
    assert r["exitflag"] == -2
    # an all-zero equality row with a nonzero right-hand side
    r = cmpc.quadprog(np.eye(2), np.zeros(2), Aeq=np.zeros((1, 2)), beq=np.array([1.0]), ctx=gpu_ctx)
    assert r["exitflag"] == -2
    # negative curvature
    r = cmpc.quadprog(-np.eye(2), np.zeros(2), lb=-np.ones(2), ub=np.ones(2), ctx=gpu_ctx)
    assert r["exitflag"] == -6
    res, feasible = cmpc.osqp_solve_qp(-np.eye(2), np.zeros(2), ctx=gpu_ctx)
    assert feasible == 0 and res.info.status_val == -7


def test_mex_gateway_column_major_batch(gpu_ctx):
    """cmpc_quadprog through the MEX gateway (mock mex.h build): MATLAB column-major
    arrays, a 3-page batch, the quadprog output/lambda structs."""
    import cmpc
    import mex_harness as MH

    rng = np.random.default_rng(7)
    probs = [_rand_qp(rng, 12, 9, 3) for _ in range(3)]
    H, f, A, b, Aeq, beq, lb, ub = (np.stack([p[i] for p in probs]) for i in range(8))
    # MATLAB layout: pages on the trailing axis
    page = lambda a: np.moveaxis(a, 0, -1)
    out, err = MH.call((page(H), page(f), page(A), page(b), page(Aeq), page(beq), page(lb), page(ub)),
                       opts={"MaxIterations": 80.0, "OptimalityTolerance": 1e-9})
    assert err is None, err
    x = MH.values(out[0]).reshape(3, 12)     # n x B column-major -> B rows of n
    flag = MH.values(out[2])
    assert (flag == 1).all()
    ref = cmpc.quadprog(H, f, A, b, Aeq, beq, lb, ub, ctx=gpu_ctx)
    assert np.abs(x - ref["x"]).max() < 1e-9
    assert np.abs(MH.values(out[1]) - ref["fval"]).max() < 1e-9
    lam = out[4]
    assert np.abs(MH.values(MH.field(lam, "eqlin")).reshape(3, 3) - ref["lambda"]["eqlin"]).max() < 1e-6
    assert (MH.values(MH.field(out[3], "iterations")) > 0).all()

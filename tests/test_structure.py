"""CPU checks of the osqp_solve_qp structure recogniser (cmpc.structure): every QP captured
from the reference's PlannerLPV (tests/golden, oracle/gen_fixtures.py) is recognised, the
recovered structured problem is the oracle builder's for the same inputs, and QPs that differ
from the pattern in any entry are refused (they go to the dense kernel)."""
import numpy as np
import pytest
import scipy.sparse as sp

from conftest import LPV_CASES, lpv_qps

from cmpc import structure as St


def _args(c):
    Aall, l, u = c["A"], c["l"], c["u"]
    eq = np.isfinite(l) & (l == u)
    return sp.csr_matrix(c["P"]), c["q"], sp.csr_matrix(Aall[~eq]), u[~eq], sp.csr_matrix(Aall[eq]), u[eq]


@pytest.mark.parametrize("name", LPV_CASES)
def test_every_captured_qp_is_recognised(name):
    from oracle import lpv_ref as L

    g = L.paper_gains()
    for j, c in lpv_qps(name):
        p = St.recognize(*_args(c))
        assert p is not None, (name, j)
        N = c["N"]
        nb = c["x_agents"].shape[1]
        assert p["N"] == N and p["mc"] == 4 + nb
        np.testing.assert_array_equal(p["Q"], g["Q"])
        np.testing.assert_array_equal(p["Qs"], np.diag(g["Qs"]))
        np.testing.assert_array_equal(p["dR"], g["dR"])
        np.testing.assert_array_equal(p["x0"][0], c["x0"])
        np.testing.assert_array_equal(p["u_prev"][0], c["u_old"])
        assert list(p["row_slack"]) == [-1, 0, 1, 1] + [2] * nb
        assert list(p["row_sign"]) == [1, 1, 1, 1] + [-1] * nb
        # rebuilt reference form == the captured one (the acceptance test itself, restated)
        P2, q2, G2, h2, A2, b2 = St.reference_form(p)
        P, q, G, h, A, b = _args(c)
        assert (P != P2).nnz == 0 and (G != G2).nnz == 0 and (A != A2).nnz == 0
        assert np.array_equal(q, q2) and np.array_equal(h, h2) and np.array_equal(b, b2)


def test_perturbed_qps_are_refused():
    _, c = next(iter(lpv_qps("lpv_n10_a2")))
    P, q, G, h, A, b = _args(c)
    assert St.recognize(P, q, G, h, A, b) is not None
    P2 = P.tolil()
    P2[0, 1] = 1e-3                                      # x-x cross term the stage form lacks
    assert St.recognize(P2, q, G, h, A, b) is None
    q2 = q.copy()
    q2[-1] = 1.0                                         # linear cost on a rate
    assert St.recognize(P, q2, G, h, A, b) is None
    h2 = h.copy()
    h2[-1] += 1.0                                        # input bound differing between stages
    assert St.recognize(P, q, G, h2, A, b) is None
    A2 = A.tolil()
    A2[20, 30] = 0.5                                     # a coupling outside the dynamics pattern
    assert St.recognize(P, q, G, h, A2, b) is None
    assert St.recognize(P, q, G[:-1], h[:-1], A, b) is None   # wrong row count
    assert St.recognize(P, q, None, None, A, b) is None


def test_stack_and_shared_key():
    cs = [c for _, c in lpv_qps("lpv_n30_a3")]
    ps = [St.recognize(*_args(c)) for c in cs]
    keys = {St.shared_key(p) for p in ps}
    assert len(keys) == 1
    s = St.stack(ps)
    assert s["A"].shape == (len(cs), 30, 9, 9) and s["C"].shape[0] == len(cs)


def test_non_canonical_inputs_are_recognised_alike():
    """The fast path compares canonical csr arrays; inputs that are not canonical (COO, an entry
    split into two duplicates, stored zeros, dense arrays, unsorted indices) are canonicalised
    first and give the same structured problem."""
    _, c = next(iter(lpv_qps("lpv_n10_a2")))
    P, q, G, h, A, b = _args(c)
    ref = St.recognize(P, q, G, h, A, b)
    Gc = G.tocoo()
    split = sp.coo_matrix((np.concatenate([Gc.data * 0.5, Gc.data * 0.5, [0.0]]),
                           (np.concatenate([Gc.row, Gc.row, [0]]), np.concatenate([Gc.col, Gc.col, [1]]))),
                          shape=G.shape)
    Au = A.copy()
    Au.has_sorted_indices = False
    for i in range(Au.shape[0]):                          # reverse every row's index order
        s, e = Au.indptr[i], Au.indptr[i + 1]
        Au.indices[s:e] = Au.indices[s:e][::-1].copy()
        Au.data[s:e] = Au.data[s:e][::-1].copy()
    for args in ((P.tocoo(), q, split, h, A.toarray(), b), (P, q, G, h, Au, b)):
        p = St.recognize(*args)
        assert p is not None
        for k, v in ref.items():
            np.testing.assert_array_equal(p[k], v)


def test_zero_entries_drop_out_of_the_rebuilt_pattern():
    """reference_form fills a per-shape cached slot pattern (cmpc.structure._pattern) and drops the
    slots whose value is zero: a structured problem with zeros in C_k, A_k, B_k rebuilds into
    canonical csr (sorted, no stored zeros) with exactly that many entries fewer, and is recognised
    back into the same problem."""
    _, c = next(iter(lpv_qps("lpv_n30_a3")))
    p = St.recognize(*_args(c))
    P0, q0, G0, h0, A0, b0 = St.reference_form(p)
    p2 = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in p.items()}
    rng = np.random.default_rng(3)
    dropped = {}
    for k, mat in (("C", G0), ("A", A0), ("B", A0)):
        v = p2[k].reshape(-1)
        nzi = np.flatnonzero(v)
        pick = rng.choice(nzi, size=min(7, nzi.size), replace=False)
        v[pick] = 0.0
        dropped[k] = pick.size
    P, q, G, h, A, b = St.reference_form(p2)
    for M in (G, A):
        assert M.has_canonical_format and (M.data != 0).all()
    assert G.nnz == G0.nnz - dropped["C"]
    assert A.nnz == A0.nnz - dropped["A"] - dropped["B"]
    back = St.recognize(P, q, G, h, A, b)
    assert back is not None
    for k, v in p2.items():
        np.testing.assert_array_equal(back[k], v)


def _same_result(p, p0):
    if p is None or p0 is None:
        return p is None and p0 is None
    return p.keys() == p0.keys() and all(np.array_equal(np.asarray(p[k]), np.asarray(p0[k])) for k in p0)


def test_slot_recogniser_agrees_with_the_rebuild_on_perturbed_qps():
    """recognize reads the structured quantities from the slots of a cached pattern and checks the
    fixed slots; _recognize_rebuild extracts and rebuilds the whole QP.  On every captured QP and on
    seeded single-entry perturbations of them (values changed, entries added outside the pattern or
    removed, a later stage's slack sign or input row flipped, bounds varying by stage, b or q
    non-zero off the pattern) both accept the same QPs with the same result."""
    rng = np.random.default_rng(11)
    cases = [c for nm in ("lpv_n10_a2", "lpv_n30_a3") for _, c in list(lpv_qps(nm))[:3]]
    n_acc = n_ref = 0
    for c in cases:
        base = _args(c)
        assert _same_result(St.recognize(*base), St._recognize_rebuild(*base))
        for trial in range(40):
            P, q, G, h, A, b = (x.copy() for x in base)
            which = trial % 8
            if which in (0, 1):                        # a G entry: change, or add one anywhere
                G = G.tolil()
                r, k = rng.integers(G.shape[0]), rng.integers(G.shape[1])
                G[r, k] = G[r, k] * -1.0 if (which == 0 and G[r, k] != 0) else rng.choice([1.0, -1.0, 0.5])
                G = G.tocsr()
            elif which in (2, 3):                      # an Aeq entry: change, add or remove
                A = A.tolil()
                r, k = rng.integers(A.shape[0]), rng.integers(A.shape[1])
                A[r, k] = 0.0 if which == 2 else (A[r, k] + 1.0)
                A = A.tocsr()
            elif which == 4:                           # h anywhere
                h[rng.integers(h.size)] += rng.choice([0.0, 1.0])
            elif which == 5:                           # b anywhere
                b[rng.integers(b.size)] += rng.choice([0.0, 1e-3])
            elif which == 6:                           # q anywhere
                q[rng.integers(q.size)] += rng.choice([0.0, 2.0])
            else:                                      # an existing G entry's value scaled (slack signs, +-1 rows)
                G = G.copy()
                G.data[rng.integers(G.nnz)] *= rng.choice([-1.0, 2.0])
            p, p0 = St.recognize(P, q, G, h, A, b), St._recognize_rebuild(P, q, G, h, A, b)
            assert _same_result(p, p0), (which, trial)
            n_acc += p is not None
            n_ref += p is None
    assert n_acc > 20 and n_ref > 100   # both outcomes exercised

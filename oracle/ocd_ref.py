"""ORACLE (test infrastructure only) — numpy restatement of the reference's OCD
coupling-dual round (planner/scripts/NL_EU_N_main.py:119-162) in its own dense
(n_agents, n_agents, N) layout, and the map to the neighbour-graph layout of
cmpc_ocd_update_dev.  Pinned bit-exactly by tests/golden/ocd_rounds.npz: rounds computed by the
reference's own get_alpha / eval_constraintEU (oracle/gen_ocd_fixtures.py imports them from
plan_lib.config.NL); the only recorded lambda artefact (ini_lambdas.pkl of NL_3agents_def) is all
zeros."""
import numpy as np


def get_alpha():  # config/NL/config.py:5-8
    return 0.25


def eval_constraint_eu(x1, x2, D):  # config/NL/config.py:19-23
    return np.array(D - np.sqrt(sum((x1 - x2) ** 2)))


def ocd_update(lambdas, agents, N, dth):
    """lambdas (n, n, N); agents (N+1, n, 2) exchanged positions (NL_EU_N_main.py:125).
    Returns the updated lambdas (:127-138)."""
    n = agents.shape[1]
    cost = np.zeros((n, n, N))
    for k in range(1, N + 1):
        for i in range(0, n):
            for j in range(0, n):
                if (i != j) and i < j:
                    cost[i, j, k - 1] = eval_constraint_eu(agents[k, i, :], agents[k, j, :], dth)
    return lambdas + get_alpha() * cost


def to_neighbour_layout(lambdas, nbr):
    """(n, n, N) -> (n, nb, N) with entry [i, s] = lambdas[i, nbr[i, s]]."""
    n, nb = nbr.shape
    return np.stack([lambdas[i, nbr[i]] for i in range(n)]) if nb else np.zeros((n, 0, lambdas.shape[2]))


def allclose_agents(x_old, x_pred, atol=0.01):  # :143-149
    return np.array([np.allclose(x_old[i], x_pred[i], atol=atol) for i in range(len(x_old))])

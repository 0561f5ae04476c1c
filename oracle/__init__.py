"""ORACLE — test infrastructure only.

CPU restatements of the reference's hot path (MarcFacerias/ColaborativeMPC-,
``planner/lib/plan_lib``) used as the *checker* for the MI355X product path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import, call, link or execute anything under ``oracle/``.  The product
(``colaborativempc-_amd/``) never imports this package and has no CPU fallback.

Contents
--------
lpv_ref.py   numpy restatement of PlannerLPV's QP assembly (LPV scheduling,
             hyperplanes, weights, F/G/M builders) and of the LPV control loop.
qp_ipm.py    dense fp64 primal-dual interior-point solver for the reference-form
             (OSQP-form) QP, with a KKT certificate.  Stands in for OSQP, which
             is absent (third party, ``requirements.txt:5`` ``osqp>=0.6.2.post5``):
             the QP is strictly convex on its feasible set, so the
             optimum it certifies is the unique point OSQP converges to.
synth.py     reference-form builder for the synthetic double-integrator family
             (BASELINE configs 1-5) — same structure as the LPV QP.
cmpc_oracle.c  plain-C condensed IPM restatement (CPU baseline, OpenMP).
gen_fixtures.py  generator of tests/golden/* (imports the real reference with an
             ``osqp`` stub; runs only in the build container).

Parity pins: the assembly restatement is checked against QPs captured from the
reference's own code (tests/golden/lpv_*.npz); the solver is pinned by its KKT
certificate (no reference test pins the solver boundary — SURVEY §8c).
"""

"""CPU oracle for the batched MPC solve path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import anything from this package, and only as the checker / the timed CPU
baseline.  The product path (``vehicle-control_amd/vcmpc``) never imports it and
has no CPU fallback: it fails loudly when ``libvcmpc.so`` is missing.

What is restated here (numpy float64, batch-first arrays), each function citing
the reference file:line it follows (paths relative to the reference checkout
``neverorfrog/vehicle-control`` @ 2024-12-20):

* ``models``   -- kinematic bicycle (temporal + spatial Euler) and dynamic bicycle
                  (modified-Fiala tyre, temporal + spatial RK4), analytic
                  Jacobians of the kinematic spatial step.
* ``ltv_qp``   -- the build's LTV-QP contract (predict -> linearize -> condense ->
                  QP data) restating the reference NLP's costs and constraints.
* ``qp``       -- an exact dense convex-QP solver (primal-dual interior point to
                  1e-12 followed by an active-set polish and a KKT certificate).

Pinning status (see DESIGN.md "Oracle and parity"):

* Dynamic-car temporal RK4 plant step: PINNED against the reference's own
  recorded closed-loop traces (``experiments/data/*/*_{state,action}_traj.npy``),
  fixtures committed under ``tests/golden/`` with the script that made them.
* Kinematic-car model, Jacobians, LTV-QP and its solution: **parity unpinned** --
  the reference holds no kinematic trace and no QP (its MPC is a CasADi 3.6.7 /
  IPOPT NLP; neither CasADi nor IPOPT/HSL is importable here).  These are pinned
  only by the reference's source formulas, finite differences of the oracle's own
  model and a KKT optimality certificate of every oracle QP solution.
"""

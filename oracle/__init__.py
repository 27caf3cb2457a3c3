"""CPU oracle for the CarMPC batched-QP hot path.  TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` may import, call or link anything under ``oracle/``; the product
package ``carmpc_amd`` never does (it fails loudly without its HIP library).

Contents
--------
``assembly``   numpy restatement of the reference's constructor-time QP
               assembly (``lib/mpc.py:22-117,128-253``, ``lib/matrix_gen.py:6-82``,
               ``lib/environments.py``, ``lib/configuration.py``).
``qp``         numpy restatement of the per-step QP (``lib/mpc.py:312-349``,
               ``450-492``) solved by a dense Mehrotra IPM, plus an independent
               active-set KKT polish/certificate and a HiGHS LP feasibility
               margin (ground truth for the feasible/infeasible status).
``ipm.c``      the same IPM in plain C (OpenMP over instances), built into
               ``oracle/build/liboracle_ipm.so``: the fast checker for the GPU
               parity tests and the ``cpu_baseline`` ("port") in ``bench.py``.

Pinning
-------
* Assembly (T, S, H, h, P, K, constraint stacks): pinned to fp64 round-off
  against outputs of the reference's own, directly importable modules
  (``lib/matrix_gen.py``, ``lib/environments.py``, ``lib/simulator.py``,
  ``lib/configuration.py``) run in the build container, committed as
  ``tests/golden/assembly_*.npz`` by ``tools/make_golden.py``; and against
  the reference's data files ``terminal_sets/*.npy`` (byte-identical copies).
* QP solution u*: the reference hands the QP to cvxpy (``lib/mpc.py:334-335``),
  whose backend is absent here and unpinned upstream (no requirements file).
  **Parity for u* is therefore unpinned against the reference's solver.**  It is
  anchored instead by KKT optimality certificates: H is SPD (lambda_min ~ 10),
  so a certified KKT point is the unique optimum every correct QP solver
  (cvxpy's included, to its own tolerance) must return.
"""

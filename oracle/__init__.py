"""CPU oracle for the physics-informed ELBO hot path.

TEST INFRASTRUCTURE ONLY.  Nothing under ``oracle/`` is part of the product:
only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import it, and only as the checker / the timed CPU baseline, never as
the code path that is measured or shipped.

Modules
-------
fem      generic P1 finite-element restatement (numpy, fp64) of the FEniCS
         assembly the reference performs at setup: fine stiffness, Dirichlet
         reduction, FOM solve, ROM stiffness tensor M, prolongation W,
         F_ROM_BC, CGR residual (Gamma, alpha) and flux rows.
elbo     numpy/torch restatement of the reference's ELBO algebra: Gaussian
         log-likelihood, KL, reparametrisation, the ROM solve with
         Dirichlet-row replacement and the virtual-observable conditioning.
field    dense restatement of the reference's random-field sampler (covariance,
         KL / Cholesky factor with the adaptive truncation).
codec    torch.nn.functional restatement of the DenseNet conv encoder /
         decoder (train-mode BatchNorm) used as the fp32 reference for the
         HIP codec kernels.

Parity status (see DESIGN.md section "Oracle"):
  * torch-side semantics (codec, ELBO terms, ROM solve, VO update) are
    PINNED by golden fixtures generated from the reference's own modules
    (tests/golden/make_golden.py, stubbed FEniCS imports).
  * FE assembly vs FEniCS/DOLFIN 2018.1 is PARITY UNPINNED: FEniCS is not
    installable here; ``fem`` is pinned by analytic known-answer tests
    (tests/test_oracle_fem.py) instead.
"""

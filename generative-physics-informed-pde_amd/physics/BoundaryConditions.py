"""Boundary-condition ensembles for the NDP problem (reference physics/BoundaryConditions.py:7-147).

An NDP Dirichlet condition is encoded by four numbers (u0, u1, u2, u3):
left x=0: u0 (1 - y) + u1 y, right x=1: u2 (1 - y) + u3 y, each ~ U(-0.5, 0.5)
(physics/LinearEllipticFactories.py:239-281).
"""
import numpy as np


class BoundaryCondition(object):
    def __init__(self, u):
        self.u = np.asarray(u, dtype=np.float64).reshape(4)

    @classmethod
    def sample(cls, rng=None):
        rng = rng or np.random
        return cls(rng.uniform(-0.5, 0.5, 4))

    def encode(self):
        return self.u.copy()


class BoundaryConditionEnsemble(object):

    def __init__(self, conditions):
        self._bcs = list(conditions)
        self._physics = {}

    @classmethod
    def FromFactory(cls, N, rng=None):
        return cls([BoundaryCondition.sample(rng) for _ in range(N)])

    @classmethod
    def FromEncoding(cls, encoding, *args, **kwargs):
        return cls([BoundaryCondition(u) for u in np.asarray(encoding).reshape(-1, 4)])

    def encode(self):
        return np.stack([b.u for b in self._bcs]) if self._bcs else np.zeros((0, 4))

    @property
    def U(self):
        return self.encode()

    def __len__(self):
        return len(self._bcs)

    def __iter__(self):
        return iter(self._bcs)

    def __getitem__(self, k):
        if isinstance(k, (list, np.ndarray)):
            return BoundaryConditionEnsemble([self._bcs[i] for i in k])
        return self._bcs[k]

    def register_function_space(self, identifier, physics):
        self._physics[identifier.lower()] = physics

    def constrained_dofs(self, identifier):
        return self._physics[identifier.lower()].constrained_dofs

    def free_dofs(self, identifier):
        return self._physics[identifier.lower()].free_dofs

    def constrained_dofs_values(self, identifier):
        g = self._physics[identifier.lower()].grid
        return np.stack([g.dirichlet_values(b.u) for b in self._bcs])

    def FULL_F_WITH_APPLIED_BC(self, identifier):
        """[N, n_nodes]: zero source, Dirichlet values at constrained nodes (BoundaryConditions.py:132-147)."""
        g = self._physics[identifier.lower()].grid
        return np.stack([g.full_force(b.u) for b in self._bcs])

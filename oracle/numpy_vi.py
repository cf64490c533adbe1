"""numpy restatement of the A9 Jacobi value iteration (single thread): the CPU baseline SURVEY 8(d)
asks for beside the C oracle, and a second, independent statement of the same loop.

TEST / BASELINE INFRASTRUCTURE ONLY (like the rest of oracle/): imported by tests/ and by bench.py's
cpu_baseline leg, never by the product package.

Transition tables come from the C oracle's orc_build_table (the reference step() restated,
pinned to tables extracted from reference step(): tests/test_oracle_golden.py); the sweep is plain
numpy, vectorised over (state, action):
    Qd = done ? R : (T)(R + g * V[s'])          (oracle/mgdp_oracle.c orc_vi)
    V' = max_a Qd,  pi = argmax_a Qd (numpy: lowest index wins ties),  absorbing states V' = 0
    stop after sweep k when max |V_k - V_{k-1}| < tol
Same operation order as the oracle and the kernels, so results are bit-identical (tested).
"""
from __future__ import annotations

import numpy as np

from . import oracle


class NumpyVI:
    def __init__(self, model: int, cells: np.ndarray, gamma=0.99, tol=1e-6, dtype="f32"):
        cells = np.ascontiguousarray(cells, np.uint8)
        if cells.ndim == 2:
            cells = cells[None]
        self.B = cells.shape[0]
        self.T = np.float32 if dtype == "f32" else np.float64
        nx, rw, dn = [], [], []
        for b in range(self.B):
            n, r, d = oracle.build_table(model, cells[b])
            nx.append(n)
            rw.append(r)
            dn.append(d)
        S, A = nx[0].shape
        self.S, self.A = S, A
        nxt = np.stack(nx).reshape(self.B * S, A).astype(np.int64)
        self.absorb = nxt[:, 0] < 0
        base = (np.arange(self.B, dtype=np.int64) * S).repeat(S)[:, None]
        self.idx = np.where(nxt < 0, 0, nxt + base)  # global V index of s' (absorbing rows: dummy)
        self.R = np.stack(rw).reshape(self.B * S, A).astype(self.T)
        self.done = np.stack(dn).reshape(self.B * S, A).astype(bool)
        self.g = self.T(gamma)
        self.tol = float(tol)

    def solve(self, max_sweeps=10000):
        V = np.zeros(self.B * self.S, self.T)
        k = 0
        while True:
            k += 1
            Q = np.where(self.done, self.R, self.R + self.g * V[self.idx])
            Vn = Q.max(axis=1)
            Vn[self.absorb] = 0
            dv = float(np.abs(Vn - V).max())
            V = Vn
            if dv < self.tol or k >= max_sweeps:
                break
        pi = Q.argmax(axis=1).astype(np.int8)
        pi[self.absorb] = -1
        return {"V": V.reshape(self.B, self.S), "pi": pi.reshape(self.B, self.S), "sweeps": k, "dv": dv}

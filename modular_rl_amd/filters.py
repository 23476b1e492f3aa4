"""Running-stat filters (`filters.py` / `running_stat.py` of the reference).

The agent's ZFilter state lives on the device in the collector's ``filter_state``
(n, mean, M2 in fp64; obs dims then the reward), updated inside the fused rollout
kernel.  ``DeviceZFilter`` is the agent-facing view of that state with the
reference's ``ZFilter`` call semantics for single observations
(`filters.py:30-38`: push, then (x - mean)/(std + 1e-8), clip) -- a host-side
convenience for the per-observation API, not part of the batched hot path.
"""
import numpy as np
import torch


class DeviceZFilter:
    def __init__(self, agent, which, demean=True, destd=True, clip=10.0):
        self.agent, self.which = agent, which
        self.demean, self.destd, self.clip = demean, destd, clip

    def _state(self):
        col = self.agent._filter_owner()
        if col is None:
            raise RuntimeError("the filter state is created with the agent's first collector (make_collector)")
        return col

    @property
    def rs(self):
        return self

    @property
    def n(self):
        (n, _, _), (nr, _, _) = self._state().filter_stats()
        return n if self.which == "obs" else nr

    @property
    def mean(self):
        (_, m, _), (_, mr, _) = self._state().filter_stats()
        return m if self.which == "obs" else mr

    @property
    def var(self):
        (_, _, v), (_, _, vr) = self._state().filter_stats()
        return v if self.which == "obs" else vr

    @property
    def std(self):
        return np.sqrt(self.var)

    def __call__(self, x, update=True):
        col = self._state()
        fs = col.filter_state[:col.FS].cpu().numpy()
        D = (col.FS - 2) // 2
        cols = list(range(D - 1)) if self.which == "obs" else [D - 1]
        ci = 0 if self.which == "obs" else 1
        x = np.asarray(x, dtype=np.float64)
        if update:  # RunningStat.push (running_stat.py:10-20)
            n = fs[ci] + 1
            M, S = fs[2:2 + D][cols], fs[2 + D:2 + 2 * D][cols]
            if n == 1:
                M = np.array(x, dtype=np.float64).reshape(M.shape)
            else:
                old = M.copy()
                M = old + (x.reshape(M.shape) - old) / n
                S = S + (x.reshape(M.shape) - old) * (x.reshape(M.shape) - M)
            fs[ci] = n
            fs[2:2 + D][cols] = M
            fs[2 + D:2 + 2 * D][cols] = S
            col.filter_state[:col.FS].copy_(torch.as_tensor(fs))
        n = fs[ci]
        M, S = fs[2:2 + D][cols], fs[2 + D:2 + 2 * D][cols]
        var = S / (n - 1) if n > 1 else np.square(M)
        y = x.reshape(M.shape) if M.shape else x
        if self.demean:
            y = y - M
        if self.destd:
            y = y / (np.sqrt(var) + 1e-8)
        if self.clip:
            y = np.clip(y, -self.clip, self.clip)
        return y.reshape(np.shape(x))

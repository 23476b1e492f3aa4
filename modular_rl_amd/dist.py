"""Data-parallel communication: one process per GPU, torch.distributed over RCCL.

The reference has no distributed path (`parallel` raises NotImplementedError,
core.py:123-124,175-176).  Here every rank owns E envs, its own trajectories and
activation work; theta is replicated and the ranks take identical steps because
every reduction the update consumes is summed over ranks first:
  * the flat policy gradient g and every conjugate-gradient Fvp (sum, then the
    kernels' 1/N_global scaling makes them global means),
  * loss sums (surr / KL / entropy) of the before/after/line-search passes,
  * advantage moments (sum, sum of squares, count) for the global standardisation,
  * VF loss and gradient of every L-BFGS evaluation,
  * the ZFilter running-stat deltas once per iteration (Chan merge, rank order).
``backend="nccl"`` is RCCL on ROCm; ``gloo`` is used by the CPU tests.

``Comm(force=True)`` (or ``MRL_COMM_FORCE=1`` with ``init_from_env``) keeps every
collective on even at world size 1, so one GPU exercises the RCCL path -- its
communicator, its stream ordering against the rollout's CU-masked streams -- with
results that must equal the no-communication run bit for bit (a sum over one rank).
"""
import os

import torch
import torch.distributed as dist


class Comm:
    def __init__(self, group=None, force=False, host_group=None):
        self.group = group
        up = dist.is_available() and dist.is_initialized()
        self.enabled = up and (dist.get_world_size(group) > 1 or bool(force))
        self.rank = dist.get_rank(group) if self.enabled else 0
        self.world = dist.get_world_size(group) if self.enabled else 1
        self.host_group = host_group

    def host(self):
        """The same ranks over a host (gloo) group: collectives on host copies of the
        tensors, no GPU collective kernels.  For the VF fit that runs beside the
        persistent rollout: its per-evaluation loss / gradient sums are
        read back by the L-BFGS host loop anyway, and reducing them on the host keeps
        RCCL's kernels -- not CU-masked -- off the rollout's CUs during its hand-offs.
        Without a host group (one rank, or a gloo default group): this Comm."""
        if not self.enabled or self.world <= 1 or self.host_group is None:
            return self
        return HostComm(self.host_group)

    def allreduce_(self, t):
        """In-place sum over ranks (no-op on one rank)."""
        if self.enabled:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return t

    def allreduce_int(self, v):
        if not self.enabled:
            return int(v)
        dev = "cuda" if dist.get_backend(self.group) == "nccl" else "cpu"
        t = torch.tensor([int(v)], dtype=torch.int64, device=dev)
        dist.all_reduce(t, group=self.group)
        return int(t.item())

    def allgather(self, t):
        if not self.enabled:
            return [t]
        out = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(out, t, group=self.group)
        return out

    def barrier(self):
        if self.enabled:
            dist.barrier(group=self.group)


class HostComm(Comm):
    """Comm over a gloo group: device tensors are reduced through host copies."""

    def allreduce_(self, t):
        if self.enabled:
            if t.is_cuda:
                h = t.cpu()
                dist.all_reduce(h, op=dist.ReduceOp.SUM, group=self.group)
                t.copy_(h)
            else:
                dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return t

    def allreduce_int(self, v):
        if not self.enabled:
            return int(v)
        t = torch.tensor([int(v)], dtype=torch.int64)
        dist.all_reduce(t, group=self.group)
        return int(t.item())

    def host(self):
        return self


def init_from_env(backend=None):
    """Initialise torch.distributed from RANK/WORLD_SIZE/MASTER_* (torchrun) if present.
    ``MRL_DIST_BACKEND=gloo`` rehearses the multi-rank path with several ranks sharing
    one GPU (each rank uses device LOCAL_RANK mod the visible device count).
    ``MRL_COMM_FORCE=1`` initialises the process group even at world size 1 and keeps
    every collective on (the RCCL path on one GPU)."""
    force = os.environ.get("MRL_COMM_FORCE", "0") == "1"
    if dist.is_initialized():
        # initialised by the caller: still give the fit its host group (collective: every
        # rank reaches this call), else Comm.host() would keep RCCL on the rollout's CUs
        multi = dist.get_world_size() > 1 and dist.get_backend() == "nccl"
        host = dist.new_group(backend="gloo") if multi else None
        return Comm(force=force, host_group=host)
    if int(os.environ.get("WORLD_SIZE", "1")) <= 1 and not force:
        return Comm()
    if backend is None:
        backend = os.environ.get("MRL_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    if torch.cuda.is_available():
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
    if int(os.environ.get("WORLD_SIZE", "1")) <= 1:
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
    dist.init_process_group(backend=backend)
    # a gloo group over the same ranks (collective: every rank creates it here) for the
    # host-side reductions of the VF fit that overlaps the rollout (Comm.host)
    host = dist.new_group(backend="gloo") if backend == "nccl" and dist.get_world_size() > 1 else None
    return Comm(force=force, host_group=host)

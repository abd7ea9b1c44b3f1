"""Rank-level communication for the sharded Krylov basis.

Reference: every nekStab dot ends in Nek5000's ``glsc3 -> gop -> MPI_Allreduce`` of one fp64 per
field (core/krylov_subspace.f90:40-47), i.e. (2k+2)*n_fields scalar all-reduces per
Arnoldi step.  Here one process drives one GPU; the block kernels leave a LOCAL partial vector of
length j in device memory and a single all-reduce of that vector (RCCL over xGMI with the
``nccl`` backend, stream-ordered, no host sync) replaces the per-field scalar all-reduces.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


class Comm:
    """One process per GPU.  ``world == 1`` makes every collective a no-op."""

    def __init__(self, group=None, force_collectives: bool = False):
        self.group = group
        self.timer = None   # optional profiling.PhaseTimer: events around every all-reduce (bench.py)
        # force_collectives: issue the all-reduces even at world size 1 (an initialised world-1
        # group) — measures the collective path's cost without peers (bench.py --force-collectives)
        self.force = bool(force_collectives) and dist.is_available() and dist.is_initialized()
        if dist.is_available() and dist.is_initialized():
            self.rank = dist.get_rank(group)
            self.world = dist.get_world_size(group)
            self.backend = dist.get_backend(group)
        else:
            self.rank, self.world, self.backend = 0, 1, None

    @property
    def distributed(self) -> bool:
        return self.world > 1

    def allreduce_(self, t: torch.Tensor) -> torch.Tensor:
        """In-place SUM all-reduce of a device partial (deterministic: RCCL gives every rank the
        same bits, so host LAPACK stays replicated on identical data)."""
        if self.world > 1 or self.force:
            tm = self.timer
            if tm is not None:
                tm.begin("allreduce")
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
            if tm is not None:
                tm.end("allreduce", 8.0 * t.numel())
        return t

    def barrier(self) -> None:
        if self.world > 1:
            dist.barrier(group=self.group)

    def min_scalar(self, x: float, device=None) -> float:
        return -self.max_scalar(-x, device=device)

    def max_scalar(self, x: float, device=None) -> float:
        if self.world == 1 and not self.force:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return float(t.item())


def init_from_env(backend: str | None = None, force_collectives: bool = False) -> Comm:
    """Initialise torch.distributed from torchrun's env (RANK/WORLD_SIZE/MASTER_*) if present.
    ``force_collectives`` at world size 1: initialise a world-1 group anyway and route every
    partial through it (the cost of the collective path without peers)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world == 1 and force_collectives and not dist.is_initialized():
        import socket

        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        kw = {}
        if backend == "nccl":
            torch.cuda.set_device(0)
            kw["device_id"] = torch.device("cuda", 0)
        dist.init_process_group(backend, init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, **kw)
        return Comm(force_collectives=True)
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            local = int(os.environ.get("LOCAL_RANK", "0"))
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:  # gloo: CPU tests, or several ranks sharing one GPU (rehearsal of the sharded path)
            if torch.cuda.is_available():
                torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
            dist.init_process_group(backend)
    return Comm()

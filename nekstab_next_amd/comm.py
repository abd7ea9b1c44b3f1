"""Rank-level communication for the sharded Krylov basis.

Reference: every nekStab dot ends in Nek5000's ``glsc3 -> gop -> MPI_Allreduce`` of one fp64 per
field (core/krylov_subspace.f90:40-47), i.e. (2k+2)*n_fields scalar all-reduces per
Arnoldi step.  Here one process drives one GPU; the block kernels leave a LOCAL partial vector of
length j in device memory and a single all-reduce of that vector (RCCL over xGMI with the
``nccl`` backend, stream-ordered, no host sync) replaces the per-field scalar all-reduces.
"""
from __future__ import annotations

import datetime
import faulthandler
import os
import sys
import threading

import torch
import torch.distributed as dist

# A collective that does not complete within this bound aborts the rank with a message instead of
# blocking it for torch's default 10 min (longer than the bench budget).  RCCL: the watchdog thread
# of ProcessGroupNCCL enforces it (async error handling on); gloo: every collective honours it.
DEFAULT_COLLECTIVE_TIMEOUT_S = 120.0


def collective_timeout_s() -> float:
    return float(os.environ.get("NKV_COLLECTIVE_TIMEOUT_S", DEFAULT_COLLECTIVE_TIMEOUT_S))


def start_rank_watchdog(seconds: float | None = None, label: str = "rank"):
    """Last-resort wall clock for one rank: after ``seconds`` (``NKV_RANK_WALL_S``; unset or <= 0:
    none) dump every thread's stack to stderr and end the process with status 124 — a hang that
    no collective timeout catches (every rank blocked in a collective, under torch.distributed.run
    where bench.py's own launcher is not the parent) still ends before the driver's limit.  Ends
    the process, never execs (no program replacement after GPU initialisation)."""
    if seconds is None:
        seconds = float(os.environ.get("NKV_RANK_WALL_S", "0") or 0)
    if seconds <= 0:
        return None

    def _fire():
        print(f"{label}: wall clock of {seconds:.0f} s exceeded; aborting this rank (status 124)",
              file=sys.stderr, flush=True)
        try:
            faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
        finally:
            os._exit(124)

    t = threading.Timer(seconds, _fire)
    t.daemon = True
    t.start()
    return t


def device_identity(device=None) -> dict:
    """This rank's GPU: index, name, PCI domain:bus:device and UUID (None on a CPU-only rank)."""
    if not torch.cuda.is_available():
        return {"device": None, "name": "cpu", "pci": None, "uuid": None, "host": os.uname().nodename}
    idx = torch.cuda.current_device() if device is None else torch.device(device).index
    pr = torch.cuda.get_device_properties(idx)
    pci = f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}"
    # the marketing name comes from libdrm's amdgpu.ids, absent on some hosts: fall back to the ISA name
    name = pr.name or str(getattr(pr, "gcnArchName", "")).split(":")[0]
    return {"device": int(idx), "name": name, "pci": pci, "uuid": str(getattr(pr, "uuid", "")),
            "host": os.uname().nodename}


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

    def devices(self, device=None) -> list:
        """Every rank's :func:`device_identity`, in rank order (a collective at world > 1)."""
        me = device_identity(device)
        if self.world == 1:
            return [me]
        out = [None] * self.world
        dist.all_gather_object(out, me, group=self.group)
        return out

    def bcast_object(self, obj, src: int = 0):
        """A picklable host object from ``src`` to every rank — the reference's ``bcast`` of
        setup-time data (the restart H, eigensolvers.f90:266; a field-file set's header), or an
        error to raise on every rank."""
        if self.world == 1:
            return obj
        box = [obj]
        dist.broadcast_object_list(box, src=src, group=self.group)
        return box[0]

    def barrier(self) -> None:
        if self.world > 1:
            dist.barrier(group=self.group)

    def raise_if_any(self, err: BaseException | None) -> None:
        """Collective error agreement (a barrier when no rank failed): every rank passes its own
        failure or None; if any rank failed, EVERY rank raises — the lowest failing rank's error
        (its own exception object there, the same type and message elsewhere) — so no rank walks on
        into the next collective while a peer has left (the reference's nek_end stops all ranks)."""
        if self.world == 1:
            if err is not None:
                raise err
            return
        out = [None] * self.world
        dist.all_gather_object(out, None if err is None else (type(err).__name__, str(err)), group=self.group)
        for r, m in enumerate(out):
            if m is None:
                continue
            if r == self.rank and err is not None:
                raise err
            raise _PEER_ERRORS.get(m[0], RuntimeError)(f"rank {r}: {m[1]}")

    def min_scalar(self, x: float, device=None) -> float:
        return -self.max_scalar(-x, device=device)

    def max_scalar(self, x: float, device=None) -> float:
        if self.world == 1 and not self.force:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return float(t.item())


# error types a peer's failure is re-raised as (anything else: RuntimeError with the peer's message)
_PEER_ERRORS = {c.__name__: c for c in (FileNotFoundError, ValueError, OSError, EOFError, KeyError, TypeError,
                                         PermissionError, IsADirectoryError, RuntimeError)}


def init_from_env(backend: str | None = None, force_collectives: bool = False) -> Comm:
    """Initialise torch.distributed from torchrun's env (RANK/WORLD_SIZE/MASTER_*) if present.
    ``force_collectives`` at world size 1: initialise a world-1 group anyway and route every
    partial through it (the cost of the collective path without peers)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    # bounded collectives: set before the process group exists (RCCL reads it at creation)
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    tmo = datetime.timedelta(seconds=collective_timeout_s())
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
        dist.init_process_group(backend, init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                timeout=tmo, **kw)
        return Comm(force_collectives=True)
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            local = int(os.environ.get("LOCAL_RANK", "0"))
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local), timeout=tmo)
        else:  # gloo: CPU tests, or several ranks sharing one GPU (rehearsal of the sharded path)
            if torch.cuda.is_available():
                torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
            dist.init_process_group(backend, timeout=tmo)
    return Comm()

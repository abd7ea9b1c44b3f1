"""Per-phase device timing with HIP events (stream-ordered, no host sync until ``summary``).

The reference's only instrumentation is a wall-clock print around matvec + Gram–Schmidt per Arnoldi
step (core/krylov_decomposition.f90:72,87-94).  Here each phase of the Gram–Schmidt step is
bracketed by events recorded on the stream the kernels run on, together with the algorithmic
bytes that phase moves, so achieved GB/s per kernel family is measured live.
"""
from __future__ import annotations

from collections import defaultdict

import torch


class PhaseTimer:
    def __init__(self, device=None):
        self.device = device
        self._open = {}
        self.records = defaultdict(list)  # name -> [(start_event, end_event, bytes)]

    def begin(self, name: str) -> None:
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(torch.cuda.current_stream(self.device))
        self._open[name] = ev

    def end(self, name: str, nbytes: float) -> None:
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(torch.cuda.current_stream(self.device))
        self.records[name].append((self._open.pop(name), ev, float(nbytes)))

    def last_ms(self, name: str) -> float:
        """Duration of the most recent launch of ``name`` (synchronises)."""
        torch.cuda.synchronize(self.device)
        a, b, _ = self.records[name][-1]
        return a.elapsed_time(b)

    def reset(self) -> None:
        self._open.clear()
        self.records.clear()

    def summary(self) -> dict:
        """{name: {launches, total_ms, avg_ms, avg_bytes, gbps}} (synchronises)."""
        torch.cuda.synchronize(self.device)
        out = {}
        for name, recs in self.records.items():
            ms = [a.elapsed_time(b) for a, b, _ in recs]
            by = [n for _, _, n in recs]
            tot_ms, tot_b = sum(ms), sum(by)
            out[name] = dict(launches=len(recs), total_ms=tot_ms, avg_ms=tot_ms / len(recs),
                             avg_bytes=tot_b / len(recs), gbps=(tot_b / (tot_ms * 1e-3) / 1e9) if tot_ms > 0 else 0.0)
        return out

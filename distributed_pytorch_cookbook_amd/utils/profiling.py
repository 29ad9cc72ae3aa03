"""Tracing / profiling helpers (absent in the reference).

* ``mark(name)``: a roctx range (``torch.cuda.nvtx`` is roctx on ROCm builds) around step
  phases, visible in ``rocprofv3 --marker-trace`` timelines; a no-op on CPU.
* ``StepProfiler``: ``--profile DIR`` records a window of training steps with
  ``torch.profiler`` (CPU + HIP activity) and writes a Chrome trace per rank.
* Fault injection for resilience tests: ``DPC_FAULT_STEP=k [DPC_FAULT_RANK=r]`` makes rank r
  exit abruptly (code 13) at training step k, to exercise torchrun elastic restarts with
  ``--resume latest``.
"""
from __future__ import annotations

import contextlib
import os

import torch


# roctx ranges (torch.cuda.nvtx maps to roctx on ROCm): usable or not is decided ONCE, at the
# first range -- not per call on the hot path (every collective and pipeline micro-batch opens
# one) -- and DPC_ROCTX=0 turns them off entirely.
_ROCTX: bool | None = None if os.environ.get("DPC_ROCTX", "1") != "0" else False


def _roctx_usable() -> bool:
    global _ROCTX
    if _ROCTX is None:
        _ROCTX = False
        if torch.cuda.is_available():
            try:
                torch.cuda.nvtx.range_push("dpc")
                torch.cuda.nvtx.range_pop()
                _ROCTX = True
            except Exception:  # a build whose nvtx module is a stub
                pass
    return _ROCTX


@contextlib.contextmanager
def _range(name: str):
    torch.cuda.nvtx.range_push(name)
    try:
        yield
    finally:
        torch.cuda.nvtx.range_pop()


_NULL = contextlib.nullcontext()


def mark(name: str):
    """A roctx range around a step phase (``rocprofv3 --marker-trace`` shows them), or a no-op
    context when ranges are unavailable or disabled (DPC_ROCTX=0)."""
    return _range(name) if _roctx_usable() else _NULL


class StepProfiler:
    def __init__(self, out_dir: str | None, rank: int = 0, wait: int = 2, warmup: int = 1, active: int = 3):
        self.prof = None
        if not out_dir:
            return
        from torch.profiler import ProfilerActivity, profile, schedule

        os.makedirs(out_dir, exist_ok=True)
        acts = [ProfilerActivity.CPU]
        if torch.cuda.is_available():
            acts.append(ProfilerActivity.CUDA)

        def on_ready(p):
            p.export_chrome_trace(os.path.join(out_dir, f"trace_rank{rank}_step{p.step_num}.json"))

        self.prof = profile(activities=acts, schedule=schedule(wait=wait, warmup=warmup, active=active),
                            on_trace_ready=on_ready, record_shapes=False)
        self.prof.__enter__()

    def step(self):
        if self.prof is not None:
            self.prof.step()

    def close(self):
        if self.prof is not None:
            self.prof.__exit__(None, None, None)
            self.prof = None


def maybe_inject_fault(step: int, rank: int) -> None:
    s = os.environ.get("DPC_FAULT_STEP")
    if s is None or int(s) != step:
        return
    r = int(os.environ.get("DPC_FAULT_RANK", "0"))
    if r == rank:
        print(f"[fault-injection] rank {rank} exiting at step {step}", flush=True)
        os._exit(13)

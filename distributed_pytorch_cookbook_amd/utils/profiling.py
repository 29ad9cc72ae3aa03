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


@contextlib.contextmanager
def mark(name: str):
    use = torch.cuda.is_available()
    if use:
        try:
            torch.cuda.nvtx.range_push(name)
        except Exception:
            use = False
    try:
        yield
    finally:
        if use:
            torch.cuda.nvtx.range_pop()


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

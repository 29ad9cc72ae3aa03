"""Safety of the native RCCL path on CPU, through a host-side fake RCCL / HIP library
(``tests/fakes/fake_rccl_hip.cpp``): the collective watchdog (deadline / async error ->
ncclCommAbort -> non-zero exit), ``--coll_check`` fingerprints through ``NativeTransport``,
bring-up agreement across ranks, and the HIP-graph capture-failure fallback of every engine.
Reference behaviour replaced: c10d's watchdog and ``destroy_process_group``
(``/root/reference/main-ddp.py:26,34-35``)."""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
import time

import pytest
import torch

from dist_helpers import ROOT, free_port, run_workers
from dist_workers import (worker_capture_fallback, worker_native_agreement, worker_native_fingerprint,
                          worker_native_fingerprint_p2p)

pytestmark = pytest.mark.slow


@pytest.fixture(scope="module")
def fake_lib(tmp_path_factory):
    cxx = shutil.which("g++") or shutil.which("c++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    out = tmp_path_factory.mktemp("fake") / "libfake_rccl_hip.so"
    src = os.path.join(ROOT, "tests", "fakes", "fake_rccl_hip.cpp")
    subprocess.run([cxx, "-O1", "-shared", "-fPIC", src, "-o", str(out)], check=True)
    return str(out)


_STALL = r"""
import os, sys, time
sys.path.insert(0, os.environ["ROOT"])
import torch, torch.distributed as dist
from distributed_pytorch_cookbook_amd.parallel.transport import NativeTransport
dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%s" % os.environ["PORT"], rank=0, world_size=1)
tp = NativeTransport(None, device="cpu")
tp.all_reduce(torch.ones(4))       # enqueued, watched, never completes (fake event)
print("enqueued", flush=True)
time.sleep(60)
print("the watchdog did not fire", flush=True)
"""


def _watchdog_run(fake, tmp_path, **env):
    mark = tmp_path / "abort.txt"
    e = dict(os.environ, ROOT=ROOT, PORT=str(free_port()), DPC_RCCL_LIB=fake, DPC_HIP_LIB=fake,
             DPC_COLL_TIMEOUT="1.0", DPC_WATCHDOG_POLL_MS="50", FAKE_ABORT_MARK=str(mark), **env)
    e.pop("DPC_WATCHDOG", None)
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, "-c", _STALL], env=e, capture_output=True, text=True, timeout=120)
    return r, time.monotonic() - t0, mark


def test_watchdog_aborts_stalled_collective(fake_lib, tmp_path):
    r, dt, mark = _watchdog_run(fake_lib, tmp_path, FAKE_EVENT_STALL="1")
    assert r.returncode == 17, (r.returncode, r.stdout, r.stderr[-2000:])
    assert "enqueued" in r.stdout and "did not fire" not in r.stdout
    assert "[dpc watchdog]" in r.stderr and "all_reduce(4,)" in r.stderr and "still pending" in r.stderr
    assert mark.read_text().count("abort") == 1  # ncclCommAbort on the communicator
    assert dt < 40, dt


def test_watchdog_aborts_on_rccl_async_error(fake_lib, tmp_path):
    r, dt, mark = _watchdog_run(fake_lib, tmp_path, FAKE_ASYNC_ERR="5")
    assert r.returncode == 17, (r.returncode, r.stdout, r.stderr[-2000:])
    assert "asynchronous error" in r.stderr and mark.exists()


def test_watchdog_quiet_when_collectives_complete(fake_lib, tmp_path):
    code = _STALL.replace("time.sleep(60)", "time.sleep(1.5)").replace(
        'print("the watchdog did not fire", flush=True)',
        "from distributed_pytorch_cookbook_amd.parallel import native_comm\n"
        "assert native_comm.watchdog_pending() == 0\n"
        "from distributed_pytorch_cookbook_amd.parallel.comm import cleanup_dist\ncleanup_dist()\nprint('clean')")
    e = dict(os.environ, ROOT=ROOT, PORT=str(free_port()), DPC_RCCL_LIB=fake_lib, DPC_HIP_LIB=fake_lib,
             DPC_COLL_TIMEOUT="1.0", DPC_WATCHDOG_POLL_MS="50", FAKE_LOG=str(tmp_path / "log"))
    e.pop("DPC_WATCHDOG", None)
    r = subprocess.run([sys.executable, "-c", code], env=e, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "clean" in r.stdout, (r.stdout, r.stderr[-2000:])
    # cleanup_dist destroyed the communicator (ncclCommDestroy)
    assert (tmp_path / "log").read_text().split() == ["all_reduce", "destroy"]


def test_coll_check_through_native_transport(fake_lib, tmp_path):
    run_workers(worker_native_fingerprint, 2, fake_lib, str(tmp_path / "log"))
    for r in range(2):
        assert (tmp_path / f"log.{r}").read_text().split() == ["all_reduce", "all_gather"]


def test_coll_check_skips_p2p_on_native_transport(fake_lib, tmp_path):
    run_workers(worker_native_fingerprint_p2p, 2, fake_lib, str(tmp_path / "log"))
    for r in range(2):
        ops = (tmp_path / f"log.{r}").read_text().split()
        assert ops[-2:] == ["all_reduce", "all_gather"], ops


@pytest.mark.parametrize("mode", ["uid", "init"])
def test_native_bringup_failure_is_agreed(fake_lib, tmp_path, mode):
    run_workers(worker_native_agreement, 2, fake_lib, mode, str(tmp_path / "log"))
    if mode == "init":  # rank 0's communicator came up and was destroyed again
        assert "destroy" in (tmp_path / "log.0").read_text().split()


@pytest.mark.parametrize("kind,world", [("ddp", 2), ("fsdp", 2), ("pipe", 2), ("pipe", 4)],
                         ids=["ddp", "fsdp", "pipe", "pipe_ddp"])
def test_capture_failure_fallback_matches_eager(tmp_path, kind, world):
    ref, got = tmp_path / "eager.pt", tmp_path / "fallback.pt"
    run_workers(worker_capture_fallback, world, str(ref), kind, False, False)
    run_workers(worker_capture_fallback, world, str(got), kind, True, False)
    a, b = torch.load(ref, weights_only=True), torch.load(got, weights_only=True)
    for k in a:
        assert torch.equal(a[k], b[k]), (k, (a[k] - b[k]).abs().max().item())


@pytest.mark.parametrize("kind", ["ddp"])
def test_capture_failure_without_reset_diverges(tmp_path, kind):
    """Negative control: without Engine.reset_step_state the retried DDP step finds its
    buckets marked as launched by the failed capture, never all-reduces them and the ranks
    diverge -- the test above has teeth.  (FSDP's stale gathered units hold valid weights on
    CPU, where the 'recorded' gathers did run, so only the GPU would show that case.)"""
    ref, got = tmp_path / "eager.pt", tmp_path / "broken.pt"
    run_workers(worker_capture_fallback, 2, str(ref), kind, False, False)
    run_workers(worker_capture_fallback, 2, str(got), kind, True, True)
    a, b = torch.load(ref, weights_only=True), torch.load(got, weights_only=True)
    assert any(not torch.equal(a[k], b[k]) for k in a)


def test_process_with_running_watchdog_exits_cleanly(fake_lib, tmp_path):
    """No explicit teardown: the atexit hook joins the watchdog thread (a joinable std::thread
    left at exit would std::terminate the process)."""
    code = _STALL.replace("time.sleep(60)", "time.sleep(0.3)").replace(
        'print("the watchdog did not fire", flush=True)', "print('bye', flush=True)")
    e = dict(os.environ, ROOT=ROOT, PORT=str(free_port()), DPC_RCCL_LIB=fake_lib, DPC_HIP_LIB=fake_lib)
    e.pop("DPC_WATCHDOG", None)
    r = subprocess.run([sys.executable, "-c", code], env=e, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "bye" in r.stdout, (r.returncode, r.stderr[-2000:])
    assert "terminate" not in r.stderr


_DESTROY_STUCK = r"""
import os, sys, time
sys.path.insert(0, os.environ["ROOT"])
import torch, torch.distributed as dist
from distributed_pytorch_cookbook_amd.parallel.native_comm import NativeComm
dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%s" % os.environ["PORT"], rank=0, world_size=1)
world = NativeComm(None, device="cpu")
sub = world.split(color=0, key=0)
world.all_reduce(torch.ones(4), stream=0)
from distributed_pytorch_cookbook_amd.parallel import native_comm
native_comm.watchdog_track(0, "all_reduce(4,)")   # stalls (fake event): the watchdog fires at 1 s
print("destroying", flush=True)
sub.destroy()                                     # ncclCommDestroy hangs (FAKE_DESTROY_SLEEP)
print("destroy returned", flush=True)
"""


def test_watchdog_aborts_others_while_a_destroy_hangs(fake_lib, tmp_path):
    """the watchdog fires while the main thread is stuck inside ncclCommDestroy (it
    holds the `life` lock): after its 2 s grace the watchdog still aborts every OTHER registered
    communicator (the parent here) and exits 17, instead of leaving them all live."""
    mark = tmp_path / "abort.txt"
    e = dict(os.environ, ROOT=ROOT, PORT=str(free_port()), DPC_RCCL_LIB=fake_lib, DPC_HIP_LIB=fake_lib,
             DPC_COLL_TIMEOUT="1.0", DPC_WATCHDOG_POLL_MS="50", FAKE_ABORT_MARK=str(mark), FAKE_EVENT_STALL="1",
             FAKE_DESTROY_SLEEP="60")
    e.pop("DPC_WATCHDOG", None)
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, "-c", _DESTROY_STUCK], env=e, capture_output=True, text=True, timeout=120)
    dt = time.monotonic() - t0
    assert r.returncode == 17, (r.returncode, r.stdout, r.stderr[-2000:])
    assert "destroying" in r.stdout and "destroy returned" not in r.stdout
    assert "destroy is stuck; aborting the other 1" in r.stderr, r.stderr[-2000:]
    assert mark.read_text().count("abort") == 1  # the parent, not the communicator being destroyed
    assert dt < 40, dt

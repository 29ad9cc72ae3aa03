"""The production multi-rank transport (``NativeTransport`` over ``NativeComm`` over
``runtime/csrc/rccl_comm.cpp``) driven end to end at 2 and 4 ranks on CPU.

The RCCL underneath is ``tests/fakes/fake_rccl_hip.cpp`` in its data-moving mode
(``FAKE_DIR``): all-reduce / reduce-scatter / all-gather / broadcast are rendezvous over
files that carry every rank's buffer, send / recv go through per-pair mailboxes with
blocking receives, ``ncclGroupStart/End`` fuse a group, and ``ncclCommSplit`` really
partitions the ranks.  So everything the 8-GPU run relies on above RCCL is executed with
more than one rank: element counts (``count`` / ``recvcount`` of every call), the
sub-communicator ranks of the (pp, dp) mesh after ``ncclCommSplit``, the pipeline peer
numbering on the split communicator, the grouped send/recv order of GPipe / 1F1B, and the
checkpoint gathers -- with ``--coll_check`` (group-wide fingerprints) and ``--stream_check``
on.  Every recipe's final checkpoint must equal the same recipe over gloo (``--comm
torch``): bit for bit with f32 gradient reduction, within bf16 rounding with
``--reduce_dtype bf16``.  Reference: the NCCL collectives of ``/root/reference/main-ddp.py:55,124``
and ``/root/reference/main-fsdp.py:64-69``.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

import pytest
import torch

from dist_helpers import ROOT, free_port

pytestmark = pytest.mark.slow

L = 2
COMMON = ["--cpu", "--synthetic_data", "--sequence_length", "16", "--dim", "32", "--heads", "2",
          "--head_dim", "16", "--num_layers", str(L), "--train_samples", "48", "--val_samples", "16",
          "--num_workers", "0", "--learning_rate", "1e-3", "--epochs", "1", "--seed", "0",
          "--coll_check", "--stream_check"]


@pytest.fixture(scope="module")
def fake_lib(tmp_path_factory):
    cxx = shutil.which("g++") or shutil.which("c++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    out = tmp_path_factory.mktemp("fake") / "libfake_rccl_hip.so"
    src = os.path.join(ROOT, "tests", "fakes", "fake_rccl_hip.cpp")
    subprocess.run([cxx, "-O2", "-shared", "-fPIC", src, "-o", str(out)], check=True)
    return str(out)


def _env(**extra):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1", MASTER_ADDR="127.0.0.1")
    for k in ("DPC_FAULT_STEP", "DPC_FAULT_RANK", "RANK", "WORLD_SIZE", "LOCAL_RANK", "DPC_COMM", "DPC_RCCL_LIB",
              "DPC_HIP_LIB", "FAKE_DIR", "FAKE_LOG"):
        env.pop(k, None)
    env.update(extra)
    return env


def _run(script, nproc, args, cwd, env):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(ROOT, script), *args]
    r = subprocess.run(cmd, cwd=cwd, env=env, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, (script, nproc, r.returncode, r.stdout[-3000:], r.stderr[-3000:])
    return r


def _final(ckdir):
    from distributed_pytorch_cookbook_amd.utils.checkpoint import load_model_state

    files = sorted(f for f in os.listdir(ckdir) if f.endswith(".pt") and not f.endswith(".train.pt")
                   and "_step" not in f)
    assert len(files) == 1, files
    return load_model_state(os.path.join(ckdir, files[0]))


# (script, ranks, per-replica batch, extra flags, ops the native log must show, exact)
CASES = [
    ("main-ddp.py", 2, 4, ["--bucket_mb", "0.5"], {"broadcast", "all_reduce"}, True),
    ("main-fsdp.py", 2, 4, [], {"all_gather", "reduce_scatter"}, True),
    ("main-fsdp.py", 2, 4, ["--reduce_dtype", "bf16"], {"all_gather", "reduce_scatter"}, False),
    ("main-pipe.py", 2, 8, ["--num_microbatches", "4", "--schedule", "1f1b"], {"send", "recv"}, True),
    ("main-pipe-ddp.py", 4, 4, ["--num_microbatches", "2"], {"send", "recv", "all_reduce"}, True),
    # the north-star topologies at full rank count (BASELINE.json: PP = 8 1F1B, PP 2 x DP 4) and
    # the other schedule / precision at 4 ranks
    ("main-pipe.py", 8, 16, ["--num_microbatches", "16", "--schedule", "1f1b", "--num_layers", "8"],
     {"send", "recv"}, True),
    ("main-pipe.py", 4, 8, ["--num_microbatches", "8", "--schedule", "gpipe"], {"send", "recv"}, True),
    # (4 f32 gradients summed in another order than gloo's ring: equal to f32 rounding, not bitwise)
    ("main-pipe-ddp.py", 8, 4, ["--num_microbatches", "2", "--dp_size", "4"], {"send", "recv", "all_reduce"}, "f32"),
    ("main-fsdp.py", 4, 4, ["--reduce_dtype", "bf16"], {"all_gather", "reduce_scatter"}, False),
    # the zero-bubble schedule (deferred W passes; its DP buckets launch from them)
    ("main-pipe.py", 4, 8, ["--num_microbatches", "8", "--schedule", "zb"], {"send", "recv"}, True),
    ("main-pipe.py", 8, 16, ["--num_microbatches", "16", "--schedule", "zb2", "--num_layers", "8"], {"send", "recv"},
     True),
    ("main-pipe-ddp.py", 4, 4, ["--num_microbatches", "4", "--schedule", "zb"], {"send", "recv", "all_reduce"}, True),
]


@pytest.mark.parametrize("script,nproc,batch,extra,ops,exact", CASES,
                         ids=["ddp2", "fsdp2", "fsdp2_bf16", "pipe2_1f1b", "pipe2xdp2", "pipe8_1f1b", "pipe4_gpipe",
                              "pipe2xdp4", "fsdp4_bf16", "pipe4_zb", "pipe8_zb2", "pipe2xdp2_zb"])
def test_native_transport_multirank_matches_gloo(tmp_path, fake_lib, script, nproc, batch, extra, ops, exact):
    args = [*COMMON, "--batch_size", str(batch), *extra]
    ref_dir, nat_dir, fake_dir = tmp_path / "gloo", tmp_path / "native", tmp_path / "fake"
    for d in (ref_dir, nat_dir, fake_dir):
        d.mkdir()
    _run(script, nproc, [*args, "--comm", "torch", "--checkpoint_dir", str(ref_dir / "ck")], ref_dir, _env())
    log = tmp_path / "ops.log"
    r = _run(script, nproc, [*args, "--comm", "native", "--checkpoint_dir", str(nat_dir / "ck")], nat_dir,
             _env(DPC_RCCL_LIB=fake_lib, DPC_HIP_LIB=fake_lib, FAKE_DIR=str(fake_dir), FAKE_LOG=str(log),
                  FAKE_TIMEOUT_S="300"))
    assert "native RCCL" not in r.stdout, r.stdout[-2000:]  # no fallback to torch.distributed
    assert "[validation] Epoch 1/1" in r.stdout, r.stdout[-2000:]
    seen = set(log.read_text().split())
    assert ops <= seen, (ops, seen)
    a, b = _final(nat_dir / "ck"), _final(ref_dir / "ck")
    assert list(a) == list(b)
    for k in a:
        if exact == "f32":
            torch.testing.assert_close(a[k], b[k], atol=1e-5, rtol=1e-5)
        elif exact:
            assert torch.equal(a[k], b[k]), (k, (a[k] - b[k]).abs().max().item())
        else:
            torch.testing.assert_close(a[k], b[k], atol=2e-3, rtol=2e-2)


def test_fake_rccl_moves_data_and_splits(fake_lib, tmp_path):
    """The fake's own semantics at 4 ranks (so the recipe tests above test the engines, not
    the fake): reductions / gathers / broadcast by dtype, grouped send/recv in a ring, and a
    2 x 2 split whose sub-communicators reduce only over their members."""
    from dist_helpers import run_workers
    from dist_workers import worker_fake_rccl_semantics

    run_workers(worker_fake_rccl_semantics, 4, fake_lib, str(tmp_path / "fake"))


def test_fake_rccl_blocking_send_rule(fake_lib, tmp_path):
    """Negative test of the fake itself: an exchange ordered so that it deadlocks under RCCL's
    blocking sends (both ranks send first, ungrouped) must fail, not pass -- so the recipe tests
    above would catch a cross-group ordering that hangs on xGMI."""
    from dist_helpers import run_workers
    from dist_workers import worker_fake_rccl_p2p_completion

    run_workers(worker_fake_rccl_p2p_completion, 2, fake_lib, str(tmp_path / "fake"))

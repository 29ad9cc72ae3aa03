"""Host-side parts of the peer-access collectives (parallel/ipc_comm.py): chunk sizing against
the kernel's staging layout (ops/csrc/ipc_coll.hip: dpc_ipc_coll's size check), and the
transport / CLI plumbing.  The kernels themselves: tests/test_ipc_gpu.py."""
import torch

from distributed_pytorch_cookbook_amd.parallel import ipc_comm as ic


def _need(op, n, W, es, A=64):
    """Bytes of one staging half the kernel needs (mirror of dpc_ipc_coll)."""
    if op == ic.ALLREDUCE:
        return W * (((n + W - 1) // W + A - 1) // A * A) * es
    if op == ic.REDUCE_SCATTER:
        return W * ((n + A - 1) // A * A) * es
    return ((n + A - 1) // A * A) * es


def test_chunk_capacity_fits_a_staging_half():
    c = object.__new__(ic.IpcComm)
    for W in (1, 2, 3, 7, 8):
        for half in (256, 4096, 262144, 64 << 20):
            for es in (2, 4):
                c.size, c.half_bytes = W, half
                for op in (ic.ALLREDUCE, ic.REDUCE_SCATTER, ic.ALLGATHER, ic.BROADCAST):
                    cap = c._cap(op, es)
                    if cap == 0:  # (a half too small for one aligned shard per rank)
                        assert _need(op, 1, W, es) > half
                        continue
                    assert cap % 64 == 0, (W, half, es, op, cap)  # chunk starts stay 16-B aligned
                    assert _need(op, cap, W, es) <= half, (W, half, es, op, cap)
                    # and it is the largest such multiple of the alignment (no needless chunks)
                    step = 64 * (W if op == ic.ALLREDUCE else 1)
                    assert _need(op, cap + step, W, es) > half, (W, half, es, op, cap)


def test_comm_flag_accepts_ipc_and_cpu_falls_back():
    from distributed_pytorch_cookbook_amd.config import build_parser
    from distributed_pytorch_cookbook_amd.parallel.transport import TorchTransport, make_transport

    assert build_parser().parse_args(["--comm", "ipc"]).comm == "ipc"
    # no process group, CPU tensors: the peer-access transport is never chosen
    assert isinstance(make_transport(None, torch.device("cpu"), "ipc"), TorchTransport)

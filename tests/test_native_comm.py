"""Native RCCL communicator (parallel/native_comm.py over runtime/csrc/rccl_comm.cpp)."""
import socket

import pytest
import torch
import torch.distributed as dist


def test_rccl_symbols_resolve():
    """The runtime library finds torch's librccl and every entry point the engines use."""
    from distributed_pytorch_cookbook_amd.parallel import native_comm

    h = native_comm._lib()
    assert h.dpc_rccl_error() is not None


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
def test_native_comm_single_rank_collectives():
    from distributed_pytorch_cookbook_amd.parallel.native_comm import NativeComm

    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=torch.device("cuda:0"))
    try:
        c = NativeComm(device=torch.device("cuda:0"))
        assert (c.rank, c.size) == (0, 1)
        x = torch.randn(1000, device="cuda")
        y = x.clone()
        c.all_reduce(y)
        torch.testing.assert_close(y, x)
        b = torch.randn(512, device="cuda").bfloat16()
        c.all_reduce(b, op="max")
        out = torch.empty(1000, device="cuda")
        c.all_gather(out, x)
        torch.testing.assert_close(out, x)
        rs = torch.empty(1000, device="cuda")
        c.reduce_scatter(rs, x)
        torch.testing.assert_close(rs, x)
        c.broadcast(y, src=0)
        r = torch.empty_like(x)
        with c.grouped():
            c.send(x, 0)
            c.recv(r, 0)
        torch.testing.assert_close(r, x)
        sub = c.split(color=0, key=0)
        assert (sub.rank, sub.size) == (0, 1)
        sub.all_reduce(y)
        torch.cuda.synchronize()
        c.check_async()
        sub.destroy()
        c.destroy()
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_native_transport_ddp_hip_graph():
    """The DDP step with its bucket all-reduces on the native RCCL transport (one rank, so
    the collectives are real RCCL calls that change nothing) captured into a HIP graph:
    same parameters as the plain single-GPU engine."""
    from distributed_pytorch_cookbook_amd.engine.data_parallel import DataParallelEngine
    from distributed_pytorch_cookbook_amd.models.gpt import TransformerDecoderLM

    def make():
        torch.manual_seed(0)
        with torch.device("cuda"):
            return TransformerDecoderLM(dim=256, head_dim=64, heads=4, num_layers=3, vocab_size=4000,
                                        max_position_embeddings=128, activation="gelu")

    def batch(step):
        g = torch.Generator(device="cpu").manual_seed(step)
        ids = torch.randint(0, 4000, (8, 128), generator=g).cuda()
        pos = torch.arange(127, device="cuda").expand(8, -1)
        return dict(input_ids=ids[:, :-1], position_ids=pos, mask=None), ids[:, 1:]

    ref = DataParallelEngine(make(), "cuda", lr=1e-3)
    for s in range(3):
        ref.train_step(*batch(s))
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=torch.device("cuda:0"))
    try:
        eng = DataParallelEngine(make(), "cuda", lr=1e-3, graph=True, comm_kind="native", force_ddp_store=True,
                                 bucket_mb=4.0)
        assert eng.store.tp.kind == "native" and len(eng.store.buckets) > 1
        for s in range(3):
            eng.train_step(*batch(s))
        torch.cuda.synchronize()
        assert eng.graph and eng._stepper.graph is not None, "the native-transport step was not captured"
        a, b = eng.store.master, ref.store.master
        assert ((a - b).norm() / b.norm()).item() < 1e-3
        eng.store.tp.nc.check_async()
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("graph", [False, True])
def test_native_fsdp_sharded_unitwise_adamw(graph):
    """FSDP on its N > 1 code path at one rank (native RCCL communicator, sharded store): the
    reduce-scatters complete unit by unit and AdamW updates each unit's shard as its
    reduce-scatter lands (FSDPStore.finish_grads_and_update), eager and HIP-graph captured;
    the rank-0 checkpoint gather goes through grouped point-to-point.  Same weights as the
    unsharded FSDP engine."""
    from distributed_pytorch_cookbook_amd.engine.fsdp import FSDPEngine
    from distributed_pytorch_cookbook_amd.models.gpt import TransformerDecoderLM

    def make():
        torch.manual_seed(0)
        with torch.device("cuda"):
            return TransformerDecoderLM(dim=256, head_dim=64, heads=4, num_layers=3, vocab_size=4000,
                                        max_position_embeddings=128, activation="gelu")

    def batch(step):
        g = torch.Generator(device="cpu").manual_seed(step)
        ids = torch.randint(0, 4000, (8, 128), generator=g).cuda()
        pos = torch.arange(127, device="cuda").expand(8, -1)
        return dict(input_ids=ids[:, :-1], position_ids=pos, mask=None), ids[:, 1:]

    ref = FSDPEngine(make(), "cuda", lr=1e-3)
    for s in range(3):
        ref.train_step(*batch(s))
    ref_sd = ref.full_state_dict()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=torch.device("cuda:0"))
    try:
        eng = FSDPEngine(make(), "cuda:0", lr=1e-3, comm_kind="native", force_sharded=True, graph=graph)
        assert eng.store.sharded and eng.store.tp.kind == "native"
        for s in range(3):
            eng.train_step(*batch(s))
        torch.cuda.synchronize()
        sd = eng.full_state_dict()
        for k in ref_sd:
            a, b = sd[k].float(), ref_sd[k].float()
            scale = max(b.norm().item(), 3e-3 * b.numel() ** 0.5)
            assert (a - b).norm().item() / scale < 1e-2, k
        eng.store.tp.nc.check_async()
    finally:
        dist.destroy_process_group()

"""ctypes binding of ``libdpc_kernels.so`` (the gfx950 kernels in ``ops/csrc``).

Each C launcher takes a pointer to an argument struct plus the raw ``hipStream_t`` of
the caller's current torch stream, so the kernels are ordered with torch's own work and
are captured by HIP graphs exactly like torch's kernels.  The structs below mirror the C
structs field-for-field (standard C layout on both sides).

Loading is strict on a GPU: if the library is missing it is built in-tree with hipcc;
if that fails the error propagates -- there is no silent fallback to torch ops.
"""
from __future__ import annotations

import ctypes
import os
import threading
from ctypes import c_float, c_int, c_longlong, c_uint, c_void_p

import torch

from . import build as _build

P = c_void_p
LL = c_longlong


class GemmArgs(ctypes.Structure):
    _fields_ = [
        ("A", P), ("B", P), ("C", P), ("bias", P), ("residual", P), ("aux_in", P),
        ("aux_out", P), ("alpha_ptr", P), ("colsum", P),
        ("lda", LL), ("ldb", LL), ("ldc", LL), ("ldr", LL), ("ld_aux_in", LL), ("ld_aux_out", LL),
        ("M", c_int), ("N", c_int), ("K", c_int),
        ("alpha", c_float),
        ("act", c_int), ("act_bwd", c_int), ("out_f32", c_int), ("accumulate", c_int),
        ("a_kmaj", c_int), ("b_kmaj", c_int),
        ("a_r", c_int), ("a_c", c_int), ("b_r", c_int), ("b_c", c_int),
        ("ksplit", c_int),  # dispatcher-owned (pass 0)
        ("impl", c_int),    # 0 = dispatcher policy, else a measured per-shape choice
        ("aux_f32", c_int),  # dpc_gemm_f32: f32 aux_in / aux_out (else bf16)
        ("ws", P), ("ws_bytes", LL),  # split-K workspace (v7 slab split instead of atomics)
        ("nt_store", c_int),  # dispatcher-owned (pass 0): non-temporal epilogue stores
        ("aux_deriv", c_int),  # aux_out = bf16(act'(v)) instead of the pre-activation (GELU only)
    ]


IPC_MAXW = 8


class IpcCollArgs(ctypes.Structure):
    """``ipc_coll.hip:IpcCollArgs``."""
    _fields_ = [
        ("slot", P * IPC_MAXW), ("flags", P * IPC_MAXW), ("ep", P), ("error", P),
        ("inp", P), ("out", P),
        ("n", LL), ("half_bytes", LL), ("spin_limit", LL),
        ("op", c_int), ("bf16", c_int), ("rank", c_int), ("world", c_int), ("root", c_int),
    ]


IPC_P2P_MAX = 8


class IpcP2PArgs(ctypes.Structure):
    """``ipc_coll.hip:IpcP2PArgs``."""
    _fields_ = [
        ("slot", P * IPC_MAXW), ("flags", P * IPC_MAXW), ("cnt", P), ("error", P),
        ("send_ptr", P * IPC_P2P_MAX), ("recv_ptr", P * IPC_P2P_MAX),
        ("send_n", LL * IPC_P2P_MAX), ("recv_n", LL * IPC_P2P_MAX),
        ("send_peer", c_int * IPC_P2P_MAX), ("recv_peer", c_int * IPC_P2P_MAX),
        ("region_bytes", LL), ("spin_limit", LL),
        ("nsend", c_int), ("nrecv", c_int), ("rank", c_int), ("world", c_int),
    ]


class AttnArgs(ctypes.Structure):
    _fields_ = [
        ("q", P), ("k", P), ("v", P), ("o", P), ("lse", P), ("pad", P), ("dout", P),
        ("dq", P), ("dk", P), ("dv", P), ("delta", P),
        ("ld_qkv", LL), ("ld_o", LL), ("ld_dqkv", LL),
        ("N", c_int), ("S", c_int), ("H", c_int),
        ("scale", c_float),
        ("causal", c_int),
        ("hd", c_int),
        ("order", c_int),  # (attention.hip's backward launcher sets it: DPC_ATTN_ORDER)
    ]


class LNArgs(ctypes.Structure):
    _fields_ = [
        ("x", P), ("gamma", P), ("beta", P), ("y", P), ("mean", P), ("rstd", P),
        ("dy", P), ("dx", P), ("dgamma", P), ("dbeta", P),
        ("ldx", LL), ("ldy", LL), ("lddy", LL), ("lddx", LL),
        ("T", c_int), ("D", c_int),
        ("eps", c_float),
        ("y_f32", c_int),
        ("gout", P), ("gsum", P), ("ld_gout", LL),
        ("drop_key", c_uint), ("drop_thresh", c_uint), ("drop_scale", c_float),
        ("dy_bf16", c_int),
        ("add_y", P), ("add_bias", P), ("x_out", P), ("ld_add", LL), ("ld_xout", LL),
        ("drop_seed", P), ("drop_site", c_uint),
        ("gz", P), ("ld_gz", LL), ("gact", c_int),
        ("dx_set", c_int),
        ("add_act", c_int),  # fwd fused add: xs = x + keep * act(add_y + add_bias)
    ]


class EmbArgs(ctypes.Structure):
    _fields_ = [
        ("ids", P), ("pos", P), ("tok", P), ("ptab", P), ("out", P), ("dout", P),
        ("dtok", P), ("dpos", P),
        ("T", c_int), ("D", c_int), ("V", c_int), ("P", c_int),
        ("table_bf16", c_int),
    ]


class CEArgs(ctypes.Structure):
    _fields_ = [
        ("logits", P), ("dlogits", P), ("targets", P), ("inv_count", P), ("row_loss", P),
        ("row_correct", P),
        ("ld", LL),
        ("T", c_int), ("V", c_int),
        ("write_grad", c_int), ("ignore_index", c_int),
    ]


class AdamArgs(ctypes.Structure):
    _fields_ = [
        ("param", P), ("grad", P), ("exp_avg", P), ("exp_avg_sq", P), ("shadow", P),
        ("grad_scale_ptr", P),
        ("n", LL),
        ("lr", c_float), ("beta1", c_float), ("beta2", c_float), ("eps", c_float),
        ("weight_decay", c_float), ("bias_correction1", c_float),
        ("bias_correction2_sqrt", c_float), ("grad_scale", c_float),
        ("step_ptr", P), ("skip_ptr", P),
    ]


class AmpCheckArgs(ctypes.Structure):
    _fields_ = [("g", P), ("n", LL), ("found_inf", P)]


class AmpUpdateArgs(ctypes.Structure):
    _fields_ = [("scale", P), ("inv_scale", P), ("found_inf", P), ("tracker", P),
                ("growth", c_float), ("backoff", c_float), ("interval", c_int)]


class CastArgs(ctypes.Structure):
    _fields_ = [("src", P), ("dst", P), ("n", LL)]


class BiasActArgs(ctypes.Structure):
    _fields_ = [
        ("dy", P), ("z", P), ("dz", P), ("db", P),
        ("lddy", LL), ("ldz", LL), ("lddz", LL),
        ("T", c_int), ("N", c_int),
        ("act", c_int),
        ("drop_key", c_uint), ("drop_thresh", c_uint), ("drop_scale", c_float),
        ("drop_seed", P), ("drop_site", c_uint),
    ]


class DropResArgs(ctypes.Structure):
    _fields_ = [
        ("y", P), ("res", P), ("out", P),
        ("ldy", LL), ("ldr", LL), ("ldo", LL),
        ("T", c_int), ("N", c_int),
        ("key", c_uint), ("thresh", c_uint),
        ("scale", c_float),
        ("seed", P), ("site", c_uint),
    ]


class DecodeAttnArgs(ctypes.Structure):
    _fields_ = [
        ("qkv", P), ("kc", P), ("vc", P), ("o", P), ("len", P),
        ("ldqkv", LL), ("ldo", LL),
        ("N", c_int), ("H", c_int), ("hd", c_int), ("Smax", c_int),
        ("scale", c_float),
    ]


class EmbBwdArgs(ctypes.Structure):
    _fields_ = [
        ("ids", P), ("pos", P), ("dout", P), ("dtok", P), ("dpos", P), ("ws", P),
        ("ws_bytes", ctypes.c_ulonglong),
        ("T", c_int), ("D", c_int), ("V", c_int), ("P", c_int),
    ]


class GemvArgs(ctypes.Structure):
    _fields_ = [
        ("x", P), ("w", P), ("bias", P), ("residual", P), ("y", P),
        ("ldx", LL), ("ldw", LL), ("ldr", LL), ("ldy", LL),
        ("M", c_int), ("N", c_int), ("Nw", c_int), ("K", c_int),
        ("act", c_int), ("y_f32", c_int),
    ]


_FUNCS = {
    "dpc_decode_attn": DecodeAttnArgs,
    "dpc_gemv": GemvArgs,
    "dpc_embedding_bwd_sorted": EmbBwdArgs,
    "dpc_gemm": GemmArgs,
    "dpc_gemm_f32": GemmArgs,
    "dpc_attn_fwd": AttnArgs,
    "dpc_attn_bwd": AttnArgs,
    "dpc_attn_fwd_f32": AttnArgs,
    "dpc_attn_bwd_f32": AttnArgs,
    "dpc_layernorm_fwd": LNArgs,
    "dpc_layernorm_bwd": LNArgs,
    "dpc_embedding_fwd": EmbArgs,
    "dpc_embedding_bwd": EmbArgs,
    "dpc_cross_entropy": CEArgs,
    "dpc_adamw": AdamArgs,
    "dpc_amp_check": AmpCheckArgs,
    "dpc_amp_update": AmpUpdateArgs,
    "dpc_cast_f32_bf16": CastArgs,
    "dpc_bias_act_bwd": BiasActArgs,
    "dpc_dropout_residual": DropResArgs,
}

_lock = threading.Lock()
_lib = None
_error = None


def lib() -> ctypes.CDLL:
    """Load (building if needed) the kernel library. Raises if it cannot be had."""
    global _lib, _error
    if _lib is not None:
        return _lib
    if _error is not None:  # fail fast: do not re-run a failed build on every call
        raise RuntimeError(f"kernel library unavailable: {_error}")
    with _lock:
        if _lib is None:
            if _build.needs_build():
                try:
                    _build.build()
                except Exception as exc:
                    _error = exc
                    raise
            handle = ctypes.CDLL(str(_build.LIB_PATH), mode=ctypes.RTLD_GLOBAL)
            for name, st in _FUNCS.items():
                fn = getattr(handle, name)
                fn.argtypes = [ctypes.POINTER(st), c_void_p]
                fn.restype = c_int
            handle.dpc_gemm_set_impl.argtypes = [c_int]
            handle.dpc_gemm_set_impl.restype = None
            handle.dpc_gemm_set_variant.argtypes = [c_int, c_int]
            handle.dpc_gemm_set_variant.restype = None
            handle.dpc_gemm_last_kernel.argtypes = []
            handle.dpc_gemm_last_kernel.restype = c_int
            handle.dpc_gemm_set_xcd_split.argtypes = [c_int]
            handle.dpc_gemm_set_xcd_split.restype = None
            handle.dpc_gemm_set_splits.argtypes = [c_int]
            handle.dpc_gemm_set_splits.restype = None
            handle.dpc_set_cu_reserve.argtypes = [c_int]
            handle.dpc_set_cu_reserve.restype = None
            handle.dpc_get_cu_reserve.argtypes = []
            handle.dpc_get_cu_reserve.restype = c_int
            handle.dpc_occupy.argtypes = [c_int, ctypes.c_longlong, c_void_p, c_void_p]
            handle.dpc_occupy.restype = c_int
            handle.dpc_embedding_bwd_ws.argtypes = [c_int, c_int]
            handle.dpc_embedding_bwd_ws.restype = ctypes.c_ulonglong
            # intra-node peer-access collectives (ipc_coll.hip, parallel/ipc_comm.py)
            handle.dpc_ipc_alloc.argtypes = [ctypes.c_longlong, c_int, ctypes.POINTER(c_void_p)]
            handle.dpc_ipc_free.argtypes = [c_void_p]
            handle.dpc_ipc_handle.argtypes = [c_void_p, c_void_p]
            handle.dpc_ipc_open.argtypes = [c_void_p, ctypes.POINTER(c_void_p)]
            handle.dpc_ipc_close.argtypes = [c_void_p]
            handle.dpc_ipc_coll.argtypes = [ctypes.POINTER(IpcCollArgs), c_void_p]
            handle.dpc_ipc_p2p.argtypes = [ctypes.POINTER(IpcP2PArgs), c_void_p]
            for f in ("dpc_ipc_alloc", "dpc_ipc_free", "dpc_ipc_handle", "dpc_ipc_open", "dpc_ipc_close",
                      "dpc_ipc_coll", "dpc_ipc_p2p", "dpc_ipc_handle_size", "dpc_ipc_max_world", "dpc_ipc_groups"):
                getattr(handle, f).restype = c_int
            _lib = handle
    return _lib


forced_gemm_impl = -1


def set_gemm_impl(impl: int) -> None:
    """Force a GEMM implementation (tests / sweeps): -1 auto (default), 1 register-staged v1,
    2-4 LDS-DMA 128x128 v2 variants, 10 the 256x128 v3, 16-26 the persistent 256x256 v7 / v8 / v9
    placements (table at the dispatcher, ``csrc/gemm.hip``)."""
    global forced_gemm_impl
    forced_gemm_impl = int(impl)
    lib().dpc_gemm_set_impl(int(impl))


def gemm_last_kernel() -> int:
    """Family + epilogue of the last product the persistent-GEMM dispatcher launched (900 + EPI:
    v9, 700 + EPI: v7, 750 + EPI: v8 / v7d; 0: it launched nothing -- a fallback ran)."""
    return int(lib().dpc_gemm_last_kernel())


def set_gemm_variant(key: int, value: int) -> None:
    """Lab switch for same-process A/Bs of one kernel's variants (``gemm7.hip:g_variant``):
    key 0 = v9 EPI 1 store layout (1: the round-4 half-line form); -1 = default."""
    lib().dpc_gemm_set_variant(int(key), int(value))


def set_gemm_splits(n: int) -> None:
    """Force the split-K count of plain f32 products (0 = automatic; sweeps)."""
    lib().dpc_gemm_set_splits(int(n))


def set_gemm_xcd_split(on: bool) -> None:
    """Split-K with one k-range per XCD instead of the default remap (experiments)."""
    lib().dpc_gemm_set_xcd_split(int(bool(on)))


def set_cu_reserve(r: int) -> None:
    """CUs the persistent GEMMs (v7 / v8) leave free for a kernel resident beside them -- an
    RCCL collective in flight on the comm stream (``parallel/transport.py`` drives it)."""
    lib().dpc_set_cu_reserve(int(r))


def get_cu_reserve() -> int:
    return int(lib().dpc_get_cu_reserve())


def occupy(nwg: int, ns: int, sink: torch.Tensor, stream=None) -> None:
    """Launch ``nwg`` workgroups spinning ``ns`` nanoseconds (measurements only)."""
    s = (stream or torch.cuda.current_stream()).cuda_stream
    rc = lib().dpc_occupy(int(nwg), int(ns), sink.data_ptr(), s)
    if rc != 0:
        raise RuntimeError(f"dpc_occupy failed: hipError {rc}")


def is_loaded() -> bool:
    return _lib is not None


def stream_ptr(device: torch.device | None = None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


# SURVEY.md §5.2 serialize switch (``--serialize_kernels`` / DPC_SERIALIZE=1): the HIP runtime
# serialises every launch and copy (AMD_SERIALIZE_KERNEL / AMD_SERIALIZE_COPY / HIP_LAUNCH_BLOCKING,
# which must be in the environment before the runtime starts -- ``enable_serialize``), and
# every native launch is followed by a stream synchronize, so a faulting kernel is reported
# by name at its own launch instead of at a later synchronisation point.
SERIALIZE = os.environ.get("DPC_SERIALIZE", "0") == "1"


def enable_serialize() -> None:
    global SERIALIZE
    SERIALIZE = True
    os.environ["DPC_SERIALIZE"] = "1"
    for k, v in (("AMD_SERIALIZE_KERNEL", "3"), ("AMD_SERIALIZE_COPY", "3"), ("HIP_LAUNCH_BLOCKING", "1")):
        os.environ.setdefault(k, v)


def call(name: str, args: ctypes.Structure, device: torch.device | None = None) -> None:
    rc = getattr(lib(), name)(ctypes.byref(args), stream_ptr(device))
    if rc != 0:
        raise RuntimeError(f"{name} launch failed: hipError {rc}")
    if SERIALIZE and not torch.cuda.is_current_stream_capturing():
        try:
            torch.cuda.current_stream(device).synchronize()
        except RuntimeError as exc:  # the fault of THIS launch
            raise RuntimeError(f"{name} failed on the device: {exc}") from exc


def ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()

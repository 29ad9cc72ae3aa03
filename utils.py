"""Reference-compatible ``utils`` module (``prepare_batch``, ``generate``)."""
from distributed_pytorch_cookbook_amd.utils.batch import generate, prepare_batch  # noqa: F401

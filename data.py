"""Reference-compatible ``data`` module (``get_dataset``, ``get_tokenizer``, ``transform_dataset``)."""
from distributed_pytorch_cookbook_amd.utils.data import (  # noqa: F401
    SyntheticTokenDataset, get_dataset, get_tokenizer, transform_dataset)
from distributed_pytorch_cookbook_amd.utils.tokenizer import ByteTokenizer  # noqa: F401

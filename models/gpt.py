"""Reference-compatible import path ``models.gpt`` (definition lives in the package)."""
from distributed_pytorch_cookbook_amd.models.gpt import (  # noqa: F401
    PRESETS, DecoderLayer, Embeddings, FeedForward, SelfAttention, TransformerDecoder,
    TransformerDecoderLM)

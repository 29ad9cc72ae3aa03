"""Reference-compatible import path: ``from models import TransformerDecoderLM``."""
from distributed_pytorch_cookbook_amd.models.gpt import TransformerDecoderLM  # noqa: F401

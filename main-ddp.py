#!/usr/bin/env python
"""MI355X cookbook recipe: ddp.

Same flags as the reference's main-ddp.py (plus the new ones in
distributed_pytorch_cookbook_amd/config.py); see README.md for launch commands.
"""
from distributed_pytorch_cookbook_amd.recipes import run

if __name__ == "__main__":
    run("ddp")

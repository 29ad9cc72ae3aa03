#!/usr/bin/env python
"""MI355X cookbook recipe: pipe.

Same flags as the reference's main-pipe.py (plus the new ones in
distributed_pytorch_cookbook_amd/config.py); see README.md for launch commands.
"""
from distributed_pytorch_cookbook_amd.recipes import run

if __name__ == "__main__":
    run("pipe")

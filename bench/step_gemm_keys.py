"""The GEMM table signatures (ops/gemm.py:_sig) one bench.py step looks up, with their call
counts and the table's choice -- which entries a retune must cover to move the step.

    python bench/step_gemm_keys.py [bench.py args]
"""
import atexit
import collections
import os
import runpy
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_cookbook_amd.ops import gemm as G  # noqa: E402

seen = collections.Counter()


class _Spy(dict):
    def get(self, k, d=None):
        seen[k] += 1
        return super().get(k, d)


G._table = _Spy(G._table)


@atexit.register
def _report():
    for k, n in sorted(seen.items()):
        print(f"{n:5d}  {k}  table={dict.get(G._table, k)}", file=sys.stderr)


root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.argv = [os.path.join(root, "bench.py")] + (sys.argv[1:] or ["--steps", "1", "--warmup", "1"])
runpy.run_path(sys.argv[0], run_name="__main__")

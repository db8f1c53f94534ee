"""Round-6 timing diagnostic for the patch embedding inside bench.py's two-stream step (VERDICT r5
item 5, "measure, don't argue").

    python tools/embed_diag.py [bench.py arguments]

runs bench.py unchanged except that every `nqk_embed_q` call is skipped, so the captured hipGraph
holds the forward without the patch embedding.  Timing only: the logits are computed from an
uninitialised residual stream, so the line reports "verified": false.  The step-time difference
against a normal bench.py run on the same box is the embedding's cost in the step; the difference
against the whole-batch launch's standalone time is what the two streams' overlap already hides.
"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "numpy-quant_amd"))
sys.path.insert(0, ROOT)

from numpy_quant import _lib  # noqa: E402

_call = _lib.call


def _call_without_embedding(name, *args):
    if name == "nqk_embed_q":
        return None
    return _call(name, *args)


_lib.call = _call_without_embedding
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[1:]
runpy.run_path(sys.argv[0], run_name="__main__")

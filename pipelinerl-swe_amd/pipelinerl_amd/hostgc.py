"""Host garbage collection around the trainer's hot loop.

After the imports (torch, transformers, the model) the interpreter holds ~220 000 tracked
objects, and CPython's generation-2 collection walks all of them: ~90 ms with the host thread
stopped (measured in this container), long enough to drain the GPU's launch queue, which then
sits idle until the host enqueues again.  The C3 7B kernel trace shows such 80-180 ms host
stalls mid-step (profiles/r02_host_gaps.txt), and a collection counted inside the timed steps
cost 184.5 ms of one run (tools/c3_step.py's host_gc).  Freezing the set-up heap once (``gc.freeze``:
those objects move to a permanent generation no collection scans) leaves collections only the
step's own short-lived objects to walk.  Nothing the step allocates is affected: reference cycles
it creates are still collected.  C3 7B step, 4 runs each interleaved: 1545.7 -> 1534.4 ms mean
(profiles/r02_gc_freeze_ab.jsonl; the first two pairs counted collections over the whole process).
PRL_GC_FREEZE=0 turns it off (A/B)."""

from __future__ import annotations

import gc
import os


def freeze_setup_heap() -> bool:
    """Collect once, then move every surviving object to the permanent generation.  Call after
    the model, optimizer and data path exist, before the first step.  Returns whether it froze."""
    if os.environ.get("PRL_GC_FREEZE", "1") == "0":
        return False
    gc.collect()
    gc.freeze()
    return True

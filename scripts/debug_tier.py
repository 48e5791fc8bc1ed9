"""Diagnostics of the tiered flow (per pass: staged / live / exported / host)."""
import sys

import torch

sys.path.insert(0, ".")
from tests.test_gpu_tiered import PASSES, _box, _pass_batches  # noqa: E402
from paddlebox_amd.ops import reference as ref  # noqa: E402

DEV = torch.device("cuda:0")
tb = _box("tiered", 2400)
passes = [_pass_batches(p) for p in range(PASSES)]
keys_of = [torch.cat([b.keys for b in bs]) for bs in passes]
uniq = [torch.unique(ref.mix64(k[k != -1])) for k in keys_of]
tb.feed_pass(keys_of[0])
for p in range(PASSES):
    tb.begin_pass()
    live = tb.engine.table
    print(p, "pass keys", uniq[p].numel(), "live size", live.size(),
          "missing in live", int((live.probe(uniq[p].to(DEV)) < 0).sum()), flush=True)
    if p + 1 < PASSES:
        tb.feed_pass(keys_of[p + 1])
    tb.end_pass()
    tb.tier.wait_writeback()
    hs = tb.host.size()
    miss = int((tb.host.probe(uniq[p]) < 0).sum())
    print(p, "host size", hs, "pass keys missing in host", miss, flush=True)

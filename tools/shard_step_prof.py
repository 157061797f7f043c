"""Per-stage host timing of ShardedMatcher.match at world 1 (diagnosis for DESIGN §6): each
stage bracketed by torch.cuda.synchronize(); config B generator, 10M filters, 1M topics."""
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from emqx_amd import workloads as W  # noqa: E402
from emqx_amd import dist as D  # noqa: E402

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29561")
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
wl = W.config_b(n_filters=10_000_000, n_topics=1_000_000, seed=2)
sm = D.ShardedMatcher(wl.filters, device=dev)
tb = torch.from_numpy(wl.topics[0]).to(dev)
to = torch.from_numpy(wl.topics[1].view(np.int64)).to(dev)
sm.match((tb, to))
T = {}


def mark(name, t0):
    torch.cuda.synchronize()
    t = time.perf_counter()
    T[name] = T.get(name, 0.0) + (t - t0) * 1e3
    return t


for _ in range(5):
    t = time.perf_counter()
    owner = D.topic_owner(tb, to, 1)
    t = mark("owner", t)
    perm, lens_p, bytes_p, n_to, bytes_to = D.partition(tb, to, owner, 1)
    t = mark("partition", t)
    n = to.numel() - 1
    offs = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    offs[1:] = torch.cumsum(lens_p, 0)
    t = mark("offsets", t)
    counts, ids = sm.match_fn(bytes_p, offs)
    t = mark("engine match", t)
    off, out = D.merge_csr(counts.to(torch.int64), ids, perm)
    t = mark("merge", t)
    tt = time.perf_counter()
    sm.match((tb, to))
    mark("whole match()", tt)
print({k: round(v / 5, 3) for k, v in T.items()})
dist.destroy_process_group()

"""Walk-order check on one GPU (diagnosis): per (level bits, sort bits, deal) setting, the
ordered device call against the unordered one on a config-D sample — totals, per-topic
count differences, deferred topics, max stack."""
import sys, time, numpy as np
sys.path.insert(0, '.')
import torch
from emqx_amd.engine import Engine
from emqx_amd import workloads as W
d = W.config_d(n_filters=30_000, n_topics=20_000)
dev = torch.device("cuda", 0)
tb = torch.from_numpy(d.topics[0]).to(dev); to = torch.from_numpy(d.topics[1].view(np.int64)).to(dev)
n = len(d.topics[1]) - 1; cap = 1 << 24
e = Engine(); e.insert_packed(*d.filters); e.commit()
print("max_depth", e.stats()["max_depth"])
d_off = torch.zeros(n + 1, dtype=torch.int64, device=dev); d_ids = torch.zeros(cap, dtype=torch.int32, device=dev)
e.set_tuning("order", 0)
t0 = e.match_device(tb.data_ptr(), to.data_ptr(), n, d_off.data_ptr(), d_ids.data_ptr(), cap)
b = d_off.cpu().numpy().copy(); bc = np.diff(b)
for lb, sb, deal in ((8, 64, 1), (4, 64, 1), (4, 64, 0), (4, 16, 1), (2, 64, 1)):
    e.set_tuning("order", 1); e.set_tuning("order_level_bits", lb); e.set_tuning("order_sort_bits", sb); e.set_tuning("order_deal", deal)
    for k in range(2):
        tot = e.match_device(tb.data_ptr(), to.data_ptr(), n, d_off.data_ptr(), d_ids.data_ptr(), cap)
        o = d_off.cpu().numpy(); c = np.diff(o); st = e.stats()
        bad = np.nonzero(c != bc)[0]
        print(lb, sb, deal, k, "tot", tot, "base", t0, "off[n]", o[-1], "count diffs", bad.size, bad[:5], "deferred", st["last_deferred"], "maxstack", st["last_max_stack"], flush=True)

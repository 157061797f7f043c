"""Single-process replay of ShardedMatcher.match_all at world 2 (no collectives): both sources'
batches (config B, rank 1 with topic_seed 1001 as in bench.py --sharded), device partition by
owner, the parts each owner would receive, host-side checks of every part before any engine
call, then each shard engine's counts against the full-table engine on the same topics."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from emqx_amd import dist as D  # noqa: E402
from emqx_amd import workloads as W  # noqa: E402
from emqx_amd.engine import Engine  # noqa: E402

G = 2
NF = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
NT = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
dev = torch.device("cuda:0")
t0 = time.time()
wls = [W.config_b(n_filters=NF, n_topics=NT, seed=2, topic_seed=None if r == 0 else 1000 + r) for r in range(G)]
print(f"workloads {time.time() - t0:.1f}s", flush=True)
filters = wls[0].filters
for r in range(1, G):
    assert np.array_equal(wls[r].filters[1], filters[1]), "tables differ between ranks"


def check_batch(name, tb, to):
    to_h = to.cpu().numpy()
    lens = np.diff(to_h)
    print(f"{name}: n={len(lens)} bytes={tb.numel()} to[0]={to_h[0]} to[-1]={to_h[-1]} "
          f"minlen={lens.min()} maxlen={lens.max()} dtype={to.dtype}", flush=True)
    assert (lens >= 0).all() and to_h[-1] <= tb.numel() and lens.max() < 65536


parts = [[None] * G for _ in range(G)]  # parts[src][owner] = (lens, bytes, batch index)
for src in range(G):
    tb = torch.from_numpy(wls[src].topics[0]).to(dev)
    to = torch.from_numpy(wls[src].topics[1].view(np.int64)).to(dev)
    check_batch(f"src{src}", tb, to)
    owner = D.topic_owner(tb, to, G)
    perm, lens_p, bytes_p, n_to, bytes_to = D.partition(tb, to, owner, G)
    torch.cuda.synchronize()
    p = perm.cpu().numpy()
    own = owner.cpu().numpy()
    assert np.array_equal(np.sort(p), np.arange(len(p))), "perm is not a permutation"
    assert (np.diff(own[p]) >= 0).all(), "perm does not sort by owner"
    nt, bt, lp = n_to.cpu().numpy(), bytes_to.cpu().numpy(), lens_p.cpu().numpy()
    print(f"src{src}: n_to={nt.tolist()} bytes_to={bt.tolist()}", flush=True)
    assert nt.tolist() == np.bincount(own, minlength=G).tolist()
    nb0 = 0
    ni0 = 0
    for o in range(G):
        seg = lp[ni0:ni0 + nt[o]]
        assert int(seg.sum()) == int(bt[o]), (src, o, int(seg.sum()), int(bt[o]))
        parts[src][o] = (lens_p[ni0:ni0 + nt[o]], bytes_p[nb0:nb0 + bt[o]], p[ni0:ni0 + nt[o]])
        ni0 += int(nt[o])
        nb0 += int(bt[o])
    # byte content of a sample
    to_h, tb_h, bp = wls[src].topics[1].view(np.int64), wls[src].topics[0], bytes_p.cpu().numpy()
    oo = np.concatenate([[0], np.cumsum(lp)])
    for k in np.random.default_rng(0).integers(0, len(p), 2000):
        i = p[k]
        assert bytes(bp[oo[k]:oo[k + 1]]) == bytes(tb_h[to_h[i]:to_h[i + 1]]), (src, k)
print("partition checks ok", flush=True)

full = Engine(0)
full.insert_packed(*filters)
full.commit()


def run(eng, tb, to):
    n = to.numel() - 1
    off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    cap = 1 << 24
    while True:
        ids = torch.empty(cap, dtype=torch.int32, device=dev)
        try:
            m = eng.match_device(tb.data_ptr(), to.data_ptr(), n, off.data_ptr(), ids.data_ptr(), cap)
            break
        except Exception as e:
            if getattr(e, "needed", None) is None:
                raise
            cap = e.needed + 1
    torch.cuda.synchronize()
    return (off[1:] - off[:-1]).cpu().numpy(), ids[:m].cpu().numpy()


for o in range(G):
    lf, gids = D.shard_filters(filters, o, G)
    eng = Engine(0)
    eng.insert_packed_ext(*lf, gids)
    eng.commit()
    my_lens = torch.cat([parts[s][o][0] for s in range(G)])
    my_bytes = torch.cat([parts[s][o][1] for s in range(G)])
    my_offs = torch.zeros(my_lens.numel() + 1, dtype=torch.int64, device=dev)
    my_offs[1:] = torch.cumsum(my_lens, 0)
    last = int(my_offs[-1].item())
    print(f"owner{o}: shard {len(gids)} filters, {my_lens.numel()} topics, {my_bytes.numel()} bytes, "
          f"offs[-1]={last} maxlen={int(my_lens.max().item())}", flush=True)
    assert last == my_bytes.numel() and int(my_lens.max().item()) < 65536
    mb = torch.empty(max(my_bytes.numel(), 1), dtype=torch.uint8, device=dev)
    mb[:my_bytes.numel()] = my_bytes
    c_sh, _ = run(eng, mb, my_offs)
    c_full, _ = run(full, mb, my_offs)
    bad = int((c_sh != c_full).sum())
    print(f"owner{o}: shard total {int(c_sh.sum())} full total {int(c_full.sum())} mismatching topics {bad}",
          flush=True)
    eng.close()
print("done", flush=True)

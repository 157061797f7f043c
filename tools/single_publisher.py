"""One publisher, one emqx_publish_batch call of 1M messages on config E's tables (VERDICT r3 #3:
a bridge's publish_batch/4 with every message from one publisher, round_robin / sticky).

Times the call (host buffers in and out, match + fan-out on the device) and checks the
per-publisher state semantics on the result: for round_robin every $share group's picks over the
batch are consecutive rotation steps in message order (emqx_shared_sub.erl:279-285), for sticky
one member per group.  Prints one JSON line.

Usage (GPU box): python tools/single_publisher.py [--strategy round_robin] [--n 1000000]
"""

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--strategy", default="round_robin", choices=["round_robin", "sticky"])
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch
    assert torch.cuda.is_available()
    from emqx_amd import workloads as W
    from emqx_amd.engine import Engine
    from emqx_amd.fanout import FANOUT_SHARED_BIT, SubTable, publish_packed
    fw = W.config_e(n_topics=args.n)
    eng = Engine(0)
    eng.insert_packed(*fw.wl.filters)
    eng.commit()
    st = SubTable(0)
    st.add(fw.sub_filter, fw.sub_id, fw.sub_group)
    st.commit()
    buf, offs = fw.wl.topics
    offs = offs.astype(np.uint64)
    keys = np.full(args.n, 7, np.uint32)  # one publisher
    cap = 64 * args.n
    times = []
    res = None
    for _ in range(args.reps):
        t0 = time.perf_counter()
        res = publish_packed(eng, st, args.strategy, buf, offs, keys, cap_hint=cap)
        times.append(time.perf_counter() - t0)
    off, subs, fils = res
    # per-group check: the picks of each (filter, group) in message order
    shared = (fils & FANOUT_SHARED_BIT) != 0
    topic_of = np.repeat(np.arange(args.n), np.diff(off.astype(np.int64)))
    f_sh = (fils[shared] & ~np.uint32(FANOUT_SHARED_BIT | 0x40000000)).astype(np.int64)
    s_sh = subs[shared].astype(np.int64)
    t_sh = topic_of[shared]
    # member lists per (filter, group) in subscription order; a filter's groups in the order of
    # their first subscription (the device's group list order, fanout.cpp fslots)
    g_idx = np.flatnonzero(fw.sub_group != W.NO_GROUP)
    members, groups_of = {}, {}
    for i in g_idx:
        f, g = int(fw.sub_filter[i]), int(fw.sub_group[i])
        if (f, g) not in members:
            groups_of.setdefault(f, []).append(g)
        members.setdefault((f, g), []).append(int(fw.sub_id[i]))
    pos_of = {k: {s: j for j, s in enumerate(m)} for k, m in members.items()}
    # the k-th $share delivery of filter f in a topic's row is f's k-th group
    bad = checked = 0
    seqs = {}
    seen = {}
    for f, s, t in zip(f_sh.tolist(), s_sh.tolist(), t_sh.tolist()):
        k = seen.get((t, f), 0)
        seen[(t, f)] = k + 1
        g = groups_of[f][k]
        seqs.setdefault((f, g), []).append((t, pos_of[(f, g)].get(s, -1), len(members[(f, g)])))
    for key, seq in seqs.items():
        seq.sort()
        idx = [p for _, p, _ in seq]
        n = seq[0][2]
        checked += len(idx)
        if args.strategy == "round_robin" and n > 1:
            bad += sum(1 for a, b in zip(idx, idx[1:]) if (a + 1) % n != b)
        elif args.strategy == "sticky":
            bad += sum(1 for a, b in zip(idx, idx[1:]) if a != b)
    out = {"metric": "one-publisher emqx_publish_batch call (config E tables, host buffers)",
           "strategy": args.strategy, "messages": args.n, "deliveries": int(off[-1]),
           "shared_picks": int(shared.sum()), "groups_picked": len(seqs),
           "call_s": [round(x, 4) for x in times], "messages_per_s": round(args.n / min(times), 1),
           "state_check": {"picks_checked": checked, "violations": bad,
                           "rule": "round_robin: consecutive picks of a group are consecutive rotation steps; "
                                   "sticky: one member per group"}}
    print(json.dumps(out), flush=True)
    if bad:
        raise SystemExit("state violations")


if __name__ == "__main__":
    main()

"""Config C at its real size (BASELINE configs[2]: 100M filters, generator B with vocab x4, seed 3),
ID-for-ID on the first 12K topics of the C1 bench batch, in the default GPU suite:

1. the whole table on one GPU (the replicated layout: one engine, ids = row numbers);
2. the same table through the filter-sharded device step (emqx_shard_step_*) at world 1 over
   RCCL: route, fold, pack, the exchanges, answer and merge on the 100M table.  The table is
   generated and built ONCE: at world 1 every request is an engine-slot AB request (dist.py
   fold_requests) and the AB engine holds every filter, so leg 1's engine is adopted as it.

Expected ids: tests/golden/c100m_slice.npz — the oracle (oracle/trie_oracle.cpp, the emqx_trie DFS
+ match_routes/1 union, apps/emqx/src/emqx_trie.erl:315-334) restated on the filters that can
match the slice (oracle/pruned.py), made by tests/golden/make_c100m.py; the file's fingerprint
of the generated table and batch is checked first, so a generator that drifted fails loudly
instead of comparing against another table's answers.

A progress line goes to gpurun_out/c100m_progress.log every 20 s (generation and the build take
minutes).  EMQX_GPU_C100M=0 skips the module (iteration on other tests only).
"""

import os
import threading
import time

import numpy as np
import pytest

from oracle import cpp as C

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(os.environ.get("EMQX_GPU_C100M") == "0", reason="EMQX_GPU_C100M=0")]

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden", "c100m_slice.npz")


class _Beat:
    """Heartbeat lines while the long steps run (a silent test looks hung)."""

    def __init__(self, what):
        self.what, self.t0, self.stop = what, time.time(), threading.Event()
        os.makedirs("gpurun_out", exist_ok=True)
        self.th = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        while not self.stop.wait(20):
            self._line(f"{self.what}: {time.time() - self.t0:.0f} s")

    @staticmethod
    def _line(s):
        with open("gpurun_out/c100m_progress.log", "a") as f:
            f.write(s + "\n")

    def __enter__(self):
        self.th.start()
        return self

    def __exit__(self, *a):
        self.stop.set()
        self._line(f"{self.what}: done in {time.time() - self.t0:.0f} s")


def _fingerprint(packed):
    import xxhash
    buf, offs = packed
    return [xxhash.xxh3_64_intdigest(np.ascontiguousarray(buf).data),
            xxhash.xxh3_64_intdigest(np.ascontiguousarray(np.asarray(offs, np.uint64)).data)]


@pytest.fixture(scope="module")
def c100m():
    """(workload, golden, slice) generated once for the module; the engine of leg 1 is handed to
    leg 2 through the dict."""
    from emqx_amd import workloads as W
    g = dict(np.load(GOLDEN))
    with _Beat("generate"):
        wl = W.config_b(n_filters=int(g["n_filters"]), n_topics=int(g["n_topics"]), seed=int(g["seed"]),
                        vocab_scale=int(g["vocab_scale"]))
    k = int(g["slice"])
    sl = W.take(wl.topics, np.arange(k))
    assert _fingerprint(wl.filters) == [int(x) for x in g["table_fp"]], "generated table differs from the golden's"
    assert _fingerprint(sl) == [int(x) for x in g["batch_fp"]], "generated batch differs from the golden's"
    st = {"wl": wl, "golden": g, "slice": sl, "k": k}
    yield st
    e = st.pop("engine", None)
    if e is not None:
        e.close()


def _dev_slice(st):
    import torch
    dev = torch.device("cuda:0")
    sl = st["slice"]
    return dev, torch.from_numpy(sl[0]).to(dev), torch.from_numpy(sl[1].astype(np.int64)).to(dev)


def test_config_c_100m_replicated_id_for_id(c100m):
    import torch
    from emqx_amd.engine import Engine
    st = c100m
    g, k = st["golden"], st["k"]
    dev, tb, to = _dev_slice(st)
    with _Beat("build replicated"):
        e = Engine(0)
        e.insert_packed(*st["wl"].filters)
        e.commit()
    st["engine"] = e
    cap = int(g["off"][-1]) + 1024
    d_off = torch.empty(k + 1, dtype=torch.int64, device=dev)
    d_ids = torch.empty(cap, dtype=torch.int32, device=dev)
    m = e.match_device(tb.data_ptr(), to.data_ptr(), k, d_off.data_ptr(), d_ids.data_ptr(), cap, mode=0,
                       stream=torch.cuda.current_stream(dev).cuda_stream)
    assert m == int(g["off"][-1])
    bad = C.csr_mismatches(d_off.cpu().numpy().astype(np.uint64), d_ids[:m].cpu().numpy().view(np.uint32),
                           g["off"], g["ids"])
    assert bad.size == 0, bad[:10]
    _Beat._line(f"replicated ok: {int(g['n_filters'])} filters, {k} topics, {m} ids ID-for-ID")


def test_config_c_100m_sharded_step_id_for_id(c100m):
    import torch
    import torch.distributed as dist
    from emqx_amd import dist as D
    st = c100m
    e = st.pop("engine", None)
    if e is None:
        pytest.skip("the replicated leg did not build the table")
    g, k, wl = st["golden"], st["k"], st["wl"]
    dev, tb, to = _dev_slice(st)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = "29571"
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        plan = D.shard_plan(wl.filters, 1)
        ids_a, ids_b, ids_ab = D.shard_local_ids(wl.filters, 0, 1, plan)
        assert len(ids_a) + len(ids_b) == len(ids_ab) == wl.n_filters and len(ids_b) > 0
        sm = D.ShardedMatcher(wl.filters, device=dev, engines=[None, None, e])
        off, ids = sm.match_all((tb, to))
        assert sm.last_local_topics == k  # one (AB) request per topic
        assert int(off[-1]) == int(g["off"][-1])
        bad = C.csr_mismatches(off.cpu().numpy().astype(np.uint64), ids.cpu().numpy().view(np.uint32),
                               g["off"], g["ids"])
        assert bad.size == 0, bad[:10]
        _Beat._line(f"sharded step ok: A {len(ids_a)} + B {len(ids_b)} filters on the AB engine, "
                    f"{k} topics, {int(off[-1])} ids ID-for-ID")
        sm._step.close()
    finally:
        dist.destroy_process_group()
        e.close()

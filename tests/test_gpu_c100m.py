"""Config C at its real size (BASELINE configs[2]: 100M filters, generator B with vocab x4, seed
3), ID-for-ID on a topic slice: the whole table on one GPU (replicated layout) and the same table
through the filter-sharded device step at world 1, against the oracle (oracle/trie_oracle.cpp,
the emqx_trie DFS + match_routes/1 union, apps/emqx/src/emqx_trie.erl:315-334) restated on the
filters that can match the slice (oracle/pruned.py — exact for the slice).

Generating and building the 100M table takes minutes, so this test runs only with
EMQX_GPU_C100M=1 (tools/r4_c100m.sh; its log is under profiles/): the default GPU suite stays
within a couple of minutes.  A progress line goes to gpurun_out/c100m_progress.log every 20 s.
"""

import os
import threading
import time

import numpy as np
import pytest

from oracle import cpp as C

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(os.environ.get("EMQX_GPU_C100M") != "1",
                                 reason="100M-filter table: set EMQX_GPU_C100M=1 (minutes of generation and build)")]

N_FILTERS = int(os.environ.get("EMQX_C100M_FILTERS", "100000000"))
SLICE = 20_000


class _Beat:
    """Heartbeat lines while the long steps run (a silent test looks hung)."""

    def __init__(self, what):
        self.what, self.t0, self.stop = what, time.time(), threading.Event()
        os.makedirs("gpurun_out", exist_ok=True)
        self.th = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        while not self.stop.wait(20):
            with open("gpurun_out/c100m_progress.log", "a") as f:
                f.write(f"{self.what}: {time.time() - self.t0:.0f} s\n")

    def __enter__(self):
        self.th.start()
        return self

    def __exit__(self, *a):
        self.stop.set()
        with open("gpurun_out/c100m_progress.log", "a") as f:
            f.write(f"{self.what}: done in {time.time() - self.t0:.0f} s\n")


def test_config_c_100m_slice_id_for_id():
    import torch
    import torch.distributed as dist
    from emqx_amd import workloads as W
    from emqx_amd.dist import ShardedMatcher
    from emqx_amd.engine import Engine
    from oracle import pruned
    with _Beat("generate"):
        wl = W.config_b(n_filters=N_FILTERS, n_topics=1_000_000, seed=3, vocab_scale=4)  # the C1 bench batch
    k = SLICE
    sl = W.take(wl.topics, np.arange(k))
    with _Beat("oracle"):
        off_o, ids_o, cand = pruned.slice_csr(wl.filters, wl.fcodes, sl, wl.tcodes[:k], threads=16)
    assert int(off_o[-1]) > 0
    dev = torch.device("cuda:0")
    tb = torch.from_numpy(sl[0]).to(dev)
    to = torch.from_numpy(sl[1].astype(np.int64)).to(dev)
    # 1. the whole table on the GPU
    with _Beat("build replicated"):
        e = Engine(0)
        e.insert_packed(*wl.filters)
        e.commit()
    cap = int(off_o[-1]) + 1024
    d_off = torch.empty(k + 1, dtype=torch.int64, device=dev)
    d_ids = torch.empty(cap, dtype=torch.int32, device=dev)
    m = e.match_device(tb.data_ptr(), to.data_ptr(), k, d_off.data_ptr(), d_ids.data_ptr(), cap, mode=0,
                       stream=torch.cuda.current_stream(dev).cuda_stream)
    bad = C.csr_mismatches(d_off.cpu().numpy().astype(np.uint64), d_ids[:m].cpu().numpy().view(np.uint32), off_o, ids_o)
    assert bad.size == 0, bad[:10]
    e.close()
    del e
    # 2. the same table through the sharded device step (two engines, world 1 over RCCL)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = "29571"
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        with _Beat("build sharded"):
            sm = ShardedMatcher(wl.filters, device=dev)
        off, ids = sm.match_all((tb, to))
        bad = C.csr_mismatches(off.cpu().numpy().astype(np.uint64), ids.cpu().numpy().view(np.uint32), off_o, ids_o)
        assert bad.size == 0, bad[:10]
    finally:
        dist.destroy_process_group()
    with open("gpurun_out/c100m_progress.log", "a") as f:
        f.write(f"ok: {N_FILTERS} filters, {k} topics, {int(off_o[-1])} ids ID-for-ID (replicated and sharded), "
                f"oracle table {len(cand)} filters\n")

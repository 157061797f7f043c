"""Benchmark: published topics matched/s (and match evals/s) at 10M subscriptions.

Workload (BASELINE.json configs[1], SURVEY §8 d config B): 10M distinct mixed exact/'+'/'#'
filters (depth 4-8, Zipf vocab), batches of 1M published topics (depth 4-8, 50% instantiated
from filters).  A step = one batched match (emqx_match_batch_device) of one batch already
resident in HBM -> CSR of matching filter ids in HBM (kernels, scan, scatter, the per-call
host readback included).

Multi-GPU (``torchrun --nproc-per-node N``): the table is REPLICATED on every GPU (10M
filters = a few GB, SURVEY §8 e) and each rank matches its own batch — weak scaling, no
collective on the data path; one barrier + a MAX of the per-rank time brackets the timed
region.

Prints ONE JSON line (rank 0).  Extra keys: evals_per_s, roofline (HBM, algorithmic bytes of
the fused match kernel per launch ÷ its HIP-event duration), cpu_baseline (the oracle's C++
restatement of emqx_trie's compact DFS, timed on host cores on a bounded topic sample).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

D_BATCH = 1_000_000  # config D: ~5000 node visits and ~1100 matches per topic
HBM_PEAK_GBS = 8000.0  # MI355X spec, /opt/skills/guides/MI355X_MICROARCH.md


def log(*a):
    print(*a, file=sys.stderr, flush=True)


class progress:
    """Logs `label: N s` every `every` seconds while a long host phase runs (workload
    generation, table build at 100M filters), so a live run is never silent for minutes."""

    def __init__(self, label, every=30.0):
        import threading
        self.label, self.every, self.done = label, every, threading.Event()
        self.t = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        t0 = time.time()
        while not self.done.wait(self.every):
            log(f"{self.label}: {time.time() - t0:.0f} s")

    def __enter__(self):
        self.t.start()
        return self

    def __exit__(self, *exc):
        self.done.set()
        self.t.join()


WORKLOAD_NAMES = {
    "A": "A: 100k filters site{i%1000}/+/dev{i/1000}/#, 1M-topic stream (configs[0] table on 1xMI355X)",
    "B": "B: 10M mixed exact/'+'/'#' subscriptions, 1xMI355X, batched topics of depth 4-8",
    "D": "D: adversarial '#'/'+'-rich table, 1M filters, depth-16 topics, 1xMI355X",
    "C1": "C on one GPU: config-C table (B generator, vocab x4, seed 3) held whole on 1xMI355X, 1M-topic batches",
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (default: 1000 for the batch-match workloads A / B / C1, so the timed "
                         "region lasts ~0.1-1 s rather than ~10 ms; 20 for the others)")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n-filters", type=int, default=10_000_000)
    ap.add_argument("--batch", type=int, default=None,
                    help="topics per batch (default 1M; --workload D: D_BATCH)")
    ap.add_argument("--mode", type=int, default=0, help="0 routes, 1 trie, 2 trie_wildcard")
    ap.add_argument("--cpu-sample", type=int, default=None,
                    help="topics in the CPU baseline sample, also the topics whose GPU match sets are compared "
                         "ID-for-ID with the oracle (default: the whole 1M batch; --workload D: 40k, ~15 s)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU-baseline threads (default 0: every host core this process may use)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-api", action="store_true", help="skip the host-buffer (PCIe-inclusive) rates")
    ap.add_argument("--cache", type=str, default=None,
                    help="npz path: reuse the generated workload across runs (profiling passes)")
    ap.add_argument("--ab", type=str, default=None,
                    help="comma list of fast-kernel variants: interleaved A/B rounds in this process, "
                         "prints per-variant kernel/call times instead of the bench line")
    ap.add_argument("--ab-rounds", type=int, default=5)
    ap.add_argument("--diag", action="store_true", help="one extra call with kernel counters, added as 'diag'")
    ap.add_argument("--workload", type=str, default="B", choices=["A", "B", "D", "E", "U", "R", "L", "P", "S", "T"],
                    help="B = the headline (BASELINE configs[1]); A = configs[0]'s 100k-filter table, "
                         "D = the adversarial depth-16 table (configs[3], 1M-topic batches), "
                         "E = publish fan-out (configs[4]): match + fan-out per step, "
                         "U = route updates (SURVEY §8 f2): subscribe/unsubscribe churn + incremental "
                         "commits on config B's table, R = retained-message lookup (SURVEY §8 f4): a batch "
                         "of subscription filters against 1M stored retained topics, L = the drop-in "
                         "per-PUBLISH path: concurrent single-topic callers through the batcher on config "
                         "B's table, P = the drop-in emqx_broker:publish/1 path: concurrent single-message "
                         "callers through the publish batcher (match + fan-out) on config E's 10M "
                         "subscriptions, S = subscription churn: subscribe/unsubscribe ops committed to "
                         "config E's 10M-subscription table, T = the per-call subscribe / route boundary: "
                         "closed-loop callers through the commit coalescer on config E's tables, single-op "
                         "latency, throughput at --callers, and P's throughput during a subscribe storm")
    ap.add_argument("--callers", type=str, default="64,512,4096",
                    help="--workload L: concurrent single-topic callers per run")
    ap.add_argument("--max-batch", type=int, default=4096, help="--workload L: batcher max_batch")
    ap.add_argument("--small-clock", action="store_true",
                    help="--workload L/P: per-phase clocks of the one-launch small-batch kernel in each run")
    ap.add_argument("--max-wait-us", type=str, default="200", help="--workload L: batcher max_wait_us (comma list)")
    ap.add_argument("--retained", type=int, default=1_000_000, help="--workload R: stored retained topics")
    ap.add_argument("--retain-tile", type=int, default=None, help="--workload R: filters per walk tile")
    ap.add_argument("--retain-budget", type=int, default=None, help="--workload R: walk step budget (0 = none)")
    ap.add_argument("--churn", type=int, default=10_000, help="--workload U: inserts and deletes per commit")
    ap.add_argument("--with-matches", action="store_true",
                    help="--workload U: a 1M-topic match in flight on a second stream during every commit")
    ap.add_argument("--rounds", type=int, default=50, help="--workload U: commits timed")
    ap.add_argument("--strategy", type=str, default="hash_clientid",
                    help="$share strategy for --workload E / P")
    ap.add_argument("--publishers", type=int, default=0,
                    help="--workload E / P with round_robin / sticky: publishers the messages come from "
                         "(message key = generated key mod N; 0: the generated keys, ~1M distinct)")
    ap.add_argument("--parity-sample", type=int, default=10000,
                    help="--sharded past 10M filters: topics of rank 0's batch checked against the oracle")
    ap.add_argument("--sharded", action="store_true",
                    help="filter-sharded table (filters by a hash of their first two levels, wildcard-keyed "
                         "ones replicated): rank 0's batch is partitioned by owner rank, exchanged with one "
                         "RCCL all-to-all, matched on one shard per topic, and the results return with a "
                         "second all-to-all (strong scaling)")
    ap.add_argument("--vocab-scale", type=int, default=1, help="4 = config C's vocabulary")
    ap.add_argument("--emulate-world", type=str, default="",
                    help="--sharded: G ranks of the G-way plan in this one process on one GPU (dist.py "
                         "EmulatedWorld): every rank's step timed, exchanges projected over xGMI links; a "
                         "comma list runs each G in turn over one generated table (one JSON line each)")
    ap.add_argument("--p-space", type=str, default="auto", choices=["auto", "sharded", "replicated"],
                    help="--sharded: space-P layout of the plan (dist.py shard_plan): '+/x/...' filters sharded "
                         "by x (two requests a topic) or on every rank (one request a topic)")
    ap.add_argument("--xgmi-gbs", type=float, default=153.0,
                    help="--emulate-world: GB/s of one xGMI link, one direction (7 links per MI355X)")
    ap.add_argument("--a2a-us", type=float, default=30.0,
                    help="--emulate-world: fixed cost (us) of one all-to-all call, added per exchange")
    ap.add_argument("--streams", type=int, default=None,
                    help="HIP streams the timed batches alternate over (pipelined calls; default 3, "
                         "see DESIGN.md §5)")
    ap.add_argument("--order", type=str, default="none", choices=["none", "sorted", "xcd"],
                    help="experiment: host-side permutation of the topic batch (sorted = lexicographic; "
                         "xcd = sorted, cut into 8 key-range segments, dealt 256 topics at a time so each "
                         "XCD's blocks see one segment)")
    ap.add_argument("--batches", type=int, default=4,
                    help="distinct topic batches the timed steps rotate over (config B / C generator; "
                         "4 x 44 MB of topic bytes, so steps do not replay one cache-resident batch)")
    ap.add_argument("--walk-order", type=str, default="auto", choices=["auto", "on", "off"],
                    help="engine walk order (emqx_set_tuning 'order'): the batch is walked in prefix-key "
                         "order with XCD-contiguous tile ranges, inside the call (auto: deep tables)")
    ap.add_argument("--walk-level-bits", type=int, default=0, help="walk order: key bits per level (0 = auto)")
    ap.add_argument("--walk-sort-bits", type=int, default=64, help="walk order: top key bits sorted on")
    ap.add_argument("--walk-deal", type=int, default=1, help="walk order: deal tile ranges to XCDs (1) or not (0)")
    ap.add_argument("--traffic-bytes", type=float, default=None,
                    help="HBM bytes per kernel launch from PMC (rocprofv3 FETCH_SIZE/WRITE_SIZE)")
    args = ap.parse_args()
    if args.batch is None:
        args.batch = D_BATCH if args.workload == "D" else 1_000_000
    if args.streams is None:
        # R: two concurrent callers (r4_q27: 1 / 2 / 3 / 4 callers 88.1 / 92.5 / 89.6 / 88.5 M filters/s)
        args.streams = 2 if args.workload == "R" else 3
    if args.cpu_sample is None:
        args.cpu_sample = {"D": 40_000}.get(args.workload, 1_000_000)
    if args.steps is None:
        args.steps = 1000 if args.workload in ("A", "B") and not args.sharded and not args.ab else 20

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # EMQX_BENCH_REHEARSE=1: rehearsal of the N-rank path on a box with fewer GPUs (ranks share
    # devices round robin, gloo instead of RCCL); never used for a reported number
    rehearse = os.environ.get("EMQX_BENCH_REHEARSE") == "1"
    if rehearse:
        local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    from emqx_amd import workloads as W
    from emqx_amd.engine import Engine, EngineError

    t0 = time.time()
    # every rank replicates the table (seed 2); each rank draws its own topic stream (weak scaling)
    if args.sharded and args.emulate_world:
        return emulated_bench(args, dev)
    if args.sharded:
        return sharded_bench(args, rank, world, dev)
    if args.workload == "E":
        return fanout_bench(args, rank, world, dev)
    if args.workload == "U":
        return update_bench(args, rank, world, dev)
    if args.workload == "R":
        return retain_bench(args, rank, world, dev)
    if args.workload == "L":
        return batcher_bench(args, rank, world, dev)
    if args.workload == "P":
        return pub_batcher_bench(args, rank, world, dev)
    if args.workload == "S":
        return subscribe_bench(args, rank, world, dev)
    if args.workload == "T":
        return storm_bench(args, rank, world, dev)
    if args.workload == "A":
        wl = load_or_make(args, rank, lambda: W.config_a(n_topics=args.batch, seed=1 if rank == 0 else 1000 + rank))
    elif args.workload == "D":
        wl = load_or_make(args, rank, lambda: W.config_d(n_topics=args.batch, seed=4))
    else:
        with progress(f"[rank {rank}] generating workload"):
            extra_seeds = tuple(5000 + 100 * rank + j for j in range(1, max(args.batches, 1)))
            wl = load_or_make(args, rank, lambda: W.config_b(n_filters=args.n_filters, n_topics=args.batch,
                                                             seed=3 if args.vocab_scale > 1 else 2,
                                                             vocab_scale=args.vocab_scale,
                                                             topic_seed=None if rank == 0 else 1000 + rank,
                                                             extra_topic_seeds=extra_seeds),
                              batches=max(args.batches, 1))
    log(f"[rank {rank}] workload: {wl.n_filters} filters, {wl.n_topics} topics ({time.time() - t0:.1f}s)")
    if args.order != "none":
        wl = reorder_topics(wl, args.order)

    t0 = time.time()
    eng = Engine(local)
    set_walk_order(eng, args)
    with progress(f"[rank {rank}] building table"):
        eng.insert_packed(*wl.filters)
        eng.commit()
    st = eng.stats()
    log(f"[rank {rank}] table: {st['n_nodes']} nodes, {st['n_slots']} slots, {st['n_words']} words, "
        f"{st['table_bytes'] / 1e9:.2f} GB, build {st['last_build_ms'] / 1e3:.1f}s ({time.time() - t0:.1f}s)")

    tb = torch.from_numpy(wl.topics[0]).to(dev)
    to = torch.from_numpy(wl.topics[1].view(np.int64)).to(dev)
    n = wl.n_topics
    # the timed steps rotate over distinct batches (batch 0 = the one the baselines and the
    # parity check use); every batch has n topics
    batches = [(tb, to)] + [(torch.from_numpy(b[0]).to(dev), torch.from_numpy(b[1].view(np.int64)).to(dev))
                            for b in getattr(wl, "extra_topics", [])[: max(args.batches, 1) - 1]
                            if len(b[1]) - 1 == n]
    d_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    cap = max(64 * n, 1 << 20)
    d_ids = torch.empty(cap, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream().cuda_stream

    def step():
        return eng.match_device(tb.data_ptr(), to.data_ptr(), n, d_off.data_ptr(), d_ids.data_ptr(), cap,
                                mode=args.mode, stream=stream)

    nout = 0
    for _ in range(max(args.warmup, 1)):  # synchronous calls: size the scratch areas once
        try:
            nout = step()
        except EngineError as err:  # id buffer too small for this workload: size it and redo
            if getattr(err, "needed", None) is None:
                raise
            cap = int(err.needed * 1.25) + 1024
            d_ids = torch.empty(cap, dtype=torch.int32, device=dev)
            nout = step()
    if args.ab:
        return ab_variants(eng, step, args, wl)
    # Timed steps are enqueued with emqx_match_batch_device_async, as a pipelined caller
    # would: every step runs the whole pipeline (fast + deep kernels, scan, scatter) and
    # writes its own summary; nothing is skipped, only the host no longer blocks per batch.
    # Consecutive batches alternate over `--streams` HIP streams (own output buffers each), so
    # one batch's output assembly overlaps the next batch's match kernel.
    summ = torch.zeros((max(args.steps, 1), eng.SUMMARY_WORDS), dtype=torch.int64, device=dev)
    # dedicated streams (not the null stream: the engine maps a null stream to its own one, so
    # events recorded there would not follow the calls)
    streams = [torch.cuda.Stream(device=dev) for _ in range(args.streams)]
    outs = [(d_off, d_ids)] + [(torch.empty_like(d_off), torch.empty_like(d_ids)) for _ in range(args.streams - 1)]
    nouts = []
    for j, (btb, bto) in enumerate(batches):  # each batch's id total; size each stream's workspace
        for k in range(len(streams)):           # (a synchronous call learns its slab)
            try:
                m = eng.match_device(btb.data_ptr(), bto.data_ptr(), n, outs[k][0].data_ptr(), outs[k][1].data_ptr(),
                                     cap, mode=args.mode, stream=streams[k].cuda_stream)
            except EngineError as err:
                if getattr(err, "needed", None) is None:
                    raise
                raise SystemExit(f"batch {j} needs {err.needed} ids, over the {cap}-id buffers")
        nouts.append(m)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    t_start = time.perf_counter()
    ev0.record(streams[0])
    for k in range(args.steps):
        j = k % len(streams)
        btb, bto = batches[k % len(batches)]
        if 0 < k < len(streams):  # the other streams start after the timed region began
            streams[j].wait_event(ev0)
        eng.match_device_async(btb.data_ptr(), bto.data_ptr(), n, outs[j][0].data_ptr(), outs[j][1].data_ptr(), cap,
                               summ[k].data_ptr(), mode=args.mode, stream=streams[j].cuda_stream)
        evs[k].record(streams[j])
    t_enq = time.perf_counter() - t_start  # host time to enqueue the steps (async calls)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    sm = summ.cpu().numpy()
    want_tot = np.array([nouts[k % len(batches)] for k in range(args.steps)], dtype=np.int64)
    if args.steps and not ((sm[:, 0] == 0).all() and (sm[:, 1] == want_tot).all()):
        raise SystemExit(f"async steps incomplete or inconsistent: flags {set(sm[:, 0].tolist())}, "
                         f"totals {set(sm[:, 1].tolist())} vs {set(want_tot.tolist())}")
    if nouts[0] != nout:
        raise SystemExit(f"batch 0 total {nouts[0]} != {nout}")
    # kernel / call times from synchronous calls (HIP events on the engine's stream)
    kern_ms, call_ms, order_ms = [], [], []
    for _ in range(min(max(args.steps, 1), 10)):
        step()
        st = eng.stats()
        kern_ms.append(st["last_kernel_ms"])
        call_ms.append(st["last_match_ms"])
        order_ms.append(st["last_order_ms"])
    evals = eng.stats()["last_evals"]
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
        tot = torch.tensor([float(evals), float(nout)], dtype=torch.float64, device=dev)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        evals_all, nout_all = float(tot[0].item()), float(tot[1].item())
    else:
        evals_all, nout_all = float(evals), float(nout)

    topics_total = float(n) * world * args.steps
    value = topics_total / elapsed
    ms_per_step = 1e3 * elapsed / args.steps
    # completion times of the steps (events on their streams), as intervals between completions
    done = np.sort([ev0.elapsed_time(e) for e in evs]) if args.steps else np.zeros(0)
    gaps = np.diff(np.concatenate([[0.0], done]))

    # roofline of the fused match kernel (rank 0's launch), live kernel time (HIP events)
    offs = wl.topics[1].astype(np.int64)
    tbytes = int(offs[-1] - offs[0])
    levels = int(np.count_nonzero(wl.topics[0][: tbytes] == ord("/"))) + n
    kms = float(np.mean(kern_ms)) if kern_ms else float("nan")
    traffic, traffic_src = args.traffic_bytes, "--traffic-bytes"
    if traffic is None:
        traffic, traffic_src = measured_traffic(n, args)
    roofline = match_roofline(n, kms, args, tbytes, levels, evals, nout, traffic, traffic_src)

    result = {
        "metric": "published topics matched/sec (and match evals/sec) at 10M subs; % of HBM BW",
        "value": round(value, 1),
        "unit": "topics/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic",
        "config": {"workload": WORKLOAD_NAMES["C1" if args.vocab_scale > 1 else args.workload],
                   "n_filters": wl.n_filters, "batch_topics_per_gpu": n, "mode": ["routes", "trie", "trie_wildcard"][args.mode],
                   "parallelism": f"replicated table, topic stream split x{world}",
                   "walk_order": walk_order_desc(args, st),
                   "timed_batches": len(batches)},
        **({"rehearsal": "ranks sharing GPUs over gloo (EMQX_BENCH_REHEARSE): not a measurement"}
           if os.environ.get("EMQX_BENCH_REHEARSE") == "1" else {}),
        "evals_per_s": round(evals_all * args.steps / elapsed, 1),
        "matches_per_topic": round(nout_all / (n * world), 3),
        "evals_per_topic": round(evals_all / (n * world), 3),
        "call_ms_avg": round(float(np.mean(call_ms)), 4),
        "order_ms_avg": round(float(np.mean(order_ms)), 4),
        "step_completion_gap_ms": {"p50": round(float(np.median(gaps)), 4) if gaps.size else None,
                                   "max": round(float(np.max(gaps)), 4) if gaps.size else None},
        "host_enqueue_ms_per_step": round(1e3 * t_enq / max(args.steps, 1), 4),
        "step_gaps_ms": [round(float(g), 3) for g in gaps] if args.steps <= 64 else None,
        "roofline": roofline,
    }

    if world == 1 and not args.no_host_api:
        result["host_api"] = host_api_rates(eng, wl, args, nout)

    if args.diag:
        eng.set_tuning("diag", 1)
        eng.diag(reset=True)
        step()
        d = eng.diag(reset=True)
        eng.set_tuning("diag", 0)
        result["diag_per_topic"] = {k: round(v / n, 3) for k, v in d.items() if not k.startswith(("ticks", "waves"))}
        w = max(d.get("waves", 0), 1)
        result["diag_per_wave"] = {"phase_a_us": round(d["ticks_a"] / w / 100.0, 3),  # 100 MHz wall clock
                                   "phase_b_us": round(d["ticks_b"] / w / 100.0, 3),
                                   "steps": round(d["steps"] / w, 2), "waves": d.get("waves", 0)}
        result["diag_per_topic"]["kernel_ms_diag_call"] = round(eng.stats()["last_kernel_ms"], 4)

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # the GPU CSR of the last synchronous call (the whole batch), compared ID-for-ID
        k = min(args.cpu_sample, n)
        off_g = d_off[: k + 1].cpu().numpy()
        ids_g = d_ids[: int(off_g[-1])].cpu().numpy().view(np.uint32)
        result["cpu_baseline"] = cpu_baseline(wl, args, (off_g, ids_g))
        result["parity"] = result["cpu_baseline"].pop("parity")
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def sharded_bench(args, rank, world, dev):
    """Config C style: the table is split over the ranks (emqx_amd/dist.py); every rank
    publishes its own batch each step (ShardedMatcher.match_all): it partitions the batch by
    owner rank, one all-to-all sends every part to its owner, every rank matches what it
    received against its shard, and the results come back to their source in batch order.
    Weak scaling: per-rank batch fixed as the world grows."""
    import torch
    import torch.distributed as dist
    from emqx_amd import workloads as W
    from emqx_amd.dist import ShardedMatcher, fixed_steps, stream_depth
    from emqx_amd.dist import plan_p_replicated as D_p_repl
    seed = 3 if args.vocab_scale > 1 else 2
    t0 = time.time()
    with progress(f"[rank {rank}] generating workload"):
        wl = W.config_b(n_filters=args.n_filters, n_topics=args.batch, seed=seed, vocab_scale=args.vocab_scale,
                        topic_seed=None if rank == 0 else 1000 + rank)
    log(f"[rank {rank}] workload {wl.n_filters} filters ({time.time() - t0:.1f}s)")
    if world == 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    with progress(f"[rank {rank}] building shard"):
        sm = ShardedMatcher(wl.filters, device=dev, mode=args.mode, p_space=args.p_space)
    sts = [e.stats() for e in sm.engines if e is not None]
    shard_bytes = sum(x["table_bytes"] for x in sts)
    log(f"[rank {rank}] shard: {sm.n_local_filters} filters, {shard_bytes / 1e9:.2f} GB, plan {len(sm.plan)} keys")
    topics = (torch.from_numpy(wl.topics[0]).to(dev), torch.from_numpy(wl.topics[1].view(np.int64)).to(dev))
    res = None
    for _ in range(max(args.warmup, 1)):
        res = sm.match_all(topics)
    sm.match_stream([topics] * max(2, stream_depth()))  # (every lane's buffers and workspaces)
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    # the timed steps: stream_depth() in flight (ShardedMatcher.match_stream), every step's CSR kept
    t_start = time.perf_counter()
    res = sm.match_stream([topics] * args.steps)[-1] if args.steps else res
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    elapsed = float(tt.item())
    n = wl.n_topics
    # parity, per rank, ID-for-ID per topic (oracle/cpp.py csr_mismatches): up to 10M filters
    # every rank's whole batch against a replicated table of the whole filter set on its GPU;
    # past that (config C's 100M) rank 0's first --parity-sample topics against the oracle
    # (oracle/trie_oracle.cpp) restated on the filters that can match them (oracle/pruned.py)
    from oracle import cpp as C
    bad_rank = torch.zeros(world, dtype=torch.float64, device=dev)
    checked = torch.zeros(world, dtype=torch.float64, device=dev)
    if args.n_filters <= 10_000_000:
        from emqx_amd.engine import Engine
        full = Engine(dev.index)
        full.insert_packed(*wl.filters)
        full.commit()
        cap = max(64 * n, 1 << 20)
        d_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
        d_ids = torch.empty(cap, dtype=torch.int32, device=dev)
        m = full.match_device(topics[0].data_ptr(), topics[1].data_ptr(), n, d_off.data_ptr(), d_ids.data_ptr(), cap,
                              mode=args.mode, stream=torch.cuda.current_stream(dev).cuda_stream)
        off_r, ids_r = d_off.cpu().numpy(), d_ids[:m].cpu().numpy().view(np.uint32)
        # the replicated CSR sorted per topic (the oracle-side argument of csr_mismatches)
        tt = np.repeat(np.arange(n, dtype=np.int64), np.diff(off_r.astype(np.int64)))
        ids_r = (np.sort((tt << 32) | ids_r.astype(np.int64)) & 0xFFFFFFFF).astype(np.uint32)
        bad = C.csr_mismatches(res[0].cpu().numpy().astype(np.uint64), res[1].cpu().numpy().view(np.uint32),
                               off_r.astype(np.uint64), ids_r)
        bad_rank[rank] = float(bad.size)
        checked[rank] = float(n)
        parity_rule = "every rank's whole batch vs a replicated table of all filters on its GPU, ID-for-ID per topic"
        del full
    else:
        k = min(args.parity_sample, n)
        if rank == 0:
            from oracle import pruned
            with progress(f"[rank 0] parity: oracle over the filters that can match {k} topics"):
                off_o, ids_o, cand = pruned.slice_csr(wl.filters, wl.fcodes, W.take(wl.topics, np.arange(k)),
                                                      wl.tcodes[:k], mode=args.mode, threads=host_threads()[0])
            off_g = res[0][: k + 1].cpu().numpy().astype(np.uint64)
            ids_g = res[1][: int(off_g[-1])].cpu().numpy().view(np.uint32)
            bad_rank[0] = float(C.csr_mismatches(off_g, ids_g, off_o, ids_o).size)
            checked[0] = float(k)
            log(f"[rank 0] parity: {k} topics, {int(off_o[-1])} ids, oracle table {len(cand)} of {wl.n_filters} filters")
        parity_rule = (f"rank 0's first {k} topics vs the oracle (emqx_trie DFS + match_routes/1 union, "
                       f"oracle/trie_oracle.cpp) over the filters that can match them (oracle/pruned.py), ID-for-ID")
    dist.all_reduce(bad_rank, op=dist.ReduceOp.SUM)
    dist.all_reduce(checked, op=dist.ReduceOp.SUM)
    mism = int(bad_rank[rank].item())
    mt = torch.tensor([float(res[0][-1].item()), float(sm.last_local_topics), 0.0, float(sm.n_local_filters)]
                      + [float(x) for x in sm.last_slot_topics], dtype=torch.float64, device=dev)
    most = mt[3:4].clone()
    dist.all_reduce(mt, op=dist.ReduceOp.SUM)
    dist.all_reduce(most, op=dist.ReduceOp.MAX)
    rehearse = os.environ.get("EMQX_BENCH_REHEARSE") == "1"
    if rank == 0:
        print(json.dumps({
            "metric": "published topics matched/sec at a filter-sharded table (SURVEY §8 e)",
            "value": round(n * world * args.steps / elapsed, 1), "unit": "topics/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic",
            "config": {"workload": f"{'C' if args.vocab_scale > 1 else 'B'}-generator table of {wl.n_filters} "
                                   f"filters sharded x{world}, every rank publishing its own {n}-topic batch per step",
                       "parallelism": f"filter-sharded x{world}: two key spaces (first level; second level under a "
                                      f"root '+'), hot keys split by the next level, "
                                      f"{'gloo (rehearsal)' if rehearse else 'RCCL'} all-to-all out and back"},
            "shard_filters_max_rank": int(most.item()), "shard_filters_max_frac": round(float(most.item()) / wl.n_filters, 4),
            "shard_plan_keys": len(sm.plan), "p_space": "replicated" if D_p_repl(sm.plan) else "sharded",
            "shard_table_bytes_rank0": int(shard_bytes),
            "requests_per_topic_by_slot": {k: round(float(mt[4 + i].item()) / (n * world), 4)
                                           for i, k in enumerate(("A", "B", "AB"))},
            "matches_per_topic": round(float(mt[0].item()) / (n * world), 3),
            "parity": {"rule": parity_rule,
                       "topics_checked_per_rank": [int(x) for x in checked.cpu().tolist()],
                       "mismatching_topics_per_rank": [int(x) for x in bad_rank.cpu().tolist()]},
            "step": "device kernels (emqx_shard_step_*: route + fold onto the engine slots A / B / AB + sort + "
                    "pack, unpack, answer, merge), engines async with learnt capacities, "
                    + ("fixed-capacity chunks agreed beforehand: no size exchange, no host read between steps, "
                       "one flag word a step (a flagged step redone classically)" if fixed_steps() else
                       "two host syncs a step (split sizes)")
                    + f", {stream_depth()} steps in flight (match_stream)",
            "steps_in_flight": stream_depth(),
            "fixed_capacity_steps": fixed_steps(),
            "fixed_steps_redone": int(getattr(sm, "last_fixed_redo", 0)),
            "fixed_host_enqueue_ms_per_step": round(float(getattr(sm, "last_fixed_enqueue_ms", 0.0)), 4),
            **({"rehearsal": "ranks sharing GPUs over gloo (EMQX_BENCH_REHEARSE): not a measurement"}
               if rehearse else {}),
        }), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    if mism:
        raise SystemExit(f"rank {rank}: sharded CSR differs on {mism} topics")


def emulated_bench(args, dev):
    """One rank's step of the filter-sharded layout at world G, measured on ONE GPU
    (VERDICT r5 #1): the G-way plan of the table (config C: 100M filters, vocab x4, seed 3), G
    ranks' engines built on this GPU, G sources' batches (source s draws the stream rank s of a
    real G-rank run would: batch 0 = the C1 batch, then topic seeds 1000 + s), and every rank's
    step run through the product's step (dist.py ShardedMatcher._step_gen) one rank at a time,
    chunks read in place of being moved (dist.py EmulatedWorld).  Reported per rank and phase:
    wall time (host-inclusive) and kernel time (HIP events), the bytes each (source,
    destination) pair exchanges, and a projection of the G-GPU step: the slowest rank per phase
    plus each exchange's largest pair at --xgmi-gbs per link (xGMI is point to point: a pair's
    bytes go over its own link) plus --a2a-us per all-to-all.  Parity: every source's merged CSR
    ID-for-ID against the whole table on this GPU (the replicated layout), and source 0's first
    12K topics against the committed oracle slice (tests/golden/c100m_slice.npz) when the table
    is the golden's."""
    import torch
    from emqx_amd import workloads as W
    from emqx_amd.dist import EmulatedWorld
    from emqx_amd.engine import Engine
    from oracle import cpp as C
    worlds = [int(x) for x in str(args.emulate_world).split(",") if x.strip()]
    G = max(worlds)
    seed = 3 if args.vocab_scale > 1 else 2
    n = args.batch
    t0 = time.time()
    with progress("generating workload"):
        wl = W.config_b(n_filters=args.n_filters, n_topics=n, seed=seed, vocab_scale=args.vocab_scale,
                        extra_topic_seeds=tuple(1000 + s for s in range(1, G)))
    log(f"workload {wl.n_filters} filters, {G} batches of {n} topics ({time.time() - t0:.1f}s)")
    srcs = [wl.topics] + list(wl.extra_topics[: G - 1])
    batches = [(torch.from_numpy(b[0]).to(dev), torch.from_numpy(b[1].view(np.int64)).to(dev)) for b in srcs]
    stream = torch.cuda.current_stream(dev).cuda_stream
    # the replicated layout on this GPU: every source's expected CSR, and the 1-GPU step time
    t0 = time.time()
    with progress("building the whole table (replicated reference)"):
        full = Engine(dev.index)
        full.insert_packed(*wl.filters)
        full.commit()
    log(f"whole table built ({time.time() - t0:.1f}s)")
    cap = max(64 * n, 1 << 20)
    d_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    d_ids = torch.empty(cap, dtype=torch.int32, device=dev)
    refs, rep_ms = [], []
    for j, (tb, to) in enumerate(batches):
        m = full.match_device(tb.data_ptr(), to.data_ptr(), n, d_off.data_ptr(), d_ids.data_ptr(), cap,
                              mode=args.mode, stream=stream)
        off_r = d_off.cpu().numpy()
        ids_r = d_ids[:m].cpu().numpy().view(np.uint32)
        tt = np.repeat(np.arange(n, dtype=np.int64), np.diff(off_r.astype(np.int64)))
        refs.append((off_r.astype(np.uint64), (np.sort((tt << 32) | ids_r.astype(np.int64)) & 0xFFFFFFFF).astype(np.uint32)))
        del tt
    for _ in range(5):
        full.match_device(batches[0][0].data_ptr(), batches[0][1].data_ptr(), n, d_off.data_ptr(), d_ids.data_ptr(),
                          cap, mode=args.mode, stream=stream)
        rep_ms.append(full.stats()["last_match_ms"])
    golden = None
    gpath = os.path.join(ROOT, "tests", "golden", "c100m_slice.npz")
    if os.path.exists(gpath):
        g = dict(np.load(gpath))
        if (int(g["n_filters"]), int(g["n_topics"]), int(g["seed"]), int(g["vocab_scale"])) == (
                args.n_filters, n, seed, args.vocab_scale):
            golden = g
    full.close()
    del full, d_ids
    torch.cuda.empty_cache()
    failed = []
    for G in worlds:
        failed += _emulated_world(args, dev, wl, batches[:G], refs, rep_ms, golden, G)
    if failed:
        raise SystemExit(f"emulated sharded CSR differs: {failed}")


def _emulated_world(args, dev, wl, batches, refs, rep_ms, golden, G):
    """One --emulate-world line (emulated_bench) at world G; returns the parity failures."""
    import torch
    from emqx_amd.dist import EmulatedWorld, fixed_steps
    from oracle import cpp as C
    n = args.batch
    fx = fixed_steps()  # the fixed-capacity form (its capacities learnt from the classic warm-up)
    t0 = time.time()
    with progress(f"building the {G} ranks' engines"):
        ew = EmulatedWorld(wl.filters, G, dev, mode=args.mode, p_space=args.p_space,
                           on_rank=lambda r: log(f"rank {r} built ({time.time() - t0:.0f}s)"))
    log(f"{G} ranks built ({time.time() - t0:.1f}s): filters per rank [A, B, AB] {ew.filters_per_rank}")
    for _ in range(max(args.warmup, 1)):
        res = ew.step(batches)
    if fx:
        ew.learn_fixed()
        res = ew.step(batches, fixed=True)
    torch.cuda.synchronize()
    # the whole emulated step, back to back (all G ranks' work on one GPU, exchanges free)
    t_all = time.perf_counter()
    for _ in range(args.steps):
        ew.step(batches, fixed=fx)
    torch.cuda.synchronize()
    all_ms = 1e3 * (time.perf_counter() - t_all) / max(args.steps, 1)
    if fx:
        phases = EmulatedWorld.PHASES_FIXED if G > 1 else EmulatedWorld.PHASES_FIXED_1
    else:
        phases = EmulatedWorld.PHASES if G > 1 else EmulatedWorld.PHASES_1
    per = {}
    for mode in ("wall", "gpu"):
        acc = np.zeros((G, len(phases)))
        for _ in range(args.steps):
            ew.step(batches, timing=mode, fixed=fx)
            t = np.array(ew.last_times, dtype=np.float64)
            if t.shape != acc.shape:
                raise SystemExit(f"unexpected exchange rounds {t.shape} (a redo during the timed steps)")
            acc += t
        per[mode] = acc / max(args.steps, 1)
    res = ew.step(batches, fixed=fx)
    torch.cuda.synchronize()
    # parity
    bad, ids_checked = [], 0
    for s in range(G):
        off_g = res[s][0].cpu().numpy().astype(np.uint64)
        ids_g = res[s][1].cpu().numpy().view(np.uint32)
        bad.append(int(C.csr_mismatches(off_g, ids_g, *refs[s]).size))
        ids_checked += int(off_g[-1])
    # each rank alone with two steps in flight (ShardedMatcher.match_stream; the other ranks'
    # side replayed from the step above), its last result checked too
    stream_ms, bad_stream, stream_ms_classic, enq_ms = [], [], [], []
    for r in range(G):
        ms, rs = ew.rank_stream(r, batches[r], args.steps, fixed=fx)
        stream_ms.append(ms)
        enq_ms.append(getattr(ew.matchers[r], "last_fixed_enqueue_ms", 0.0))
        if fx:  # (the classic form on the same ranks, for an A/B on one box)
            stream_ms_classic.append(ew.rank_stream(r, batches[r], args.steps, fixed=False)[0])
        bad_stream.append(int(C.csr_mismatches(rs[-1][0].cpu().numpy().astype(np.uint64),
                                               rs[-1][1].cpu().numpy().view(np.uint32), *refs[r]).size))
        del rs
    gold = None
    if golden is not None:
        k = int(golden["slice"])
        off_g = res[0][0][: k + 1].cpu().numpy().astype(np.uint64)
        ids_g = res[0][1][: int(off_g[-1])].cpu().numpy().view(np.uint32)
        gold = {"topics": k, "ids": int(golden["off"][-1]),
                "mismatches": int(C.csr_mismatches(off_g, ids_g, golden["off"], golden["ids"]).size)}
    # projection of the G-GPU step: per phase the slowest rank; per exchange the largest pair
    link = args.xgmi_gbs * 1e9
    bo = ew.bytes_out.copy()
    for k in range(2):
        np.fill_diagonal(bo[k], 0)  # (a rank's own chunk is never moved)
    exch_ms = [float(bo[k].max()) / link * 1e3 for k in range(2)]
    # two size exchanges + two chunk exchanges (the fixed form: the chunk exchanges only)
    fixed_ms = (2 if fx else 4) * args.a2a_us / 1e3 if G > 1 else 0.0
    proj = {}
    for mode in ("wall", "gpu"):
        slow = per[mode].max(axis=0)
        step_ms = float(slow.sum()) + sum(exch_ms) + fixed_ms
        proj[mode] = {"step_ms": round(step_ms, 4), "topics_per_s": round(G * n / step_ms * 1e3, 1),
                      "slowest_rank_phase_ms": {p: round(float(v), 4) for p, v in zip(phases, slow)}}
    step_ms = max(stream_ms) + sum(exch_ms) + fixed_ms
    proj["pipelined"] = {"step_ms": round(step_ms, 4), "topics_per_s": round(G * n / step_ms * 1e3, 1),
                         "slowest_rank_stream_ms": round(max(stream_ms), 4),
                         "rule": "slowest rank's pipelined step + both exchanges' largest pair + fixed costs "
                                 "(exchanges not overlapped)"}
    rep = float(np.median(rep_ms))
    rep_rate = n / rep * 1e3
    out = {
        "metric": f"one rank's filter-sharded step at world {G}, measured on 1xMI355X (all {G} ranks emulated), "
                  f"and the projected {G}-GPU rate",
        "value": proj["pipelined"]["topics_per_s"], "unit": "topics/s (projected)", "n_gpus": 1, "emulated_world": G,
        "steps": args.steps, "warmup": args.warmup, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u32", "data": "synthetic",
        "config": {"workload": f"{'C' if args.vocab_scale > 1 else 'B'}-generator table of {wl.n_filters} filters, "
                               f"{G}-way plan, every rank publishing its own {n}-topic batch per step",
                   "parallelism": f"filter-sharded x{G} emulated on one GPU (dist.py EmulatedWorld)"},
        "p_space": "replicated" if ew.p_replicated else "sharded",
        "fixed_capacity_steps": fx,
        **({"fixed_capacities": {"request_chunk_bytes": ew.matchers[0]._fixed["chunk"],
                                 "answer_chunk_words": ew.matchers[0]._fixed["answer"],
                                 "slot_requests_rank0": ew.matchers[0]._fixed["q"]}} if fx else {}),
        "filters_per_rank_A_B_AB": ew.filters_per_rank,
        "shard_plan_keys": int(len(ew.plan)),
        "requests_per_rank_by_slot": [list(m.last_slot_topics) for m in ew.matchers],
        "rank_phase_ms_wall": [[round(float(x), 4) for x in row] for row in per["wall"]],
        "rank_phase_ms_gpu": [[round(float(x), 4) for x in row] for row in per["gpu"]],
        "rank_step_ms_wall": [round(float(x), 4) for x in per["wall"].sum(axis=1)],
        "rank_step_ms_gpu": [round(float(x), 4) for x in per["gpu"].sum(axis=1)],
        "rank_stream_ms": [round(float(x), 4) for x in stream_ms],
        **({"rank_stream_ms_classic_form": [round(float(x), 4) for x in stream_ms_classic],
            "rank_stream_host_enqueue_ms": [round(float(x), 4) for x in enq_ms]} if fx else {}),
        "phases": list(phases),
        "exchange_bytes_out": {"requests": bo[0].tolist(), "answers": bo[1].tolist()},
        "exchange_max_pair_bytes": {"requests": int(bo[0].max()), "answers": int(bo[1].max())},
        "projection": {"xgmi_gbs_per_link": args.xgmi_gbs, "a2a_fixed_us": args.a2a_us,
                       "exchange_ms": [round(x, 4) for x in exch_ms], **proj},
        "emulated_step_ms_all_ranks_one_gpu": round(all_ms, 4),
        "replicated_one_gpu": {"call_ms": round(rep, 4), "topics_per_s": round(rep_rate, 1),
                               "x_G": round(G * rep_rate, 1)},
        "projected_vs_G_replicated": {m: round(proj[m]["topics_per_s"] / (G * rep_rate), 4) for m in proj},
        "parity": {"rule": "every source's merged CSR vs the whole table on this GPU, ID-for-ID per topic",
                   "topics_checked": G * n, "ids_checked": ids_checked, "mismatching_topics_per_source": bad,
                   "mismatching_topics_per_rank_stream": bad_stream, "golden_slice_source0": gold},
    }
    print(json.dumps(out), flush=True)
    ew.close()
    del ew, res
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return [(G, bad, bad_stream, gold)] if any(bad) or any(bad_stream) or (gold and gold["mismatches"]) else []


def retain_traffic(nf, n_retained):
    """HBM bytes of one config-R call from the committed PMC passes (profiles/pmc_retain.json,
    tools/pmc_retain.py), when they were taken on this same workload; else (None, None)."""
    path = os.path.join(ROOT, "profiles", "pmc_retain.json")
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        p = json.load(f)
    if p.get("filters_per_call") != nf or p.get("retained_topics") != n_retained or p.get("traffic_bytes_per_call") is None:
        return None, None
    return round(p["traffic_bytes_per_call"]), "profiles/pmc_retain.json (%s; %s)" % (p["traffic_rule"], p["source"])


def pmc_file(args):
    """The committed PMC summary of the fast kernel for this exact workload (B, D, or config C's
    100M-filter table on one GPU), or None."""
    if args.mode != 0:
        return None
    if args.workload == "D" and args.vocab_scale == 1:
        return "pmc_match_fast_D.json"
    if args.workload == "B" and args.vocab_scale == 1 and args.n_filters == 10_000_000:
        return "pmc_match_fast.json"
    if args.workload == "B" and args.vocab_scale == 4 and args.n_filters == 100_000_000:
        return "pmc_match_fast_C1.json"
    return None


def measured_traffic(n, args):
    """HBM bytes per launch of the fused match kernel from the committed rocprofv3 PMC passes
    (profiles/pmc_match_fast.json, written from tools/gpu_round.sh's counter runs on the same
    workload), scaled to this batch.  None when the file is absent or the workload differs."""
    fname = pmc_file(args)
    if fname is None:
        return None, None
    path = os.path.join(ROOT, "profiles", fname)
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        p = json.load(f)
    per_topic = p["traffic_bytes_per_launch"] / p["batch_topics"]
    return round(per_topic * n), "profiles/%s (%s; %s)" % (fname, p["traffic_rule"], p["source"])


def host_api_rates(eng, wl, args, nout):
    """The same batch through the host-memory entry points (PCIe included; never `value`):
    emqx_match_batch from pageable numpy buffers (chunks staged through two pinned host
    batches), and pinned host batches (emqx_host_batch_*, the NIF's buffers) with four
    quarter-batches in flight."""
    from emqx_amd import workloads as W
    from emqx_amd.engine import HostBatch
    n = wl.n_topics
    tb, to = wl.topics
    out_off = np.zeros(n + 1, dtype=np.uint64)
    reps = 5
    off, ids = eng.match_packed(tb, to, mode=args.mode)  # sizes the pool's buffers
    if int(off[-1]) != nout:
        raise SystemExit(f"host API total {int(off[-1])} != device total {nout}")
    t = time.perf_counter()
    for _ in range(reps):
        eng.match_packed(tb, to, mode=args.mode)
    pageable = reps * n / (time.perf_counter() - t)
    q = 4
    parts = [W.take(wl.topics, np.arange(n * k // q, n * (k + 1) // q)) for k in range(q)]
    hbs = []
    for p_ in parts:
        hb = HostBatch(eng, cap_topics=len(p_[1]), cap_bytes=int(p_[1][-1]) + 64, cap_ids=4 * nout // q + (1 << 20))
        hb.pack(*p_)
        hbs.append(hb)
    tot = 0
    for hb in hbs:
        hb.submit(args.mode)
    for hb in hbs:
        tot += int(hb.wait(copy=False)[0][-1])
    if tot != nout:
        raise SystemExit(f"pinned host batches total {tot} != device total {nout}")
    t = time.perf_counter()
    for _ in range(reps):
        for hb in hbs:
            hb.submit(args.mode)
        for hb in hbs:
            hb.wait(copy=False)
    pinned = reps * n / (time.perf_counter() - t)
    for hb in hbs:
        hb.close()
    in_b = int(to[-1] - to[0]) + 8 * (n + 1)
    out_b = 8 * (n + 1) + 4 * nout
    return {"pageable_emqx_match_batch_topics_per_s": round(pageable, 1),
            "pinned_host_batches_topics_per_s": round(pinned, 1),
            "bytes_in_per_batch": in_b, "bytes_out_per_batch": out_b,
            "pinned_pcie_gb_per_s": round((in_b + out_b) * pinned / n / 1e9, 2),
            "note": "same 1M-topic batch from host memory: H2D + match + CSR back to host; pinned = 4 "
                    "quarter-batches in flight (emqx_host_batch_*), pageable = emqx_match_batch on numpy "
                    "arrays (2 pinned chunk buffers inside)"}


def batcher_bench(args, rank, world, dev):
    """The drop-in per-PUBLISH path (emqx_broker.erl:213 -> emqx_router:match_routes/1 per
    message): C concurrent single-topic callers in a closed loop through the cross-caller
    batcher (emqx_batcher_*, two pinned batches in flight) on config B's 10M-filter table.
    tools/batch_load.cpp drives the callers natively; per C: topics/s and latency
    percentiles (submit -> ids delivered to the caller's callback)."""
    import ctypes
    from emqx_amd import workloads as W
    from emqx_amd.engine import Engine
    t0 = time.time()
    with progress(f"[rank {rank}] generating workload"):
        wl = load_or_make(args, rank, lambda: W.config_b(n_filters=args.n_filters, n_topics=args.batch, seed=2,
                                                         topic_seed=None if rank == 0 else 1000 + rank))
    eng = Engine(dev.index)
    with progress(f"[rank {rank}] building table"):
        eng.insert_packed(*wl.filters)
        eng.commit()
    log(f"[rank {rank}] table ready ({time.time() - t0:.1f}s)")
    L = ctypes.CDLL(os.path.join(ROOT, "tools", "_build", "libbatchload.so"))
    L.batch_load.restype = ctypes.c_int
    L.batch_load.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                             ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_double, ctypes.c_double,
                             ctypes.c_void_p]
    tb, to = wl.topics
    to = np.ascontiguousarray(to.astype(np.uint64))
    runs = []
    waits = [int(x) for x in str(args.max_wait_us).split(",")]
    for c, wus in [(int(x), w) for x in args.callers.split(",") for w in waits]:
        out = np.zeros(12, dtype=np.float64)
        small_clock_start(eng, args)
        rc = L.batch_load(eng._h, args.mode, tb.ctypes.data, to.ctypes.data, wl.n_topics, c, args.max_batch,
                          wus, 500.0, 3000.0, out.ctypes.data)
        if rc != 0:
            raise SystemExit(f"batch_load failed: {rc}")
        runs.append({"callers": c, "max_wait_us": wus, "topics_per_s": round(out[0] / out[1], 1), "p50_us": round(out[2], 1),
                     "p90_us": round(out[3], 1), "p99_us": round(out[4], 1), "max_us": round(out[5], 1),
                     "batches": int(out[6]), "topics_per_batch": round(out[7], 1),
                     "max_in_flight": int(out[8]), "us_per_batch_device_wait": round(out[9], 1),
                     "us_per_batch_callbacks": round(out[10], 1), "us_per_batch_submit": round(out[11], 1)})
        clk = small_clock_read(eng, args)
        if clk:
            runs[-1]["small_clock"] = clk
        log(f"[rank {rank}] callers {c}: {runs[-1]}")
    best = max(runs, key=lambda r: r["topics_per_s"])
    res = {"metric": "per-PUBLISH match_routes/1 calls served/sec through the batcher (10M subs)",
           "value": best["topics_per_s"], "unit": "topics/s", "n_gpus": world, "steps": len(runs),
           "warmup": 1, "ms_per_step": 3000.0, "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "u32", "data": "synthetic",
           "config": {"workload": "L: concurrent single-topic callers -> emqx_batcher -> pinned host batches, "
                                  "config B table", "n_filters": wl.n_filters, "max_batch": args.max_batch,
                      "parallelism": "replicated table"},
           "runs": runs}
    if rank == 0:
        print(json.dumps(res), flush=True)


SMALL_CLK = ("copy_in", "walk", "deep", "scan", "scatter", "out", "fo_pass1", "fo_pass2")


def small_clock_start(eng, args):
    """--small-clock: the one-launch small-batch kernel accumulates its per-phase wall clocks
    (kernels.h SMALL_CLK_*) into the engine's timeline buffer while the run lasts."""
    if args.small_clock:
        eng.set_tuning("timeline", 0)
        eng.set_tuning("timeline", 5)


def small_clock_read(eng, args):
    """Average microseconds per launch of each small-kernel phase, and the launches counted."""
    if not args.small_clock:
        return None
    import ctypes
    from emqx_amd import _lib
    buf = np.zeros(10, dtype=np.uint64)
    got = ctypes.c_uint64(0)
    _lib.check(_lib.lib().emqx_diag_timeline(eng._h, buf.ctypes.data, 5, ctypes.byref(got)), "emqx_diag_timeline")
    eng.set_tuning("timeline", 0)
    k = int(buf[8])
    out = {"launches": k}
    for i, name in enumerate(SMALL_CLK):
        out[name + "_us"] = round(float(buf[i]) * 0.01 / max(k, 1), 2)  # 100 MHz ticks
    out["kernel_us"] = round(float(buf[:8].sum()) * 0.01 / max(k, 1), 2)
    return out


def config_e_tables(args, rank, dev):
    """Config E's tables on this rank's device: the 2M-filter route table and the 10M-subscription
    table (one full commit)."""
    from emqx_amd import workloads as W
    from emqx_amd.engine import Engine
    from emqx_amd.fanout import SubTable
    t0 = time.time()
    with progress(f"[rank {rank}] generating config E"):
        fw = W.config_e(n_topics=args.batch)
        publisher_keys(fw, args)
    eng = Engine(dev.index)
    with progress(f"[rank {rank}] building tables"):
        eng.insert_packed(*fw.wl.filters)
        eng.commit()
        st = SubTable(dev.index)
        st.add(fw.sub_filter, fw.sub_id, fw.sub_group)
        t1 = time.perf_counter()
        st.commit()
        full_ms = 1e3 * (time.perf_counter() - t1)
    log(f"[rank {rank}] config E: {fw.wl.n_filters} filters, {fw.n_subscriptions} subscriptions, "
        f"subtab {st.stats()} ({time.time() - t0:.1f}s)")
    return fw, eng, st, full_ms


def pub_batcher_bench(args, rank, world, dev):
    """The drop-in per-PUBLISH fan-out (emqx_channel -> emqx_broker:publish/1, emqx_broker.erl:
    203-214, once per message from each publisher process): C concurrent single-message callers
    in a closed loop through the publish batcher (emqx_pub_batcher_*: pinned batches, match +
    fan-out on the device with no host sync in between, two batches in flight) on config E's
    10M subscriptions.  Per C: messages/s and latency percentiles (submit -> deliveries in the
    caller's callback)."""
    import ctypes
    from emqx_amd import _lib
    fw, eng, st, _ = config_e_tables(args, rank, dev)
    L = ctypes.CDLL(os.path.join(ROOT, "tools", "_build", "libbatchload.so"))
    L.pub_load.restype = ctypes.c_int
    L.pub_load.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                           ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                           ctypes.c_double, ctypes.c_double, ctypes.c_void_p]
    from emqx_amd.fanout import STRATEGIES
    strat = STRATEGIES[args.strategy]
    tb, to = fw.wl.topics
    to = np.ascontiguousarray(to.astype(np.uint64))
    keys = np.ascontiguousarray(fw.keys.astype(np.uint32))
    runs = []
    waits = [int(x) for x in str(args.max_wait_us).split(",")]
    for c, wus in [(int(x), w) for x in args.callers.split(",") for w in waits]:
        out = np.zeros(13, dtype=np.float64)
        small_clock_start(eng, args)
        rc = L.pub_load(eng._h, st.handle, strat, tb.ctypes.data, to.ctypes.data, keys.ctypes.data, fw.wl.n_topics, c,
                        args.max_batch, wus, 500.0, 3000.0, out.ctypes.data)
        if rc != 0:
            raise SystemExit(f"pub_load failed: {rc} ({_lib.lib().emqx_strerror(rc).decode()})")
        runs.append({"callers": c, "max_wait_us": wus, "messages_per_s": round(out[0] / out[1], 1),
                     "p50_us": round(out[2], 1), "p90_us": round(out[3], 1), "p99_us": round(out[4], 1),
                     "max_us": round(out[5], 1), "batches": int(out[6]), "messages_per_batch": round(out[7], 1),
                     "deliveries_per_message": round(out[12], 3), "max_in_flight": int(out[8]),
                     "us_per_batch_device_wait": round(out[9], 1), "us_per_batch_callbacks": round(out[10], 1),
                     "us_per_batch_submit": round(out[11], 1)})
        clk = small_clock_read(eng, args)
        if clk:
            runs[-1]["small_clock"] = clk
        log(f"[rank {rank}] callers {c}: {runs[-1]}")
    best = max(runs, key=lambda r: r["messages_per_s"])
    res = {"metric": "per-PUBLISH emqx_broker:publish/1 fan-outs served/sec through the publish batcher "
                     "(config E, 10M subscriptions)",
           "value": best["messages_per_s"], "unit": "messages/s", "n_gpus": world, "steps": len(runs),
           "warmup": 1, "ms_per_step": 3000.0, "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "u32", "data": "synthetic",
           "config": {"workload": "P: concurrent single-message publishers -> emqx_pub_batcher -> pinned publish "
                                  "batches (match + fan-out) on config E's tables",
                      "n_filters": fw.wl.n_filters, "subscriptions": fw.n_subscriptions,
                      "strategy": args.strategy, "max_batch": args.max_batch, "parallelism": "replicated tables"},
           "runs": runs}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        args.cpu_sample = min(args.cpu_sample, 200_000)
        res["cpu_baseline"] = fanout_cpu_baseline(fw, args)
    if rank == 0:
        print(json.dumps(res), flush=True)


def storm_bench(args, rank, world, dev):
    """The per-call boundary for subscription and route changes: EMQX applies each
    SUBSCRIBE as its own ETS write (emqx_broker.erl:124-164) and each new topic's route as its own
    mria transaction (emqx_router.erl:111-124, emqx_router_utils.erl:97-125).  Here closed-loop
    callers (tools/batch_load.cpp sub_load) subscribe / unsubscribe one (filter, subscriber) pair
    per call, or add / delete one route per call, through the commit coalescer
    (emqx_coalescer_*: group commit; a call returns when the commit carrying it has reached the
    device) on config E's tables (2M filters, 10M subscriptions).  Reports single-op latency
    (1 caller), ops/s and latency at --callers, and the publish batcher's throughput (P, 512
    callers, round_robin) alone and while 512 callers subscribe and unsubscribe."""
    import ctypes
    import threading
    from emqx_amd import _lib
    from emqx_amd.fanout import STRATEGIES
    fw, eng, st, _ = config_e_tables(args, rank, dev)
    L = ctypes.CDLL(os.path.join(ROOT, "tools", "_build", "libbatchload.so"))
    L.sub_load.restype = ctypes.c_int
    L.sub_load.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                           ctypes.c_int, ctypes.c_uint32, ctypes.c_double, ctypes.c_double, ctypes.c_void_p]
    L.pub_load.restype = ctypes.c_int
    L.pub_load.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                           ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                           ctypes.c_double, ctypes.c_double, ctypes.c_void_p]
    nf = int(fw.wl.n_filters)
    first_sub = int(fw.sub_id.max()) + 1

    def sub_run(callers, route=0, dur_ms=2000.0, base=first_sub):
        out = np.zeros(13, dtype=np.float64)
        rc = L.sub_load(eng._h, st.handle, callers, nf, base, route, 0, 300.0, dur_ms, out.ctypes.data)
        if rc != 0:
            raise SystemExit(f"sub_load failed: {rc} ({_lib.lib().emqx_strerror(rc).decode()})")
        r = {"callers": callers, "op": "route add/delete" if route else "subscribe/unsubscribe",
             "ops_per_s": round(out[0] / out[1], 1), "p50_us": round(out[2], 1), "p90_us": round(out[3], 1),
             "p99_us": round(out[4], 1), "max_us": round(out[5], 1), "commits": int(out[6]),
             "ops_per_commit": round(out[7], 1), "us_per_commit": round(out[12], 1)}
        log(f"[rank {rank}] {r}")
        return r

    tb, to = fw.wl.topics
    to = np.ascontiguousarray(to.astype(np.uint64))
    keys = np.ascontiguousarray(fw.keys.astype(np.uint32))
    strat = STRATEGIES["round_robin"]

    def pub_run(callers, dur_ms=2000.0):
        out = np.zeros(13, dtype=np.float64)
        rc = L.pub_load(eng._h, st.handle, strat, tb.ctypes.data, to.ctypes.data, keys.ctypes.data, fw.wl.n_topics,
                        callers, args.max_batch, 200, 500.0, dur_ms, out.ctypes.data)
        if rc != 0:
            raise SystemExit(f"pub_load failed: {rc} ({_lib.lib().emqx_strerror(rc).decode()})")
        return {"callers": callers, "messages_per_s": round(out[0] / out[1], 1), "p50_us": round(out[2], 1),
                "p99_us": round(out[4], 1)}

    single_sub = sub_run(1)
    single_route = sub_run(1, route=1)
    storms = [sub_run(int(c)) for c in args.callers.split(",")]
    p_alone = pub_run(512)
    storm_box = {}

    def storm():
        storm_box["r"] = sub_run(512, dur_ms=3500.0, base=first_sub + 100_000)

    th = threading.Thread(target=storm)
    th.start()
    time.sleep(0.5)
    p_storm = pub_run(512)
    th.join()
    p_storm["storm"] = storm_box.get("r")
    best = storms[-1]
    res = {"metric": "per-call subscribe/unsubscribe operations committed/sec through the commit coalescer "
                     "(config E, 10M subscriptions)",
           "value": best["ops_per_s"], "unit": "ops/s", "n_gpus": world, "steps": len(storms) + 4, "warmup": 1,
           "ms_per_step": 2000.0, "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
           "data": "synthetic",
           "config": {"workload": "T: closed-loop per-call subscribe / route changes -> emqx_coalescer (group "
                                  "commit) on config E's tables; P beside it", "n_filters": nf,
                      "subscriptions": fw.n_subscriptions, "callers": args.callers, "parallelism": "replicated tables"},
           "single_op": {"subscribe": single_sub, "route_add_delete": single_route},
           "storm": storms, "publish_alone": p_alone, "publish_during_storm": p_storm}
    if rank == 0:
        print(json.dumps(res), flush=True)


def subscribe_bench(args, rank, world, dev):
    """Subscription churn on config E's 10M-subscription table (emqx_broker:subscribe/3 and
    unsubscribe/1, emqx_broker.erl:124-195; emqx_shared_sub's subscribe/unsubscribe,
    emqx_shared_sub.erl:308-322): `--rounds` commits of `--churn` unsubscribes of live
    subscriptions plus `--churn` new subscriptions (10% into existing $share groups), each round
    = emqx_subtab_remove + emqx_subtab_add + emqx_subtab_commit (patched in place on the device).
    After the rounds the device fan-out of a topic sample is compared with the oracle's after
    the same ops (count + order-free checksum per topic, hash_clientid picks); the CPU baseline
    is the oracle applying the same ops to its ETS-bag restatement on the host cores."""
    import torch
    from emqx_amd import workloads as W
    from oracle import cpp as C
    fw, eng, st, full_ms = config_e_tables(args, rank, dev)
    rng = np.random.default_rng(21)
    k = args.churn
    n_sub = len(fw.sub_id)
    present = np.ones(n_sub, bool)
    shared_idx = np.flatnonzero(fw.sub_group != W.NO_GROUP)
    next_sub = int(fw.sub_id.max()) + 1
    nf = int(fw.wl.n_filters)
    ops_f, ops_s, ops_g, ops_a = [], [], [], []
    times, commit_ms, rem_ms, add_ms = [], [], [], []
    c0 = None
    warm = max(0, args.warmup)
    for r in range(warm + args.rounds):
        if r == warm:  # the first rounds (first-time allocations, pool start) are not timed
            c0 = st.commit_stats()
            times, commit_ms, rem_ms, add_ms = [], [], [], []
        idx = rng.choice(n_sub, k + k // 4, replace=False)
        rem = idx[present[idx]][:k]
        present[rem] = False
        # new subscriptions: 90% plain to random filters, 10% new members of existing groups
        n_sh = k // 10
        gi = rng.choice(shared_idx, n_sh)
        af = np.concatenate([rng.integers(0, nf, k - n_sh).astype(np.uint32), fw.sub_filter[gi]])
        asub = np.arange(next_sub, next_sub + k, dtype=np.uint32)
        next_sub += k
        ag = np.concatenate([np.full(k - n_sh, W.NO_GROUP, np.uint32), fw.sub_group[gi]])
        rf, rs, rg = fw.sub_filter[rem], fw.sub_id[rem], fw.sub_group[rem]
        t = time.perf_counter()
        st.remove(rf, rs, rg)
        ta = time.perf_counter()
        st.add(af, asub, ag)
        tc = time.perf_counter()
        st.commit()
        t_end = time.perf_counter()
        times.append(t_end - t)
        commit_ms.append(1e3 * (t_end - tc))
        rem_ms.append(1e3 * (ta - t))
        add_ms.append(1e3 * (tc - ta))
        ops_f += [rf, af]
        ops_s += [rs, asub]
        ops_g += [rg, ag]
        ops_a += [np.zeros(len(rf), np.uint8), np.ones(len(af), np.uint8)]
    c1 = st.commit_stats()
    n_ops = int(sum(len(a) for a in ops_a))  # every round's ops (the parity check applies them all)
    timed_ops = 2 * k * args.rounds
    value = timed_ops / sum(times)
    # parity after the churn: device fan-out of a topic sample vs the oracle with the same ops
    n = fw.wl.n_topics
    sample = min(args.cpu_sample, n, 200_000)
    tb = torch.from_numpy(fw.wl.topics[0]).to(dev)
    to = torch.from_numpy(fw.wl.topics[1].view(np.int64)).to(dev)
    moff = torch.empty(sample + 1, dtype=torch.int64, device=dev)
    mcap = 64 * sample
    mids = torch.empty(mcap, dtype=torch.int32, device=dev)
    nm = eng.match_device(tb.data_ptr(), to.data_ptr(), sample, moff.data_ptr(), mids.data_ptr(), mcap)
    keys = torch.from_numpy(fw.keys[:sample].view(np.int32)).to(dev)
    ooff = torch.empty(sample + 1, dtype=torch.int64, device=dev)
    ocap = 256 * sample
    osubs = torch.empty(ocap, dtype=torch.int32, device=dev)
    ofil = torch.empty(ocap, dtype=torch.int32, device=dev)
    tot = st.fanout_device("hash_clientid", moff.data_ptr(), mids.data_ptr(), sample, keys.data_ptr(), ooff.data_ptr(),
                           osubs.data_ptr(), ofil.data_ptr(), ocap)
    off_g = ooff.cpu().numpy().view(np.uint64)
    gsum = C.delivery_checksums(off_g, osubs[:tot].cpu().numpy().view(np.uint32), ofil[:tot].cpu().numpy().view(np.uint32))
    fo = C.FanoutOracle(fw.sub_filter, fw.sub_id, fw.sub_group)
    threads = args.cpu_threads or host_threads()[0]
    of, os_, og, oa = (np.concatenate(x) for x in (ops_f, ops_s, ops_g, ops_a))
    t = time.perf_counter()
    changed = fo.churn(of, os_, og, oa, threads=threads)
    cpu_s = time.perf_counter() - t
    mo, mi = moff.cpu().numpy().view(np.uint64), mids[:nm].cpu().numpy().view(np.uint32)
    counts, sums, total = fo.publish(mo, mi, fw.keys[:sample], threads=threads)
    bad = np.nonzero((np.diff(off_g.astype(np.int64)) != counts.astype(np.int64)) | (gsum != sums))[0]
    if bad.size:
        raise SystemExit(f"fan-out after churn differs from the oracle on {bad.size} topics, first {bad[:10].tolist()}")
    res = {"metric": "subscription ops/s (subscribe + unsubscribe, committed to the device) at 10M subscriptions",
           "value": round(value, 1), "unit": "ops/s", "n_gpus": world, "steps": args.rounds, "warmup": warm,
           "ms_per_step": round(1e3 * float(np.mean(times)), 4), "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "u32", "data": "synthetic", "warmup_rounds": warm,
           "round_ms": [round(1e3 * x, 3) for x in times],
           "config": {"workload": "S: subscription churn on config E's 10M-subscription table",
                      "subscriptions": fw.n_subscriptions, "ops_per_commit": timed_ops // args.rounds,
                      "shared_fraction_of_new": 0.1, "parallelism": "replicated tables"},
           "commit_ms": {"p50": round(float(np.median(commit_ms)), 3), "p99": round(float(np.percentile(commit_ms, 99)), 3),
                         "first": round(commit_ms[0], 3), "last": round(commit_ms[-1], 3)},
           "host_ms_p50": {"remove": round(float(np.median(rem_ms)), 3), "add": round(float(np.median(add_ms)), 3),
                           "commit_host_half": round(float(np.median(commit_ms)), 3),
                           "note": "emqx_subtab_commit returns after its host half; its device half overlaps the "
                                   "next round and is waited for by the next commit"},
           "full_build_commit_ms": round(full_ms, 1),
           "commit_stats": {"incremental_commits": int(c1["commits"] - c0["commits"] - (c1["full_commits"] - c0["full_commits"])),
                            "full_commits": int(c1["full_commits"] - c0["full_commits"]),
                            "words_per_commit": round((c1["words"] - c0["words"]) / args.rounds, 1),
                            "records_per_commit": round((c1["records"] - c0["records"]) / args.rounds, 1),
                            "extents_moved_per_commit": round((c1["moves"] - c0["moves"]) / args.rounds, 1),
                            "host_us_last_commit": c1["host_us"]},
           "cpu_baseline": {"value": round(n_ops / cpu_s, 1), "unit": "ops/s", "cores": threads, "kind": "port",
                            "sample": f"the same {n_ops} ops (oracle/fanout_oracle.cpp orf_churn: ETS-bag insert / "
                                      "delete_object restatement, ops split by filter over the threads, no mria)",
                            "changed": changed},
           "parity": {"topics_checked": int(sample), "deliveries_checked": int(total), "mismatches": 0,
                      "rule": "after all rounds: per-topic delivery count + order-free multiset checksum of "
                              "(subscriber, filter), device fan-out vs the oracle with the same ops"}}
    if rank == 0:
        print(json.dumps(res), flush=True)


def gather_ceiling():
    """Random-access ceiling of the chip: the best rate of independent random 16-B reads from
    a 1 GiB HBM-resident table (tools/gather_bench.hip, profiles/r1_gather16_ceiling.jsonl):
    one L2 miss per read, so it is also the ceiling on L2 misses/s."""
    path = os.path.join(ROOT, "profiles", "r1_gather16_ceiling.jsonl")
    best = None
    if os.path.exists(path):
        with open(path) as f:
            for line in f:
                r = json.loads(line)
                if r.get("shape") == "indep" and r.get("table_mb", 0) >= 1024:
                    best = max(best or 0.0, float(r["records_per_s"]))
    return best


def request_roofline(n, kms, args):
    """The request-rate roofline beside the byte one: the fused kernel's L2 misses per launch
    (committed PMC passes, scaled to this batch) / its HIP-event time, against the measured
    random-access ceiling.  The walk is a chain of dependent random 16-B probes, so this, not
    the byte rate, is what bounds it."""
    fname = pmc_file(args)
    if fname is None:
        return None
    path = os.path.join(ROOT, "profiles", fname)
    ceil = gather_ceiling()
    if not os.path.exists(path) or not ceil:
        return None
    with open(path) as f:
        p = json.load(f)
    misses = p["l2_misses_per_launch"] / p["batch_topics"] * n
    got = misses / (kms * 1e-3)
    return {"bound": "random-gather ceiling", "l2_misses_per_launch": round(misses),
            "l2_misses_per_topic": round(misses / n, 2), "l2_hit_rate": round(p["l2_hit_rate"], 4),
            "achieved": round(got / 1e9, 2), "peak": round(ceil / 1e9, 2), "unit": "G misses/s",
            "frac": round(got / ceil, 4),
            "source": f"profiles/{fname} (TCC_MISS per launch); ceiling profiles/r1_gather16_ceiling.jsonl"}


def match_roofline(n, kms, args, tbytes, levels, evals, nout, traffic, traffic_src):
    """The match kernel's roofline on SURVEY §8(d)'s basis: `achieved` = the ALGORITHMIC bytes
    of one launch (per topic len(T) + 64*L(T) + 64*evals(T) + 4*(|M(T)|+1): the topic bytes, one
    64-B intern probe per level, one 64-B transaction per trie-node visit, the CSR ids and offset)
    over the kernel's live HIP-event time, against the 8 TB/s HBM peak; `traffic` = the HBM bytes
    the counters saw per launch (FETCH_SIZE + WRITE_SIZE, committed PMC passes, scaled to the
    batch).  The model charges L2 hits as HBM bytes, so counted traffic can sit below it (config
    B: 46 % of the probes hit in L2).

    What actually bounds the walk is the rate of random line requests the chip serves (a chain of
    dependent random 16-B probes): `request_rate` sets the kernel's L2 misses per launch against
    the measured random-gather ceiling (55.8 G independent random 16-B reads/s of a 1 GiB table,
    tools/gather_bench.hip, one L2 miss each), labelled "random-gather ceiling"."""
    alg_bytes = tbytes + 64 * levels + 64 * evals + 4 * (nout + n)
    gbs = alg_bytes / (kms * 1e-3) / 1e9
    out = {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_src,
           "kernel": "match_fast_kernel", "kernel_ms_avg": round(kms, 4), "alg_bytes_per_launch": alg_bytes,
           "basis": "algorithmic bytes per launch (SURVEY §8 d: len(T) + 64*L(T) + 64*evals(T) + 4*(|M(T)|+1) "
                    "per topic) / live kernel time (HIP events on the engine's stream), against 8 TB/s"}
    if traffic:
        tgbs = traffic / (kms * 1e-3) / 1e9
        out["traffic_frac"] = round(tgbs / HBM_PEAK_GBS, 4)
        out["traffic_vs_alg"] = round(traffic / alg_bytes, 4)
    rr = request_roofline(n, kms, args)
    if rr is not None:
        rr["bound"] = "random-gather ceiling"
        out["request_rate"] = rr
    return out


def publisher_keys(fw, args):
    """round_robin / sticky take the publisher as the message key: `--publishers N` folds the
    generated keys onto N publishers (N = 1: one publisher sends the whole batch, a bridge)."""
    if args.publishers and args.strategy in ("round_robin", "sticky"):
        fw.keys = (fw.keys % np.uint32(args.publishers)).astype(np.uint32)


def fanout_bench(args, rank, world, dev):
    """Config E: 10M subscriptions (1M subscribers x 10 filters over a 2M-filter config-B table,
    10% in $share groups of 2-16 members).  A step = match (emqx_match_batch_device) + fan-out
    (emqx_fanout_batch_device) of one 1M-topic batch resident in HBM -> per-topic CSR of
    (subscriber, filter) deliveries in HBM.  Replicated tables, weak scaling over ranks."""
    import torch
    import torch.distributed as dist
    from emqx_amd import workloads as W
    from emqx_amd.engine import Engine
    from emqx_amd.fanout import SubTable
    t0 = time.time()
    fw = W.config_e(n_topics=args.batch)
    publisher_keys(fw, args)
    log(f"[rank {rank}] config E: {fw.wl.n_filters} filters, {fw.n_subscriptions} subscriptions ({time.time() - t0:.1f}s)")
    eng = Engine(dev.index)
    eng.insert_packed(*fw.wl.filters)
    eng.commit()
    st = SubTable(dev.index)
    if args.strategy == "round_robin":  # SURVEY §8 d: config E's round_robin has its counter seeded 0
        st.set_tuning("rr_seed0", 1)
    st.add(fw.sub_filter, fw.sub_id, fw.sub_group)
    st.commit()
    log(f"[rank {rank}] subtab {st.stats()}")
    n = fw.wl.n_topics
    tb = torch.from_numpy(fw.wl.topics[0]).to(dev)
    to = torch.from_numpy(fw.wl.topics[1].view(np.int64)).to(dev)
    keys = torch.from_numpy(fw.keys.view(np.int32)).to(dev)
    moff = torch.empty(n + 1, dtype=torch.int64, device=dev)
    mcap = 32 * n
    mids = torch.empty(mcap, dtype=torch.int32, device=dev)
    ooff = torch.empty(n + 1, dtype=torch.int64, device=dev)
    ocap = 128 * n
    osubs = torch.empty(ocap, dtype=torch.int32, device=dev)
    ofil = torch.empty(ocap, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    fo_ms = []

    def step():
        nm = eng.match_device(tb.data_ptr(), to.data_ptr(), n, moff.data_ptr(), mids.data_ptr(), mcap, mode=0,
                              stream=stream)
        ev[0].record()
        nd = st.fanout_device(args.strategy, moff.data_ptr(), mids.data_ptr(), n, keys.data_ptr(), ooff.data_ptr(),
                              osubs.data_ptr(), ofil.data_ptr(), ocap, stream=stream)
        ev[1].record()
        return nm, nd

    nm = nd = 0
    for _ in range(max(args.warmup, 1)):
        nm, nd = step()
    # Timed steps: match (emqx_match_batch_device_async) + fan-out (emqx_fanout_batch_device_async)
    # of one batch each, enqueued with no host synchronisation; consecutive batches alternate
    # over `--streams` HIP streams with their own buffers, so one batch's fan-out overlaps the
    # next batch's match kernel.  Every step writes both summaries; all must be complete.
    # dedicated streams (not the null stream: the engine maps a null stream to its own one, so
    # events recorded there would not follow the calls)
    streams = [torch.cuda.Stream(device=dev) for _ in range(args.streams)]
    bufs = [(moff, mids, ooff, osubs, ofil)] + [tuple(torch.empty_like(t) for t in (moff, mids, ooff, osubs, ofil))
                                                for _ in range(args.streams - 1)]
    msum = torch.zeros((max(args.steps, 1), eng.SUMMARY_WORDS), dtype=torch.int64, device=dev)
    fsum = torch.zeros((max(args.steps, 1), st.SUMMARY_WORDS), dtype=torch.int64, device=dev)
    for j in range(1, len(streams)):  # size each stream's workspace once
        b = bufs[j]
        eng.match_device(tb.data_ptr(), to.data_ptr(), n, b[0].data_ptr(), b[1].data_ptr(), mcap, mode=0,
                         stream=streams[j].cuda_stream)
        st.fanout_device(args.strategy, b[0].data_ptr(), b[1].data_ptr(), n, keys.data_ptr(), b[2].data_ptr(),
                         b[3].data_ptr(), b[4].data_ptr(), ocap, stream=streams[j].cuda_stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for k in range(args.steps):
        j = k % len(streams)
        b, s = bufs[j], streams[j].cuda_stream
        eng.match_device_async(tb.data_ptr(), to.data_ptr(), n, b[0].data_ptr(), b[1].data_ptr(), mcap,
                               msum[k].data_ptr(), mode=0, stream=s)
        st.fanout_device_async(args.strategy, b[0].data_ptr(), b[1].data_ptr(), n, mcap, keys.data_ptr(),
                               b[2].data_ptr(), b[3].data_ptr(), b[4].data_ptr(), ocap, fsum[k].data_ptr(), stream=s)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    ms_, fs_ = msum.cpu().numpy(), fsum.cpu().numpy()
    if args.steps and not ((ms_[:, 0] == 0).all() and (ms_[:, 1] == nm).all() and (fs_[:, 0] == 0).all()
                           and (fs_[:, 1] == nd).all()):
        raise SystemExit("async match/fan-out steps incomplete or inconsistent")
    # call times from synchronous steps
    kern = []
    for _ in range(min(max(args.steps, 1), 10)):
        step()
        ev[1].synchronize()
        fo_ms.append(ev[0].elapsed_time(ev[1]))
        kern.append(eng.stats()["last_match_ms"])
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    fo = float(np.median(fo_ms))
    froof = fanout_roofline(fo, nm, nd, n, args)
    res = {
        "metric": "published topics matched and fanned out/sec (config E, 10M subscriptions)",
        "value": round(n * world * args.steps / elapsed, 1), "unit": "topics/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32", "data": "synthetic",
        "config": {"workload": "E: end-to-end publish fan-out, match -> subscriber ids incl. $share, 10M subs",
                   "n_filters": fw.wl.n_filters, "subscriptions": fw.n_subscriptions, "batch_topics_per_gpu": n,
                   "strategy": args.strategy, "publishers": args.publishers or "generated keys (~1M)",
                   "parallelism": f"replicated tables, topic stream split x{world}"},
        "deliveries_per_s": round(nd * world * args.steps / elapsed, 1),
        "matches_per_topic": round(nm / n, 3), "deliveries_per_topic": round(nd / n, 3),
        "match_call_ms": round(float(np.median(kern)), 4), "fanout_call_ms": round(fo, 4),
        "roofline": froof,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        k = min(args.cpu_sample, n)
        off_g = ooff[: k + 1].cpu().numpy().view(np.uint64)
        tot_k = int(off_g[-1])
        gpu = (off_g, osubs[:tot_k].cpu().numpy().view(np.uint32), ofil[:tot_k].cpu().numpy().view(np.uint32))
        res["cpu_baseline"] = fanout_cpu_baseline(fw, args, gpu)
        if "parity" in res["cpu_baseline"]:
            res["parity"] = res["cpu_baseline"].pop("parity")
        if args.strategy == "round_robin":
            res["parity"] = round_robin_parity(fw, args, st, moff, mids, keys, ooff, osubs, ofil, ocap, stream, n)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def round_robin_parity(fw, args, st, moff, mids, keys, ooff, osubs, ofil, ocap, stream, n):
    """Config E's round_robin pick by pick: the round_robin state of every
    publisher forgotten on the device, then two fan-out calls over the batch's match CSR (the
    second continues the state of the first), each against the oracle's restatement of
    do_pick_subscriber/6 with the counter seeded 0 (oracle/fanout_oracle.cpp
    orf_publish_list_rr; apps/emqx/src/emqx_shared_sub.erl:265-285) run over the oracle's own
    match of the same topics: every (subscriber, filter | shared) delivery of every topic, as a
    per-topic multiset (oracle/cpp.py pair_csr_mismatches)."""
    from emqx_amd import workloads as W
    from oracle import cpp as C
    k = min(args.cpu_sample, n)
    o = C.CppOracle(True)
    with progress("E round_robin parity: building the oracle table"):
        o.add_packed(*fw.wl.filters)
        o.freeze()
    m_off, m_ids, _ = o.match_csr(*W.take(fw.wl.topics, np.arange(k)), mode=0, threads=host_threads()[0])
    fo = C.FanoutOracle(fw.sub_filter, fw.sub_id, fw.sub_group)
    st.forget_publishers(np.unique(fw.keys))
    nm = int(moff[k].item())
    bad, checked, picks = [], 0, 0
    for call in range(2):
        nd = st.fanout_device("round_robin", moff.data_ptr(), mids.data_ptr(), k, keys.data_ptr(), ooff.data_ptr(),
                              osubs.data_ptr(), ofil.data_ptr(), ocap, stream=stream)
        off_g = ooff[: k + 1].cpu().numpy().view(np.uint64)
        subs_g = osubs[:nd].cpu().numpy().view(np.uint32)
        fils_g = ofil[:nd].cpu().numpy().view(np.uint32)
        off_o, subs_o, fils_o = fo.publish_list(m_off, m_ids, fw.keys[:k], round_robin=True)
        bad.append(int(C.pair_csr_mismatches(off_g, subs_g, fils_g, off_o, subs_o, fils_o).size))
        checked += int(nd)
        picks += int(np.count_nonzero(fils_o & np.uint32(0x80000000)))
    res = {"rule": "round_robin (counter seeded 0) pick by pick: every (subscriber, filter|shared) delivery per "
                   "topic vs oracle/fanout_oracle.cpp orf_publish_list_rr, two calls carrying the state",
           "topics_checked": int(k), "calls": 2, "match_ids": nm, "deliveries_checked": checked,
           "share_picks_checked": picks, "mismatches": int(sum(bad)), "mismatches_per_call": bad}
    if sum(bad):
        raise SystemExit(f"round_robin fan-out differs from the oracle: {bad}")
    return res


def fanout_roofline(fo_ms, nm, nd, n, args):
    """The fan-out call's roofline: streaming HBM work (entry scan, record loads, plain-list
    copies, delivery writes).  `traffic` = FETCH_SIZE + WRITE_SIZE summed over the call's
    kernels from the committed PMC passes on this workload (profiles/pmc_fanout_E.json,
    tools/pmc_fanout.py), scaled to the batch; `achieved` = those bytes / the call's live time
    (HIP events around the synchronous call); peak = 8 TB/s.  The algorithmic model (32 B per
    match entry + 12 B per delivery) is kept as `model_bytes`."""
    alg = 32 * nm + 12 * nd
    model_gbs = alg / (fo_ms * 1e-3) / 1e9
    model = {"achieved": round(model_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
             "frac": round(model_gbs / HBM_PEAK_GBS, 4), "alg_bytes_per_call": alg,
             "rule": "32 B per match entry (id, record, offsets, topic) + 12 B per delivery (plain-list read, two writes)"}
    path = os.path.join(ROOT, "profiles", "pmc_fanout_E.json")
    p = None
    if os.path.exists(path):
        with open(path) as f:
            p = json.load(f)
        if p.get("strategy") != args.strategy or p.get("batch_topics") != n:
            p = None
    if p is None:
        return {"bound": "hbm", "achieved": model["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": model["frac"], "traffic": None, "kernel": "fan-out call (all its kernels)",
                "kernel_ms_avg": round(fo_ms, 4), "basis": "model bytes (no committed PMC passes for this workload)",
                "model_bytes": model}
    traffic = p["traffic_bytes_per_call"]
    gbs = traffic / (fo_ms * 1e-3) / 1e9
    return {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": traffic,
            "traffic_source": "profiles/pmc_fanout_E.json (%s; %s)" % (p["traffic_rule"], p["source"]),
            "kernel": "fan-out call (all its kernels)", "kernel_ms_avg": round(fo_ms, 4),
            "basis": "counted HBM bytes (FETCH_SIZE + WRITE_SIZE over the call's kernels) / call time",
            "per_kernel_bytes": p.get("per_kernel_bytes"), "model_bytes": model}


def fanout_cpu_baseline(fw, args, gpu=None):
    """Host restatement of publish/1's lookup + dispatch on a bounded sample, one thread per
    host core: the C++ port of emqx_trie's DFS + match_routes/1 (oracle/trie_oracle.cpp), then
    route/aggre/do_dispatch and the hash $share pick per matched filter
    (oracle/fanout_oracle.cpp).  `gpu` = (offsets, subs, filters) of the GPU's fan-out of the
    same batch: per-topic delivery counts and multiset checksums must be equal (hash
    strategies are deterministic given the caller's phash2 key)."""
    from emqx_amd import workloads as W
    from oracle import cpp as C
    o = C.CppOracle(True)
    with progress("E baseline: building the oracle table"):
        o.add_packed(*fw.wl.filters)
        o.freeze()
    fo = C.FanoutOracle(fw.sub_filter, fw.sub_id, fw.sub_group)
    sample = min(args.cpu_sample, fw.wl.n_topics)
    s = W.take(fw.wl.topics, np.arange(sample))
    threads = args.cpu_threads or host_threads()[0]
    t0 = time.perf_counter()
    moff, mids, _ = o.match_csr(*s, mode=0, threads=threads)
    counts, sums, total = fo.publish(moff, mids, fw.keys[:sample], threads=threads)
    dt = time.perf_counter() - t0
    res = {"value": round(sample / dt, 1), "unit": "topics/s", "cores": threads, "kind": "port",
           "sample": f"first {sample} topics; C++ DFS match + C++ route/dispatch with hash $share picks",
           "deliveries_per_topic": round(total / max(sample, 1), 3)}
    if gpu is not None:
        off_g, subs_g, fils_g = gpu
        off_g = off_g[: sample + 1]
        cnt_bad = np.diff(off_g.astype(np.int64)) != counts.astype(np.int64)
        if args.strategy in ("hash_clientid", "hash_topic", "hash"):
            gsum = C.delivery_checksums(off_g, subs_g, fils_g)
            bad = np.nonzero(cnt_bad | (gsum != sums))[0]
            rule = "per-topic delivery count + order-free multiset checksum of (subscriber, filter)"
        else:  # round_robin / sticky / random picks: exact parity is the GPU tests' (replayed draws)
            bad = np.nonzero(cnt_bad)[0]
            rule = ("per-topic delivery count (the picks of stateful / random strategies are checked pick by "
                    "pick in tests/test_gpu_share_parity.py)")
        res["parity"] = {"topics_checked": int(sample), "deliveries_checked": int(total), "mismatches": int(bad.size),
                         "rule": rule}
        if bad.size:
            raise SystemExit(f"GPU fan-out differs from the oracle on {bad.size} topics, first {bad[:10].tolist()}")
    return res


def update_bench(args, rank, world, dev):
    """Route updates (emqx_router:do_add_route/do_delete_route ->
    emqx_trie:insert/delete in a mria transaction, emqx_router_utils.erl:33-70): on config B's
    10M-filter table, each step unsubscribes `churn` random live filters, subscribes `churn`
    new ones and commits (incremental: flag flips for the deletes, the new filters patched into
    the committed table in place, emqx_amd/csrc/live_trie.cpp).  value =
    (inserts + deletes) / (time of the ops and their commits).  After the last commit the batch
    is matched on the patched table and again after a full rebuild: the two CSRs must be
    identical (ids sorted per topic), and both throughputs are reported.  --with-matches keeps
    a 1M-topic match call in flight on a second stream during every commit (commits no longer
    drain the device)."""
    import torch
    import torch.distributed as dist
    from emqx_amd import workloads as W
    from emqx_amd.engine import Engine
    k, R = args.churn, args.rounds
    t0 = time.time()
    wl = load_or_make(args, rank, lambda: W.config_b(n_filters=args.n_filters + (R + 1) * k, n_topics=args.batch,
                                                     seed=2, topic_seed=None if rank == 0 else 1000 + rank))
    nb = wl.n_filters - (R + 1) * k
    base = W.take(wl.filters, np.arange(nb))
    log(f"[rank {rank}] workload: {nb} base filters + {(R + 1) * k} to subscribe ({time.time() - t0:.1f}s)")
    eng = Engine(dev.index)
    eng.insert_packed(*base)
    eng.commit()
    full_ms = eng.stats()["last_build_ms"]
    rng = np.random.default_rng(7 + rank)
    live = np.ones(nb, dtype=bool)
    nxt = nb

    side = None
    if args.with_matches:  # a match call in flight on another stream during each commit
        side_stream = torch.cuda.Stream(device=dev)
        stb = torch.from_numpy(wl.topics[0]).to(dev)
        sto = torch.from_numpy(wl.topics[1].view(np.int64)).to(dev)
        sn = wl.n_topics
        soff = torch.empty(sn + 1, dtype=torch.int64, device=dev)
        scap = max(64 * sn, 1 << 20)
        sids = torch.empty(scap, dtype=torch.int32, device=dev)
        ssum = torch.zeros(eng.SUMMARY_WORDS, dtype=torch.int64, device=dev)
        eng.match_device(stb.data_ptr(), sto.data_ptr(), sn, soff.data_ptr(), sids.data_ptr(), scap, mode=0,
                         stream=side_stream.cuda_stream)
        side = lambda: eng.match_device_async(stb.data_ptr(), sto.data_ptr(), sn, soff.data_ptr(), sids.data_ptr(),
                                              scap, ssum.data_ptr(), mode=0, stream=side_stream.cuda_stream)

    def churn_once():
        nonlocal nxt
        dels = np.sort(rng.choice(np.nonzero(live)[0], k, replace=False)).astype(np.uint32)
        adds = W.take(wl.filters, np.arange(nxt, nxt + k))
        nxt += k
        if side is not None:
            side()
        t = time.perf_counter()
        eng.delete(dels)
        ids = eng.insert_packed(*adds)
        eng.commit()
        dt = time.perf_counter() - t
        live[dels[dels < nb]] = False
        return dt, ids

    churn_once()  # warm-up commit
    if world > 1:
        dist.barrier()
    times, kinds, commit_ms, cst = [], [], [], []
    for r in range(R):
        dt, _ = churn_once()
        st = eng.stats()
        times.append(dt)
        kinds.append(st["last_commit_kind"])
        commit_ms.append(st["last_build_ms"])
        cst.append(eng.commit_stats())
        if r % 10 == 9:
            log(f"[rank {rank}] commit {r + 1}/{R}: {dt * 1e3:.1f} ms ({cst[-1]})")
    elapsed = float(np.sum(times))
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    if not all(x == 1 for x in kinds):
        raise SystemExit(f"expected incremental commits, got kinds {kinds}")
    delta_filters = eng.stats()["delta_filters"]

    tb = torch.from_numpy(wl.topics[0]).to(dev)
    to = torch.from_numpy(wl.topics[1].view(np.int64)).to(dev)
    n = wl.n_topics
    # the timed steps rotate over distinct batches (batch 0 = the one the baselines and the
    # parity check use); every batch has n topics
    batches = [(tb, to)] + [(torch.from_numpy(b[0]).to(dev), torch.from_numpy(b[1].view(np.int64)).to(dev))
                            for b in getattr(wl, "extra_topics", [])[: max(args.batches, 1) - 1]
                            if len(b[1]) - 1 == n]
    stream = torch.cuda.current_stream().cuda_stream

    def match_rate():
        d_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
        cap = max(64 * n, 1 << 20)
        d_ids = torch.empty(cap, dtype=torch.int32, device=dev)
        nout = eng.match_device(tb.data_ptr(), to.data_ptr(), n, d_off.data_ptr(), d_ids.data_ptr(), cap,
                                mode=0, stream=stream)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(args.steps):
            eng.match_device(tb.data_ptr(), to.data_ptr(), n, d_off.data_ptr(), d_ids.data_ptr(), cap,
                             mode=0, stream=stream)
        torch.cuda.synchronize()
        rate = n * args.steps / (time.perf_counter() - t)
        off = d_off.cpu().numpy()
        ids = d_ids[:nout].cpu().numpy().view(np.uint32).astype(np.int64)
        topic = np.repeat(np.arange(n, dtype=np.int64), np.diff(off))
        key = np.sort(topic << 32 | ids)  # per-topic sorted id sets, as one array
        return rate, eng.stats()["last_kernel_ms"], off, key

    torch.cuda.synchronize()
    rate_delta, kms_delta, off_d, key_d = match_rate()
    eng.set_tuning("incremental", 0)
    eng.commit()
    rebuild_ms = eng.stats()["last_build_ms"]
    rate_full, kms_full, off_f, key_f = match_rate()
    if not (np.array_equal(off_d, off_f) and np.array_equal(key_d, key_f)):
        raise SystemExit("match CSR of the patched table differs from the one after a full rebuild")

    value = 2.0 * k * R * world / elapsed
    result = {
        "metric": "route updates committed/sec (subscribe + unsubscribe, incremental commit) at 10M subs",
        "value": round(value, 1),
        "unit": "updates/s",
        "n_gpus": world,
        "steps": R,
        "warmup": 1,
        "ms_per_step": round(1e3 * elapsed / R, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic",
        "config": {"workload": "U: config B table, churn of subscribe/unsubscribe batches with a commit each",
                   "n_filters": nb, "churn_per_commit": k, "commits": R,
                   "parallelism": f"replicated table x{world} (each rank commits its own copy)"},
        "commit_ms_avg": round(float(np.mean(commit_ms)), 3),
        "commit_ms_p50": round(float(np.median(commit_ms)), 3),
        "commit_ms_max": round(float(np.max(commit_ms)), 3),
        "commit_ms_first5": round(float(np.mean(commit_ms[:5])), 3),
        "commit_ms_last5": round(float(np.mean(commit_ms[-5:])), 3),
        "step_ms_first5": round(1e3 * float(np.mean(times[:5])), 3),
        "step_ms_last5": round(1e3 * float(np.mean(times[-5:])), 3),
        "per_commit": {k: round(float(np.mean([c[k] for c in cst])), 1)
                       for k in ("relocations", "in_place", "patches", "new_slots", "host_us", "extents",
                                 "vocab_slots", "upload_us")},
        "spare_used_at_end": cst[-1]["spare_used"], "spare_cap": cst[-1]["spare_cap"],
        "full_rebuild_ms": round(min(full_ms, rebuild_ms), 1),
        "filters_patched_in_since_build": delta_filters,
        "match_topics_per_s_after_patches": round(rate_delta, 1),
        "match_topics_per_s_after_rebuild": round(rate_full, 1),
        "kernel_ms_after_patches": round(kms_delta, 4),
        "kernel_ms_after_rebuild": round(kms_full, 4),
        "matches_in_flight_during_commits": bool(args.with_matches),
        "parity": "CSR of the patched table == CSR after a full rebuild (per-topic sorted ids)",
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = update_cpu_baseline(wl, nb, k, args)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def retain_bench(args, rank, world, dev):
    """Retained-message lookup (emqx_retainer:dispatch/4 ->
    emqx_retainer_mnesia:match_messages/3 / read_message/2): a subscribe burst of
    `--batch` (default 100k) config-B subscription filters (exact / '+' / '#' mix) against
    `--retained` stored retained topics (config B's topic generator, 10% with an expiry).
    A step = one emqx_retain_match_batch_device call on the resident batch -> CSR of topic
    ids in HBM.  Replicated store: each rank answers its own filter batch (weak scaling)."""
    import torch
    import torch.distributed as dist
    from emqx_amd import workloads as W
    from emqx_amd.engine import pack
    from emqx_amd.retainer import RetainIndex
    from emqx_amd._lib import EngineError
    nf = args.batch if args.batch != 1_000_000 else 100_000
    t0 = time.time()
    topics_wl = W.config_b(n_filters=max(args.retained // 10, 1000), n_topics=int(args.retained * 1.15), seed=41)
    names = W.unpack(topics_wl.topics)
    names = list(dict.fromkeys(names))[: args.retained]
    filt_wl = W.config_b(n_filters=nf, n_topics=1000, seed=42 + rank)
    rng = np.random.default_rng(5)
    now = 1_000_000
    expiry = np.where(rng.random(len(names)) < 0.1, now - 500 + rng.integers(0, 1000, len(names)), 0).astype(np.int64)
    log(f"[rank {rank}] retained store: {len(names)} topics, {nf} filters ({time.time() - t0:.1f}s)")
    idx = RetainIndex(dev.index)
    for key, v in (("tile", args.retain_tile), ("step_budget", args.retain_budget)):
        if v is not None:
            idx.set_tuning(key, v)
    tb, to = pack(names)
    idx.store_packed(tb, to, expiry)
    idx.commit()
    st = idx.stats()
    log(f"[rank {rank}] index: {st['n_nodes']} nodes, {st['n_words']} words, {st['table_bytes'] / 1e6:.1f} MB, "
        f"build {st['last_build_ms']:.0f} ms")
    fb, fo = filt_wl.filters
    d_fb = torch.from_numpy(fb.copy()).to(dev)
    d_fo = torch.from_numpy(fo.view(np.int64).copy()).to(dev)
    d_off = torch.empty(nf + 1, dtype=torch.int64, device=dev)
    cap = 1 << 24
    d_ids = torch.empty(cap, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream().cuda_stream

    def step(o=None, ids=None, st_=None):
        o = d_off if o is None else o
        ids = d_ids if ids is None else ids
        return idx.match_device(d_fb.data_ptr(), d_fo.data_ptr(), nf, now, o.data_ptr(), ids.data_ptr(), cap,
                                stream=stream if st_ is None else st_)

    try:
        nout = step()
    except EngineError as err:
        cap = int(err.needed * 1.25) + 1024
        d_ids = torch.empty(cap, dtype=torch.int32, device=dev)
        nout = step()
    for _ in range(max(args.warmup, 1)):
        step()
    torch.cuda.synchronize()
    # the call's own time (HIP events, one caller): roofline and the per-call fields
    call_ms, walk_ms = [], []
    for _ in range(min(args.steps, 10)):
        step()
        s2 = idx.stats()
        call_ms.append(s2["last_match_ms"])
        walk_ms.append(s2["last_walk_ms"])
    # throughput: `--streams` concurrent callers (host threads, each its own stream and output
    # buffers; a call holds one of the index's work areas and synchronizes its own stream), as a
    # subscribe burst from many channels reaches the retainer; ctypes releases the GIL in a call
    import threading
    ncall = max(1, min(args.streams, args.steps))
    cstreams = [torch.cuda.Stream(device=dev) for _ in range(ncall)]
    cbufs = [(d_off, d_ids)] + [(torch.empty_like(d_off), torch.empty_like(d_ids)) for _ in range(ncall - 1)]
    per = [args.steps // ncall + (1 if i < args.steps % ncall else 0) for i in range(ncall)]
    errs = []

    def worker(i):
        try:
            for _ in range(per[i]):
                step(cbufs[i][0], cbufs[i][1], cstreams[i].cuda_stream)
        except Exception as e:  # noqa: BLE001 - re-raised below
            errs.append(e)

    for i in range(ncall):  # each caller's first call outside the timed region
        step(cbufs[i][0], cbufs[i][1], cstreams[i].cuda_stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t_start = time.perf_counter()
    threads = [threading.Thread(target=worker, args=(i,)) for i in range(ncall)]
    for th in threads:
        th.start()
    for th in threads:
        th.join()
    torch.cuda.synchronize()
    if errs:
        raise errs[0]
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    st = idx.stats()
    visits, ranges = st["last_visits"], st["last_ranges"]
    levels = int(np.count_nonzero(fb[: int(fo[-1])] == ord("/"))) + nf
    # algorithmic bytes of one call: filter bytes, one 32-B vocab slot per level, per node visit
    # its 16-B record and one 16-B edge probe, 16 B per range written + read twice, and per id
    # out: rank_id read + id write (+ 8 B expiry read under the guard), offsets
    alg = int(fo[-1]) + 32 * levels + 32 * visits + 48 * ranges + 16 * nout + 16 * nf
    cms = float(np.median(call_ms))
    achieved = alg / (cms * 1e-3) / 1e9
    value = nf * args.steps * world / elapsed
    result = {
        "metric": "subscription filters resolved against the retained store /sec (retained lookup, 1M retained topics)",
        "value": round(value, 1), "unit": "filters/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u32", "data": "synthetic",
        "config": {"workload": "R: retained lookup, config-B subscription filters vs config-B topics stored retained",
                   "retained_topics": len(names), "filters_per_call": nf,
                   "parallelism": f"replicated store x{world}"},
        "ids_per_s": round(nout * args.steps * world / elapsed, 1),
        "ids_per_filter": round(nout / nf, 3), "node_visits_per_filter": round(visits / nf, 3),
        "ranges_per_filter": round(ranges / nf, 3), "call_ms_median": round(cms, 4),
        "callers": ncall, "callers_note": "value: `callers` concurrent callers (threads, one stream each); "
                                          "call_ms_median / walk_ms_median / roofline: one caller alone",
        "walk_ms_median": round(float(np.median(walk_ms)), 4),
        "walk_balance": "spill rounds" if os.environ.get("EMQX_RETAIN_BALANCE") == "0" else "work-sharing queue",
        "walk_spill_rounds": int(st["last_spill_rounds"]), "walk_spilled_items": int(st["last_spilled"]),
        "walk_shares": int(st.get("last_shares", 0)), "walk_queue_aborts": int(st.get("queue_aborts", 0)),
        "walk_step_budget": (args.retain_budget if args.retain_budget is not None else "24, spill rounds 64 (default)")
        if os.environ.get("EMQX_RETAIN_BALANCE") == "0" else None,
        "walk_spill_full": int(st.get("last_spill_full", 0)),
        "walk_tile_filters": args.retain_tile if args.retain_tile is not None
        else (10 if os.environ.get("EMQX_RETAIN_BALANCE") == "0" else 16),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": retain_traffic(nf, len(names))[0],
                     "traffic_source": retain_traffic(nf, len(names))[1],
                     "kernel": ("retain_walk_kernel (+ spill rounds)" if os.environ.get("EMQX_RETAIN_BALANCE") == "0"
                                else "retain_walk_queue_kernel (work-sharing walk) + retain_queue_clear_kernel")
                     + " + retain_out_kernel<0,1> (whole call, one host sync)",
                     "alg_bytes_per_launch": alg,
                     "alg_bytes_model": "len(F) + 32*L(F) + 32*visits + 48*ranges + 16*ids + 16 per filter"},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import cpp as C
        sc = C.RetainScan(tb, to, expiry)
        sample = min(2000, nf)
        sfb, sfo = W.take(filt_wl.filters, np.arange(sample))
        threads = args.cpu_threads or host_threads()[0]
        t1 = time.perf_counter()
        counts, sums = sc.select_packed(sfb, sfo, now, threads=threads)
        dt = time.perf_counter() - t1
        off = d_off[: sample + 1].cpu().numpy()
        ids = d_ids[: int(off[-1])].cpu().numpy().view(np.uint32).astype(np.uint64)
        cs = np.concatenate([np.zeros(1, np.uint64), np.cumsum(ids, dtype=np.uint64)])
        gsum = cs[off[1:]] - cs[off[:-1]]
        gcnt = np.diff(off)
        if not (np.array_equal(gcnt, counts.astype(np.int64)) and np.array_equal(gsum, sums)):
            raise SystemExit("retained lookup differs from the CPU port on the baseline sample")
        result["cpu_baseline"] = {"value": round(sample / dt, 1), "unit": "filters/s", "cores": threads,
                                  "kind": "port",
                                  "sample": f"first {sample} filters; full-table match-spec scan per wildcard "
                                            "filter, key read per plain one (mnesia set table), C++",
                                  "parity": "per-filter count and id sum equal the GPU's"}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def update_cpu_baseline(wl, nb, k, args):
    """emqx_trie:insert/delete (refcounted TOPIC/PREFIX keys in one ordered key set,
    oracle/trie_oracle.cpp) for the same churn on the same base table, one writer thread (the
    reference serialises each route change in a mria transaction; one ordered set takes one
    writer at a time): rounds of `k` deletes + `k` inserts for about 10 s."""
    from emqx_amd import workloads as W
    from oracle import cpp as C
    o = C.CppOracle(True)
    with progress("update baseline: building the oracle table"):
        o.add_packed(*W.take(wl.filters, np.arange(nb)))
    rng = np.random.default_rng(11)
    pool = wl.n_filters - k
    t_total, ops, r = 0.0, 0, 0
    while t_total < 10.0 and r < 50:
        dels = W.unpack(wl.filters, rng.choice(nb, k, replace=False))
        adds = W.take(wl.filters, np.arange(pool, pool + k))
        t = time.perf_counter()
        o.delete(dels)
        o.add_packed(*adds)
        t_total += time.perf_counter() - t
        o.delete(W.unpack(adds))
        o.add(dels)
        ops += 2 * k
        r += 1
    return {"value": round(ops / t_total, 1), "unit": "updates/s", "cores": 1, "kind": "port",
            "sample": f"{r} rounds of {k} deletes + {k} inserts on the same {nb}-filter table (C++ restatement "
                      "of emqx_trie:insert/delete key maintenance, no mnesia transaction, one writer)"}


def set_walk_order(eng, args):
    eng.set_tuning("order", {"auto": -1, "on": 1, "off": 0}[args.walk_order])
    eng.set_tuning("order_level_bits", args.walk_level_bits)
    eng.set_tuning("order_sort_bits", args.walk_sort_bits)
    eng.set_tuning("order_deal", args.walk_deal)


def walk_order_desc(args, st):
    """The engine's walk order for this table (engine.cpp use_order: auto = tables deeper than
    12 levels, batches of >= 65536 topics)."""
    on = args.walk_order == "on" or (args.walk_order == "auto" and st.get("max_depth", 0) > 12)
    if not on:
        return "batch order"
    lb = args.walk_level_bits or (4 if st.get("max_depth", 0) > 12 else 8)
    return (f"prefix-key order inside the call ({lb} bits per level, top {args.walk_sort_bits} bits sorted"
            f"{', tile ranges dealt to XCDs' if args.walk_deal else ''})")


def reorder_topics(wl, order):
    """A permutation of the same batch (the match sets per topic are unchanged)."""
    from emqx_amd import workloads as W
    names = W.unpack(wl.topics)
    idx = sorted(range(len(names)), key=names.__getitem__)
    if order == "xcd":
        n = len(idx)
        seg = [idx[k * n // 8:(k + 1) * n // 8] for k in range(8)]
        out, pos = [], [0] * 8
        while len(out) < n:
            for k in range(8):
                out.extend(seg[k][pos[k]:pos[k] + 256])
                pos[k] += 256
        idx = out
    return W.Workload(wl.name, wl.filters, W.take(wl.topics, np.asarray(idx)))


def load_or_make(args, rank, make, batches=1):
    from emqx_amd.workloads import Workload
    path = f"{args.cache}.{rank}.npz" if args.cache else None
    if path and os.path.exists(path):
        z = np.load(path)
        wl = Workload("B", (z["fb"], z["fo"]), (z["tb"], z["to"]))
        wl.extra_topics = [(z[f"tb{j}"], z[f"to{j}"]) for j in range(1, 64) if f"tb{j}" in z]
        if len(wl.extra_topics) + 1 >= batches:
            return wl
    wl = make()
    if path:
        extra = {}
        for j, (tb, to) in enumerate(getattr(wl, "extra_topics", []), 1):
            extra[f"tb{j}"], extra[f"to{j}"] = tb, to
        np.savez(path, fb=wl.filters[0], fo=wl.filters[1], tb=wl.topics[0], to=wl.topics[1], **extra)
    return wl


def ab_variants(eng, step, args, wl):
    """Interleaved rounds of every variant in one process (cdna_hip_programming.md §5.4
    rule 24): median/min of the fused kernel's HIP-event time and of the whole call."""
    import torch
    variants = [int(v) for v in args.ab.split(",")]
    res = {v: {"kernel_ms": [], "call_ms": [], "nout": None, "deferred": 0, "max_stack": 0} for v in variants}
    for v in variants:  # warm each variant once
        eng.set_tuning("fast_variant", v)
        step()
    for _ in range(args.ab_rounds):
        for v in variants:
            eng.set_tuning("fast_variant", v)
            for _ in range(max(1, args.steps // args.ab_rounds)):
                nout = step()
                st = eng.stats()
                r = res[v]
                r["kernel_ms"].append(st["last_kernel_ms"])
                r["call_ms"].append(st["last_match_ms"])
                r["nout"] = nout
                r["deferred"] = max(r["deferred"], st["last_deferred"])
                r["max_stack"] = max(r["max_stack"], st["last_max_stack"])
    torch.cuda.synchronize()
    out = {}
    for v, r in res.items():
        out[v] = {"kernel_ms_median": round(float(np.median(r["kernel_ms"])), 4),
                  "kernel_ms_min": round(float(np.min(r["kernel_ms"])), 4),
                  "call_ms_median": round(float(np.median(r["call_ms"])), 4),
                  "topics_per_s_call": round(wl.n_topics / (float(np.median(r["call_ms"])) * 1e-3), 1),
                  "nout": r["nout"], "deferred": r["deferred"], "max_stack": r["max_stack"]}
    eng.set_tuning("fast_variant", -1)
    print(json.dumps({"ab": out, "n_filters": wl.n_filters, "batch": wl.n_topics}), flush=True)


def host_threads():
    """Threads for the CPU baseline: the host cores this process may use (its affinity set,
    capped by a cgroup CPU quota when one is set, as on the GPU box's per-GPU CPU share);
    `nproc` (os.cpu_count()) is reported beside it."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = nproc
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or None
    t = aff
    for cap in (quota, share):
        if cap:
            t = min(t, cap)
    return max(1, t), {"nproc": nproc, "affinity": aff, "cgroup_quota": quota, "omp_num_threads": share}


def cpu_baseline(wl, args, gpu_csr=None):
    """emqx_trie compact-mode DFS (oracle/trie_oracle.cpp) + emqx_router exact union, timed on
    a bounded sample of the same batch with one thread per host core (kind "port": Erlang is
    absent on the GPU box).  The oracle emits the full sorted id set of every sampled topic
    (as match_routes/1 returns it); `gpu_csr` = (offsets, ids) of the GPU's call on the whole
    batch is compared with it ID-for-ID and the bench fails on any mismatch."""
    from emqx_amd import workloads as W
    from oracle import cpp as C
    t0 = time.time()
    o = C.CppOracle(True, trie_all=(args.mode == C.MODE_TRIE))
    with progress("cpu baseline: building the oracle table"):
        o.add_packed(*wl.filters)
        o.freeze()
    build_s = time.time() - t0
    sample = min(args.cpu_sample, wl.n_topics)
    s = W.take(wl.topics, np.arange(sample))
    threads, host = host_threads()
    if args.cpu_threads:
        threads = args.cpu_threads
    t0 = time.perf_counter()
    off_o, ids_o, lookups = o.match_csr(*s, mode=args.mode, threads=threads)
    dt = time.perf_counter() - t0
    log(f"cpu baseline: {sample} topics in {dt:.2f}s on {threads} threads (table build {build_s:.1f}s)")
    res = {"value": round(sample / dt, 1), "unit": "topics/s", "cores": threads, "kind": "port",
           "sample": f"first {sample} topics of the batch vs the full {wl.n_filters}-filter table",
           "host": host,
           "ets_lookups_per_topic": round(lookups / sample, 2),
           "matches_per_topic": round(float(off_o[-1]) / max(sample, 1), 3)}
    if gpu_csr is not None:
        off_g, ids_g = gpu_csr
        off_g = off_g[: sample + 1]
        bad = C.csr_mismatches(off_g, ids_g, off_o, ids_o)
        res["parity"] = {"topics_checked": int(sample), "ids_checked": int(off_o[-1]),
                         "mismatches": int(bad.size),
                         "rule": "per-topic sorted filter-id sets, GPU CSR vs the oracle (SURVEY §8 S7)"}
        if bad.size:
            raise SystemExit(f"GPU match sets differ from the oracle on {bad.size} of {sample} topics, "
                             f"first {bad[:10].tolist()}")
    return res

if __name__ == "__main__":
    main()

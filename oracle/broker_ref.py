"""CPU restatement of the reference's publish fan-out — TEST INFRASTRUCTURE ONLY.

Parity oracle for the GPU fan-out stage (emqx_amd/csrc/fanout_kernels.hip).  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it.

Restates (EMQX 5.0.0-beta.3, paths relative to ``/root/reference``):

* ``apps/emqx/src/emqx_broker.erl``
    - subscribe/3, do_subscribe/3,4   :124-163  (?SUBSCRIBER bag, {shard, I} buckets)
    - unsubscribe/1, do_unsubscribe   :169-195
    - publish/1                       :203-214  (route(aggre(match_routes(Topic))))
    - route/2, do_route/2, aggre/1    :244-272
    - dispatch/2, do_dispatch/2,3     :275-286,500-524
* ``apps/emqx/src/emqx_shared_sub.erl``
    - subscribe/unsubscribe handlers  :300-322  (bag keyed by Group; first member adds the
                                                 {Group, node()} route, the last one removes it)
    - dispatch/3,4                    :113-130  (a failed delivery retries with [SubPid | FailedSubs])
    - dispatch_per_qos/4              :147-163  (a {retry, Sub} pick is sent without an ack)
    - pick/6, do_pick/6               :234-263  (sticky: kept while is_active_sub/2; All -- FailedSubs,
                                                 [] -> {retry, pick over All})
    - pick_subscriber/6               :265-268
    - do_pick_subscriber/6            :270-285
    - subscribers/2                   :287-288  (ets:select -> members in insertion order)
    - cleanup_down/1                  :369-376  (a dead subscriber's shared subscriptions go)
    - is_active_sub/2, is_alive_sub/1 :385-393  (erlang:is_process_alive/1: liveness, not membership)
* ``apps/emqx/src/emqx_broker_helper.erl:81-86`` (get_sub_shard: storage split only)

``erlang:phash2`` (ERTS C, OTP 24.1.5) is NOT restated: the hash strategies take the
caller's phash2 value as ``key`` (the NIF computes ``erlang:phash2(ClientId)`` /
``erlang:phash2(Topic)`` in Erlang), so the pick ``lists:nth(1 + Key rem N, Subs)`` is exact.

``round_robin`` and ``sticky`` keep their state in the *publishing process's* dictionary under
``{shared_sub_round_robin | shared_sub_sticky, Group, Topic}`` (emqx_shared_sub.erl:234-247,
279-285): here a dict keyed ``(publisher, group, topic)``, where the publisher is the message's
``key`` (the engine's C ABI takes the publisher handle in the same per-message key slot for
these two strategies).  ``rand:uniform/1`` draws (round_robin's first index, random picks,
sticky's re-picks) come from ``draw(candidates) -> 0-based index`` (default 0), so a test can
replay the draw the device made: it returns the index of the device's pick among the candidate
list, which also checks that the device drew from the right candidates.
"""

from __future__ import annotations

from typing import Dict, List, Optional, Tuple

from .emqx_ref import Router

NODE = "emqx@127.0.0.1"

RANDOM, ROUND_ROBIN, STICKY, HASH_CLIENTID, HASH_TOPIC = 0, 1, 2, 3, 4


class SharedSub:
    """emqx_shared_sub's table: a bag of {Group, Topic, SubPid}; select order = insertion order
    among the objects of one key (ETS bag semantics).  ``dead``: subscribers whose process is
    down (is_alive_sub/1 false) and not yet cleaned up."""

    def __init__(self):
        self.tab: List[Tuple[object, bytes, object]] = []
        self.rr: Dict[Tuple[object, object, bytes], int] = {}      # (publisher, group, topic) -> Rem
        self.sticky: Dict[Tuple[object, object, bytes], object] = {}  # (publisher, group, topic) -> Sub
        self.dead: set = set()

    def subscribe(self, group, topic: bytes, sub) -> bool:
        """Returns True when this is the group's first member on `topic` (route to add)."""
        rec = (group, topic, sub)
        first = not any(g == group and t == topic for g, t, _ in self.tab)
        if rec not in self.tab:
            self.tab.append(rec)
        self.dead.discard(sub)  # a subscribing process is alive
        return first

    def unsubscribe(self, group, topic: bytes, sub) -> bool:
        """Returns True when the group has no member left on `topic` (route to delete)."""
        rec = (group, topic, sub)
        if rec in self.tab:
            self.tab.remove(rec)
        return not self.subscribers(group, topic)

    def subscribers(self, group, topic: bytes) -> list:
        return [s for g, t, s in self.tab if g == group and t == topic]

    def is_alive(self, sub) -> bool:
        """is_alive_sub/1 (:390-393); ``undefined`` (None: no sticky pick yet) is not a pid."""
        return sub is not None and sub not in self.dead

    def pick(self, strategy: int, key: int, group, topic: bytes, first=None, failed=(), draw=None):
        """pick/6 with FailedSubs = ``failed``: ``False`` when the group has no member, else the
        picked member (see ``pick_typed`` for the {fresh | retry, Sub} form).  ``first(n)``: the
        older form of ``draw`` (the 0-based index of a draw over n candidates)."""
        r = self.pick_typed(strategy, key, group, topic, failed, _draw(first, draw))
        return False if r is False else r[1]

    def pick_typed(self, strategy: int, key: int, group, topic: bytes, failed=(), draw=None):
        """pick/6 (:234-249): ``False`` or ``(type, sub)`` with type "fresh" | "retry"."""
        draw = draw or (lambda cands: 0)
        if strategy == STICKY:
            sk = (key, group, topic)
            sub0 = self.sticky.get(sk)
            if self.is_alive(sub0) and sub0 not in failed:  # is_active_sub(Sub0, FailedSubs)
                return ("fresh", sub0)
            r = self.do_pick(RANDOM, key, group, topic, [sub0] + list(failed), draw)
            if r is False:  # the reference would fail its {Type, Sub} match here
                return False
            self.sticky[sk] = r[1]
            return r
        return self.do_pick(strategy, key, group, topic, failed, draw)

    def do_pick(self, strategy: int, key: int, group, topic: bytes, failed, draw):
        """do_pick/6 (:251-263): Subs = All -- FailedSubs."""
        every = self.subscribers(group, topic)
        if not every:
            return False
        subs = [s for s in every if s not in failed]
        if not subs:  # all offline? pick one anyway
            return ("retry", self.pick_subscriber(group, topic, strategy, key, every, draw))
        return ("fresh", self.pick_subscriber(group, topic, strategy, key, subs, draw))

    def pick_subscriber(self, group, topic: bytes, strategy: int, key: int, subs: list, draw):
        """pick_subscriber/6 + do_pick_subscriber/6 (:265-285)."""
        if len(subs) == 1:  # the strategy is not consulted
            return subs[0]
        n = len(subs)
        if strategy in (HASH_CLIENTID, HASH_TOPIC):
            nth = 1 + key % n
        elif strategy == ROUND_ROBIN:
            rk = (key, group, topic)
            rem = (self.rr[rk] + 1) % n if rk in self.rr else draw(subs) % n
            self.rr[rk] = rem
            nth = rem + 1
        else:  # random (and sticky's re-pick): rand:uniform(Count)
            nth = 1 + draw(subs) % n
        return subs[nth - 1]

    def dispatch(self, strategy: int, key: int, group, topic: bytes, deliver, draw=None):
        """dispatch/3,4 (:113-130) with dispatch_per_qos/4 (:147-163): ``deliver(sub)`` is the
        outcome of a fresh delivery (dispatch_with_ack: True = acked); a {retry, Sub} pick is sent
        without an ack and succeeds.  Returns (attempts [(type, sub)], result)."""
        failed: list = []
        attempts = []
        while True:
            r = self.pick_typed(strategy, key, group, topic, failed, draw)
            if r is False:
                return attempts, ("error", "no_subscribers")
            attempts.append(r)
            typ, sub = r
            if typ == "retry" or deliver(sub):
                return attempts, ("ok", 1)
            failed = [sub] + failed

    def down(self, sub) -> None:
        """The subscriber's process ended; its records stay until cleanup_down/1 runs."""
        self.dead.add(sub)

    def cleanup_down(self, sub) -> list:
        """cleanup_down/1 (:369-376): the dead subscriber's shared subscriptions; returns the
        (group, topic) pairs left without members (routes to delete)."""
        gone = [(g, t) for g, t, s in self.tab if s == sub]
        for g, t in gone:
            self.tab.remove((g, t, sub))
        return [(g, t) for g, t in gone if not self.subscribers(g, t)]


def _draw(first, draw):
    if draw is not None:
        return draw
    if first is not None:
        return lambda cands: first(len(cands))
    return None


class Broker:
    """One node: the router, the ?SUBSCRIBER bag and the shared-subscription table."""

    def __init__(self, compact: bool = True):
        self.router = Router(compact)
        self.subscriber: Dict[bytes, list] = {}
        self.shared = SharedSub()

    def subscribe(self, topic: bytes, sub, group=None) -> None:
        if group is None:
            lst = self.subscriber.setdefault(topic, [])
            if sub not in lst:
                lst.append(sub)
                self.router.add_route(topic, NODE)  # emqx_broker: call(pick(Topic), {subscribe, Topic})
        else:
            if self.shared.subscribe(group, topic, sub):
                self.router.add_route(topic, (group, NODE))

    def unsubscribe(self, topic: bytes, sub, group=None) -> None:
        if group is None:
            lst = self.subscriber.get(topic, [])
            if sub in lst:
                lst.remove(sub)
                if not lst:
                    del self.subscriber[topic]
                    self.router.delete_route(topic, NODE)
        else:
            if self.shared.unsubscribe(group, topic, sub):
                self.router.delete_route(topic, (group, NODE))

    @staticmethod
    def aggre(routes) -> list:
        """emqx_broker.erl:261-272 (fold prepends; with >1 routes a group route usorts the acc)."""
        if not routes:
            return []
        if len(routes) == 1:
            to, dest = routes[0]
            return [(to, dest)] if isinstance(dest, str) else [(to, dest[0])]
        acc: list = []
        for to, dest in routes:
            if isinstance(dest, str):
                acc = [(to, dest)] + acc
            else:
                acc = sorted(set([(to, dest[0])] + acc), key=repr)
        return acc

    def down(self, sub) -> None:
        """A subscriber process ended (shared-subscription liveness; cleanup is separate)."""
        self.shared.down(sub)

    def cleanup_down(self, sub) -> None:
        """emqx_shared_sub:cleanup_down/1 for a dead subscriber (routes of emptied groups go)."""
        for group, topic in self.shared.cleanup_down(sub):
            self.router.delete_route(topic, (group, NODE))

    def publish(self, topic: bytes, key: int = 0, strategy: int = HASH_CLIENTID, first=None, draw=None):
        """Deliveries of one PUBLISH: list of (filter, subscriber, shared).  ``key`` as in
        SharedSub.pick; ``draw(candidates)`` (or the older ``first(n)``) replays rand draws."""
        out = []
        d = _draw(first, draw)
        for to, dest in self.aggre(self.router.match_routes(topic)):
            if dest == NODE:
                for sub in self.subscriber.get(to, []):  # do_dispatch/2 (shards flattened)
                    out.append((to, sub, False))
            else:
                sub = self.shared.pick(strategy, key, dest, to, draw=d)
                if sub is not False:
                    out.append((to, sub, True))
        return out

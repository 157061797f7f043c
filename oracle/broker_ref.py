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
    - subscribe/unsubscribe handlers  :300-314  (bag keyed by Group; first member adds the
                                                 {Group, node()} route, the last one removes it)
    - dispatch/3,4                    :113-126
    - pick/6, do_pick/6               :234-264
    - pick_subscriber/6               :266-269
    - do_pick_subscriber/6            :271-285
    - subscribers/2                   :287-288  (ets:select -> members in insertion order)
* ``apps/emqx/src/emqx_broker_helper.erl:81-86`` (get_sub_shard: storage split only)

``erlang:phash2`` (ERTS C, OTP 24.1.5) is NOT restated: the hash strategies take the
caller's phash2 value as ``key`` (the NIF computes ``erlang:phash2(ClientId)`` /
``erlang:phash2(Topic)`` in Erlang), so the pick ``lists:nth(1 + Key rem N, Subs)`` is exact.

``round_robin`` and ``sticky`` keep their state in the *publishing process's* dictionary under
``{shared_sub_round_robin | shared_sub_sticky, Group, Topic}`` (emqx_shared_sub.erl:234-247,
279-285): here a dict keyed ``(publisher, group, topic)``, where the publisher is the message's
``key`` (the engine's C ABI takes the publisher handle in the same per-message key slot for
these two strategies).  Their first pick is ``rand:uniform(N) - 1`` / a random member: the
oracle takes it from ``first(n)`` (default 0), so a test can seed it with the pick the device
made and check every later pick exactly.  ``random`` is checked by its distribution only.
"""

from __future__ import annotations

from typing import Dict, List, Optional, Tuple

from .emqx_ref import Router

NODE = "emqx@127.0.0.1"

RANDOM, ROUND_ROBIN, STICKY, HASH_CLIENTID, HASH_TOPIC = 0, 1, 2, 3, 4


class SharedSub:
    """emqx_shared_sub's table: a bag of {Group, Topic, SubPid}; select order = insertion order
    among the objects of one key (ETS bag semantics)."""

    def __init__(self):
        self.tab: List[Tuple[object, bytes, object]] = []
        self.rr: Dict[Tuple[object, object, bytes], int] = {}      # (publisher, group, topic) -> Rem
        self.sticky: Dict[Tuple[object, object, bytes], object] = {}  # (publisher, group, topic) -> Sub

    def subscribe(self, group, topic: bytes, sub) -> bool:
        """Returns True when this is the group's first member on `topic` (route to add)."""
        rec = (group, topic, sub)
        first = not any(g == group and t == topic for g, t, _ in self.tab)
        if rec not in self.tab:
            self.tab.append(rec)
        return first

    def unsubscribe(self, group, topic: bytes, sub) -> bool:
        """Returns True when the group has no member left on `topic` (route to delete)."""
        rec = (group, topic, sub)
        if rec in self.tab:
            self.tab.remove(rec)
        return not self.subscribers(group, topic)

    def subscribers(self, group, topic: bytes) -> list:
        return [s for g, t, s in self.tab if g == group and t == topic]

    def pick(self, strategy: int, key: int, group, topic: bytes, first=None):
        """pick/6 -> do_pick/6 with FailedSubs = [] (dispatch never fails here): ``False`` when
        the group has no member, else the picked member.  ``key``: phash2 value (hash
        strategies) or the publisher (round_robin, sticky).  ``first(n)``: the 0-based index the
        reference draws with rand:uniform(N) (default 0)."""
        subs = self.subscribers(group, topic)
        if not subs:
            return False
        n = len(subs)
        draw = (lambda k: 0) if first is None else first
        if strategy == STICKY:  # pick/6 :234-247; "active" = still subscribed to the group here
            sk = (key, group, topic)
            cur = self.sticky.get(sk)
            if cur is not None and cur in subs:
                return cur
            sub = subs[draw(n) % n] if n > 1 else subs[0]
            self.sticky[sk] = sub
            return sub
        if n == 1:  # pick_subscriber/6, first clause: the strategy is not consulted
            return subs[0]
        if strategy in (HASH_CLIENTID, HASH_TOPIC):
            nth = 1 + key % n
        elif strategy == ROUND_ROBIN:  # do_pick_subscriber/6 :279-285
            rk = (key, group, topic)
            rem = (self.rr[rk] + 1) % n if rk in self.rr else draw(n) % n
            self.rr[rk] = rem
            nth = rem + 1
        else:
            raise ValueError("random picks are not deterministic; test their distribution")
        return subs[nth - 1]


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

    def publish(self, topic: bytes, key: int = 0, strategy: int = HASH_CLIENTID, first=None):
        """Deliveries of one PUBLISH: list of (filter, subscriber, shared).  ``key`` as in
        SharedSub.pick; ``first(n)`` seeds a publisher's first round_robin / sticky pick."""
        out = []
        for to, dest in self.aggre(self.router.match_routes(topic)):
            if dest == NODE:
                for sub in self.subscriber.get(to, []):  # do_dispatch/2 (shards flattened)
                    out.append((to, sub, False))
            else:
                sub = self.shared.pick(strategy, key, dest, to, first)
                if sub is not False:
                    out.append((to, sub, True))
        return out

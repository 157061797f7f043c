"""``emqx_router`` API mirror (apps/emqx/src/emqx_router.erl:35-54) on the device engine.

The route table (a ``bag`` of ``#route{topic, dest}``, emqx_router.erl:75-83) stays on the
host as ``filter id -> [dest]``; the filter set itself lives in one engine snapshot that
holds every routed filter (exact and wildcard), so ``match_routes/1`` is one device match
in ``EMQX_MODE_ROUTES``: the exact filter equal to the topic ∪ the wildcard filters that
match it (emqx_router.erl:128-133), and only the exact filter for a wildcard topic (S3).
"""

from __future__ import annotations

import threading
from typing import Dict, List, NamedTuple, Optional, Sequence

from .engine import MODE_ROUTES, MODE_TRIE_WILDCARD, Engine, pack


class Route(NamedTuple):
    """#route{topic, dest} (apps/emqx/include/emqx.hrl)."""
    topic: bytes
    dest: object


class Router:
    def __init__(self, device: int = -1, node: object = "emqx@127.0.0.1"):
        self.node = node
        self._eng = Engine(device)
        self._dests: Dict[int, List[object]] = {}
        self._names: Dict[int, bytes] = {}
        self._dirty = False
        self._lock = threading.Lock()

    # emqx_router.erl:98-124
    def add_route(self, topic: bytes, dest: object = None) -> None:
        dest = self.node if dest is None else dest
        with self._lock:
            fid = self._eng.lookup(topic)
            lst = self._dests.get(fid) if fid is not None else None
            if lst and dest in lst:
                return
            if not lst:
                fid = int(self._eng.insert([topic])[0])
                self._names[fid] = topic
                self._dests[fid] = []
                self._dirty = True
            self._dests[fid].append(dest)

    do_add_route = add_route

    # emqx_router.erl:150-171
    def delete_route(self, topic: bytes, dest: object = None) -> None:
        dest = self.node if dest is None else dest
        with self._lock:
            fid = self._eng.lookup(topic)
            if fid is None:
                return
            lst = self._dests.get(fid, [])
            if dest not in lst:
                return
            lst.remove(dest)
            if not lst:
                del self._dests[fid]
                self._eng.delete([fid])
                self._dirty = True

    do_delete_route = delete_route

    def _sync(self) -> None:
        if self._dirty:
            with self._lock:
                if self._dirty:
                    self._eng.commit()
                    self._dirty = False

    # emqx_router.erl:142-148
    def lookup_routes(self, topic: bytes) -> List[Route]:
        fid = self._eng.lookup(topic)
        return [Route(topic, d) for d in self._dests.get(fid, [])] if fid is not None else []

    def has_routes(self, topic: bytes) -> bool:
        fid = self._eng.lookup(topic)
        return fid is not None and bool(self._dests.get(fid))

    def topics(self) -> List[bytes]:
        """emqx_router.erl:173-175."""
        return [self._names[f] for f in self._dests]

    # emqx_router.erl:127-133
    def match_routes(self, topic: bytes) -> List[Route]:
        return self.match_routes_batch([topic])[0]

    def match_filter_ids(self, topics: Sequence[bytes]):
        """CSR (offsets, ids) of the filters whose routes match_routes/1 returns."""
        self._sync()
        return self._eng.match_packed(*pack(list(topics)), mode=MODE_ROUTES)

    def match_routes_batch(self, topics: Sequence[bytes]) -> List[List[Route]]:
        off, ids = self.match_filter_ids(topics)
        out = []
        for i in range(len(topics)):
            routes: List[Route] = []
            for f in ids[off[i]:off[i + 1]]:
                name = self._names[int(f)]
                routes.extend(Route(name, d) for d in self._dests.get(int(f), []))
            out.append(routes)
        return out

    # emqx_router.erl:136-140 (private match_trie/1: wildcard filters only)
    def match_trie(self, topic: bytes) -> List[bytes]:
        self._sync()
        off, ids = self._eng.match_packed(*pack([topic]), mode=MODE_TRIE_WILDCARD)
        return [self._names[int(f)] for f in ids[off[0]:off[1]]]

    # emqx_router.erl:177-182
    def print_routes(self, topic: bytes) -> None:
        for r in self.match_routes(topic):
            print("%s -> %s" % (r.topic.decode(errors="replace"), r.dest))

    @property
    def engine(self) -> Engine:
        return self._eng


_default: Optional[Router] = None


def _router() -> Router:
    global _default
    if _default is None:
        _default = Router()
    return _default


def add_route(topic: bytes, dest=None) -> None:
    _router().add_route(topic, dest)


def delete_route(topic: bytes, dest=None) -> None:
    _router().delete_route(topic, dest)


def match_routes(topic: bytes) -> List[Route]:
    return _router().match_routes(topic)


def lookup_routes(topic: bytes) -> List[Route]:
    return _router().lookup_routes(topic)


def has_routes(topic: bytes) -> bool:
    return _router().has_routes(topic)


def topics() -> List[bytes]:
    return _router().topics()

"""``emqx_trie`` API mirror (apps/emqx/src/emqx_trie.erl:28-43) on the device engine.

The reference keeps one global trie table (plus session tries, emqx_trie.erl:50-52,
144-146); here a :class:`Trie` owns one engine snapshot, and the module-level functions
use a default instance for the main trie and a second one for the session trie.

Mutations are buffered and published by one batched rebuild (``commit``) the next time a
match needs them — the reference applies each insert/delete in its own mria transaction
(emqx_router_utils.erl:97-125).  ``match/1`` returns the filters ``emqx_trie:match/1``
returns (wildcard filters matching the topic; ``[]`` for wildcard topics), ``match_batch``
is the batched form the NIF serves.
"""

from __future__ import annotations

import threading
from typing import Dict, List, Optional, Sequence

from .engine import MODE_TRIE, Engine, pack


class Trie:
    def __init__(self, device: int = -1, compact: bool = True):
        # broker.perf.trie_compaction (emqx_trie.erl:336-340) changes the reference's DFS
        # order and cost only, never its result (emqx_trie_SUITE.erl:27-41); kept as a flag.
        self.compact = compact
        self._eng = Engine(device)
        self._dirty = False
        self._lock = threading.Lock()
        self._names: Dict[int, bytes] = {}

    # emqx_trie.erl:106-120 — idempotent insert
    def insert(self, topic: bytes) -> None:
        with self._lock:
            fid = int(self._eng.insert([topic])[0])
            self._names[fid] = topic
            self._dirty = True

    # emqx_trie.erl:122-137 — delete if present
    def delete(self, topic: bytes) -> None:
        with self._lock:
            fid = self._eng.lookup(topic)
            if fid is not None:
                self._eng.delete([fid])
                self._dirty = True

    def empty(self) -> bool:
        """emqx_trie.erl:164-171."""
        return self._eng.stats()["n_filters"] == 0

    def _sync(self) -> None:
        if self._dirty:
            with self._lock:
                if self._dirty:
                    self._eng.commit()
                    self._dirty = False

    def match(self, topic: bytes) -> List[bytes]:
        return self.match_batch([topic])[0]

    def match_batch(self, topics: Sequence[bytes]) -> List[List[bytes]]:
        self._sync()
        off, ids = self._eng.match_packed(*pack(list(topics)), mode=MODE_TRIE)
        names = self._names
        return [[names[int(f)] for f in ids[off[i]:off[i + 1]]] for i in range(len(topics))]

    def lookup_topic(self, topic: bytes) -> List[bytes]:
        """emqx_trie.erl:259-263: [Topic] when the filter is present."""
        return [topic] if self._eng.lookup(topic) is not None else []

    @property
    def engine(self) -> Engine:
        return self._eng


_default: Optional[Trie] = None
_session: Optional[Trie] = None


def _trie() -> Trie:
    global _default
    if _default is None:
        _default = Trie()
    return _default


def _session_trie() -> Trie:
    global _session
    if _session is None:
        _session = Trie()
    return _session


def insert(topic: bytes) -> None:
    _trie().insert(topic)


def delete(topic: bytes) -> None:
    _trie().delete(topic)


def match(topic: bytes) -> List[bytes]:
    return _trie().match(topic)


def empty() -> bool:
    return _trie().empty()


def insert_session(topic: bytes) -> None:
    _session_trie().insert(topic)


def delete_session(topic: bytes) -> None:
    _session_trie().delete(topic)


def match_session(topic: bytes) -> List[bytes]:
    return _session_trie().match(topic)


def empty_session() -> bool:
    return _session_trie().empty()

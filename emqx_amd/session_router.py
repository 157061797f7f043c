"""``emqx_session_router`` API mirror (apps/emqx/src/emqx_session_router.erl:104-150) on the
device engine: the persistent-session route table, a second engine handle beside the
broker's.

Routes are ``#route{topic, dest = SessionID}``.  Wildcard filters go through the session trie
(``emqx_router_utils:insert_session_trie_route/2`` -> ``emqx_trie:insert_session/1``), exact
ones are direct routes; both live in one engine snapshot here, and ``match_routes/1``
(emqx_session_router.erl:122-128: ``lookup_routes(Topic)`` plus the routes of every session-
trie match) is one device match in ``EMQX_MODE_ROUTES`` — the same set, since a wildcard
topic only ever matches its byte-identical filter (S3).
"""

from __future__ import annotations

from typing import List, Optional, Sequence

from . import topic as _topic
from .router import Route, Router


class SessionRouter(Router):
    def __init__(self, device: int = -1):
        super().__init__(device, node=None)

    # emqx_session_router.erl:104-118: dest is the SessionID (no default node)
    def do_add_route(self, topic: bytes, session_id) -> None:  # type: ignore[override]
        super().add_route(topic, session_id)

    add_route = do_add_route

    # emqx_session_router.erl:141-150
    def do_delete_route(self, topic: bytes, session_id) -> None:  # type: ignore[override]
        super().delete_route(topic, session_id)

    delete_route = do_delete_route

    def delete_routes(self, session_id, subscriptions: Sequence[bytes]) -> None:
        """emqx_session_router.erl:136-138 (a cast there; applied in place here)."""
        for t in subscriptions:
            self.do_delete_route(t, session_id)

    # match_trie/1 (emqx_session_router.erl:130-134, emqx_trie:match_session/1) is
    # Router.match_trie: EMQX_MODE_TRIE_WILDCARD on this handle's snapshot.

    def empty_session(self) -> bool:
        """emqx_trie:empty_session/0: no wildcard session route."""
        return not any(_topic.wildcard(self._names[f]) for f in self._dests)


_default: Optional[SessionRouter] = None


def _router() -> SessionRouter:
    global _default
    if _default is None:
        _default = SessionRouter()
    return _default


def do_add_route(topic: bytes, session_id) -> None:
    _router().do_add_route(topic, session_id)


def do_delete_route(topic: bytes, session_id) -> None:
    _router().do_delete_route(topic, session_id)


def match_routes(topic: bytes) -> List[Route]:
    return _router().match_routes(topic)


def delete_routes(session_id, subscriptions: Sequence[bytes]) -> None:
    _router().delete_routes(session_id, subscriptions)


__all__ = ["SessionRouter", "Route", "do_add_route", "do_delete_route", "match_routes", "delete_routes"]

"""Persistent-session routes: emqx_session_router:do_add_route/match_routes/
do_delete_route (emqx_session_router.erl:104-150) and emqx_trie:insert_session/match_session
(emqx_trie.erl:111-146) on their own engine handle, checked against brute-force
emqx_topic:match over the live session routes."""

import random

import pytest

from oracle import emqx_ref as R
from tests.test_oracle_fuzz import rand_filter, rand_topic

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mods():
    import torch  # noqa: F401
    from emqx_amd import _lib, session_router, trie
    _lib.lib()
    return session_router, trie


def test_session_routes_fuzz(mods):
    session_router, _ = mods
    rng = random.Random(61)
    sr = session_router.SessionRouter()
    routes = {}  # filter -> set(session ids)
    for step in range(5):
        for _ in range(80):
            f, sid = rand_filter(rng), b"s%d" % rng.randrange(20)
            sr.do_add_route(f, sid)
            routes.setdefault(f, set()).add(sid)
        for f in rng.sample(sorted(routes), min(len(routes), 15)):
            for sid in sorted(routes[f])[:1]:
                sr.do_delete_route(f, sid)
                routes[f].discard(sid)
        for t in [rand_topic(rng) for _ in range(200)] + [b"$SYS/a", b"a/+"]:
            got = sorted((r.topic, r.dest) for r in sr.match_routes(t))
            fl = sorted(f for f, ss in routes.items() if ss)
            exp = sorted((fl[i], s) for i in R.brute_force_routes(fl, t) for s in routes[fl[i]])
            assert got == exp, (step, t)
    sr.delete_routes(b"s1", sorted(routes))
    assert all(r.dest != b"s1" for r in sr.match_routes(b"a/b"))


def test_session_trie_is_its_own_handle(mods):
    _, trie = mods
    trie.insert_session(b"sess/+/x")
    trie.insert(b"main/#")
    assert trie.match_session(b"sess/1/x") == [b"sess/+/x"]
    assert trie.match_session(b"main/1") == []
    assert trie.match(b"sess/1/x") == []
    assert not trie.empty_session()
    trie.delete_session(b"sess/+/x")
    assert trie.match_session(b"sess/1/x") == []
    assert trie.empty_session()
    trie.delete(b"main/#")

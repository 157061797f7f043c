"""ORACLE (test infrastructure only — never imported by the product path).

CPU restatement of the retained-message lookup of the reference's mnesia retainer backend
("inverse match": a subscription filter -> the stored retained topics it
matches).  Pure Python, for small tables:

  * topic2tokens/1            apps/emqx_retainer/src/emqx_retainer_mnesia.erl:178-179
                              (= emqx_topic:words/1, apps/emqx/src/emqx_topic.erl:153-164)
  * condition/1               emqx_retainer_mnesia.erl:225-231: '+' -> '_' (any one token,
                              the empty level included); a final '#' is dropped (`Ws1 --
                              ['#']` removes the FIRST '#') and the list gets the improper
                              tail '_' (any tail, the empty one included).  Unlike routing
                              (emqx_topic:match/2) there is NO '$' rule: the match spec
                              never looks at the first level, so '#' and '+/...' match
                              '$SYS/...' topics too.
  * make_match_spec/1         emqx_retainer_mnesia.erl:233-245: live iff expiry_time =:= 0
                              or expiry_time > NowMs
  * read_messages/1           emqx_retainer_mnesia.erl:199-208: exact key, live iff
                              Et =:= 0 orelse Et >= NowMs   (note >= here, > above)
  * dispatch/4                apps/emqx_retainer/src/emqx_retainer.erl:119-131: plain
                              filter -> read_message/2, wildcard filter -> match_messages/3
  * match_delete_messages/1   emqx_retainer_mnesia.erl:217-223: condition/1 without the
                              expiry guard
"""

from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

from .emqx_ref import HASH, PLUS, wildcard, words

ANY = object()  # the match-spec wildcard '_'


def topic2tokens(topic: bytes) -> list:
    return words(topic)


def condition(ws: list):
    """emqx_retainer_mnesia.erl:225-231.  Returns (prefix, open_tail): the pattern matches a
    token list L iff len(prefix) elements match pairwise (ANY matches anything) and either
    len(L) == len(prefix) or open_tail."""
    ws1 = [ANY if w == PLUS else w for w in ws]
    if ws1 and ws1[-1] == HASH:
        i = ws1.index(HASH)  # `--` removes the first occurrence
        return ws1[:i] + ws1[i + 1:], True
    return ws1, False


def cond_match(cond, tokens: list) -> bool:
    prefix, open_tail = cond
    if len(tokens) < len(prefix) or (not open_tail and len(tokens) != len(prefix)):
        return False
    return all(p is ANY or p == t for p, t in zip(prefix, tokens))


class RetainTable:
    """The ?TAB set keyed by token list (one retained message per topic)."""

    def __init__(self):
        self.ids: Dict[bytes, int] = {}
        self.names: List[bytes] = []
        self.expiry: List[int] = []
        self.live: List[bool] = []

    def store(self, topic: bytes, expiry_ms: int = 0) -> int:
        i = self.ids.get(topic)
        if i is None:
            i = len(self.names)
            self.ids[topic] = i
            self.names.append(topic)
            self.expiry.append(0)
            self.live.append(False)
        self.expiry[i] = int(expiry_ms)
        self.live[i] = True
        return i

    def delete_ids(self, ids: Sequence[int]) -> None:
        for i in ids:
            self.live[i] = False

    def match_messages(self, filt: bytes, now_ms: Optional[int]) -> List[int]:
        """mnesia:dirty_select(?TAB, make_match_spec(Filter)); now_ms None = no guard
        (match_delete_messages/1)."""
        cond = condition(words(filt))
        out = []
        for i, t in enumerate(self.names):
            if not self.live[i] or not cond_match(cond, topic2tokens(t)):
                continue
            e = self.expiry[i]
            if now_ms is None or e == 0 or e > now_ms:
                out.append(i)
        return out

    def read_messages(self, topic: bytes, now_ms: int) -> List[int]:
        i = self.ids.get(topic)
        if i is None or not self.live[i]:
            return []
        e = self.expiry[i]
        return [i] if (e == 0 or e >= now_ms) else []

    def dispatch(self, filt: bytes, now_ms: int) -> List[int]:
        """emqx_retainer.erl:119-131 (the ids whose messages are delivered, unordered)."""
        if wildcard(filt):
            return self.match_messages(filt, now_ms)
        return self.read_messages(filt, now_ms)

    def delete_message(self, topic: bytes) -> None:
        """emqx_retainer_mnesia.erl:117-128."""
        if wildcard(topic):
            self.delete_ids(self.match_messages(topic, None))
        else:
            i = self.ids.get(topic)
            if i is not None:
                self.live[i] = False


def brute_force(names: Sequence[bytes], expiry: Sequence[int], live: Sequence[bool],
                filters: Sequence[bytes], now_ms: int) -> List[List[int]]:
    """dispatch/4 for every filter against a packed table (ids = positions)."""
    t = RetainTable()
    for n, e in zip(names, expiry):
        t.store(n, e)
    for i, v in enumerate(live):
        if not v:
            t.live[i] = False
    return [sorted(t.dispatch(f, now_ms)) for f in filters]


def pairs(table: RetainTable, filters: Sequence[bytes], now_ms: int) -> List[Tuple[int, ...]]:
    return [tuple(sorted(table.dispatch(f, now_ms))) for f in filters]


class TokenTrie:
    """The same select as RetainTable.match_messages/dispatch, evaluated by walking a dict
    trie of token lists instead of testing every record — for tables too large for the
    brute-force form (cross-checked against it in tests/test_retain_oracle.py)."""

    def __init__(self, names: Sequence[bytes], expiry: Sequence[int], live: Optional[Sequence[bool]] = None):
        self.root: dict = {}
        self.expiry = list(expiry)
        self.ids: Dict[bytes, int] = {}
        for i, n in enumerate(names):
            if live is not None and not live[i]:
                continue
            self.ids[n] = i
            node = self.root
            for w in topic2tokens(n):
                node = node.setdefault(w, {})
            node[None] = i  # None key: the topic ending here

    def _subtree(self, node, out):
        stack = [node]
        while stack:
            v = stack.pop()
            for k, c in v.items():
                if k is None:
                    out.append(c)
                else:
                    stack.append(c)

    def select(self, filt: bytes) -> List[int]:
        prefix, open_tail = condition(words(filt))
        out: List[int] = []
        frontier = [self.root]
        for p in prefix:
            nxt = []
            for v in frontier:
                if p is ANY:
                    nxt.extend(c for k, c in v.items() if k is not None)
                elif p in v:
                    nxt.append(v[p])
            frontier = nxt
        for v in frontier:
            if open_tail:
                self._subtree(v, out)
            elif None in v:
                out.append(v[None])
        return out

    def dispatch(self, filt: bytes, now_ms: int) -> List[int]:
        if wildcard(filt):
            ids = self.select(filt)
            return sorted(i for i in ids if now_ms < 0 or self.expiry[i] == 0 or self.expiry[i] > now_ms)
        i = self.ids.get(filt)
        if i is None:
            return []
        e = self.expiry[i]
        return [i] if (now_ms < 0 or e == 0 or e >= now_ms) else []

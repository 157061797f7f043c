"""CPU restatement of the reference's route-lookup algorithm — TEST INFRASTRUCTURE ONLY.

This module is the parity oracle.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import it, and only as the checker.  The
product path (``emqx_amd``) never imports anything from ``oracle/``.

It restates, function by function, the Erlang reference (EMQX 5.0.0-beta.3, paths
relative to ``/root/reference``):

* ``apps/emqx/src/emqx_topic.erl``   — tokens/words/wildcard/match/join/validate/parse
* ``apps/emqx/src/emqx_trie.erl``    — key layout, compaction, refcounted insert/delete,
  the ``$`` root rule and BOTH DFS match modes (compact / non-compact)
* ``apps/emqx/src/emqx_router.erl``  — ``match_routes/1`` (exact lookup ∪ trie matches)

Representation: Erlang binaries are Python ``bytes``; the atoms that
``emqx_topic:word/1`` produces (``''``, ``'+'``, ``'#'``) are the Python ``str``
objects ``EMPTY``, ``PLUS``, ``HASH``.  The trie's virtual root ``empty`` is ``ROOT``.

Pinning: every function here is checked against the reference's own known-answer
tests (``tests/golden/kats.json``, transcribed by ``tests/golden/make_kats.py`` from
``emqx_trie.erl:345-395``, ``emqx_trie_SUITE.erl:63-186``,
``emqx_topic_SUITE.erl:42-213``, ``emqx_router_SUITE.erl:81-95``,
``emqx_client_SUITE.erl:28-43,165-238``) and against the brute-force predicate
(``emqx_topic:match/2``) on fuzzed tables, in both compaction modes.
"""

from __future__ import annotations

from typing import Dict, Iterable, List, Sequence, Tuple, Union

EMPTY = ""   # atom ''   (emqx_topic.erl:161)
PLUS = "+"   # atom '+'  (emqx_topic.erl:162)
HASH = "#"   # atom '#'  (emqx_topic.erl:163)
ROOT = None  # atom `empty`, the trie's virtual root prefix (emqx_trie.erl:209,218-221,265)

Word = Union[bytes, str]
MAX_TOPIC_LEN = 65535  # emqx_topic.erl:45


class TopicError(Exception):
    """Mirrors ``error(Reason)`` raised by emqx_topic:validate/parse."""


# --------------------------------------------------------------------------
# emqx_topic
# --------------------------------------------------------------------------

def tokens(topic: bytes) -> List[bytes]:
    """``binary:split(Topic, <<"/">>, [global])`` — emqx_topic.erl:153-154."""
    return topic.split(b"/")


def word(w: bytes) -> Word:
    """emqx_topic.erl:161-164."""
    if w == b"":
        return EMPTY
    if w == b"+":
        return PLUS
    if w == b"#":
        return HASH
    return w


def words(topic: bytes) -> List[Word]:
    """emqx_topic.erl:158-159."""
    return [word(w) for w in tokens(topic)]


def levels(topic: bytes) -> int:
    """emqx_topic.erl:147-148."""
    return len(tokens(topic))


def wildcard(topic_or_words) -> bool:
    """emqx_topic.erl:53-62: true iff some level is exactly '+' or '#'."""
    ws = words(topic_or_words) if isinstance(topic_or_words, (bytes, bytearray)) else topic_or_words
    for w in ws:
        if w == HASH or w == PLUS:
            return True
    return False


def match(name, filt) -> bool:
    """``emqx_topic:match/2`` — the normative predicate, emqx_topic.erl:68-87.

    The ``$`` rule is applied on raw binaries (first byte of name is ``$`` and first
    byte of filter is ``+`` or ``#`` => false), exactly as clauses 68-71 do, and only
    when both arguments are binaries.
    """
    if isinstance(name, (bytes, bytearray)) and isinstance(filt, (bytes, bytearray)):
        if name[:1] == b"$" and filt[:1] in (b"+", b"#"):
            return False
        return _match_words(words(bytes(name)), words(bytes(filt)))
    return _match_words(list(name), list(filt))


def _match_words(n: Sequence[Word], f: Sequence[Word]) -> bool:
    # Iterative form of the clause sequence at emqx_topic.erl:74-87.
    i = 0
    while True:
        if i == len(n) and i == len(f):
            return True                                  # match([], [])
        if i < len(n) and i < len(f) and n[i] == f[i]:
            i += 1                                       # match([H|T1], [H|T2])
            continue
        if i < len(n) and i < len(f) and f[i] == PLUS:
            i += 1                                       # match([_H|T1], ['+'|T2])
            continue
        if len(f) - i == 1 and f[i] == HASH:
            return True                                  # match(_, ['#'])
        return False                                     # remaining clauses


def _bin(w) -> bytes:
    """emqx_topic.erl:140-144."""
    if w == EMPTY:
        return b""
    if w == PLUS:
        return b"+"
    if w == HASH:
        return b"#"
    if isinstance(w, (bytes, bytearray)):
        return bytes(w)
    if isinstance(w, str):
        return w.encode()
    raise TypeError(w)


def join(ws: Iterable) -> bytes:
    """emqx_topic.erl:184-195."""
    return b"/".join(_bin(w) for w in ws)


def prepend(parent, w) -> bytes:
    """emqx_topic.erl:131-138."""
    if parent is None or parent == b"":
        return _bin(w)
    p = _bin(parent)
    if p[-1:] == b"/":
        return p + _bin(w)
    return p + b"/" + _bin(w)


def feed_var(var: bytes, val: bytes, topic: bytes) -> bytes:
    """emqx_topic.erl:174-181."""
    return join([val if w == var else w for w in words(topic)])


def validate(arg, topic: bytes = None) -> bool:
    """emqx_topic.erl:91-127.  ``validate(T)`` == ``validate(filter, T)``."""
    if topic is None:
        if isinstance(arg, tuple):
            kind, topic = arg
        else:
            kind, topic = "filter", arg
    else:
        kind = arg
    if topic == b"":
        raise TopicError("empty_topic")
    if len(topic) > MAX_TOPIC_LEN:
        raise TopicError("topic_too_long")
    ws = words(topic)
    if kind == "filter":
        return _validate2(ws)
    if kind == "name":
        if _validate2(ws) and not wildcard(ws):
            return True
        raise TopicError("topic_name_error")
    raise ValueError(kind)


def _validate2(ws: List[Word]) -> bool:
    for i, w in enumerate(ws):
        if w == HASH:
            if i != len(ws) - 1:
                raise TopicError("topic_invalid_#")          # emqx_topic.erl:113-114
            return True
        if w in (EMPTY, PLUS):
            continue
        _validate3(w)
    return True


def _validate3(w: bytes) -> None:
    """emqx_topic.erl:122-127: reject '#', '+' and NUL characters (UTF-8 decoded)."""
    s = w.decode("utf-8")
    for c in s:
        if c in ("#", "+", "\x00"):
            raise TopicError("topic_invalid_char")


def parse(topic_filter, options=None):
    """emqx_topic.erl:198-220 — strips ``$queue/`` and ``$share/<g>/``."""
    if isinstance(topic_filter, tuple):
        topic_filter, options = topic_filter
    options = dict(options or {})
    tf = topic_filter
    if "share" in options and (tf.startswith(b"$queue/") or tf.startswith(b"$share/")):
        raise TopicError(("invalid_topic_filter", tf))
    if tf.startswith(b"$queue/"):
        options["share"] = b"$queue"
        return parse(tf[len(b"$queue/"):], options)
    if tf.startswith(b"$share/"):
        rest = tf[len(b"$share/"):]
        parts = rest.split(b"/", 1)
        if len(parts) == 1:
            raise TopicError(("invalid_topic_filter", tf))
        share_name, filt = parts
        if b"+" in share_name or b"#" in share_name:
            raise TopicError(("invalid_topic_filter", tf))
        options["share"] = share_name
        return parse(filt, options)
    return tf, options


# --------------------------------------------------------------------------
# emqx_trie
# --------------------------------------------------------------------------

PREFIX_TAG = 0   # ?PREFIX(P) = {P, 0}  emqx_trie.erl:53
TOPIC_TAG = 1    # ?TOPIC(T)  = {T, 1}  emqx_trie.erl:54


def trie_join(prefix, w) -> bytes:
    """``join/2`` of emqx_trie.erl:218-222 (root-aware)."""
    if prefix is ROOT:
        if w == PLUS:
            return b"+"
        if w == HASH:
            return b"#"
        if w == EMPTY:
            return b""
        return w
    return join([prefix, w])


def do_compact(ws: List[Word]) -> List[bytes]:
    """emqx_trie.erl:208-216: segments, each ending at one wildcard word."""
    seg = ROOT
    acc: List[bytes] = []
    for w in ws:
        if w == PLUS or w == HASH:
            acc.append(trie_join(seg, w))
            seg = ROOT
        else:
            seg = trie_join(seg, w)
    if seg is not ROOT:
        acc.append(seg)
    return acc


class Trie:
    """The ETS ``ordered_set`` of ``{Key, Count}`` records (emqx_trie.erl:56-59,67-77).

    ``compact`` is ``broker.perf.trie_compaction`` (default true, emqx_trie.erl:336-337).
    ``lookups`` counts ETS lookups (lookup_topic / has_prefix) for cost accounting.
    """

    def __init__(self, compact: bool = True):
        self.compact = compact
        self.tab: Dict[Tuple[bytes, int], int] = {}
        self.lookups = 0

    # -- key construction -------------------------------------------------
    def _compact(self, ws):
        return do_compact(ws) if self.compact else ws           # emqx_trie.erl:196-200

    def make_prefixes(self, ws: List[Word]) -> List[bytes]:
        """emqx_trie.erl:224-233."""
        segs = self._compact(ws)
        acc = []
        prefix: List = []
        for h in segs[:-1]:
            prefix = prefix + [h]
            acc.insert(0, list(prefix))
        return [join(p) for p in acc]

    def make_keys(self, topic: bytes):
        """emqx_trie.erl:192-194."""
        ws = words(topic)
        return (topic, TOPIC_TAG), [(p, PREFIX_TAG) for p in self.make_prefixes(ws)]

    # -- mutation -----------------------------------------------------------
    def insert(self, topic: bytes) -> None:
        """emqx_trie.erl:115-120 + insert_key :235-242."""
        tkey, pkeys = self.make_keys(topic)
        if tkey in self.tab:
            return
        for k in [tkey] + pkeys:
            self.tab[k] = self.tab.get(k, 0) + 1

    def delete(self, topic: bytes) -> None:
        """emqx_trie.erl:132-137 + delete_key :244-252."""
        tkey, pkeys = self.make_keys(topic)
        if tkey not in self.tab:
            return
        for k in [tkey] + pkeys:
            c = self.tab.get(k)
            if c is None:
                continue
            if c > 1:
                self.tab[k] = c - 1
            else:
                del self.tab[k]

    def empty(self) -> bool:
        """emqx_trie.erl:171."""
        return not self.tab

    # -- lookups ------------------------------------------------------------
    def lookup_topic(self, topic: bytes, is_wildcard: bool = True) -> List[bytes]:
        """emqx_trie.erl:256-263 (the 3-arity form skips the lookup for non-wildcards)."""
        if not is_wildcard:
            return []
        self.lookups += 1
        c = self.tab.get((topic, TOPIC_TAG))
        return [topic] if c is not None and c > 0 else []

    def has_prefix(self, prefix) -> bool:
        """emqx_trie.erl:265-270."""
        if prefix is ROOT:
            return True
        self.lookups += 1
        c = self.tab.get((prefix, PREFIX_TAG))
        return c is not None and c > 0

    def _match_hash(self, prefix) -> List[bytes]:
        """'match_#' — emqx_trie.erl:332-334 (2-arity lookup_topic: no wildcard gate)."""
        return self.lookup_topic(trie_join(prefix, HASH), True)

    # -- match ----------------------------------------------------------------
    def match(self, topic: bytes) -> List[bytes]:
        """emqx_trie.erl:148-162 + do_match :272-287."""
        ws = words(topic)
        if wildcard(ws):
            return []
        first = ws[0]
        if isinstance(first, bytes) and first[:1] == b"$":
            rest = ws[1:]
            head = self.lookup_topic(first, True) if not rest else []
            return head + self._do_match(rest, first)
        return self._do_match(ws, ROOT)

    def _do_match(self, ws, prefix):
        if self.compact:
            return self._match_compact(ws, 0, prefix, False, [])
        return self._match_no_compact(ws, 0, prefix, False, [])

    def _match_no_compact(self, ws, i, prefix, is_wild, acc):
        """emqx_trie.erl:289-313."""
        if i == len(ws):
            return self._match_hash(prefix) + self.lookup_topic(prefix, is_wild) + acc
        if not self.has_prefix(prefix):
            return acc
        acc1 = self._match_hash(prefix) + acc
        acc2 = self._match_no_compact(ws, i + 1, trie_join(prefix, PLUS), True, acc1)
        return self._match_no_compact(ws, i + 1, trie_join(prefix, ws[i]), is_wild, acc2)

    def _match_compact(self, ws, i, prefix, is_wild, acc):
        """emqx_trie.erl:315-330 (default mode)."""
        if i == len(ws):
            return self._match_hash(prefix) + self.lookup_topic(prefix, is_wild) + acc
        acc1 = self._match_hash(prefix) + acc
        acc2 = self._match_compact(ws, i + 1, trie_join(prefix, ws[i]), is_wild, acc1)
        wprefix = trie_join(prefix, PLUS)
        if i + 1 == len(ws) or self.has_prefix(wprefix):
            return self._match_compact(ws, i + 1, wprefix, True, acc2)
        return acc2


# --------------------------------------------------------------------------
# emqx_router
# --------------------------------------------------------------------------

class Router:
    """Route table (``bag`` of ``#route{topic, dest}``) + trie of wildcard filters.

    emqx_router.erl:75-83 (table), :110-124 (do_add_route: only wildcard filters
    enter the trie), :127-140 (match_routes), :142-148 (lookup/has), :162-171 (delete).
    """

    def __init__(self, compact: bool = True):
        self.routes: Dict[bytes, List] = {}
        self.trie = Trie(compact)

    def add_route(self, topic: bytes, dest="node@local") -> None:
        lst = self.routes.setdefault(topic, [])
        if dest in lst:
            return
        if wildcard(topic) and not lst:
            self.trie.insert(topic)   # insert_trie_route: trie insert on first route
        lst.append(dest)

    def delete_route(self, topic: bytes, dest="node@local") -> None:
        lst = self.routes.get(topic)
        if not lst or dest not in lst:
            return
        lst.remove(dest)
        if not lst:
            del self.routes[topic]
            if wildcard(topic):
                self.trie.delete(topic)  # delete_trie_route: trie delete on last route

    def lookup_routes(self, topic: bytes):
        return [(topic, d) for d in self.routes.get(topic, [])]

    def has_routes(self, topic: bytes) -> bool:
        return topic in self.routes

    def topics(self) -> List[bytes]:
        return list(self.routes.keys())

    def match_trie(self, topic: bytes) -> List[bytes]:
        return [] if self.trie.empty() else self.trie.match(topic)

    def match_routes(self, topic: bytes):
        matched = self.match_trie(topic)
        if not matched:
            return self.lookup_routes(topic)
        out = []
        for to in [topic] + matched:
            out.extend(self.lookup_routes(to))
        return out


# --------------------------------------------------------------------------
# Set-level helpers used by the parity tests (filter-ID formulation)
# --------------------------------------------------------------------------

def brute_force_trie(filters: Sequence[bytes], topic: bytes) -> List[int]:
    """IDs that ``emqx_trie:match`` returns for a trie holding every filter in
    ``filters`` (exact ones included, as emqx_trie_SUITE does): wildcard filters
    satisfying emqx_topic:match/2, plus the one-level ``$`` quirk of
    emqx_trie.erl:276-277 (an exact ``$x`` filter matches topic ``$x``)."""
    ws = words(topic)
    if wildcard(ws):
        return []
    out = []
    for i, f in enumerate(filters):
        if wildcard(f):
            if match(topic, f):
                out.append(i)
        elif len(ws) == 1 and topic[:1] == b"$" and f == topic:
            out.append(i)
    return out


def brute_force_routes(filters: Sequence[bytes], topic: bytes) -> List[int]:
    """IDs of the filters whose routes ``emqx_router:match_routes/1`` returns."""
    out = []
    wt = wildcard(topic)
    for i, f in enumerate(filters):
        if f == topic:
            out.append(i)
        elif not wt and wildcard(f) and match(topic, f):
            out.append(i)
    return out


def trie_match_ids(trie: Trie, index: Dict[bytes, int], topic: bytes) -> List[int]:
    return sorted(index[f] for f in trie.match(topic))


def router_match_ids(router: Router, index: Dict[bytes, int], topic: bytes) -> List[int]:
    return sorted({index[t] for t, _ in router.match_routes(topic)})


def evals(filters: Sequence[bytes], topics: Sequence[bytes]) -> List[int]:
    """SURVEY §8(d) cost model: node visits in the uncompacted level trie of ALL
    filters.  evals(T) = sum_{i=0..L} |F_i|, F_0 = {root},
    F_{i+1} = {n/w_i, n/'+' : present}; the root '+' is skipped for '$' topics.
    Wildcard topics are rejected by the trie (emqx_trie.erl:150-159) and count 0."""
    nodes = set()
    for f in filters:
        ws = words(f)
        for k in range(1, len(ws) + 1):
            nodes.add(tuple(ws[:k]))
    out = []
    for t in topics:
        ws = words(t)
        if wildcard(ws):
            out.append(0)
            continue
        frontier = [()]
        total = 1
        dollar = isinstance(ws[0], bytes) and ws[0][:1] == b"$"
        for i, w in enumerate(ws):
            nxt = []
            for n in frontier:
                c = n + (w,)
                if c in nodes:
                    nxt.append(c)
                if not (i == 0 and dollar):
                    p = n + (PLUS,)
                    if p in nodes:
                        nxt.append(p)
            frontier = nxt
            total += len(frontier)
            if not frontier:
                break
        out.append(total)
    return out

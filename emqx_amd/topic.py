"""``emqx_topic`` API mirror (apps/emqx/src/emqx_topic.erl:20-33).

``match/2`` and ``wildcard/1`` call the library's CPU implementation (emqx_topic_match /
emqx_topic_wildcard in emqx_amd/csrc/topic.cpp) — per-pair callers stay on the CPU, as in
the reference; batched routing goes through :mod:`emqx_amd.router` / :mod:`emqx_amd.trie`.
Words use the reference's representation: binaries are ``bytes``; the atoms ``''``,
``'+'`` and ``'#'`` are the str constants EMPTY, PLUS, HASH.
"""

from __future__ import annotations

import ctypes
from typing import Iterable, List, Union

from . import _lib

EMPTY, PLUS, HASH = "", "+", "#"
MAX_TOPIC_LEN = 65535  # emqx_topic.erl:45


class TopicError(ValueError):
    """Raised where the reference calls ``error(Reason)``; ``.reason`` holds Reason."""

    def __init__(self, reason):
        super().__init__(reason)
        self.reason = reason


def _buf(b: bytes):
    return ctypes.c_char_p(b) if b else ctypes.c_char_p(b"\0")


def match(name: bytes, filt: bytes) -> bool:
    """emqx_topic:match/2 (emqx_topic.erl:68-87) on binaries."""
    return bool(_lib.lib().emqx_topic_match(_buf(name), len(name), _buf(filt), len(filt)))


def tokens(topic: bytes) -> List[bytes]:
    """emqx_topic.erl:153-154."""
    return topic.split(b"/")


_ATOM = {b"": EMPTY, b"+": PLUS, b"#": HASH}


def words(topic: bytes) -> List[Union[bytes, str]]:
    """emqx_topic.erl:158-164."""
    return [_ATOM.get(w, w) for w in topic.split(b"/")]


def levels(topic: bytes) -> int:
    return topic.count(b"/") + 1


def wildcard(topic) -> bool:
    """emqx_topic.erl:53-62 — accepts a binary or a words list."""
    if isinstance(topic, (bytes, bytearray)):
        return bool(_lib.lib().emqx_topic_wildcard(_buf(bytes(topic)), len(topic)))
    return any(w == PLUS or w == HASH for w in topic)


def _bin(w) -> bytes:
    if isinstance(w, str):
        return w.encode()
    return bytes(w)


def join(ws: Iterable) -> bytes:
    """emqx_topic.erl:184-195."""
    return b"/".join(_bin(w) for w in ws)


def prepend(parent, w) -> bytes:
    """emqx_topic.erl:131-138."""
    if parent is None or parent == b"":
        return _bin(w)
    p = _bin(parent)
    return p + _bin(w) if p.endswith(b"/") else p + b"/" + _bin(w)


def feed_var(var: bytes, val: bytes, topic: bytes) -> bytes:
    """emqx_topic.erl:174-181."""
    return join(val if w == var else w for w in words(topic))


def systop(name, node: bytes = b"emqx@127.0.0.1") -> bytes:
    """emqx_topic.erl:167-171 (node() passed explicitly)."""
    return b"$SYS/brokers/" + node + b"/" + _bin(name)


def validate(arg, topic: bytes = None) -> bool:
    """emqx_topic.erl:91-127 — ``validate(T)``, ``validate((kind, T))`` or ``validate(kind, T)``."""
    if topic is None:
        kind, topic = arg if isinstance(arg, tuple) else ("filter", arg)
    else:
        kind = arg
    if topic == b"":
        raise TopicError("empty_topic")
    if len(topic) > MAX_TOPIC_LEN:
        raise TopicError("topic_too_long")
    ws = words(topic)
    last = len(ws) - 1
    for i, w in enumerate(ws):
        if w == HASH:
            if i != last:
                raise TopicError("topic_invalid_#")
        elif w in (EMPTY, PLUS):
            continue
        else:
            text = w.decode("utf-8")
            if "#" in text or "+" in text or "\x00" in text:
                raise TopicError("topic_invalid_char")
    if kind == "name" and wildcard(ws):
        raise TopicError("topic_name_error")
    if kind not in ("name", "filter"):
        raise ValueError(kind)
    return True


def parse(topic_filter, options=None):
    """emqx_topic.erl:197-220: ``$queue/`` and ``$share/<group>/`` prefixes -> options."""
    if isinstance(topic_filter, tuple):
        topic_filter, options = topic_filter
    opts = dict(options or {})
    tf = topic_filter
    while True:
        is_q, is_s = tf.startswith(b"$queue/"), tf.startswith(b"$share/")
        if (is_q or is_s) and "share" in opts:
            raise TopicError(("invalid_topic_filter", tf))
        if is_q:
            opts["share"] = b"$queue"
            tf = tf[7:]
            continue
        if is_s:
            rest = tf[7:]
            if b"/" not in rest:
                raise TopicError(("invalid_topic_filter", tf))
            group, filt = rest.split(b"/", 1)
            if b"+" in group or b"#" in group:
                raise TopicError(("invalid_topic_filter", tf))
            opts["share"] = group
            tf = filt
            continue
        return tf, opts

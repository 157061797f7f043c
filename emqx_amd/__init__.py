"""emqx_amd — MI355X-native route lookup for EMQX (topic -> matching filters).

Modules mirror the reference's Erlang modules on the hot path:
  :mod:`emqx_amd.topic`   emqx_topic   (CPU topic algebra, match/2)
  :mod:`emqx_amd.trie`    emqx_trie    (insert/delete/match/empty on the device engine)
  :mod:`emqx_amd.router`  emqx_router  (add/delete/match_routes/lookup_routes)
  :mod:`emqx_amd.engine`  the C-ABI engine handle (batched, device-resident matching)
  :mod:`emqx_amd.workloads` synthetic subscription tables / topic streams (BASELINE configs)
  :mod:`emqx_amd.dist`    multi-GPU: replicated tables + data-parallel topic split,
                          filter-sharded tables with broadcast + gather
"""

__version__ = "0.1.0"

from ._lib import EngineError, MODE_ROUTES, MODE_TRIE, MODE_TRIE_WILDCARD  # noqa: F401

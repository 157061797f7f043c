// C ABI of the retained-message index (include/emqx_retain.h): host topic store, trie build
// with DFS-preorder ranks, snapshot upload/swap, and the match pipeline
//   walk -> spill rounds -> count -> scan -> write -> [one D2H: control words + id total],
// all enqueued at once (the device reads every count it needs).
// Reference semantics: apps/emqx_retainer/src/emqx_retainer_mnesia.erl (see retain.h and
// oracle/retain_ref.py).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/emqx_retain.h"
#include "kernels.h"
#include "retain.h"
#include "streams.h"
#include "tables.h"

using namespace emqx;

namespace {

#define RT_TRY(expr)                             \
  do {                                           \
    hipError_t _e = (expr);                      \
    if (_e != hipSuccess) return EMQX_EDEVICE;   \
  } while (0)

template <class T>
void rfree(T*& p) {
  if (p) (void)hipFree(p);
  p = nullptr;
}

template <class T>
hipError_t ralloc(T*& p, uint64_t count) {
  rfree(p);
  return hipMalloc(reinterpret_cast<void**>(&p), std::max<uint64_t>(count, 1) * sizeof(T));
}

// Device arrays of one committed snapshot (freed after draining the device).
struct RSnapshot {
  int device = 0;
  REdgeBucket* edges = nullptr;
  VocabSlot* vocab = nullptr;
  uint8_t* arena = nullptr;
  uint32_t* rank_id = nullptr;
  int64_t* rank_exp = nullptr;
  RPostKey* pkeys = nullptr;
  uint4* posts = nullptr;
  uint32_t* pst = nullptr;  // RSTree levels
  uint32_t* dst = nullptr;
  uint32_t* pfence = nullptr;
  uint32_t* dfence = nullptr;
  uint32_t* dterm_off = nullptr;
  uint32_t* dterm = nullptr;
  uint16_t* rank_depth = nullptr;
  RetainView rv{};
  uint64_t n_nodes = 0, n_words = 0, bytes = 0;
  ~RSnapshot() {
    int cur = 0;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(device);
    (void)hipDeviceSynchronize();
    rfree(edges);
    rfree(vocab);
    rfree(arena);
    rfree(rank_id);
    rfree(rank_exp);
    rfree(pkeys);
    rfree(posts);
    rfree(pst);
    rfree(dst);
    rfree(pfence);
    rfree(dfence);
    rfree(dterm_off);
    rfree(dterm);
    rfree(rank_depth);
    (void)hipSetDevice(cur);
  }
};

// Per-call scratch, grown on demand (one per concurrent caller).
struct RWork {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr, evw = nullptr;
  uint32_t* wids = nullptr;
  uint64_t wids_cap = 0;
  uint4* stack = nullptr;
  uint64_t stack_items = 0;
  uint32_t stack_cap = 1024;  // items per wave beyond the LDS part (grows on overflow)
  RRange* ranges = nullptr;
  uint32_t* rcount = nullptr;
  uint64_t* rlive = nullptr;
  uint32_t range_cap = 0;
  uint32_t* ctrl = nullptr;
  uint32_t* fcount = nullptr;
  uint32_t* fcursor = nullptr;
  uint64_t f_cap = 0;
  uint4* wdesc = nullptr;  // per-level step descriptors for the spill rounds
  uint64_t wdesc_cap = 0;
  uint4* spill[2] = {nullptr, nullptr};  // spill rounds: items in / items out, alternating
  uint32_t spill_cap = 0;
  uint4* queue = nullptr;  // queue mode's shared pieces (all zero when a call starts)
  uint32_t queue_cap = 0;
  uint32_t* qctl = nullptr;  // queue mode's per-shard control words (likewise)
  uint64_t* partials = nullptr;
  uint64_t partials_cap = 0;
  uint64_t* h_pinned = nullptr;  // [RC_WORDS / 2 + 1] readbacks: ctrl words, then the id total
  uint64_t* prof = nullptr;      // [16] RETAIN_PROF builds with EMQX_RETAIN_PROF=1
  // host-API staging (device copies of the caller's buffers)
  uint8_t* d_fb = nullptr;
  uint64_t d_fb_cap = 0;
  uint64_t* d_fo = nullptr;
  uint64_t* d_oo = nullptr;
  uint64_t d_n_cap = 0;
  uint32_t* d_ids = nullptr;
  uint64_t d_ids_cap = 0;
  ~RWork() {
    (void)hipSetDevice(device);
    if (stream) (void)hipStreamSynchronize(stream);
    rfree(wids);
    rfree(stack);
    rfree(ranges);
    rfree(rcount);
    rfree(rlive);
    rfree(ctrl);
    rfree(fcount);
    rfree(fcursor);
    rfree(wdesc);
    rfree(spill[0]);
    rfree(spill[1]);
    rfree(queue);
    rfree(qctl);
    rfree(partials);
    rfree(prof);
    rfree(d_fb);
    rfree(d_fo);
    rfree(d_oo);
    rfree(d_ids);
    if (h_pinned) (void)hipHostFree(h_pinned);
    if (ev0) (void)hipEventDestroy(ev0);
    if (ev1) (void)hipEventDestroy(ev1);
    if (evw) (void)hipEventDestroy(evw);
    if (stream) (void)hipStreamDestroy(stream);
  }
};

constexpr uint32_t MAX_WAVES = 8192;
// Load balance of the walk: a wave that has not emptied its stack after STEP_BUDGET steps
// spills the rest as 64-node pieces, and the next round deals them evenly over up to
// SPILL_WAVES waves.  The heavy filters' work is wide '+' slices (thousands of nodes per item):
// config R's walk drops from 10.7 to 3.8 ms in 2 rounds (profiles/r1_v8_retain_sweep.txt).
// A round lasts as long as its busiest wave, so short budgets rebalance sooner: 24 steps for
// the first round and 64 for the spill rounds run the config-R walk in 1.38-1.41 ms against
// 1.95-1.96 ms for 128/128 (32: 1.40-1.43 ms; profiles/r3_retain_budget_sweep/; small budgets only paid once the
// spill reservation stopped being a compare-and-swap loop, see spill_reserve).
// emqx_retain_set_tuning "step_budget" / "spill_budget" override them (0 = no budget / the same).
constexpr uint32_t STEP_BUDGET = 24;
constexpr uint32_t SPILL_BUDGET = 64;
constexpr uint32_t SPILL_WAVES = 4096;
constexpr uint32_t SPILL_PER_WAVE = 4;  // spilled pieces dealt to each wave of a spill round
constexpr uint32_t SPILL_CAP = 1u << 22;  // items per spill buffer (a full one: waves keep walking)
constexpr uint32_t SPILL_ROUNDS = 4;      // budgeted spill rounds per call, then one without a
                                          // budget; all enqueued up front, empty ones exit at once
// Queue mode (balance 1, the default): no rounds; a wave that runs out of tiles waits on a ticket
// of the shared-work queue, and busy waves share the bottom of their stacks while waves wait
// (retain_walk_queue_kernel).  A round lasts as long as its busiest wave; the queue has no rounds.
enum : uint32_t { BALANCE_SPILL = 0, BALANCE_QUEUE = 1 };
constexpr uint32_t QUEUE_CAP = 1u << 22;   // shared pieces per call at most (a full queue: waves keep walking)
constexpr uint32_t QUEUE_PIECE = 512;      // nodes per shared piece (8 wave steps)
constexpr uint32_t QUEUE_CHECK = 4;        // steps between a busy wave's looks at the waiting count
constexpr uint32_t QUEUE_POLL_LIMIT = 1u << 20;  // ~1 s of polls: then RC_QABORT, rerun in spill mode
constexpr uint32_t QUEUE_MAX_WAIT = 1u << 16;   // waves waiting on tickets at most (no cap: r4_q7)
constexpr uint32_t QUEUE_SLEEP = 1;              // s_sleep(16) per poll
constexpr uint32_t QUEUE_SHARDS = 512;           // queue shards (waves w % 512 share with each other)
constexpr uint32_t QUEUE_ROAM = 4;               // other shards a wave helps once its own is done

// Filters per wave tile.  The walk is latency-bound (one dependent round trip per step), so the
// number of waves in flight, not lane fill, sets its rate: 64 filters per tile leaves ~6 waves
// per CU for a 100K-filter batch.  With tiles taken first come first served, 10 (10K tiles over
// 8192 waves) runs the config-R walk + spill in 1.96-1.99 ms against 2.23-2.25 ms for 8
// (profiles/r2_retain_sweeps.txt).  The work-sharing walk: 16 (1.055 ms per call against 1.16
// for 10, 1.10 for 14, 1.19 for 20; profiles/r4_retain_queue_sweep.txt, r4_q24/q25).
constexpr uint32_t TILE_FILTERS = 10;
constexpr uint32_t QUEUE_TILE_FILTERS = 16;

uint32_t env_u32(const char* name, uint32_t dflt) {
  const char* e = std::getenv(name);
  if (!e || !*e) return dflt;
  return static_cast<uint32_t>(std::min<unsigned long>(std::strtoul(e, nullptr, 10), 0xFFFFFFFFul));
}

bool has_wild_level(const uint8_t* p, uint64_t n) {
  uint64_t s = 0;
  for (uint64_t i = 0; i <= n; ++i) {
    if (i == n || p[i] == '/') {
      if (i - s == 1 && (p[s] == '+' || p[s] == '#')) return true;
      s = i + 1;
    }
  }
  return false;
}

}  // namespace

struct emqx_retain {
  int device = 0;
  std::mutex writer;
  FilterStore store;           // topic bytes <-> id, liveness
  std::vector<int64_t> expiry;  // per id
  uint64_t epoch = 0;
  double last_build_ms = 0;
  std::mutex snap_mu;
  std::shared_ptr<RSnapshot> snap;
  std::mutex ws_mu;
  std::vector<RWork*> free_ws;
  std::vector<std::unique_ptr<RWork>> all_ws;
  std::atomic<uint64_t> last_ranges{0}, last_visits{0}, last_total{0}, last_spill_rounds{0}, last_spilled{0}, last_spill_full{0},
      last_shares{0}, queue_aborts{0};
  std::atomic<double> last_match_ms{0}, last_walk_ms{0};
  // walk tuning (emqx_retain_set_tuning; the EMQX_RETAIN_* variables give the initial values)
  bool prof_on = false;
  uint32_t ablate = 0;  // EMQX_RETAIN_ABLATE (profiling builds only)  // EMQX_RETAIN_PROF=1 (a RETAIN_PROF build fills the phase counters)
  // tile 0: the balance mode's default
  std::atomic<uint32_t> tile{0}, step_budget{STEP_BUDGET}, spill_budget{SPILL_BUDGET}, spill_decay{0}, spill_per_wave{SPILL_PER_WAVE}, spill_rounds{SPILL_ROUNDS}, search{RSEARCH_STREE},
      walk_waves{MAX_WAVES}, spill_waves{SPILL_WAVES}, spill_cap{SPILL_CAP}, balance{BALANCE_QUEUE},
      lane_map{1}, queue_piece{QUEUE_PIECE}, queue_check{QUEUE_CHECK}, queue_cap{QUEUE_CAP}, queue_wait{QUEUE_MAX_WAIT},
      queue_sleep{QUEUE_SLEEP}, queue_shards{QUEUE_SHARDS}, queue_roam{QUEUE_ROAM}, queue_poll_limit{QUEUE_POLL_LIMIT};
};

namespace {

// The levels of an RSTree over `k0` (level 0 = k0, level k = every 16^k-th key, until a level
// has <= 16 entries), each rst_level_words long: 64-B aligned, with one spare block behind it
// (a scan may read the block just past a level's end); t->n/levels set.
std::vector<uint32_t> build_stree(const std::vector<uint32_t>& k0, RSTree* t) {
  std::vector<uint32_t> buf;
  uint64_t n = k0.size();
  uint32_t k = 0;
  for (;; ++k) {
    const uint64_t base = buf.size(), step = 1ull << (RST_SH * k);
    buf.resize(base + rst_level_words(static_cast<uint32_t>(n)), 0xFFFFFFFFu);
    for (uint64_t i = 0; i < n; ++i) buf[base + i] = k0[i * step];
    if (n <= RST_FAN || k + 1 == RST_MAX) break;
    n = (n + RST_FAN - 1) / RST_FAN;
  }
  t->n = static_cast<uint32_t>(k0.size());
  t->levels = k + 1;
  return buf;
}

// Builds the trie of the live topics: BFS node ids (contiguous children), DFS preorder ranks.
int build_and_upload(emqx_retain* r, std::shared_ptr<RSnapshot>* out) {
  const FilterStore& fs = r->store;
  VocabState vs;
  // pass 1: temporary trie, children as (parent, wid) -> node in a hash map
  std::vector<uint32_t> first_child{WID_NONE}, next_sib{WID_NONE}, term{WID_NONE}, wid_of{WID_NONE};
  std::vector<uint64_t> hkeys;
  std::vector<uint32_t> hvals;
  uint64_t hmask = 0, hsize = 0;
  auto hrehash = [&](uint64_t cap) {
    std::vector<uint64_t> ok;
    std::vector<uint32_t> ov;
    ok.swap(hkeys);
    ov.swap(hvals);
    hkeys.assign(cap, ~0ull);
    hvals.assign(cap, 0);
    hmask = cap - 1;
    for (uint64_t i = 0; i < ok.size(); ++i) {
      if (ok[i] == ~0ull) continue;
      uint64_t j = (ok[i] * 0x9E3779B97F4A7C15ull >> 20) & hmask;
      while (hkeys[j] != ~0ull) j = (j + 1) & hmask;
      hkeys[j] = ok[i];
      hvals[j] = ov[i];
    }
  };
  hrehash(1024);
  auto child_of = [&](uint32_t parent, uint32_t wid) -> uint32_t {
    const uint64_t key = static_cast<uint64_t>(parent) << 32 | wid;
    uint64_t j = (key * 0x9E3779B97F4A7C15ull >> 20) & hmask;
    while (hkeys[j] != ~0ull) {
      if (hkeys[j] == key) return hvals[j];
      j = (j + 1) & hmask;
    }
    const uint32_t c = static_cast<uint32_t>(term.size());
    first_child.push_back(WID_NONE);
    term.push_back(WID_NONE);
    wid_of.push_back(wid);
    next_sib.push_back(first_child[parent]);
    first_child[parent] = c;
    hkeys[j] = key;
    hvals[j] = c;
    if (++hsize * 2 > hkeys.size()) hrehash(hkeys.size() * 2);
    return c;
  };
  const uint64_t n_ids = fs.n_ids();
  for (uint64_t id = 0; id < n_ids; ++id) {
    if (!fs.live[id]) continue;
    const uint8_t* p = fs.bytes.data() + fs.off[id];
    const uint64_t n = fs.off[id + 1] - fs.off[id];
    uint32_t node = 0;
    uint64_t s = 0;
    for (uint64_t i = 0; i <= n; ++i) {
      if (i == n || p[i] == '/') {
        node = child_of(node, vs.intern(p + s, i - s));
        s = i + 1;
      }
    }
    term[node] = static_cast<uint32_t>(id);
  }
  const uint64_t nn = term.size();
  if (nn >= 0x7FFFFFFFull) return EMQX_ENOMEM;
  // pass 2: BFS ids (children contiguous)
  std::vector<uint32_t> order;  // bfs index -> temp node
  order.reserve(nn);
  std::vector<RNode> nodes(nn);
  order.push_back(0);
  std::vector<uint32_t> depth(nn, 0);
  for (uint64_t k = 0; k < order.size(); ++k) {
    const uint32_t v = order[k];
    const uint32_t cb = static_cast<uint32_t>(order.size());
    uint32_t nc = 0;
    for (uint32_t c = first_child[v]; c != WID_NONE; c = next_sib[c]) {
      depth[order.size()] = depth[k] + 1;
      order.push_back(c);
      ++nc;
    }
    nodes[k].cbeg = cb;
    nodes[k].ncld = nc | (term[v] != WID_NONE ? RNODE_TERM : 0u);
  }
  // pass 3: DFS preorder ranks (a node's own topic, then its children's subtrees)
  std::vector<uint32_t> rank_id;
  rank_id.reserve(fs.n_live);
  {
    std::vector<std::pair<uint32_t, uint32_t>> st;  // (bfs node, next child index)
    st.push_back({0, 0});
    nodes[0].lo = 0;
    while (!st.empty()) {
      auto& [v, ci] = st.back();
      RNode& rn = nodes[v];
      const uint32_t nc = rn.ncld & ~RNODE_TERM;
      if (ci < nc) {
        const uint32_t c = rn.cbeg + ci;
        ++ci;
        RNode& cn = nodes[c];
        cn.lo = static_cast<uint32_t>(rank_id.size());
        if (cn.ncld & RNODE_TERM) rank_id.push_back(term[order[c]]);
        st.push_back({c, 0});
      } else {
        rn.hi = static_cast<uint32_t>(rank_id.size());
        st.pop_back();
      }
    }
  }
  // per-depth rank lists (ascending: ranks follow DFS preorder)
  uint32_t max_depth = 0;
  for (uint64_t k = 0; k < nn; ++k)
    if (nodes[k].ncld & RNODE_TERM) max_depth = std::max(max_depth, depth[k]);
  std::vector<uint32_t> dterm_off(max_depth + 2, 0), dterm(std::max<uint64_t>(rank_id.size(), 1));
  std::vector<uint16_t> rank_depth;
  for (uint64_t k = 0; k < nn; ++k)
    if (nodes[k].ncld & RNODE_TERM) dterm_off[depth[k] + 1] += 1;
  for (uint32_t d = 0; d <= max_depth; ++d) dterm_off[d + 1] += dterm_off[d];
  {
    std::vector<uint32_t> cur(dterm_off.begin(), dterm_off.end() - 1);
    std::vector<uint32_t> depth_of_rank(rank_id.size());
    for (uint64_t k = 0; k < nn; ++k)
      if (nodes[k].ncld & RNODE_TERM) depth_of_rank[nodes[k].lo] = depth[k];
    for (uint64_t rk = 0; rk < rank_id.size(); ++rk) dterm[cur[depth_of_rank[rk]]++] = static_cast<uint32_t>(rk);
    rank_depth.resize(std::max<uint64_t>(rank_id.size(), 1), 0);
    for (uint64_t rk = 0; rk < rank_id.size(); ++rk)
      rank_depth[rk] = static_cast<uint16_t>(std::min<uint32_t>(depth_of_rank[rk], 65535));
  }
  std::vector<int64_t> rank_exp(rank_id.size());
  uint32_t has_exp = 0;
  for (uint64_t i = 0; i < rank_id.size(); ++i) {
    rank_exp[i] = r->expiry[rank_id[i]];
    has_exp |= rank_exp[i] != 0;
  }
  // level postings: nodes grouped by (depth, word), each group sorted by lo
  std::vector<uint32_t> pid(nn > 0 ? nn - 1 : 0);
  for (uint64_t k = 1; k < nn; ++k) pid[k - 1] = static_cast<uint32_t>(k);
  std::sort(pid.begin(), pid.end(), [&](uint32_t x, uint32_t y) {
    if (depth[x] != depth[y]) return depth[x] < depth[y];
    const uint32_t wx = wid_of[order[x]], wy = wid_of[order[y]];
    if (wx != wy) return wx < wy;
    return nodes[x].lo < nodes[y].lo;
  });
  std::vector<uint4> posts(std::max<uint64_t>(pid.size(), 1), make_uint4(0, 0, 0, 0));
  std::vector<RPostKey> groups;
  for (uint64_t i = 0; i < pid.size(); ++i) {
    const uint32_t x = pid[i];
    posts[i] = make_uint4(nodes[x].lo, x, nodes[x].ncld, nodes[x].hi);
    const uint32_t d = depth[x], w = wid_of[order[x]];
    if (groups.empty() || groups.back().depth != d || groups.back().wid != w)
      groups.push_back(RPostKey{d, w, static_cast<uint32_t>(i), 0});
    groups.back().len += 1;
  }
  uint64_t pcap = 1024;
  while (pcap < 2 * groups.size()) pcap <<= 1;
  std::vector<RPostKey> pkeys(pcap, RPostKey{WID_NONE, 0, 0, 0});
  const uint32_t pmask = static_cast<uint32_t>(pcap - 1);
  for (const RPostKey& g : groups) {
    uint32_t sl = rpost_slot0(g.depth, g.wid) & pmask;
    while (pkeys[sl].depth != WID_NONE) sl = (sl + 1) & pmask;
    pkeys[sl] = g;
  }
  // a node's name: its postings index (the root: RNAME_ROOT)
  std::vector<uint32_t> name(nn, RNAME_ROOT);
  for (uint64_t i = 0; i < pid.size(); ++i) name[pid[i]] = static_cast<uint32_t>(i);
  // literal lookup table (parent name, wid) -> child name: buckets of REDGE_BUCKET edges at
  // load <= 3/8; an edge goes to the first bucket from its hash with a free slot, flagging
  // every full bucket it passes (REDGE_OVF)
  uint64_t nbk = 256;
  while (nbk * REDGE_BUCKET * 3 < 8 * nn) nbk <<= 1;
  REdgeBucket empty{};
  for (uint32_t i = 0; i < REDGE_BUCKET; ++i) {
    empty.key[i] = make_uint2(WID_NONE, 0);
    empty.child[i] = 0;
  }
  std::vector<REdgeBucket> edges(nbk, empty);
  const uint32_t emask = static_cast<uint32_t>(nbk - 1);
  for (uint64_t v = 0; v < nn; ++v) {
    const uint32_t nc = nodes[v].ncld & ~RNODE_TERM;
    for (uint32_t j = 0; j < nc; ++j) {
      const uint32_t c = nodes[v].cbeg + j;
      const uint32_t w = wid_of[order[c]];
      uint32_t bk = redge_slot0(name[v], w) & emask;
      uint32_t i = 0;
      for (;;) {
        i = 0;
        while (i < REDGE_BUCKET && edges[bk].key[i].x != WID_NONE) ++i;
        if (i < REDGE_BUCKET) break;
        edges[bk].key[0].y |= REDGE_OVF;
        bk = (bk + 1) & emask;
      }
      edges[bk].key[i] = make_uint2(name[v], w | (edges[bk].key[i].y & REDGE_OVF));
      edges[bk].child[i] = name[c];
    }
  }
  vs.build_table();

  auto sn = std::make_shared<RSnapshot>();
  sn->device = r->device;
  const uint64_t nr = std::max<uint64_t>(rank_id.size(), 1);
  RT_TRY(ralloc(sn->edges, nbk));
  RT_TRY(ralloc(sn->vocab, vs.table.size()));
  RT_TRY(ralloc(sn->arena, vs.arena.size() + 16));
  RT_TRY(ralloc(sn->rank_id, nr));
  RT_TRY(ralloc(sn->rank_exp, nr));
  RT_TRY(ralloc(sn->pkeys, pcap));
  RT_TRY(ralloc(sn->posts, posts.size()));
  RT_TRY(hipMemcpy(sn->pkeys, pkeys.data(), pcap * sizeof(RPostKey), hipMemcpyHostToDevice));
  RT_TRY(hipMemcpy(sn->posts, posts.data(), posts.size() * sizeof(uint4), hipMemcpyHostToDevice));
  RT_TRY(ralloc(sn->dterm_off, dterm_off.size()));
  RT_TRY(ralloc(sn->dterm, dterm.size()));
  RT_TRY(hipMemcpy(sn->dterm_off, dterm_off.data(), dterm_off.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
  RT_TRY(hipMemcpy(sn->dterm, dterm.data(), dterm.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
  // search trees of the postings keys and the per-depth rank lists (RSTree)
  std::vector<uint32_t> pkey(posts.size());
  for (uint64_t i = 0; i < posts.size(); ++i) pkey[i] = posts[i].x;
  RSTree pst{}, dst{};
  const std::vector<uint32_t> pst_h = build_stree(pkey, &pst), dst_h = build_stree(dterm, &dst);
  RT_TRY(ralloc(sn->pst, pst_h.size()));
  RT_TRY(ralloc(sn->dst, dst_h.size()));
  RT_TRY(hipMemcpy(sn->pst, pst_h.data(), pst_h.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
  RT_TRY(hipMemcpy(sn->dst, dst_h.data(), dst_h.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
  pst.keys = sn->pst;
  dst.keys = sn->dst;
  std::vector<uint32_t> pfence((posts.size() + RFENCE - 1) / RFENCE), dfence((dterm.size() + RFENCE - 1) / RFENCE);
  for (uint64_t b = 0; b < pfence.size(); ++b) pfence[b] = posts[b * RFENCE].x;
  for (uint64_t b = 0; b < dfence.size(); ++b) dfence[b] = dterm[b * RFENCE];
  RT_TRY(ralloc(sn->pfence, pfence.size()));
  RT_TRY(ralloc(sn->dfence, dfence.size()));
  RT_TRY(hipMemcpy(sn->pfence, pfence.data(), pfence.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
  RT_TRY(hipMemcpy(sn->dfence, dfence.data(), dfence.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
  RT_TRY(ralloc(sn->rank_depth, rank_depth.size()));
  RT_TRY(hipMemcpy(sn->rank_depth, rank_depth.data(), rank_depth.size() * sizeof(uint16_t), hipMemcpyHostToDevice));
  RT_TRY(hipMemcpy(sn->edges, edges.data(), nbk * sizeof(REdgeBucket), hipMemcpyHostToDevice));
  RT_TRY(hipMemcpy(sn->vocab, vs.table.data(), vs.table.size() * sizeof(VocabSlot), hipMemcpyHostToDevice));
  if (!vs.arena.empty()) RT_TRY(hipMemcpy(sn->arena, vs.arena.data(), vs.arena.size(), hipMemcpyHostToDevice));
  if (!rank_id.empty()) {
    RT_TRY(hipMemcpy(sn->rank_id, rank_id.data(), rank_id.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    RT_TRY(hipMemcpy(sn->rank_exp, rank_exp.data(), rank_exp.size() * sizeof(int64_t), hipMemcpyHostToDevice));
  }
  // the copies' DMA has landed before the snapshot is used from another stream (pageable
  // copies may return early; the walk streams do not follow the null stream)
  RT_TRY(hipStreamSynchronize(nullptr));
  RetainView& rv = sn->rv;
  rv.root_ncld = nn ? nodes[0].ncld : 0u;
  rv.root_lo = nn ? nodes[0].lo : 0u;
  rv.root_hi = nn ? nodes[0].hi : 0u;
  rv.edges = sn->edges;
  rv.edge_mask = emask;
  rv.vocab = sn->vocab;
  rv.arena = sn->arena;
  rv.vocab_mask = vs.mask;
  rv.rank_id = sn->rank_id;
  rv.rank_exp = sn->rank_exp;
  rv.pkeys = sn->pkeys;
  rv.pkey_mask = pmask;
  rv.posts = sn->posts;
  rv.dterm_off = sn->dterm_off;
  rv.dterm = sn->dterm;
  rv.pst = pst;
  rv.dst = dst;
  rv.pfence = sn->pfence;
  rv.dfence = sn->dfence;
  rv.max_depth = max_depth;
  rv.rank_depth = sn->rank_depth;
  rv.n_nodes = rank_id.empty() ? 0u : static_cast<uint32_t>(nn);
  rv.has_expiring = has_exp;
  sn->n_nodes = nn;
  sn->n_words = vs.n_words();
  sn->bytes = nbk * sizeof(REdgeBucket) + vs.table.size() * sizeof(VocabSlot) + vs.arena.size() +
              nr * (sizeof(uint32_t) + sizeof(int64_t)) + pcap * sizeof(RPostKey) + posts.size() * sizeof(uint4) +
              (dterm_off.size() + dterm.size() + pst_h.size() + dst_h.size() + pfence.size() + dfence.size()) *
                  sizeof(uint32_t) +
              rank_depth.size() * sizeof(uint16_t);
  *out = std::move(sn);
  return EMQX_OK;
}

std::shared_ptr<RSnapshot> current(emqx_retain* r) {
  std::lock_guard<std::mutex> g(r->snap_mu);
  return r->snap;
}

int acquire(emqx_retain* r, RWork** out) {
  {
    std::lock_guard<std::mutex> g(r->ws_mu);
    if (!r->free_ws.empty()) {
      *out = r->free_ws.back();
      r->free_ws.pop_back();
      return EMQX_OK;
    }
  }
  auto w = std::make_unique<RWork>();
  w->device = r->device;
  RT_TRY(hipStreamCreateWithFlags(&w->stream, hipStreamNonBlocking));
  RT_TRY(hipEventCreate(&w->ev0));
  RT_TRY(hipEventCreate(&w->ev1));
  RT_TRY(hipEventCreate(&w->evw));
  RT_TRY(ralloc(w->ctrl, RC_WORDS));
  RT_TRY(hipHostMalloc(reinterpret_cast<void**>(&w->h_pinned), (RC_WORDS / 2 + 1) * sizeof(uint64_t), hipHostMallocDefault));
  std::lock_guard<std::mutex> g(r->ws_mu);
  *out = w.get();
  r->all_ws.push_back(std::move(w));
  return EMQX_OK;
}

void release(emqx_retain* r, RWork* w) {
  std::lock_guard<std::mutex> g(r->ws_mu);
  r->free_ws.push_back(w);
}

// The pipeline on device buffers.  *total = ids the batch needs; ids written iff it fits.
int run_match(emqx_retain* r, RWork* w, const RSnapshot& sn, const uint8_t* d_fb, const uint64_t* d_fo,
              uint64_t n, uint64_t byte_span, int64_t now_ms, uint64_t* d_oo, uint32_t* d_ids, uint64_t cap,
              hipStream_t s, uint64_t* total, bool strict_all = false) {
  RetainArgs a{};
  a.rv = sn.rv;
  a.strict_all = strict_all ? RRANGE_STRICT : 0u;
  a.fbytes = d_fb;
  a.foffs = d_fo;
  a.n = n;
  a.now_ms = now_ms;
  a.out_off = d_oo;
  a.out_ids = d_ids;
  a.out_cap = cap;
  const uint64_t need_w = byte_span + n + 1;
  if (need_w > w->wids_cap) {
    RT_TRY(ralloc(w->wids, need_w + need_w / 4));
    w->wids_cap = need_w + need_w / 4;
  }
  const uint64_t need_d = byte_span + 2 * n + 1;
  if (need_d > w->wdesc_cap) {
    RT_TRY(ralloc(w->wdesc, need_d + need_d / 4));
    w->wdesc_cap = need_d + need_d / 4;
  }
  if (n > w->f_cap) {
    RT_TRY(ralloc(w->fcount, n + n / 4));
    RT_TRY(ralloc(w->fcursor, n + n / 4));
    w->f_cap = n + n / 4;
  }
  const uint64_t np = scan_partials(n);
  if (np > w->partials_cap) {
    RT_TRY(ralloc(w->partials, np));
    w->partials_cap = np;
  }
  if (w->range_cap == 0) {
    const uint64_t rc = std::max<uint64_t>(4 * n, 1 << 16);
    RT_TRY(ralloc(w->ranges, rc));
    RT_TRY(ralloc(w->rcount, rc));
    RT_TRY(ralloc(w->rlive, 5 * rc));
    w->range_cap = static_cast<uint32_t>(rc);
  }
  bool queue = r->balance.load() == BALANCE_QUEUE;
  const uint32_t tile = r->tile.load();
  a.tile_filters = tile ? std::min<uint32_t>(64, tile) : queue ? QUEUE_TILE_FILTERS : TILE_FILTERS;
  a.search = r->search.load();
  const uint64_t ntiles = (n + a.tile_filters - 1) / a.tile_filters;
  const uint32_t spill_waves = std::max<uint32_t>(64, r->spill_waves.load());
  a.waves = static_cast<uint32_t>(std::min<uint64_t>(ntiles, std::max<uint32_t>(64, r->walk_waves.load())));
  a.wids = w->wids;
  a.ctrl = w->ctrl;
  a.fcount = w->fcount;
  a.fcursor = w->fcursor;
  if (w->spill_cap == 0) {
    RT_TRY(ralloc(w->spill[0], SPILL_CAP));
    RT_TRY(ralloc(w->spill[1], SPILL_CAP));
    w->spill_cap = SPILL_CAP;
  }
  a.wdesc = w->wdesc;
  a.wdesc_n = need_d;
  a.spill_cap = std::min<uint32_t>(w->spill_cap, r->spill_cap.load());
  if (queue && w->queue_cap == 0) {
    RT_TRY(ralloc(w->queue, QUEUE_CAP));
    RT_TRY(hipMemsetAsync(w->queue, 0, static_cast<uint64_t>(QUEUE_CAP) * sizeof(uint4), s));
    RT_TRY(ralloc(w->qctl, static_cast<uint64_t>(QS_MAX_SHARDS) * QS_STRIDE));
    RT_TRY(hipMemsetAsync(w->qctl, 0, static_cast<uint64_t>(QS_MAX_SHARDS) * QS_STRIDE * sizeof(uint32_t), s));
    w->queue_cap = QUEUE_CAP;
  }
  a.qctl = w->qctl;
  a.qshards = r->queue_shards.load();
  a.queue = w->queue;
  a.queue_cap = std::min<uint32_t>(w->queue_cap, r->queue_cap.load());
  a.qpiece = std::max<uint32_t>(64, r->queue_piece.load());
  a.qcheck = r->queue_check.load();
  a.ownmap = r->lane_map.load();
  a.qpoll_limit = r->queue_poll_limit.load();
  a.qmaxwait = r->queue_wait.load();
  a.qsleep = r->queue_sleep.load();
  a.qroam = std::min<uint32_t>(r->queue_roam.load(), a.qshards - 1);
  a.ntiles = static_cast<uint32_t>(ntiles);
  const uint32_t budget = r->step_budget.load();
  a.step_budget = budget == 0 ? ~0u : budget;
  const uint32_t per_wave = std::max<uint32_t>(1, r->spill_per_wave.load());
  const uint32_t rounds = a.step_budget == ~0u ? 0u : r->spill_rounds.load();
  const uint32_t spill_budget = r->spill_budget.load();
  const uint32_t spill_decay = r->spill_decay.load();  // round k's budget: spill_budget >> (k * decay), >= 8
  const uint32_t* c = reinterpret_cast<const uint32_t*>(w->h_pinned);
  for (int attempt = 0;; ++attempt) {
    const uint64_t stack_waves = static_cast<uint64_t>(w->stack_cap) <= (1u << 14) ? std::max(a.waves, spill_waves) : a.waves;
    if (stack_waves * w->stack_cap > w->stack_items) {
      const uint64_t items = stack_waves * w->stack_cap;
      RT_TRY(ralloc(w->stack, items));
      w->stack_items = items;
    }
    a.stack = w->stack;
    a.stack_cap = w->stack_cap;
    a.ranges = w->ranges;
    a.rcount = w->rcount;
    a.rlive = w->rlive;
    a.range_cap = w->range_cap;
    a.spill_out = w->spill[0];
    a.spill_word = RC_SPILL;
    // the whole call is enqueued at once: walk, `rounds` budgeted spill rounds and one without
    // a budget (each reads its item count on the device; an empty round exits at once), the
    // range count, the scan, the write (skipped on the device when the ids do not fit); then
    // one readback of the control words and the total
    RT_TRY(hipEventRecord(w->ev0, s));
    RT_TRY(hipMemsetAsync(w->ctrl, 0, RC_WORDS * sizeof(uint32_t), s));
    // reserved but unused record slots must read as empty ranges
    RT_TRY(hipMemsetAsync(w->ranges, 0, static_cast<uint64_t>(w->range_cap) * sizeof(RRange), s));
    if (r->prof_on) {
      if (!w->prof) RT_TRY(ralloc(w->prof, 20));
      RT_TRY(hipMemsetAsync(w->prof, 0, 20 * sizeof(uint64_t), s));
      a.prof = w->prof;
      a.ablate = r->ablate;
    }
    const uint64_t fit = w->stack_items / w->stack_cap;
    if (queue) {
      RT_TRY(launch_retain_walk_queue(a, s));  // its last kernel zeroes the queue again
    } else {
      RT_TRY(launch_retain_walk(a, s));
    }
    for (uint32_t k = 0; !queue && k <= rounds; ++k) {
      RetainArgs b = a;
      b.waves = static_cast<uint32_t>(std::max<uint64_t>(1, std::min<uint64_t>(spill_waves, fit)));
      const uint32_t in_word = RC_SPILL + 2 * k;
      b.spill_word = in_word + 2;
      b.spill_out = w->spill[(k + 1) & 1];
      if (k == rounds) b.step_budget = ~0u;  // the last round finishes every stack
      else if (spill_budget) b.step_budget = std::max<uint32_t>(8u, spill_budget >> std::min<uint32_t>(k * spill_decay, 31u));
      RT_TRY(launch_retain_walk_spill(b, w->spill[k & 1], in_word, per_wave, s));
    }
    RT_TRY(hipEventRecord(w->evw, s));
    RT_TRY(hipMemsetAsync(w->fcount, 0, n * sizeof(uint32_t), s));
    RT_TRY(hipMemsetAsync(w->fcursor, 0, n * sizeof(uint32_t), s));
    RT_TRY(launch_retain_count(a, s));
    RT_TRY(launch_scan(w->fcount, n, d_oo, w->partials, s));
    RT_TRY(launch_retain_write(a, s));
    RT_TRY(hipEventRecord(w->ev1, s));
    RT_TRY(hipMemcpyAsync(w->h_pinned, w->ctrl, RC_WORDS * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    RT_TRY(hipMemcpyAsync(w->h_pinned + RC_WORDS / 2, d_oo + n, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    RT_TRY(hipStreamSynchronize(s));
    const uint64_t ranges = static_cast<uint64_t>(c[RC_RANGES]) + c[RC_BIG];
    uint32_t visits = 0, emitted = 0, qpieces = 0, qshares = 0;
    for (uint32_t l = 0; l < RC_STAT_LINES; ++l) {
      visits += c[RC_STAT + 16 * l];
      emitted += c[RC_STAT + 16 * l + 1];
      qpieces += c[RC_STAT + 16 * l + 2];
      qshares += c[RC_STAT + 16 * l + 3];
    }
    const uint32_t ovf = c[RC_STACK];
    bool again = false;
    if (queue && c[RC_QABORT]) {
      // a waiting wave gave up (never expected: the safety valve of the queue's termination):
      // rerun in spill mode
      r->queue_aborts.fetch_add(1);
      queue = false;
      again = true;
    }
    if (ovf) {
      if (w->stack_cap >= (1u << 24) || attempt > 8) return EMQX_ETOODEEP;
      w->stack_cap *= 4;
      again = true;
    }
    if (ranges > w->range_cap) {
      const uint64_t rc = ranges + ranges / 4 + 1024;
      if (rc > 0xFFFFFFF0ull) return EMQX_ENOMEM;
      RT_TRY(ralloc(w->ranges, rc));
      RT_TRY(ralloc(w->rcount, rc));
      RT_TRY(ralloc(w->rlive, 5 * rc));
      w->range_cap = static_cast<uint32_t>(rc);
      again = true;
    }
    if (!again && r->prof_on)
      std::fprintf(stderr, "RETAIN_CTRL spilled %u rounds %u spill_fail %u spill_max %u visits %u small %u big %u emitted %u\n",
                   c[RC_SPILLED], c[RC_ROUNDS], c[RC_SPILLFAIL], c[RC_SPILLMAX], visits, c[RC_RANGES], c[RC_BIG], emitted);
    if (!again && r->prof_on) {
      uint64_t pr[20];
      if (hipMemcpy(pr, w->prof, sizeof(pr), hipMemcpyDeviceToHost) == hipSuccess) {
        std::fprintf(stderr, "RETAIN_PROF take %llu node %llu probe %llu search %llu emitpush %llu steps %llu active %llu searching %llu\n",
                     (unsigned long long)pr[0], (unsigned long long)pr[1], (unsigned long long)pr[2],
                     (unsigned long long)pr[3], (unsigned long long)pr[4], (unsigned long long)pr[5],
                     (unsigned long long)pr[6], (unsigned long long)pr[7]);
        std::fprintf(stderr, "RETAIN_QPROF wait %llu ticket %llu retire %llu share %llu pieces %llu tilewalk %llu piecewalk %llu capped %llu\n",
                     (unsigned long long)pr[8], (unsigned long long)pr[9], (unsigned long long)pr[10],
                     (unsigned long long)pr[11], (unsigned long long)pr[12], (unsigned long long)pr[13],
                     (unsigned long long)pr[14], (unsigned long long)pr[15]);
        std::fprintf(stderr, "RETAIN_SPROF groups %llu in_ge8 %llu in_ge32 %llu\n", (unsigned long long)pr[16],
                     (unsigned long long)pr[17], (unsigned long long)pr[18]);
      }
    }
    if (!again) {
      r->last_ranges.store(emitted);
      r->last_visits.store(visits);
      r->last_spill_rounds.store(queue ? 0u : c[RC_ROUNDS]);
      r->last_spilled.store(queue ? qpieces : c[RC_SPILLED]);
      r->last_spill_full.store(queue ? 0u : c[RC_SPILLFAIL]);
      r->last_shares.store(queue ? qshares : 0u);
      break;
    }
  }
  *total = w->h_pinned[RC_WORDS / 2];
  r->last_total.store(*total);
  float ms = 0, wms = 0;
  if (hipEventElapsedTime(&ms, w->ev0, w->ev1) == hipSuccess) r->last_match_ms.store(ms);
  if (hipEventElapsedTime(&wms, w->ev0, w->evw) == hipSuccess) r->last_walk_ms.store(wms);
  return *total <= cap ? EMQX_OK : EMQX_EOVERFLOW;
}

}  // namespace

extern "C" {

int emqx_retain_create(int32_t device, emqx_retain** out) {
  if (!out) return EMQX_EINVAL;
  int nd = 0;
  if (hipGetDeviceCount(&nd) != hipSuccess || nd == 0) return EMQX_EDEVICE;
  if (device < 0) RT_TRY(hipGetDevice(&device));
  if (device >= nd) return EMQX_EINVAL;
  emqx_retain* r = new (std::nothrow) emqx_retain();
  if (!r) return EMQX_ENOMEM;
  r->device = device;
  r->tile = std::min<uint32_t>(64, env_u32("EMQX_RETAIN_TILE", 0));  // 0: the mode's default
  r->step_budget = env_u32("EMQX_RETAIN_STEP_BUDGET", STEP_BUDGET);
  r->spill_budget = env_u32("EMQX_RETAIN_SPILL_BUDGET", SPILL_BUDGET);
  r->spill_decay = std::min<uint32_t>(4, env_u32("EMQX_RETAIN_SPILL_DECAY", 0));
  r->spill_per_wave = std::max<uint32_t>(1, env_u32("EMQX_RETAIN_SPILL_PER_WAVE", SPILL_PER_WAVE));
  r->spill_rounds = std::min<uint32_t>(RC_MAX_ROUNDS, env_u32("EMQX_RETAIN_SPILL_ROUNDS", SPILL_ROUNDS));
  r->search = std::min<uint32_t>(env_u32("EMQX_RETAIN_SEARCH", RSEARCH_STREE), RSEARCH_STREE);
  r->walk_waves = env_u32("EMQX_RETAIN_WALK_WAVES", MAX_WAVES);
  r->spill_waves = env_u32("EMQX_RETAIN_SPILL_WAVES", SPILL_WAVES);
  r->balance = std::min<uint32_t>(env_u32("EMQX_RETAIN_BALANCE", BALANCE_QUEUE), BALANCE_QUEUE);
  {
    const uint32_t qc = env_u32("EMQX_RETAIN_QUEUE_CHECK", QUEUE_CHECK);
    r->lane_map = env_u32("EMQX_RETAIN_LANE_MAP", 1) ? 1u : 0u;
  r->queue_check = qc >= 1 && qc <= 1024 && (qc & (qc - 1)) == 0 ? qc : QUEUE_CHECK;
  }
  r->queue_piece = std::max<uint32_t>(64, env_u32("EMQX_RETAIN_QUEUE_PIECE", QUEUE_PIECE));
  r->queue_wait = std::max<uint32_t>(1, env_u32("EMQX_RETAIN_QUEUE_WAIT", QUEUE_MAX_WAIT));
  r->queue_sleep = std::min<uint32_t>(64, env_u32("EMQX_RETAIN_QUEUE_SLEEP", QUEUE_SLEEP));
  r->queue_shards = std::max<uint32_t>(1, std::min<uint32_t>(QS_MAX_SHARDS, env_u32("EMQX_RETAIN_QUEUE_SHARDS", QUEUE_SHARDS)));
  r->queue_roam = std::min<uint32_t>(QS_MAX_SHARDS, env_u32("EMQX_RETAIN_QUEUE_ROAM", QUEUE_ROAM));
  r->prof_on = env_u32("EMQX_RETAIN_PROF", 0) != 0;
  r->ablate = env_u32("EMQX_RETAIN_ABLATE", 0);
  *out = r;
  return EMQX_OK;
}

int emqx_retain_destroy(emqx_retain* r) {
  if (!r) return EMQX_EINVAL;
  (void)hipSetDevice(r->device);
  r->snap.reset();
  r->all_ws.clear();
  delete r;
  return EMQX_OK;
}

int emqx_retain_store(emqx_retain* r, const uint8_t* bytes, const uint64_t* offsets, uint64_t n,
                      const int64_t* expiry_ms, uint32_t* ids_out) {
  if (!r || (n && (!bytes || !offsets))) return EMQX_EINVAL;
  for (uint64_t i = 0; i < n; ++i) {
    if (offsets[i + 1] < offsets[i] || offsets[i + 1] - offsets[i] > 65535) return EMQX_EINVAL;
    if (has_wild_level(bytes + offsets[i], offsets[i + 1] - offsets[i])) return EMQX_EINVAL;
  }
  std::lock_guard<std::mutex> g(r->writer);
  for (uint64_t i = 0; i < n; ++i) {
    bool created = false;
    const uint32_t id = r->store.insert(bytes + offsets[i], offsets[i + 1] - offsets[i], &created);
    if (created) r->expiry.push_back(0);
    r->expiry[id] = expiry_ms ? expiry_ms[i] : 0;
    if (ids_out) ids_out[i] = id;
  }
  return EMQX_OK;
}

int emqx_retain_delete(emqx_retain* r, const uint32_t* ids, uint64_t n) {
  if (!r || (n && !ids)) return EMQX_EINVAL;
  std::lock_guard<std::mutex> g(r->writer);
  for (uint64_t i = 0; i < n; ++i) {
    if (ids[i] < r->store.n_ids() && r->store.live[ids[i]]) {
      r->store.live[ids[i]] = 0;
      r->store.n_live -= 1;
    }
  }
  return EMQX_OK;
}

int emqx_retain_lookup(emqx_retain* r, const uint8_t* bytes, uint64_t len, uint32_t* id_out) {
  if (!r || (len && !bytes) || !id_out) return EMQX_EINVAL;
  std::lock_guard<std::mutex> g(r->writer);
  const uint32_t id = r->store.find(bytes, len);
  if (id == WID_NONE || !r->store.live[id]) return EMQX_ENOTFOUND;
  *id_out = id;
  return EMQX_OK;
}

int emqx_retain_topic(emqx_retain* r, uint32_t id, uint8_t* buf, uint64_t cap, uint64_t* len_out) {
  if (!r || !len_out) return EMQX_EINVAL;
  std::lock_guard<std::mutex> g(r->writer);
  if (id >= r->store.n_ids()) return EMQX_ENOTFOUND;
  const uint64_t a = r->store.off[id], b = r->store.off[id + 1];
  *len_out = b - a;
  if (buf) std::memcpy(buf, r->store.bytes.data() + a, std::min(cap, b - a));
  return EMQX_OK;
}

int emqx_retain_expired(emqx_retain* r, int64_t now_ms, uint32_t* ids_out, uint64_t cap, uint64_t* n_out) {
  if (!r || !n_out) return EMQX_EINVAL;
  std::lock_guard<std::mutex> g(r->writer);
  uint64_t k = 0;
  for (uint64_t id = 0; id < r->store.n_ids(); ++id) {
    if (!r->store.live[id] || r->expiry[id] == 0 || r->expiry[id] >= now_ms) continue;
    if (ids_out && k < cap) ids_out[k] = static_cast<uint32_t>(id);
    ++k;
  }
  *n_out = k;
  return k <= cap ? EMQX_OK : EMQX_EOVERFLOW;
}

int emqx_retain_commit(emqx_retain* r) {
  if (!r) return EMQX_EINVAL;
  std::lock_guard<std::mutex> g(r->writer);
  RT_TRY(hipSetDevice(r->device));
  const auto t0 = std::chrono::steady_clock::now();
  std::shared_ptr<RSnapshot> sn;
  const int rc = build_and_upload(r, &sn);
  if (rc != EMQX_OK) return rc;
  {
    std::lock_guard<std::mutex> gs(r->snap_mu);
    r->snap = std::move(sn);
  }
  r->epoch += 1;
  r->last_build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return EMQX_OK;
}

int emqx_retain_match_batch_device(emqx_retain* r, const uint8_t* d_fb, const uint64_t* d_fo, uint64_t n,
                                   int64_t now_ms, uint64_t* d_oo, uint32_t* d_ids, uint64_t out_cap,
                                   uint64_t* n_out, void* stream) {
  if (!r || !n_out || (n && (!d_fb || !d_fo)) || !d_oo) return EMQX_EINVAL;
  RT_TRY(hipSetDevice(r->device));
  auto sn = current(r);
  if (!sn) {  // nothing committed yet: commit the (possibly empty) store
    const int rc = emqx_retain_commit(r);
    if (rc != EMQX_OK) return rc;
    sn = current(r);
  }
  RWork* w = nullptr;
  int rc = acquire(r, &w);
  if (rc != EMQX_OK) return rc;
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : w->stream;
  if (!stream && after_null_stream(s) != hipSuccess) {
    release(r, w);
    return EMQX_EDEVICE;
  }
  uint64_t span = 0;
  if (n) {
    uint64_t ends[2];
    rc = hipMemcpyAsync(&ends[0], d_fo, sizeof(uint64_t), hipMemcpyDeviceToHost, s) == hipSuccess &&
                 hipMemcpyAsync(&ends[1], d_fo + n, sizeof(uint64_t), hipMemcpyDeviceToHost, s) == hipSuccess &&
                 hipStreamSynchronize(s) == hipSuccess
             ? EMQX_OK
             : EMQX_EDEVICE;
    span = ends[1] - ends[0];
  } else {
    rc = hipMemsetAsync(d_oo, 0, sizeof(uint64_t), s) == hipSuccess && hipStreamSynchronize(s) == hipSuccess
             ? EMQX_OK
             : EMQX_EDEVICE;
    *n_out = 0;
    release(r, w);
    return rc;
  }
  uint64_t total = 0;
  if (rc == EMQX_OK) rc = run_match(r, w, *sn, d_fb, d_fo, n, span, now_ms, d_oo, d_ids, out_cap, s, &total);
  *n_out = total;
  release(r, w);
  return rc;
}

namespace {

int match_host(emqx_retain* r, const uint8_t* fb, const uint64_t* fo, uint64_t n, int64_t now_ms,
               uint64_t* out_offsets, uint32_t* out_ids, uint64_t out_cap, uint64_t* n_out, bool strict_all) {
  if (!r || !n_out || !out_offsets || (n && (!fb || !fo))) return EMQX_EINVAL;
  if (n == 0) {
    out_offsets[0] = 0;
    *n_out = 0;
    return EMQX_OK;
  }
  RT_TRY(hipSetDevice(r->device));
  auto sn = current(r);
  if (!sn) {
    const int rc0 = emqx_retain_commit(r);
    if (rc0 != EMQX_OK) return rc0;
    sn = current(r);
  }
  RWork* w = nullptr;
  int rc = acquire(r, &w);
  if (rc != EMQX_OK) return rc;
  const uint64_t span = fo[n] - fo[0];
  auto stage = [&]() -> int {
    if (span + 16 > w->d_fb_cap) {
      RT_TRY(ralloc(w->d_fb, span + span / 4 + 16));
      w->d_fb_cap = span + span / 4 + 16;
    }
    if (n + 1 > w->d_n_cap) {
      RT_TRY(ralloc(w->d_fo, n + n / 4 + 1));
      RT_TRY(ralloc(w->d_oo, n + n / 4 + 1));
      w->d_n_cap = n + n / 4 + 1;
    }
    if (out_cap > w->d_ids_cap) {
      RT_TRY(ralloc(w->d_ids, out_cap));
      w->d_ids_cap = out_cap;
    }
    RT_TRY(hipMemcpyAsync(w->d_fb, fb + fo[0], span, hipMemcpyHostToDevice, w->stream));
    // offsets rebased to the staged bytes
    std::vector<uint64_t> ro(n + 1);
    for (uint64_t i = 0; i <= n; ++i) ro[i] = fo[i] - fo[0];
    RT_TRY(hipMemcpyAsync(w->d_fo, ro.data(), (n + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, w->stream));
    RT_TRY(hipStreamSynchronize(w->stream));
    return EMQX_OK;
  };
  rc = stage();
  uint64_t total = 0;
  if (rc == EMQX_OK)
    rc = run_match(r, w, *sn, w->d_fb, w->d_fo, n, span, now_ms, w->d_oo, w->d_ids, out_cap, w->stream, &total,
                   strict_all);
  if (rc == EMQX_OK || rc == EMQX_EOVERFLOW) {
    if (hipMemcpy(out_offsets, w->d_oo, (n + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess)
      rc = EMQX_EDEVICE;
    else if (rc == EMQX_OK && total && out_ids &&
             hipMemcpy(out_ids, w->d_ids, total * sizeof(uint32_t), hipMemcpyDeviceToHost) != hipSuccess)
      rc = EMQX_EDEVICE;
  }
  *n_out = total;
  release(r, w);
  return rc;
}

}  // namespace

int emqx_retain_match_batch(emqx_retain* r, const uint8_t* fb, const uint64_t* fo, uint64_t n, int64_t now_ms,
                            uint64_t* out_offsets, uint32_t* out_ids, uint64_t out_cap, uint64_t* n_out) {
  return match_host(r, fb, fo, n, now_ms, out_offsets, out_ids, out_cap, n_out, false);
}

int emqx_retain_match_spec_batch(emqx_retain* r, const uint8_t* fb, const uint64_t* fo, uint64_t n, int64_t now_ms,
                                 uint64_t* out_offsets, uint32_t* out_ids, uint64_t out_cap, uint64_t* n_out) {
  return match_host(r, fb, fo, n, now_ms, out_offsets, out_ids, out_cap, n_out, true);
}

int emqx_retain_set_tuning(emqx_retain* r, const char* key, int64_t value) {
  if (!r || !key || value < 0 || value > 0xFFFFFFFFll) return EMQX_EINVAL;
  const uint32_t v = static_cast<uint32_t>(value);
  if (std::strcmp(key, "tile") == 0) {
    if (v < 1 || v > 64) return EMQX_EINVAL;
    r->tile = v;
  } else if (std::strcmp(key, "step_budget") == 0) {
    r->step_budget = v;  // 0 = no budget (no spill rounds)
  } else if (std::strcmp(key, "spill_budget") == 0) {
    r->spill_budget = v;  // 0 = the walk's step budget
  } else if (std::strcmp(key, "spill_per_wave") == 0) {
    if (v < 1) return EMQX_EINVAL;
    r->spill_per_wave = v;
  } else if (std::strcmp(key, "spill_rounds") == 0) {
    if (v > RC_MAX_ROUNDS) return EMQX_EINVAL;
    r->spill_rounds = v;
  } else if (std::strcmp(key, "walk_waves") == 0) {
    if (v < 64 || v > (1u << 20)) return EMQX_EINVAL;
    r->walk_waves = v;
  } else if (std::strcmp(key, "spill_waves") == 0) {
    if (v < 64 || v > (1u << 20)) return EMQX_EINVAL;
    r->spill_waves = v;
  } else if (std::strcmp(key, "spill_cap") == 0) {
    if (v < 64 || v > SPILL_CAP) return EMQX_EINVAL;
    r->spill_cap = v;
  } else if (std::strcmp(key, "search") == 0) {
    if (v > RSEARCH_STREE) return EMQX_EINVAL;
    r->search = v;
  } else if (std::strcmp(key, "balance") == 0) {
    if (v > BALANCE_QUEUE) return EMQX_EINVAL;
    r->balance = v;
  } else if (std::strcmp(key, "queue_piece") == 0) {
    if (v < 64 || v > (1u << 20)) return EMQX_EINVAL;
    r->queue_piece = v;
  } else if (std::strcmp(key, "lane_map") == 0) {
    if (v < 0 || v > 1) return EMQX_EINVAL;
    r->lane_map = static_cast<uint32_t>(v);
  } else if (std::strcmp(key, "queue_check") == 0) {
    if (v < 1 || v > 1024 || (v & (v - 1)) != 0) return EMQX_EINVAL;
    r->queue_check = v;
  } else if (std::strcmp(key, "queue_wait") == 0) {
    if (v < 1 || v > (1u << 20)) return EMQX_EINVAL;
    r->queue_wait = v;
  } else if (std::strcmp(key, "queue_sleep") == 0) {
    if (v > 64) return EMQX_EINVAL;
    r->queue_sleep = v;
  } else if (std::strcmp(key, "queue_shards") == 0) {
    if (v < 1 || v > QS_MAX_SHARDS) return EMQX_EINVAL;
    r->queue_shards = v;
  } else if (std::strcmp(key, "queue_roam") == 0) {
    if (v > QS_MAX_SHARDS) return EMQX_EINVAL;
    r->queue_roam = v;
  } else if (std::strcmp(key, "queue_cap") == 0) {
    if (v < 64 || v > QUEUE_CAP) return EMQX_EINVAL;
    r->queue_cap = v;
  } else if (std::strcmp(key, "queue_poll_limit") == 0) {  // the safety valve (tests force it: 1)
    if (v < 1) return EMQX_EINVAL;
    r->queue_poll_limit = v;
  } else {
    return EMQX_ENOTFOUND;
  }
  return EMQX_OK;
}

int emqx_retain_stats_get(emqx_retain* r, emqx_retain_stats* dst) {
  if (!r || !dst || (dst->size && dst->size < sizeof(uint64_t))) return EMQX_EINVAL;
  const uint64_t want =
      dst->size ? std::min<uint64_t>(dst->size, sizeof(emqx_retain_stats)) : sizeof(emqx_retain_stats);
  emqx_retain_stats full;
  emqx_retain_stats* out = &full;
  std::memset(out, 0, sizeof(*out));
  {
    std::lock_guard<std::mutex> g(r->writer);
    out->n_ids = r->store.n_ids();
    out->n_live = r->store.n_live;
    out->epoch = r->epoch;
    out->last_build_ms = r->last_build_ms;
  }
  auto sn = current(r);
  if (sn) {
    out->n_nodes = sn->n_nodes;
    out->n_words = sn->n_words;
    out->table_bytes = sn->bytes;
  }
  out->last_ranges = r->last_ranges.load();
  out->last_visits = r->last_visits.load();
  out->last_spill_rounds = r->last_spill_rounds.load();
  out->last_spilled = r->last_spilled.load();
  out->last_spill_full = r->last_spill_full.load();
  out->last_shares = r->last_shares.load();
  out->queue_aborts = r->queue_aborts.load();
  out->last_total = r->last_total.load();
  out->last_match_ms = r->last_match_ms.load();
  out->last_walk_ms = r->last_walk_ms.load();
  out->size = want;
  std::memcpy(dst, out, want);
  return EMQX_OK;
}

}  // extern "C"

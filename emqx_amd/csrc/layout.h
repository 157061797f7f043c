// Device-resident table layout shared by the host builder (tables.cpp) and the HIP
// kernels (match_kernels.hip).  See DESIGN.md §2 for the HBM layout.
//
// The reference stores its trie as an ETS ordered_set of joined-string keys
// {Prefix,0}/{Topic,1} (apps/emqx/src/emqx_trie.erl:53-77) and matches by probing that
// set once per visited prefix (emqx_trie.erl:315-334).  Here the same filter set is a
// *level trie over interned words*:
//
//   * vocab:  open-addressed table  word bytes -> 32-bit word id (exact byte check)
//   * nodes:  one per distinct filter prefix (all filters, exact and wildcard)
//   * edges:  each node owns a power-of-two slice of one global slot array, open-
//             addressed by word id; '+' is the reserved word WID_PLUS, a non-final '#'
//             the reserved word WID_HASH; a final '#' is the parent's hash filter.
//   * fids:   per slot, its child's {filter "<path>/#", filter "<path>"} ids (inline in
//             the slot for an edgeless child); the root's '#' filter is a table-view field.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#define EMQX_HD __host__ __device__ __forceinline__
#else
#define EMQX_HD inline
#endif

namespace emqx {

constexpr uint32_t WID_NONE = 0xFFFFFFFFu;  // unknown word / empty edge slot
constexpr uint32_t WID_PLUS = 0xFFFFFFFEu;  // '+' level
constexpr uint32_t WID_HASH = 0xFFFFFFFDu;  // '#' level (edge only when not final)
constexpr uint32_t FID_NONE = 0xFFFFFFFFu;

// EdgeSlot.meta bits (describe the CHILD the slot points to).
constexpr uint32_t META_CAPLOG2_MASK = 0x1Fu;   // child's edge-array size = 1 << caplog2
constexpr uint32_t META_HAS_PLUS = 1u << 5;     // child has a '+' edge
constexpr uint32_t META_HAS_EDGES = 1u << 6;    // child has any edge (literal/'+'/'#')
constexpr uint32_t META_HAS_HASH = 1u << 7;     // filter "<child path>/#" exists
constexpr uint32_t META_HAS_TERM = 1u << 8;     // filter "<child path>" exists
constexpr uint32_t META_TERM_WILD = 1u << 9;    // ... and that filter is a wildcard filter
constexpr uint32_t META_PH = 1u << 10;          // literal edges perfect-hashed (seed below); else 2-slot buckets
constexpr uint32_t META_LITF_EXACT = 1u << 11;  // litf = the child's only literal edge word
constexpr uint32_t META_LITF_NONE = 1u << 12;   // the child has no literal edge at all
constexpr uint32_t META_BUCKET_OVF = 1u << 13;  // (slot position, wide nodes) first slot of a 2-slot
                                                // bucket some word of which lives in its secondary bucket
constexpr uint32_t META_XFID = 1u << 14;        // litf holds the child's one filter id; the literal
                                                // filter shrinks to 8 bits in meta[31:24]
constexpr uint32_t META_XFID_TERM = 1u << 15;   // ... which is its terminal filter (else its '#' filter)
constexpr uint32_t META_F8_SHIFT = 24;          // XFID: fingerprint of the only literal (LITF_EXACT)
                                                // or an 8-bit Bloom mask of the literals
constexpr uint32_t META_SEED_SHIFT = 16;        // 8-bit perfect-hash seed
constexpr uint32_t PH_MAX_CAPLOG = 15;

// 16-byte edge slot: the child's record travels with the edge, so one probe (one dwordx4
// load per lane) yields everything the next level's walk needs: the child's edge array and
// meta, and a filter over the child's literal edges, tested against the topic's next word
// before the child is even pushed.  A node's '+' edge, when present, always sits in slot 0 of
// its array; literal edges are perfect-hashed by a per-node seed found at build time (one
// load per lookup, hit or miss), or — in wide nodes, where no seed fits — hashed into 2-slot
// buckets (two loads per lookup, two more for ~1% of words).
// The filter ids of the child behind slot i live apart, in `fids[2i]` ("<child>/#") and
// `fids[2i + 1]` ("<child>"), except
//   * for a child without edges (no META_HAS_EDGES: it is never pushed), which carries them
//     in place of child_base and litf — the common leaf emission needs no second load;
//   * for a child with edges and one filter id (META_XFID), which carries it in litf; its
//     literal filter shrinks to an 8-bit fingerprint / Bloom mask in the meta's top byte.
// For the others the walk emits the reference 2i + kind and the scatter kernel resolves it,
// so a probe moves 16 B and the walk never waits on an id.
struct alignas(16) EdgeSlot {
  uint32_t wid;         // key (WID_NONE = empty)
  uint32_t child_base;  // first slot of the child's edge array  | edgeless child: hash_fid
  uint32_t meta;        // META_* (+ seed) of the child; META_BUCKET_OVF belongs to this slot
  uint32_t litf;        // literal-edge filter of the child: its only literal word (LITF_EXACT)
                        //   or a 2-probe 32-bit Bloom mask (all ones when the child is wide)
                        //   | edgeless child: term_fid
};
static_assert(sizeof(EdgeSlot) == 16, "EdgeSlot must be 16 bytes");
constexpr uint64_t MAX_SLOTS = (1ull << 31) - 1;  // references 2i + kind fit 32 bits

// One in-place rewrite of an existing slot by an incremental commit (live_trie.cpp): the
// slot's new content and its two filter ids.
struct alignas(16) SlotPatch {
  uint32_t slot;
  uint32_t fid_h, fid_t;
  uint32_t pad;
  EdgeSlot s;
};
static_assert(sizeof(SlotPatch) == 32, "SlotPatch must be 32 bytes");

// 32-byte vocab slot; words up to 16 bytes are verified from `inl` without a second load.
struct alignas(16) VocabSlot {
  uint32_t hash;   // word_hash_bytes() of the word
  uint32_t len;    // word length in bytes
  uint32_t wid;    // word id (WID_NONE = empty slot)
  uint32_t off;    // offset of the bytes in the arena
  uint32_t inl[4]; // first 16 bytes, little-endian, zero padded
};
static_assert(sizeof(VocabSlot) == 32, "VocabSlot must be 32 bytes");

// Kernel-argument view of one committed snapshot.
struct TableView {
  const EdgeSlot* edges;
  const uint32_t* fids;  // 2 * n_slots filter ids (see EdgeSlot)
  const VocabSlot* vocab;
  const uint8_t* arena;
  uint32_t vocab_mask;
  uint32_t root_base;      // root's edge array
  uint32_t root_meta;      // META_* of the root
  uint32_t root_hash_fid;  // filter '#' or FID_NONE
  uint32_t plus_mask;      // ~(PLUS_LINE - 1) when the table holds '+' copies (plus_copies), else 0
};

// '+' copies: in a table built with them, a node with a '+' edge and an array of 8 to
// 2^PLUS_COPY_MAX_CAPLOG slots keeps a copy of that edge in slot 0 of every 64-B line
// (PLUS_LINE slots) of its array, and no literal edge sits there.  A step that probes both the
// '+' edge and a literal then reads the copy in the literal's line: two loads of one line cost
// one L2 request (tools/gather_bench pair), where slot 0 is usually another line.  Arrays of
// PLUS_LINE slots or more start on a line boundary (layout pass).  Larger arrays keep '+' in
// slot 0 alone: an incremental commit rewrites every copy when the '+' edge's record changes,
// and in the wide upper nodes that is thousands of slot patches per change (measured: commits
// 40x slower with copies in every array), while those nodes' lines are L2-resident anyway.
constexpr uint32_t PLUS_LINE = 4;
constexpr uint32_t PLUS_COPY_MAX_CAPLOG = 14;
// Does the array of a node (its meta's caplog, whether it has a '+' edge) hold '+' copies?
EMQX_HD bool plus_copies(uint32_t plus_mask, bool has_plus, uint32_t caplog) {
  return plus_mask != 0 && has_plus && caplog > 2 && caplog <= PLUS_COPY_MAX_CAPLOG;
}
// Is slot i of such an array a '+' position (slot 0, or a line head when it holds copies)?
EMQX_HD bool plus_position(uint32_t i, bool copies) { return copies ? (i & (PLUS_LINE - 1u)) == 0 : i == 0; }
// The '+' slot a step reads beside literal slot i1: the copy in i1's line, or slot 0.
EMQX_HD uint32_t plus_copy(uint32_t i1, bool copies) { return copies ? (i1 & ~(PLUS_LINE - 1u)) : 0u; }

// murmur3 fmix32: spreads word ids inside a node's edge array.
EMQX_HD uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x85ebca6bu;
  x ^= x >> 13;
  x *= 0xc2b2ae35u;
  x ^= x >> 16;
  return x;
}

// Vocab word hash: a multiply-rotate chain over the word's bytes read as little-endian
// dwords (zero padded, at least four dwords), seeded by the length, then fmix32.  A word of
// at most 16 bytes hashes from the four head dwords the kernels already hold for the exact
// byte check (VocabSlot::inl), so interning needs no per-byte loop.
EMQX_HD uint32_t whash_init(uint32_t len) { return len * 0x9E3779B1u + 0x7F4A7C15u; }
EMQX_HD uint32_t whash_step(uint32_t h, uint32_t d) {
  h = (h ^ d) * 0x85EBCA77u;
  return (h << 13) | (h >> 19);
}
EMQX_HD uint32_t word_hash16(uint32_t len, uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3) {
  return mix32(whash_step(whash_step(whash_step(whash_step(whash_init(len), w0), w1), w2), w3));
}
// Any length; p[0, n) are the word's bytes.
EMQX_HD uint32_t word_hash_bytes(const uint8_t* p, uint32_t n) {
  uint32_t h = whash_init(n);
  const uint32_t nd = n > 16 ? (n + 3) / 4 : 4;
  for (uint32_t i = 0; i < nd; ++i) {
    uint32_t d = 0;
    for (uint32_t b = 0; b < 4; ++b)
      if (4 * i + b < n) d |= static_cast<uint32_t>(p[4 * i + b]) << (8 * b);
    h = whash_step(h, d);
  }
  return mix32(h);
}

EMQX_HD uint32_t vocab_slot0(uint32_t hash) { return hash; }

// The per-node hash of a literal word (seed = the node's hashing seed): one fmix32 serves the
// perfect-hash slot and the primary bucket alike, so a walk step computes it once whatever the
// node's hashing (the kernels are bound by their per-step instruction count).
EMQX_HD uint32_t node_hash(uint32_t wid, uint32_t seed) { return mix32(wid ^ (seed * 0x9E3779B1u + 0x7F4A7C15u)); }

// Slot of a literal word with node hash h in a perfect-hashed node's array (mask = cap - 1).
// In an array that holds '+' copies (copies = plus_copies(...)) the literal slots are the 3/4
// of the array that are not line heads: a hash landing on a head moves to slot 1 or 2 of its
// line (by its top bit), so the copies cost the perfect hash no larger arrays.
EMQX_HD uint32_t ph_slot(uint32_t h, uint32_t mask, bool copies) {
  const uint32_t s = h & mask;
  return (!copies || (s & (PLUS_LINE - 1u))) ? s : s + 1u + (h >> 31);
}
EMQX_HD uint32_t lit_slot(uint32_t wid, uint32_t seed, uint32_t mask, bool copies) {
  return ph_slot(node_hash(wid, seed), mask, copies);
}


// Wide (non-perfect-hashed) nodes use 2-slot buckets: a word lives in its primary bucket,
// or — rarely, flagged by META_BUCKET_OVF on the primary bucket's first slot —
// in its secondary bucket.  Bucket 0's slot 0 is '+'.  `seed` (7 bits) is re-drawn by the
// builder until every word fits.
EMQX_HD uint32_t bucket1(uint32_t wid, uint32_t seed, uint32_t nbmask) { return node_hash(wid, seed) & nbmask; }
EMQX_HD uint32_t bucket2(uint32_t wid, uint32_t seed, uint32_t nbmask) {
  const uint32_t a = bucket1(wid, seed, nbmask), b = mix32(wid ^ (0xDAA66D2Bu + seed * 0x7F4A7C15u)) & nbmask;
  return b != a ? b : ((a + 1) & nbmask);
}
// First slot of word `wid`'s primary (second = false) or secondary 2-slot bucket in a wide
// array (mask = cap - 1).  In an array holding '+' copies, a bucket is a window of two of the
// three literal slots of a 64-B line — slots {1, 2} or {2, 3} after the line's '+' copy — so
// both candidate slots and the copy share a line, and adding '+' later finds every line head
// free.  (The windows of a line overlap; each has its own first slot for META_BUCKET_OVF.)
// Primary window / bucket from the node hash h (wide_slot(.., false) = wide_slot1(node_hash)).
EMQX_HD uint32_t wide_slot1(uint32_t h, uint32_t mask, bool copies) {
  if (!copies) return 2u * (h & (mask >> 1));
  return (((h >> 1) & ((mask + 1u) / PLUS_LINE - 1u)) * PLUS_LINE) + 1u + (h & 1u);
}
EMQX_HD uint32_t wide_slot(uint32_t wid, uint32_t seed, uint32_t mask, bool copies, bool second) {
  if (!copies) return 2u * (second ? bucket2(wid, seed, mask >> 1) : bucket1(wid, seed, mask >> 1));
  const uint32_t lm = (mask + 1u) / PLUS_LINE - 1u;  // line mask
  const uint32_t w1 = wide_slot1(node_hash(wid, seed), mask, true);
  if (!second) return w1;
  const uint32_t h2 = mix32(wid ^ (0xDAA66D2Bu + seed * 0x7F4A7C15u));
  const uint32_t w2 = (((h2 >> 1) & lm) * PLUS_LINE) + 1u + (h2 & 1u);
  return w2 != w1 ? w2 : (w1 ^ 3u);  // the same window: the line's other one ({1,2} <-> {2,3})
}
constexpr uint32_t CUCKOO_SEEDS = 128;

// Hash of a word for the literal filters (Bloom bits, fingerprints): one multiply and a fold,
// computed per walk step for the topic's next word.
EMQX_HD uint32_t litf_hash(uint32_t wid) {
  const uint32_t m = (wid ^ 0xA5A5A5A5u) * 0x9E3779B1u;
  return m ^ (m >> 15);
}

// May the child (meta, litf) have a literal edge for `wid`?  No false negatives.
EMQX_HD bool litf_may_contain(uint32_t meta, uint32_t litf, uint32_t wid) {
  if (meta & META_LITF_NONE) return false;
  if (meta & META_XFID) {
    const uint32_t f8 = meta >> META_F8_SHIFT, h = litf_hash(wid);
    if (meta & META_LITF_EXACT) return (h >> 24) == f8;
    return ((f8 >> (h & 7u)) & 1u) != 0;
  }
  if (meta & META_LITF_EXACT) return litf == wid;
  const uint32_t h = litf_hash(wid);
  return ((litf >> (h & 31u)) & (litf >> ((h >> 5) & 31u)) & 1u) != 0;
}
constexpr uint32_t LITF_BLOOM_MAX = 16;  // wider children get an all-ones filter

// Filter-sharded tables (emqx_amd/dist.py): the rank that owns a filter / topic is a hash of
// its first `levels` levels (their bytes, separators included).  A filter with a '+' or '#'
// among those levels, or with fewer levels, can match topics of more than one key, so it is
// replicated on every rank (SHARD_ALL); every other filter lives with the topics of its key,
// and each topic is matched on exactly one rank.  Topics: a key level that is '+' / '#' (a
// wildcard "topic", matched byte for byte by match_routes/1 against replicated filters) sends
// the topic to rank 0; a topic shorter than `levels` hashes the levels it has.
constexpr uint32_t SHARD_ALL = 0xFFFFFFFFu;
EMQX_HD uint32_t shard_owner(const uint8_t* p, uint64_t n, uint32_t world, uint32_t levels, bool topic) {
  uint64_t s = 0, e = 0;
  uint32_t k = 0;
  while (k < levels) {
    e = s;
    while (e < n && p[e] != '/') ++e;
    if (e - s == 1 && (p[s] == '+' || p[s] == '#')) return topic ? 0u : SHARD_ALL;
    ++k;
    if (e >= n) break;
    s = e + 1;
  }
  if (k < levels && !topic) return SHARD_ALL;
  uint32_t h = 0x811C9DC5u;  // FNV-1a over the key levels' bytes
  for (uint64_t i = 0; i < e; ++i) h = (h ^ p[i]) * 0x01000193u;
  return mix32(h ^ k) % world;
}

// ---- filter-sharded layout with two key spaces (emqx_amd/dist.py) ----------
// A topic t = l1/l2/l3/... can be matched by three kinds of filter:
//   root-wildcard  '#', '+', '+/#', '+/+/...'      -> every rank (replicated)
//   space L        a literal first level l1         -> placed by (l1, l2)
//   space P        '+' then a literal second level  -> placed by (l2, l3)
// A space's key is its first level (l1, or l2 for space P); a key with few filters lives on one
// rank (a hash of it), a hot key (the plan, emqx_shard_plan) is split over `span` consecutive
// ranks by the next level, filters whose next level is a wildcard (or who end at the key...
// see shard_place_key) going to all `span` ranks of the key.  A topic is sent to its L-space
// rank (engine "A": space L + root-wildcard filters) and, when it has two levels and does not
// start with '$', to its P-space rank (engine "B": space P filters): every filter that can match
// it lives on one of the two, exactly once, so the two answers concatenate into the match set.
constexpr uint32_t SHARD_NONE = 0xFFFFFFFFu;
constexpr uint32_t SHARD_SPACE_P = 0x80000000u;  // key bit of space P keys
constexpr uint32_t SHARD_PAIR = 0x40000000u;     // key bit of (split key, next level) entries
constexpr uint32_t SHARD_HASH_MASK = 0x3FFFFFFFu;
constexpr uint32_t SHARD_ABSENT = 0x9E3779B9u;   // the hash of "no next level"

// One plan entry: a key (space bit | 30-bit level hash; info = first rank | span << 16), or a
// next level of a split key (SHARD_PAIR | space bit | 30-bit pair hash; info = its rank).
struct ShardSplitE {
  uint32_t key, info;
};

// Space P replicated: the plan entry {SHARD_SPACE_P, SHARD_P_REPLICATED} (no real key entry has
// that info: span 0, first rank 0xFFFF).  Then every '+/x/...' filter lives
// on every rank with the root wildcards (engine A), and a topic makes ONE request, to its L-space
// rank: emqx_shard_plan chooses it when space P holds at most a rank's share of the filters
// (config C: 7 % of the table, against 12.5 % a rank at world 8), so the step carries one request
// a topic instead of two for a larger replicated part.
constexpr uint32_t SHARD_P_REPLICATED = 0x0000FFFFu;

// A level's hash: its bytes as little-endian 32-bit words (the last one zero-padded), FNV-style
// over the words, then mixed with the length — a few word steps per level where a byte-wise
// FNV took one step a byte (the device's routing scanner, shard_step.hip, was VALU-bound on it).
EMQX_HD uint32_t shard_word_step(uint32_t h, uint32_t w) { return (h ^ w) * 0x01000193u; }
EMQX_HD uint32_t shard_level_hash(const uint8_t* p, uint64_t s, uint64_t e) {
  uint32_t h = 0x811C9DC5u;
  uint64_t i = s;
  for (; i + 4 <= e; i += 4)
    h = shard_word_step(h, static_cast<uint32_t>(p[i]) | (static_cast<uint32_t>(p[i + 1]) << 8) |
                               (static_cast<uint32_t>(p[i + 2]) << 16) | (static_cast<uint32_t>(p[i + 3]) << 24));
  if (i < e) {
    uint32_t w = 0;
    for (uint32_t k = 0; i + k < e; ++k) w |= static_cast<uint32_t>(p[i + k]) << (8u * k);
    h = shard_word_step(h, w);
  }
  return mix32(h ^ static_cast<uint32_t>(e - s));
}

EMQX_HD uint32_t shard_split_find(const ShardSplitE* sp, uint32_t n, uint32_t key) {
  uint32_t lo = 0, hi = n;  // sorted by key
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (sp[mid].key < key) lo = mid + 1; else hi = mid;
  }
  return lo < n && sp[lo].key == key ? sp[lo].info : SHARD_NONE;
}

// Level k of p[0, n): bounds [*s, *e); false if the name has fewer levels.
EMQX_HD bool shard_level(const uint8_t* p, uint64_t n, uint32_t k, uint64_t* s, uint64_t* e) {
  uint64_t a = 0;
  for (uint32_t j = 0; j < k; ++j) {
    while (a < n && p[a] != '/') ++a;
    if (a >= n) return false;
    ++a;
  }
  uint64_t b = a;
  while (b < n && p[b] != '/') ++b;
  *s = a;
  *e = b;
  return true;
}

EMQX_HD bool shard_is_wild(const uint8_t* p, uint64_t s, uint64_t e) {
  return e - s == 1 && (p[s] == '+' || p[s] == '#');
}

// Rank range [*first, *first + *span) (mod world) of key hash `hk` in `space` given its next
// level: `next` = its hash, or SHARD_ABSENT (no next level), or SHARD_NONE (a wildcard: every
// rank of the key).
EMQX_HD void shard_place_key(uint32_t space, uint32_t hk, uint32_t next, uint32_t world, const ShardSplitE* sp,
                             uint32_t nsp, uint32_t* first, uint32_t* span) {
  const uint32_t info = shard_split_find(sp, nsp, space | (hk & SHARD_HASH_MASK));
  if (info == SHARD_NONE) {
    *first = mix32(hk ^ (space ? 0x5BD1E995u : 0x27D4EB2Fu)) % world;
    *span = 1;
    return;
  }
  const uint32_t base = info & 0xFFFFu, s = info >> 16;
  if (next == SHARD_NONE) {
    *first = base;
    *span = s;
    return;
  }
  const uint32_t pair = mix32(next ^ hk);
  const uint32_t pinfo = s > 1 && next != SHARD_ABSENT
                             ? shard_split_find(sp, nsp, SHARD_PAIR | space | (pair & SHARD_HASH_MASK))
                             : SHARD_NONE;
  *first = pinfo != SHARD_NONE ? (pinfo & 0xFFFFu) : (base + pair % s) % world;
  *span = 1;
}

EMQX_HD bool shard_p_replicated(const ShardSplitE* sp, uint32_t nsp) {
  return nsp && shard_split_find(sp, nsp, SHARD_SPACE_P) == SHARD_P_REPLICATED;
}

// Placement of filter p[0, n): *engine 0 (A: space L, root-wildcard) or 1 (B: space P).
EMQX_HD void shard_place_filter(const uint8_t* p, uint64_t n, uint32_t world, const ShardSplitE* sp, uint32_t nsp,
                                uint32_t* first, uint32_t* span, uint32_t* engine) {
  uint64_t s1, e1, s2, e2, s3, e3;
  shard_level(p, n, 0, &s1, &e1);
  const bool has2 = shard_level(p, n, 1, &s2, &e2);
  *engine = 0;
  if (shard_is_wild(p, s1, e1)) {
    // '#', '+', '+/#', '+/+/...'; and '+/x/...' when space P is replicated
    if (p[s1] == '#' || !has2 || shard_is_wild(p, s2, e2) || shard_p_replicated(sp, nsp)) {
      *first = 0;
      *span = world;
      return;
    }
    *engine = 1;  // '+/x/...': space P, keyed by x, split by the third level
    const bool has3 = shard_level(p, n, 2, &s3, &e3);
    const uint32_t next = !has3 ? SHARD_ABSENT : shard_is_wild(p, s3, e3) ? SHARD_NONE : shard_level_hash(p, s3, e3);
    shard_place_key(SHARD_SPACE_P, shard_level_hash(p, s2, e2), next, world, sp, nsp, first, span);
    return;
  }
  const uint32_t next = !has2 ? SHARD_ABSENT : shard_is_wild(p, s2, e2) ? SHARD_NONE : shard_level_hash(p, s2, e2);
  shard_place_key(0, shard_level_hash(p, s1, e1), next, world, sp, nsp, first, span);
}

// What routing reads of a topic name: its level count (levels 0..2 hashed), whether some level
// is a wildcard, its first byte.  One pass (shard_topic_levels here; the device's shard step
// fills it from 16-B windows, shard_step.hip).
struct ShardTopicLevels {
  uint32_t n_levels;  // '/' count + 1
  uint32_t h[3];      // shard_level_hash of levels 0..2 (those present)
  bool wild;          // some level is exactly '+' or '#'
};

EMQX_HD void shard_topic_levels(const uint8_t* p, uint64_t n, ShardTopicLevels* L) {
  L->n_levels = 0;
  L->wild = false;
  uint64_t s = 0;
  for (uint64_t i = 0; i <= n; ++i) {
    if (i < n && p[i] != '/') continue;
    if (L->n_levels < 3) L->h[L->n_levels] = shard_level_hash(p, s, i);
    if (i - s == 1 && (p[s] == '+' || p[s] == '#')) L->wild = true;
    ++L->n_levels;
    s = i + 1;
  }
}

// The requests of topic p[0, n) from its level summary: req[0] to engine A, req[1] to engine B,
// each rank * 2 + engine or SHARD_NONE.  A wildcard topic (match_routes/1 returns only its
// byte-identical filter, S3) makes one request, to the first rank of that filter.
EMQX_HD void shard_route_levels(const uint8_t* p, uint64_t n, const ShardTopicLevels& L, uint32_t world,
                                const ShardSplitE* sp, uint32_t nsp, uint32_t* req) {
  req[0] = req[1] = SHARD_NONE;
  uint32_t first, span, engine;
  if (L.wild) {
    shard_place_filter(p, n, world, sp, nsp, &first, &span, &engine);
    req[engine] = 2 * first + engine;
    return;
  }
  const bool has2 = L.n_levels >= 2, has3 = L.n_levels >= 3;
  shard_place_key(0, L.h[0], has2 ? L.h[1] : SHARD_ABSENT, world, sp, nsp, &first, &span);
  req[0] = 2 * first;
  if (!has2 || (n > 0 && p[0] == '$')) return;  // '+/x/...' never matches a '$' topic (S5)
  if (shard_p_replicated(sp, nsp)) return;       // ... and lives on every rank
  shard_place_key(SHARD_SPACE_P, L.h[1], has3 ? L.h[2] : SHARD_ABSENT, world, sp, nsp, &first, &span);
  req[1] = 2 * first + 1;
}

EMQX_HD void shard_route_topic(const uint8_t* p, uint64_t n, uint32_t world, const ShardSplitE* sp, uint32_t nsp,
                               uint32_t* req) {
  ShardTopicLevels L;
  shard_topic_levels(p, n, &L);
  shard_route_levels(p, n, L, world, sp, nsp, req);
}

}  // namespace emqx

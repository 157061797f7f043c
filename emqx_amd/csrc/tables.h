// Host-side filter store and level-trie builder (see layout.h for the device format).
#pragma once

#include <stdint.h>

#include <mutex>
#include <string>
#include <vector>

#include "layout.h"

namespace emqx {

// Sorts v ascending and drops repeats: LSD radix passes of 11 bits over the bits the largest
// value uses (commit paths: 20K filter ids, 10^5 dirty slots; std::sort took milliseconds).
void sort_unique_u32(std::vector<uint32_t>& v);

uint64_t hash64_bytes(const uint8_t* p, uint64_t n);

// Open-addressed map from byte strings (kept in an external arena) to uint32 ids.
class StrIdMap {
 public:
  // get: id or WID_NONE.  `arena_of(id)` resolves an id to (ptr, len) for verification.
  template <class Resolve>
  uint32_t find(const uint8_t* p, uint64_t n, uint64_t h, Resolve&& res) const {
    if (keys_.empty()) return WID_NONE;
    uint64_t mask = keys_.size() - 1;
    for (uint64_t i = h & mask;; i = (i + 1) & mask) {
      if (vals_[i] == WID_NONE) return WID_NONE;
      if (keys_[i] == h) {
        const uint8_t* q;
        uint64_t m;
        res(vals_[i], q, m);
        if (m == n && (n == 0 || std::char_traits<char>::compare((const char*)p, (const char*)q, n) == 0))
          return vals_[i];
      }
    }
  }
  void insert_new(uint64_t h, uint32_t id);  // caller guarantees absence
  void reserve(uint64_t n);
  uint64_t size() const { return size_; }
  void clear() {
    keys_.clear();
    vals_.clear();
    size_ = 0;
  }

 private:
  void grow();
  std::vector<uint64_t> keys_;
  std::vector<uint32_t> vals_;
  uint64_t size_ = 0;
};

// The engine's authoritative filter set (the route table's key set).  Ids are stable
// and never reused; a deleted filter keeps its id for a later re-insert.
struct FilterStore {
  std::vector<uint8_t> bytes;
  std::vector<uint64_t> off{0};  // id -> [off[id], off[id+1])
  std::vector<uint8_t> live;
  std::vector<uint32_t> ext;     // id -> the id reported by matches (default: the id itself)
  uint64_t n_live = 0;
  StrIdMap index;

  uint64_t n_ids() const { return live.size(); }
  uint32_t find(const uint8_t* p, uint64_t n) const;
  // returns id; *created = true if a new id was assigned
  uint32_t insert(const uint8_t* p, uint64_t n, bool* created);
};

// Word interner that outlives a build: incremental (delta) builds keep interning into it so
// word ids stay those of the device vocab, and `table` is the host image of that vocab.
struct VocabState {
  std::vector<uint8_t> arena;
  std::vector<uint32_t> off{0};
  std::vector<uint32_t> h32;  // word_hash_bytes per word id
  StrIdMap map;
  std::vector<VocabSlot> table;
  uint32_t mask = 0;

  uint32_t intern(const uint8_t* p, uint64_t n);
  uint64_t n_words() const { return h32.size(); }
  // (Re)builds `table` for every word, at 2x load headroom.
  void build_table();
  // Inserts words [from, n_words()) into `table`; dirty slot indices appended.  False when
  // the load would exceed 1/2 (the caller rebuilds everything).
  bool insert_table(uint64_t from, std::vector<uint32_t>* dirty);
};

// Where a filter's id lives in a built trie: slot << 2 | kind (FIDLOC_HASH / FIDLOC_TERM:
// the META_HAS_HASH / META_HAS_TERM flag of that slot), FIDLOC_ROOT_HASH (the root's '#'
// filter, in the table view), or FIDLOC_NONE.
constexpr uint64_t FIDLOC_HASH = 0, FIDLOC_TERM = 1;
constexpr uint64_t FIDLOC_ROOT_HASH = ~0ull - 1, FIDLOC_NONE = ~0ull;

struct BuildOpts {
  const std::vector<uint32_t>* ids = nullptr;  // filters to include (null: every live filter)
  uint64_t slot_offset = 0;                    // the trie's arrays start at this slot
  VocabState* vocab = nullptr;                 // persistent interner (null: a private one)
  bool vocab_table = true;                     // build the vocab table into HostTables
  std::vector<uint64_t>* fid_loc = nullptr;    // out: per filter id (sized n_ids)
  std::vector<uint32_t>* slot_ids = nullptr;   // out: per slot, the engine ids {hash, term} (2 per slot)
  int threads = 1;                             // host threads for the per-node passes
};

struct HostTables {
  std::vector<EdgeSlot> edges;
  std::vector<uint32_t> fids;  // 2 * edges.size() (see EdgeSlot)
  std::vector<VocabSlot> vocab;
  std::vector<uint8_t> arena;
  uint32_t vocab_mask = 0;
  uint32_t root_base = 0;
  uint32_t root_meta = 0;
  uint32_t root_hash_fid = FID_NONE;
  uint32_t plus_mask = 0;    // TableView::plus_mask of the build
  uint64_t n_nodes = 0;
  uint64_t n_words = 0;
  uint32_t max_depth = 0;
  uint64_t n_ph_nodes = 0;
  uint64_t slot_offset = 0;  // edges[i] is slot slot_offset + i (child_base values are absolute)
};

// Builds the level trie of the selected live filters.  Returns false on size overflow.
bool build_tables(const FilterStore& fs, const BuildOpts& opts, HostTables& out, std::string* err);
inline bool build_tables(const FilterStore& fs, HostTables& out, std::string* err) {
  return build_tables(fs, BuildOpts{}, out, err);
}
// Verifies the lookup invariants of a built table (host-side; used by tests).
bool check_tables(const HostTables& t, std::string* err);

// ---- incremental commits: the committed trie patched in place (live_trie.cpp) ---------
//
// The host keeps an image of the device slot array (edges + fids) with spare capacity behind
// the built slots.  Publishing an insert walks the image like the kernel does; the filter's
// missing tail becomes a chain of new one-edge nodes in the spare region, and its first edge is
// placed into the existing node when that node's hashing has a free slot for it, else the node
// is relocated (rebuilt one entry larger into the spare region).  Either way the device sees a
// handful of new slots plus whole-slot (16-B) rewrites of existing ones — the edge's slot and
// the parent slot that describes the node — so the cost of a commit is proportional to the
// churn, not to the table or to earlier commits.  Deletes / revivals flip the filter's flag in
// its slot.  A full rebuild (compaction) runs when the spare region is used up.
struct LiveTrie {
  struct Entry {
    uint32_t wid;
    EdgeSlot s;  // slot content without the position's META_BUCKET_OVF bit
    uint32_t fh, ft, ih, it;
  };
  // Per-thread state of a commit: spare-region chunk, line packer, rewritten slots, counters,
  // scratch.  Inserts under different first-level nodes touch disjoint parts of the table, so
  // a commit runs them on several threads, one Ctx each.
  struct Ctx {
    uint64_t cur = 0, end = 0;          // current chunk of the spare region [cur, end)
    uint64_t line = 0;
    uint32_t line_used = 0xFFu;
    std::vector<std::pair<uint64_t, uint64_t>> ranges;  // allocated extents (uploaded whole)
    size_t chunk_range = 0;             // ranges[chunk_range] is the current chunk's extent
    std::vector<uint32_t> dirty;        // slots < mark rewritten in place (may repeat)
    uint64_t relocations = 0, in_place = 0, chains = 0, flips = 0, nodes = 0, garbage = 0;
    uint64_t reloc_ns = 0, ph_ns = 0;   // EMQX_COMMIT_PROF: time in relocate / its seed search
    uint32_t max_depth = 0;
    bool failed = false;                // spare region exhausted
    std::vector<Entry> ent;
    std::vector<uint32_t> pos, w;
    std::vector<uint32_t> plus_heads;   // '+' slots flipped in place: copies synced after the flips
  };

  std::vector<EdgeSlot> edges;  // host image of device slots [0, cap)
  std::vector<uint32_t> fids;   // 2 per slot (reported ids)
  std::vector<uint32_t> sid;    // 2 per slot (engine ids, for fid_loc upkeep)
  uint64_t used = 0, cap = 0;   // spare-region cursor / capacity in slots
  uint64_t garbage = 0;         // slots of arrays superseded by relocations
  uint32_t root_base = 0, root_meta = 0, root_hash_fid = FID_NONE, root_hash_id = WID_NONE;
  uint64_t n_nodes = 0;
  uint32_t max_depth = 0;
  std::vector<uint64_t> loc;    // per engine id: FIDLOC (tables.h)
  VocabState* vocab = nullptr;
  // '+' copies (layout.h plus_copy): plus_mask of the build, and per array base slot the caplog
  // of an array whose '+' edge has copies (cap > PLUS_LINE), else 0
  uint32_t plus_mask = 0;
  std::vector<uint8_t> pcap;
  // per commit
  uint64_t mark = 0;            // `used` when the commit began: slots >= mark are new
  std::vector<uint32_t> dirty;  // slots < mark rewritten in place (may repeat)
  std::vector<std::pair<uint64_t, uint64_t>> ranges;  // new extents [begin, end) to upload
  uint64_t relocations = 0, in_place = 0, chains = 0, flips = 0;

  // Adopts a full build (moves its arrays) and reserves `spare` slots behind it.
  void adopt(HostTables& ht, std::vector<uint64_t>& fid_loc, std::vector<uint32_t>& slot_ids, uint64_t spare,
             VocabState* v);
  // Publishes the changes of `ids` (each brought in line with fs.live[id]: flag flip, or
  // insertion of a new filter) on up to `threads` threads.  False when the spare region is
  // exhausted (the caller then does a full rebuild).
  bool commit(const FilterStore& fs, const std::vector<uint32_t>& ids, int threads);
  // The commit's in-place rewrites (deduplicated slot patches for slots < mark).
  void patches(std::vector<SlotPatch>& out) const;
  uint64_t new_slots() const;

 private:
  bool find_child(uint32_t base, uint32_t meta, uint32_t wid, uint32_t* slot) const;
  bool alloc(Ctx& c, uint32_t caplog, uint64_t* at);
  void touch(Ctx& c, uint64_t slot) const {
    if (slot < mark) c.dirty.push_back(static_cast<uint32_t>(slot));
  }
  bool has_copies(uint64_t slot) const { return plus_mask && pcap[slot] && edges[slot].wid == WID_PLUS; }
  // Writes the '+' edge at array base `slot` into its copies (each keeps its own
  // META_BUCKET_OVF position bit) and touches them.
  void sync_plus(Ctx& c, uint64_t slot);
  void lit_summary(uint32_t base, uint32_t meta, uint32_t* n_lit, uint32_t* only, uint32_t* bloom,
                   uint32_t* bloom8) const;
  EdgeSlot encode(uint32_t wid, bool has_edges, uint32_t base, uint32_t smeta, uint32_t fid_h, uint32_t fid_t,
                  uint32_t fmeta) const;
  void reencode(Ctx& c, uint64_t pslot);
  void set_node(Ctx& c, bool root, uint64_t pslot, uint32_t base, uint32_t smeta);
  bool place(Ctx& c, bool root, uint64_t pslot, uint32_t wid, const EdgeSlot& child, uint32_t fh, uint32_t ft,
             uint32_t ih, uint32_t it);
  bool relocate(Ctx& c, bool root, uint64_t pslot, uint32_t wid, const EdgeSlot& child, uint32_t fh, uint32_t ft,
                uint32_t ih, uint32_t it);
  void flip(Ctx& c, uint32_t id, bool want, bool atomic);
  // Inserts filter `id` (words w, final '#' flag) starting at the node reached through
  // `pslot` (or the root) after `i` levels.
  bool insert(Ctx& c, const FilterStore& fs, uint32_t id, const std::vector<uint32_t>& w, bool wild,
              bool final_hash, bool root, uint64_t pslot, uint32_t i);
  bool tokenize(const FilterStore& fs, uint32_t id, std::vector<uint32_t>& w, bool* wild, bool* final_hash,
                bool intern) const;
  std::mutex alloc_mu_;
};

}  // namespace emqx

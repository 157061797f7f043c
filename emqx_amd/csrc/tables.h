// Host-side filter store and level-trie builder (see layout.h for the device format).
#pragma once

#include <stdint.h>

#include <string>
#include <vector>

#include "layout.h"

namespace emqx {

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

}  // namespace emqx

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
};

// Builds the level trie of every live filter.  Returns false on size overflow.
bool build_tables(const FilterStore& fs, HostTables& out, std::string* err);
// Verifies the lookup invariants of a built table (host-side; used by tests).
bool check_tables(const HostTables& t, std::string* err);

}  // namespace emqx

// Host lowering: the reference's []Variable (wire format) -> one int32 record
// per problem (include/deppy_hip.h).  This is the batched C++ counterpart of
//   newLitMapping        pkg/sat/lit_mapping.go:40-77
//   Constraint.Apply     pkg/sat/constraints.go:59-62,84-86,116-123,148-150,180-186
//   AnchorIdentifiers    pkg/sat/lit_mapping.go:163-174
//   Order()              pkg/sat/constraints.go:125-127 (search.go:59-69)
// Instead of emitting gini gates + Tseitin CNF (lit_mapping.go:132-134) it
// emits rows the kernel propagates natively; the And-inverter graph of
// gini's logic.C is still built, only to decide which constraints share one
// assumed literal (the reference's constraints[m] map, lit_mapping.go:69-72).
#include <algorithm>
#include <cstdlib>
#include <new>
#include <atomic>
#include <memory>
#include <cstring>
#include <mutex>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include "common.hpp"
#include "dlower.hpp"
#include "hostmem.hpp"
#include "placement.hpp"
#include "pool.hpp"

namespace dp {

static thread_local std::string g_err;
void set_global_error(const std::string& s) { g_err = s; }

// -------------------------------------------------------------------------
// Go %q
// -------------------------------------------------------------------------
static bool go_printable(uint32_t r) {
  if (r < 0x20 || r == 0x7f) return false;
  if (r >= 0x80 && r <= 0xa0) return false;  // C1 controls, NBSP (Zs)
  if (r == 0xad) return false;               // soft hyphen (Cf)
  if (r >= 0x600 && r <= 0x605) return false;
  if (r == 0x61c || r == 0x6dd || r == 0x70f || r == 0x180e) return false;
  if (r == 0x1680) return false;
  if (r >= 0x2000 && r <= 0x200f) return false;  // spaces, ZW*, marks
  if (r >= 0x2028 && r <= 0x202f) return false;
  if (r >= 0x205f && r <= 0x206f) return false;
  if (r == 0x3000 || r == 0xfeff) return false;
  if (r >= 0xd800 && r <= 0xf8ff) return false;  // surrogates, private use
  if (r >= 0xfff9 && r <= 0xfffb) return false;
  if (r == 0xfffe || r == 0xffff) return false;
  if (r >= 0xe0000) return false;  // tags, supplementary private use
  return true;
}

std::string go_quote(const char* s, size_t n) {
  static const char* hex = "0123456789abcdef";
  std::string o;
  o.reserve(n + 2);
  o.push_back('"');
  size_t i = 0;
  while (i < n) {
    unsigned char c = (unsigned char)s[i];
    if (c < 0x80) {
      if (c == '"' || c == '\\') {
        o.push_back('\\');
        o.push_back((char)c);
      } else if (c >= 0x20 && c < 0x7f) {
        o.push_back((char)c);
      } else {
        const char* e = nullptr;
        switch (c) {
          case 7: e = "\\a"; break;
          case 8: e = "\\b"; break;
          case 12: e = "\\f"; break;
          case 10: e = "\\n"; break;
          case 13: e = "\\r"; break;
          case 9: e = "\\t"; break;
          case 11: e = "\\v"; break;
        }
        if (e) o += e;
        else { o += "\\x"; o.push_back(hex[c >> 4]); o.push_back(hex[c & 15]); }
      }
      ++i;
      continue;
    }
    int len = (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 0;
    uint32_t r = 0;
    bool ok = len > 0 && i + len <= n;
    if (ok) {
      r = c & (0x7f >> len);
      for (int k = 1; k < len; ++k) {
        unsigned char d = (unsigned char)s[i + k];
        if ((d & 0xc0) != 0x80) { ok = false; break; }
        r = (r << 6) | (d & 0x3f);
      }
      // overlong / out of range / surrogate encodings are invalid UTF-8
      static const uint32_t minr[5] = {0, 0, 0x80, 0x800, 0x10000};
      if (ok && (r < minr[len] || r > 0x10ffff || (r >= 0xd800 && r <= 0xdfff))) ok = false;
    }
    if (!ok) {
      o += "\\x"; o.push_back(hex[c >> 4]); o.push_back(hex[c & 15]);
      ++i;
      continue;
    }
    if (go_printable(r)) {
      o.append(s + i, (size_t)len);
    } else if (r < 0x10000) {
      char b[8]; snprintf(b, sizeof b, "\\u%04x", r); o += b;
    } else {
      char b[12]; snprintf(b, sizeof b, "\\U%08x", r); o += b;
    }
    i += (size_t)len;
  }
  o.push_back('"');
  return o;
}

namespace {

constexpr int32_t kF = 0, kT = 1;

// Open-addressing hash map from 64-bit keys to int32 values, with
// generation-stamped slots: reset() is O(1), so one table serves every
// problem a worker lowers (std::unordered_map cost ~0.3 s per OLM-scale
// catalog in node allocation alone).
struct FlatMap {
  // one 16-byte slot per entry (key, generation, value): a probe touches one
  // cache line instead of one in each of three arrays
  struct Slot {
    uint64_t key;
    uint32_t gen;
    int32_t val;
  };
  std::vector<Slot> slot;
  uint32_t cur = 1;
  size_t count = 0, mask = 0;
  FlatMap() { grow(1024); }
  void grow(size_t cap) {
    std::vector<Slot> s2(cap, Slot{0, 0, 0});
    const size_t m2 = cap - 1;
    for (const Slot& e : slot)
      if (e.gen == cur) {
        size_t h = hash(e.key) & m2;
        while (s2[h].gen == cur) h = (h + 1) & m2;
        s2[h] = e;
      }
    slot.swap(s2);
    mask = m2;
  }
  static size_t hash(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33;
    return (size_t)x;
  }
  void reset() {
    count = 0;
    if (++cur == 0) {  // generation wrap: clear for real
      for (Slot& e : slot) e.gen = 0;
      cur = 1;
    }
  }
  // the value of k, or -1
  int32_t find(uint64_t k) const {
    for (size_t h = hash(k) & mask; slot[h].gen == cur; h = (h + 1) & mask)
      if (slot[h].key == k) return slot[h].val;
    return -1;
  }
  // insert k -> v (k must be absent)
  void insert(uint64_t k, int32_t v) {
    if (2 * (count + 1) > slot.size()) grow(2 * slot.size());
    size_t h = hash(k) & mask;
    while (slot[h].gen == cur) h = (h + 1) & mask;
    slot[h] = Slot{k, cur, v};
    ++count;
  }
  // the slot of k, inserted with value v when absent
  int32_t* find_or_insert(uint64_t k, int32_t v) {
    if (2 * (count + 1) > slot.size()) grow(2 * slot.size());
    size_t h = hash(k) & mask;
    for (; slot[h].gen == cur; h = (h + 1) & mask)
      if (slot[h].key == k) return &slot[h].val;
    slot[h] = Slot{k, cur, v};
    ++count;
    return &slot[h].val;
  }
  int32_t* find_slot(uint64_t k) {
    for (size_t h = hash(k) & mask; slot[h].gen == cur; h = (h + 1) & mask)
      if (slot[h].key == k) return &slot[h].val;
    return nullptr;
  }
};

// And-inverter graph with structural hashing (gini logic.C).
struct Aig {
  int32_t next_node = 1;
  FlatMap strash;
  std::vector<uint64_t> fanin;  // gate node 1 + nv + i: its strash key (a << 32 | b)
  void reset(int nv) {
    next_node = 1 + nv;
    strash.reset();
    fanin.clear();
  }
  static int32_t input(int v) { return 2 * (v + 1); }
  int32_t And(int32_t a, int32_t b) {
    if (a == kF || b == kF) return kF;
    if (a == kT) return b;
    if (b == kT) return a;
    if (a == b) return a;
    if (a == (b ^ 1)) return kF;
    if (a > b) std::swap(a, b);
    uint64_t key = ((uint64_t)(uint32_t)a << 32) | (uint32_t)b;
    const int32_t hit = strash.find(key);
    if (hit >= 0) return hit;
    int32_t g = 2 * next_node++;
    strash.insert(key, g);
    fanin.push_back(key);
    return g;
  }
  int32_t Or(int32_t a, int32_t b) { return And(a ^ 1, b ^ 1) ^ 1; }
};

// Batcher odd-even merge sort comparators for n = 2^k (gini CardSort,
// recalled).  Built once per k (k < 31), then read without a lock.
const std::vector<std::pair<int, int>>& batcher(int n) {
  static std::mutex mu;
  static std::atomic<const std::vector<std::pair<int, int>>*> table[31];
  int k = 0;
  while ((1 << k) < n) ++k;
  if (const auto* t = table[k].load(std::memory_order_acquire)) return *t;
  std::lock_guard<std::mutex> lk(mu);
  if (const auto* t = table[k].load(std::memory_order_relaxed)) return *t;
  auto* v = new std::vector<std::pair<int, int>>();  // kept for the process lifetime
  for (int p = 1; p < n; p <<= 1)
    for (int q = p; q >= 1; q >>= 1)
      for (int j = q % p; j < n - q; j += 2 * q)
        for (int i = 0; i < std::min(q, n - j - q); ++i)
          if ((i + j) / (2 * p) == (i + j + q) / (2 * p)) v->emplace_back(i + j, i + j + q);
  table[k].store(v, std::memory_order_release);
  return *v;
}

// The fast path's record under construction: raw arrays sized once per
// problem from its counts (no per-element capacity checks).
struct Fast {
  std::vector<int32_t> store;
  std::vector<int64_t> store64;
  int32_t *clause_off, *clause_lits, *clause_id, *card_off, *card_lits, *card_bound, *card_id;
  int32_t *var_choice_off, *choice_off, *choice_lits, *anchors, *owner_v, *owner_c, *first_s, *seq, *seq2;
  int32_t* list_id;  // [nch] the identity of choice list k's Dependency (-1: folded to T)
  int64_t* first_c;
  // DP_FMT_P16D sources of the choice lists (choice_sources' answer, known
  // while the lists are made): valid while src_ok
  uint8_t* src;
  bool src_ok;
  int32_t nc, ncl, nk, nkl, nch, nchl, na, nid;
  void reset(size_t nv, size_t C, size_t A) {
    const size_t need = (C + 1) + (A + C) + C + (C + 1) + A + C + C + (nv + 1) + (C + 1) + A + nv + 5 * C + 2 * (A + 1) +
                        (C + 4) / 4;
    if (store.size() < need) store.resize(need + need / 4);
    if (store64.size() < C + 1) store64.resize(C + 1 + C / 4);
    int32_t* q = store.data();
    auto take = [&](size_t n) { int32_t* r = q; q += n; return r; };
    clause_off = take(C + 1); clause_lits = take(A + C); clause_id = take(C);
    card_off = take(C + 1); card_lits = take(A); card_bound = take(C); card_id = take(C);
    var_choice_off = take(nv + 1); choice_off = take(C + 1); choice_lits = take(A); anchors = take(nv);
    owner_v = take(C); owner_c = take(C); first_s = take(C); seq2 = take(A + 1); seq = take(A + 1);
    list_id = take(C);
    src = reinterpret_cast<uint8_t*>(take((C + 4) / 4));
    (void)take(C);
    first_c = store64.data();
    nc = ncl = nk = nkl = nch = nchl = na = nid = 0;
    src_ok = true;
    clause_off[0] = card_off[0] = var_choice_off[0] = choice_off[0] = 0;
  }
  void close_clause(int32_t id) {
    clause_id[nc] = id;
    clause_off[++nc] = ncl;
  }
};

// Per-thread output and scratch: 128-byte aligned, since their vector headers
// change with every append and neighbouring threads' would share cache lines.
struct alignas(128) Out {  // per-thread output chunk
  // records: rec[0..nrec) (storage grows geometrically and is never
  // re-initialised, so appending a record writes its words once)
  std::vector<int32_t> rec;
  size_t nrec = 0;
  int32_t* extend(size_t n) {
    if (nrec + n > rec.size()) rec.resize(std::max(2 * rec.size(), nrec + n + 4096));
    int32_t* r = rec.data() + nrec;
    nrec += n;
    return r;
  }
  std::vector<int64_t> rec_len;  // per problem
  std::vector<int32_t> ivar, icon;
  std::vector<int64_t> ident_len;
  std::vector<int32_t> err;
  std::vector<std::string> msg;
};

struct alignas(128) Work {  // per-thread scratch
  Aig aig;
  // interned path: string id -> variable of the problem being lowered, valid
  // while st_tag matches the problem's tag (no clearing between problems)
  std::vector<uint64_t> st_tag;
  std::vector<int32_t> st_idx;
  // the fast path's: (problem stamp << 32 | variable) per string id, one load
  // per lookup; a stamp per problem lowered (0 never used, wrap clears)
  std::vector<uint64_t> fst;
  uint32_t fstamp = 0;
  uint32_t next_fstamp() {
    if (++fstamp == 0) {
      std::fill(fst.begin(), fst.end(), 0);
      fstamp = 1;
    }
    return fstamp;
  }
  uint64_t gen = 0;  // dp_lower call number of this scratch
  uint64_t tag_of(int32_t p, bool fast) const { return gen << 33 | (uint64_t)(p + 1) << 1 | (fast ? 1u : 0u); }
  std::unordered_map<std::string_view, int32_t> names;
  FlatMap key_ident;  // gate literal -> identity
  std::vector<int32_t> owner_v, owner_c;
  std::vector<int32_t> clause_off, clause_lits, clause_id;
  std::vector<int32_t> card_off, card_lits, card_bound, card_id;
  std::vector<int32_t> var_choice_off, choice_off, choice_lits, anchors;
  std::vector<int32_t> ms, sorted, order, mult;
  // AtMost networks (Lowerer::network_rows): next auxiliary variable, a
  // gate's cone and the walk's marks
  int32_t naux = 0;
  std::vector<int32_t> cone, walk;
  std::vector<uint8_t> vis;
  std::vector<std::string> errs;
  // fast path (lower_fast): identity keys and the record under construction
  FlatMap fkey;
  Fast fast;
};

// Canonical identity keys of the fast path (Lowerer::lower_fast).  gini's
// logic.C hash-conses And(a, b) on the unordered operand pair after folding
// constants, a == b and a == !b, so two constraints share an assumed literal
// exactly when their folded terms are equal.  The fast path names each term
// by a key without building the graph:
//   K_POS v        x_v             Mandatory(v)
//   K_NEG v        !x_v            Prohibited(v), Dependency(v;), Conflict(v,v),
//                                  AtMost(0; v)
//   K_CONF {a,b}   !And(x_a, x_b)  Conflict(a,b), AtMost(1; a,b)   (a != b)
//   K_NOR {a,b}    And(!x_a, !x_b) AtMost(0; a,b)                  (a != b)
//   K_DEP (s,d..)  the Or chain    Dependency(s; d1..dn), d1 != s  (hashed;
//                                  the term is And(..And(x_s,!x_d1)..,!x_dn):
//                                  each level splits uniquely into a node and
//                                  an input, so equal terms <=> equal sequences)
//   K_CARD n, set  !sorted[n]      AtMost(n; m distinct vars), m >= 3 (hashed)
//   K_F            F               AtMost(n < 0; ...)
// Terms of different keys compute different Boolean functions, so they are
// different terms: !sorted[n] of Batcher's network over m distinct inputs is
// "at most n of the m", antimonotone and dependent on all m (0 <= n < m); a
// Dependency chain with s not among d is increasing in every d it names (or
// the constant T once s recurs); Mandatory is increasing, the others are
// antimonotone in fewer variables.  What the keys cannot decide goes to the
// exact path (lower_one, the full AIG): an AtMost with a repeated variable,
// two AtMosts over one set and bound in different orders (same function,
// structure unknown), a hashed key that matches a different sequence, and any
// lookup error.
enum : uint64_t { K_F = 0, K_POS = 1, K_NEG = 2, K_CONF = 3, K_NOR = 4, K_DEP = 5, K_CARD = 6 };
inline uint64_t key1(uint64_t tag, uint32_t a) { return tag << 60 | a; }
inline uint64_t key2(uint64_t tag, uint32_t a, uint32_t b) {
  if (a > b) std::swap(a, b);
  return tag << 60 | (uint64_t)a << 30 | b;
}
inline uint64_t hmix(uint64_t h, uint64_t x) {
  h ^= x + 0x9e3779b97f4a7c15ULL;
  h *= 0xbf58476d1ce4e5b9ULL;
  return h ^ (h >> 31);
}
inline uint64_t keyh(uint64_t tag, uint64_t h) { return tag << 60 | (h & ((1ULL << 60) - 1)); }

// DP_FMT_P16D (include/deppy_hip.h): the choice lists a record's dependency
// rows imply.  Dependency rows are clause rows of two or more literals, the
// first negative and the others positive, in row order.  src[k] == 0: list k
// is the next dependency row's variables after its first literal; src[k] = d
// > 0: list k repeats list k - d (which took a row).  var_choice_off counts
// the lists per subject (the first literal's variable; subjects never
// decrease).  Writes vco[nv+1], co[nch+1], cl[nchl]; false unless every
// dependency row is taken once and the lists hold exactly nchl variables,
// every index in range.
bool implied_choices(const int32_t* clause_off, const int32_t* clause_lits, int32_t nc, int32_t nv, int32_t nch,
                     int32_t nchl, const uint8_t* src, int32_t* vco, int32_t* co, int32_t* cl) {
  static thread_local std::vector<int32_t> dep, rowk;
  dep.clear();
  for (int32_t r = 0; r < nc; ++r) {
    const int32_t a = clause_off[r], b = clause_off[r + 1];
    if (b - a < 2 || !(clause_lits[a] & 1)) continue;
    bool d = true;
    for (int32_t j = a + 1; j < b && d; ++j) d = !(clause_lits[j] & 1);
    if (d) dep.push_back(r);
  }
  rowk.assign((size_t)nch, -1);
  size_t j = 0;
  int32_t n = 0, filled = 0, last = 0;
  vco[0] = 0;
  co[0] = 0;
  for (int32_t k = 0; k < nch; ++k) {
    int32_t row;
    if (src[k] == 0) {
      if (j == dep.size()) return false;
      row = dep[j++];
    } else {
      if (src[k] > k || src[k - src[k]] != 0) return false;
      row = rowk[(size_t)(k - src[k])];
    }
    rowk[(size_t)k] = row;
    const int32_t a = clause_off[row], b = clause_off[row + 1];
    const int32_t s = clause_lits[a] >> 1;
    if (s < last || s >= nv || n + (b - a - 1) > nchl) return false;
    last = s;
    while (filled < s) vco[++filled] = k;
    for (int32_t q = a + 1; q < b; ++q) {
      if ((clause_lits[q] >> 1) >= nv) return false;
      cl[n++] = clause_lits[q] >> 1;
    }
    co[k + 1] = n;
  }
  while (filled < nv) vco[++filled] = nch;
  return j == dep.size() && n == nchl;
}

// The DP_FMT_P16D sources of an int32 record's choice lists (src[nch]), or
// false when its dependency rows do not imply them (a list whose row was
// folded away, a repeat more than 255 lists back, a row no list takes, ...).
// Matched greedily: list k takes the next dependency row when that row is
// (~subject, list k), else repeats an earlier list of the same subject and
// content.  Every list is checked against what it derives from, so true
// means implied_choices(src) gives back exactly the record's arrays.
bool choice_sources(const int32_t* r, const dp_rec_layout& L, uint8_t* src) {
  const int32_t nc = r[DP_H_NC], nv = r[DP_H_NV], nch = r[DP_H_NCH];
  const int32_t* clause_off = r + L.clause_off;
  const int32_t* clause_lits = r + L.clause_lits;
  const int32_t* vco = r + L.var_choice_off;
  const int32_t* co = r + L.choice_off;
  const int32_t* cl = r + L.choice_lits;
  int32_t row = 0, v = 0;
  auto next_dep = [&]() {
    for (; row < nc; ++row) {
      const int32_t a = clause_off[row], b = clause_off[row + 1];
      if (b - a < 2 || !(clause_lits[a] & 1)) continue;
      bool d = true;
      for (int32_t j = a + 1; j < b && d; ++j) d = !(clause_lits[j] & 1);
      if (d) return;
    }
  };
  auto same = [&](int32_t k, int32_t k2) {
    return co[k + 1] - co[k] == co[k2 + 1] - co[k2] && std::equal(cl + co[k], cl + co[k + 1], cl + co[k2]);
  };
  next_dep();
  for (int32_t k = 0; k < nch; ++k) {
    while (v < nv && vco[v + 1] <= k) ++v;
    bool took = false;
    if (row < nc) {
      const int32_t a = clause_off[row], b = clause_off[row + 1];
      if (clause_lits[a] == 2 * v + 1 && b - a - 1 == co[k + 1] - co[k]) {
        took = true;
        for (int32_t q = 0; q < b - a - 1 && took; ++q) took = clause_lits[a + 1 + q] == 2 * cl[co[k] + q];
      }
    }
    if (took) {
      src[k] = 0;
      ++row;
      next_dep();
      continue;
    }
    int32_t d = 1;
    for (; d <= 255 && d <= k && vco[v] <= k - d; ++d)
      if (src[k - d] == 0 && same(k, k - d)) break;
    if (d > 255 || d > k || vco[v] > k - d) return false;
    src[k] = (uint8_t)d;
  }
  return row >= nc;  // every dependency row taken
}

// DP_FMT_P8D (include/deppy_hip.h) -> the DP_FMT_P16D record it encodes,
// into p16 (header + body, DP_H_P8 cleared).  0, or < 0 when the flags are
// unknown, the body is shorter than its sections or a src value marked
// nonzero is zero (dp_rec_widen then checks the DP_FMT_P16D record).
int p8_to_p16d(const int32_t* rec, int64_t avail, std::vector<int32_t>& p16) {
  const uint32_t w14 = (uint32_t)rec[DP_H_P8];
  const int32_t f = (int32_t)(w14 & 0xffu);
  const int64_t bytes = w14 >> 8;
  if (f & ~(DP_P8_B1 | DP_P8_HI | DP_P8_NIB)) return -22;
  if (DP_H_SIZE + (bytes + 3) / 4 > avail) return -4;
  const dp_p8_layout P = dp_p8_layout_of(rec);
  const int64_t ncl = rec[DP_H_NCL], nkl = rec[DP_H_NKL], nk = rec[DP_H_NK], na = rec[DP_H_NA];
  const int64_t nc = rec[DP_H_NC], nch = rec[DP_H_NCH], nid = rec[DP_H_NID];
  if (P.srcval > bytes) return -22;
  const uint8_t* b = reinterpret_cast<const uint8_t*>(rec + DP_H_SIZE);
  auto bit = [&](int64_t at, int64_t j) -> int { return (b[at + (j >> 3)] >> (j & 7)) & 1; };
  int64_t nz = 0;
  for (int64_t k = 0; k < nch; ++k) nz += bit(P.srcnz, k);
  if (dp_p8_body_bytes(rec, nz) > bytes) return -22;
  int32_t hdr[DP_H_SIZE];
  std::memcpy(hdr, rec, sizeof hdr);
  hdr[DP_H_FMT] = DP_FMT_P16D;
  hdr[DP_H_P8] = 0;
  const int64_t at = dp_p16_tail_at(hdr), tb = dp_p16_tail_bytes(hdr);
  p16.assign((size_t)(DP_H_SIZE + (at + tb + 3) / 4), 0);
  std::memcpy(p16.data(), hdr, sizeof hdr);
  uint16_t* u = reinterpret_cast<uint16_t*>(p16.data() + DP_H_SIZE);
  const bool hi = f & DP_P8_HI;
  auto var = [&](int64_t lo, int64_t hp, int64_t j) -> int { return b[lo + j] | (hi ? bit(hp, j) << 8 : 0); };
  for (int64_t j = 0; j < ncl; ++j) *u++ = (uint16_t)(2 * var(P.cvar, P.chi, j) + bit(P.neg, j));
  for (int64_t j = 0; j < nkl; ++j) *u++ = (uint16_t)var(P.kvar, P.khi, j);
  for (int64_t k = 0; k < nk; ++k) *u++ = (uint16_t)((f & DP_P8_B1) ? 1 : b[P.bound + k]);
  for (int64_t i = 0; i < na; ++i) *u++ = (uint16_t)var(P.avar, P.ahi, i);
  uint8_t* t = reinterpret_cast<uint8_t*>(p16.data() + DP_H_SIZE) + at;
  for (int64_t i = 0; i < nc + nk; ++i)
    *t++ = (f & DP_P8_NIB) ? (uint8_t)((b[P.lens + (i >> 1)] >> (4 * (i & 1))) & 15) : b[P.lens + i];
  int64_t q = 0;
  for (int64_t k = 0; k < nch; ++k) {
    if (!bit(P.srcnz, k)) { *t++ = 0; continue; }
    if (b[P.srcval + q] == 0) return -22;
    *t++ = b[P.srcval + q++];
  }
  std::memcpy(t, b + P.srcval + nz, (size_t)((nid + 7) / 8));
  return 0;
}

// DP_FMT_P8D's body (include/deppy_hip.h) from a record's arrays given by
// accessors -- clause literal j, AtMost variable j, bound k, anchor i, the
// length of row i (clause rows, then AtMost rows), list source k, and the
// identity of AtMost row k -- in two steps: p8_plan (the flags and the body's
// bytes; false when the form does not apply: more than DP_P8_MAX_VARS
// variables or a bound above 255), then p8_write into `o` (the body, zeroed,
// plan.bytes long; sets h's DP_H_FMT and DP_H_P8).  pack8 feeds them a
// DP_FMT_P16D record, the fast lowering its own arrays (Lowerer::emit_p16d).
struct P8Plan {
  int32_t flags;
  int64_t bytes;
};
template <class KB, class LEN, class SRC>
bool p8_plan(const int32_t* h, KB kb, LEN len, SRC src, P8Plan& P) {
  if (h[DP_H_NV] > DP_P8_MAX_VARS) return false;
  const int64_t nk = h[DP_H_NK], rows = (int64_t)h[DP_H_NC] + nk, nch = h[DP_H_NCH];
  bool b1 = true, nib = true;
  for (int64_t k = 0; k < nk; ++k) {
    const int32_t b = kb(k);
    if (b < 0 || b > 255) return false;
    b1 = b1 && b == 1;
  }
  for (int64_t i = 0; i < rows && nib; ++i) nib = len(i) <= 15;
  int64_t nz = 0;
  for (int64_t k = 0; k < nch; ++k) nz += src(k) != 0;
  P.flags = (h[DP_H_NV] > 256 ? DP_P8_HI : 0) | (b1 ? DP_P8_B1 : 0) | (nib ? DP_P8_NIB : 0);
  int32_t t[DP_H_SIZE];
  std::memcpy(t, h, sizeof t);
  t[DP_H_P8] = P.flags;
  P.bytes = dp_p8_body_bytes(t, nz);
  return true;
}
template <class CL, class KL, class KB, class AN, class LEN, class SRC, class KID>
void p8_write(int32_t* h, const P8Plan& P, uint8_t* o, CL cl, KL kl, KB kb, AN an, LEN len, SRC src, KID kid) {
  const int32_t f = P.flags;
  h[DP_H_FMT] = DP_FMT_P8D;
  h[DP_H_P8] = f;
  const dp_p8_layout L = dp_p8_layout_of(h);
  const int64_t ncl = h[DP_H_NCL], nkl = h[DP_H_NKL], nk = h[DP_H_NK], na = h[DP_H_NA];
  const int64_t rows = (int64_t)h[DP_H_NC] + nk, nch = h[DP_H_NCH];
  const bool hi = f & DP_P8_HI;
  auto setbit = [&](int64_t at, int64_t j) { o[at + (j >> 3)] |= (uint8_t)(1u << (j & 7)); };
  // eight positions a step: their low bytes, then their bit-plane bytes
  // whole (no read-modify-write per bit)
  auto vars = [&](auto get, int64_t n, int64_t lo, int64_t neg, int64_t hp, int sh) {
    for (int64_t j0 = 0; j0 < n; j0 += 8) {
      uint32_t nb = 0, hb = 0;
      const int q1 = (int)std::min<int64_t>(8, n - j0);
      for (int q = 0; q < q1; ++q) {
        const int32_t x = get(j0 + q);
        o[lo + j0 + q] = (uint8_t)(x >> sh);
        nb |= (uint32_t)(x & sh) << q;  // (sh = 1: the literal's sign; 0: none)
        hb |= (uint32_t)((x >> (8 + sh)) & 1) << q;
      }
      if (neg >= 0) o[neg + (j0 >> 3)] = (uint8_t)nb;
      if (hi) o[hp + (j0 >> 3)] = (uint8_t)hb;
    }
  };
  vars(cl, ncl, L.cvar, L.neg, L.chi, 1);
  vars(kl, nkl, L.kvar, -1, L.khi, 0);
  vars(an, na, L.avar, -1, L.ahi, 0);
  if (!(f & DP_P8_B1))
    for (int64_t k = 0; k < nk; ++k) o[L.bound + k] = (uint8_t)kb(k);
  if (f & DP_P8_NIB) {
    for (int64_t i = 0; i < rows; i += 2)
      o[L.lens + (i >> 1)] = (uint8_t)(len(i) | (i + 1 < rows ? len(i + 1) << 4 : 0));
  } else {
    for (int64_t i = 0; i < rows; ++i) o[L.lens + i] = (uint8_t)len(i);
  }
  int64_t q = L.srcval;
  for (int64_t k = 0; k < nch; ++k)
    if (const int32_t x = src(k)) {
      setbit(L.srcnz, k);
      o[q++] = (uint8_t)x;
    }
  for (int64_t k = 0; k < nk; ++k) setbit(q, kid(k));
  h[DP_H_P8] = (int32_t)((uint32_t)f | ((uint32_t)P.bytes << 8));
}

// The DP_FMT_P16D record r in the DP_FMT_P8D form, in place, when it applies
// (p8_plan).  Returns its words as it lies (dp_rec_phys_words), or 0 with r
// unchanged.
int64_t pack8(int32_t* r) {
  if (r[DP_H_FMT] != DP_FMT_P16D) return 0;
  const int64_t ncl = r[DP_H_NCL], nkl = r[DP_H_NKL], nk = r[DP_H_NK], nc = r[DP_H_NC], nch = r[DP_H_NCH];
  const uint16_t* u = reinterpret_cast<const uint16_t*>(r + DP_H_SIZE);
  const uint16_t *cl = u, *kl = cl + ncl, *kb = kl + nkl, *an = kb + nk;
  const uint8_t* t = reinterpret_cast<const uint8_t*>(r + DP_H_SIZE) + dp_p16_tail_at(r);
  const uint8_t *lens = t, *src = t + nc + nk, *mask = src + nch;
  auto KB = [&](int64_t k) { return (int32_t)kb[k]; };
  auto LEN = [&](int64_t i) { return (int32_t)lens[i]; };
  auto SRC = [&](int64_t k) { return (int32_t)src[k]; };
  P8Plan P;
  if (!p8_plan(r, KB, LEN, SRC, P)) return 0;
  static thread_local std::vector<int32_t> kid;  // the AtMost identities, from the mask
  kid.clear();
  for (int32_t i = 0; i < r[DP_H_NID]; ++i)
    if ((mask[i >> 3] >> (i & 7)) & 1) kid.push_back(i);
  static thread_local std::vector<uint8_t> o;
  o.assign((size_t)P.bytes, 0);
  int32_t h[DP_H_SIZE];
  std::memcpy(h, r, sizeof h);
  p8_write(h, P, o.data(), [&](int64_t j) { return (int32_t)cl[j]; }, [&](int64_t j) { return (int32_t)kl[j]; }, KB,
           [&](int64_t i) { return (int32_t)an[i]; }, LEN, SRC, [&](int64_t k) { return kid[(size_t)k]; });
  std::memcpy(r, h, sizeof h);
  uint8_t* b = reinterpret_cast<uint8_t*>(r + DP_H_SIZE);
  std::memcpy(b, o.data(), (size_t)P.bytes);
  std::memset(b + P.bytes, 0, (size_t)((4 - P.bytes % 4) % 4));  // to the last word's end
  return dp_rec_phys_words(r);
}

struct Lowerer {
  const dp_wire& w;
  const bool narrow;  // DP_LOWER_NARROW: records that fit 16 bits in the DP_FMT_U16 form
  const bool packed;  // DP_LOWER_PACKED: ... in the DP_FMT_P16 form where they allow it
  // diagnostic DEPPY_HOST_WATCHES=1: multi-wave records above DEV_WATCH_VARS
  // variables carry host-built watch lists (DP_FMT_I32W), as before round 3
  const bool host_watches;
  const int ldsg;  // placement.hpp ldsg_env()
  const bool p8;   // packed records in DP_FMT_P8D where it applies (not DP_LOWER_NO_P8)
  Lowerer(const dp_wire& wire, bool narrow16, bool packed16, bool host_lists, bool p8d)
      : w(wire), narrow(narrow16), packed(packed16), host_watches(host_lists), ldsg(ldsg_env()), p8(p8d) {}

  // The last record appended to O (int32 words from `base`) in the 16-bit
  // form, in place (word j -> halfword j never overtakes word j).  Every
  // record of a DP_LOWER_NARROW batch then ends on a 16-byte boundary, so
  // each one's 16-bit form is the staged form as it is (runtime.cpp
  // start_chunk copies such batches to the device without staging them).
  // src: the DP_FMT_P16D sources of its choice lists when the caller knows
  // them (lower_fast), else nullptr (pack16 derives them: choice_sources).
  void narrow_last(Out& O, size_t base, const uint8_t* src = nullptr) const {
    if (!narrow || O.nrec == base) return;
    int32_t* r = O.rec.data() + base;
    const int64_t words = r[DP_H_WORDS];
    int64_t phys = words;
    if (!lds_image(r, ldsg)) {
      // an HBM-read multi-wave problem: its staged form is the int32 record as it is
      // (the device builds its watch lists, layout.hpp DEV_WATCH_VARS)
      if (host_watches && !device_watches(r)) {
        const int64_t ext = 2 * (int64_t)r[DP_H_NV] + 1 + r[DP_H_NCL] + r[DP_H_NKL];
        O.extend((size_t)ext);  // (may move the storage)
        r = O.rec.data() + base;
        build_watches_host(r);
        r[DP_H_FMT] = DP_FMT_I32W;
        phys = words + ext;
      }
    } else if (packed && pack16(r, src)) {
      const int64_t p8w = p8 ? pack8(r) : 0;
      phys = p8w ? p8w : dp_rec_phys_words(r);
    } else if (dp_rec_fits16(r)) {
      uint16_t* u = reinterpret_cast<uint16_t*>(r + DP_H_SIZE);
      for (int64_t j = 0; j < words - DP_H_SIZE; ++j) u[j] = (uint16_t)r[DP_H_SIZE + j];
      if ((words - DP_H_SIZE) & 1) u[words - DP_H_SIZE] = 0;
      r[DP_H_FMT] = DP_FMT_U16;
      phys = dp_rec_phys_words(r);
    }
    const int64_t padded = (phys + 3) & ~3LL;
    const int64_t have = (int64_t)(O.nrec - base);  // words appended for the record so far
    O.nrec = base + (size_t)std::min(have, padded);
    if (padded > have) O.extend((size_t)(padded - have));  // (may move the storage)
    r = O.rec.data() + base;
    for (int64_t j = phys; j < padded; ++j) r[j] = 0;
    O.rec_len.back() = padded;
  }

  // The int32 record r (fits16) in a packed form, in place, if it allows it
  // (every identity one row, each row kind's identities ascending, lengths
  // below 256, DP_P16_TAIL_MAX): DP_FMT_P16D when its dependency rows imply
  // its choice lists, else DP_FMT_P16.  False leaves r as it is.
  static bool pack16(int32_t* r, const uint8_t* src_known = nullptr) {
    if (!dp_rec_fits16(r) || r[DP_H_NID] != r[DP_H_NC] + r[DP_H_NK]) return false;
    const dp_rec_layout L = dp_rec_layout_of(r);
    const int32_t nc = r[DP_H_NC], nk = r[DP_H_NK], nv = r[DP_H_NV], nch = r[DP_H_NCH], nid = r[DP_H_NID];
    // DP_FMT_P16D when the dependency rows imply the choice lists exactly
    static thread_local std::vector<uint8_t> srcs;
    const uint8_t* sp = src_known;
    bool derived = !no_p16d() && sp;
    if (!no_p16d() && !sp) {
      if (srcs.size() < (size_t)nch + 1) srcs.resize((size_t)nch + 1);
      derived = choice_sources(r, L, srcs.data());
      sp = srcs.data();
    }
    for (int32_t i = 1; i < nc; ++i)
      if (r[L.clause_id + i] <= r[L.clause_id + i - 1]) return false;
    for (int32_t i = 1; i < nk; ++i)
      if (r[L.card_id + i] <= r[L.card_id + i - 1]) return false;
    for (int32_t k = 0; k < nk; ++k)
      if (r[L.card_id + k] < 0 || r[L.card_id + k] >= nid) return false;
    auto short_lens = [&](int32_t off, int32_t n) {
      for (int32_t j = 0; j < n; ++j)
        if (r[off + j + 1] - r[off + j] > 255) return false;
      return true;
    };
    if (!short_lens(L.clause_off, nc) || !short_lens(L.card_off, nk) ||
        (!derived && (!short_lens(L.var_choice_off, nv) || !short_lens(L.choice_off, nch))))
      return false;
    const int32_t fmt0 = r[DP_H_FMT];
    r[DP_H_FMT] = derived ? DP_FMT_P16D : DP_FMT_P16;  // (the tail's size depends on the form)
    if (dp_p16_tail_bytes(r) > DP_P16_TAIL_MAX) {
      r[DP_H_FMT] = fmt0;
      return false;
    }
    // the tail first (it reads the offsets arrays and the AtMost identities,
    // which the 16-bit arrays then overwrite in place: each lands at half its
    // int32 position or less, so no word is written before it is read)
    static thread_local std::vector<uint8_t> tail;
    const int64_t at = dp_p16_tail_at(r), tb = dp_p16_tail_bytes(r);
    tail.assign((size_t)tb, 0);
    uint8_t* t = tail.data();
    auto put_lens = [&](int32_t off, int32_t n) {
      for (int32_t j = 0; j < n; ++j) *t++ = (uint8_t)(r[off + j + 1] - r[off + j]);
    };
    put_lens(L.clause_off, nc);
    put_lens(L.card_off, nk);
    if (!derived) {
      put_lens(L.var_choice_off, nv);
      put_lens(L.choice_off, nch);
    } else {
      std::memcpy(t, sp, (size_t)nch);
      t += nch;
    }
    for (int32_t k = 0; k < nk; ++k) t[r[L.card_id + k] >> 3] |= (uint8_t)(1u << (r[L.card_id + k] & 7));
    uint16_t* u = reinterpret_cast<uint16_t*>(r + DP_H_SIZE);
    auto put16 = [&](int32_t off, int32_t n) {
      for (int32_t j = 0; j < n; ++j) *u++ = (uint16_t)r[off + j];
    };
    put16(L.clause_lits, r[DP_H_NCL]);
    put16(L.card_lits, r[DP_H_NKL]);
    put16(L.card_bound, nk);
    if (!derived) put16(L.choice_lits, r[DP_H_NCHL]);
    put16(L.anchors, r[DP_H_NA]);
    uint8_t* b = reinterpret_cast<uint8_t*>(r + DP_H_SIZE);
    std::memset(reinterpret_cast<uint8_t*>(u), 0, (size_t)(b + at - reinterpret_cast<uint8_t*>(u)));
    std::memcpy(b + at, tail.data(), (size_t)tb);
    std::memset(b + at + tb, 0, (size_t)((4 - (at + tb) % 4) % 4));  // to the last word's end
    return true;
  }

  static bool no_p16d() {  // diagnostic DEPPY_NO_P16D=1: explicit choice lists (DP_FMT_P16)
    static const bool v = [] {
      const char* e = std::getenv("DEPPY_NO_P16D");
      return e && *e && *e != '0';
    }();
    return v;
  }

  // The fast path's record written straight in DP_FMT_P16D, the form
  // emit_fast + narrow_last + pack16 give it, without the int32 record in
  // between (a third of the lowering's memory traffic): when the batch asks
  // for packed records, the record runs one wavefront per problem (decided
  // on its int32 header, as narrow_last does) and the form applies (every
  // identity one row -- the fast path numbers identities in row order, so
  // each row kind's are ascending -- row lengths below 256, choice lists
  // implied, tail within DP_P16_TAIL_MAX).  False: nothing written.
  bool emit_p16d(const Fast& F, Out& O, int nv) const {
    if (!narrow || !packed || !F.src_ok || no_p16d() || F.nid != F.nc + F.nk) return false;
    int32_t hdr[DP_H_SIZE] = {0};
    hdr[DP_H_MAGIC] = DP_REC_MAGIC;
    hdr[DP_H_NV] = nv;
    hdr[DP_H_NC] = F.nc;
    hdr[DP_H_NK] = F.nk;
    hdr[DP_H_NCH] = F.nch;
    hdr[DP_H_NA] = F.na;
    hdr[DP_H_NID] = F.nid;
    hdr[DP_H_NCL] = F.ncl;
    hdr[DP_H_NKL] = F.nkl;
    hdr[DP_H_NCHL] = F.nchl;
    hdr[DP_H_WORDS] = dp_rec_layout_of(hdr).words;
    if (!lds_image(hdr, ldsg)) return false;  // (fits16 included)
    for (int32_t i = 0; i < F.nc; ++i)
      if (F.clause_off[i + 1] - F.clause_off[i] > 255) return false;
    for (int32_t k = 0; k < F.nk; ++k)
      if (F.card_off[k + 1] - F.card_off[k] > 255) return false;
    hdr[DP_H_FMT] = DP_FMT_P16D;
    const int64_t tb = dp_p16_tail_bytes(hdr);
    if (tb > DP_P16_TAIL_MAX) return false;
    auto len = [&](int64_t i) {
      return i < F.nc ? F.clause_off[i + 1] - F.clause_off[i] : F.card_off[i - F.nc + 1] - F.card_off[i - F.nc];
    };
    auto kb = [&](int64_t k) { return F.card_bound[k]; };
    auto srcv = [&](int64_t k) { return (int32_t)F.src[k]; };
    P8Plan P8;
    if (p8 && p8_plan(hdr, kb, len, srcv, P8)) {  // DP_FMT_P8D straight from the arrays
      const int64_t phys = DP_H_SIZE + (P8.bytes + 3) / 4, padded = (phys + 3) & ~3LL;
      int32_t* r = O.extend((size_t)padded);
      uint8_t* b = reinterpret_cast<uint8_t*>(r + DP_H_SIZE);
      std::memset(b, 0, (size_t)(4 * (padded - DP_H_SIZE)));
      p8_write(hdr, P8, b, [&](int64_t j) { return F.clause_lits[j]; }, [&](int64_t j) { return F.card_lits[j]; }, kb,
               [&](int64_t i) { return F.anchors[i]; }, len, srcv, [&](int64_t k) { return F.card_id[k]; });
      std::memcpy(r, hdr, sizeof hdr);
      O.rec_len.push_back(padded);
      O.ivar.insert(O.ivar.end(), F.owner_v, F.owner_v + F.nid);
      O.icon.insert(O.icon.end(), F.owner_c, F.owner_c + F.nid);
      O.ident_len.push_back(F.nid);
      O.err.push_back(DP_LOWER_OK);
      O.msg.emplace_back();
      return true;
    }
    const int64_t at = dp_p16_tail_at(hdr);
    const int64_t phys = DP_H_SIZE + (at + tb + 3) / 4, padded = (phys + 3) & ~3LL;
    int32_t* r = O.extend((size_t)padded);
    std::memcpy(r, hdr, sizeof hdr);
    uint16_t* u = reinterpret_cast<uint16_t*>(r + DP_H_SIZE);
    auto put16 = [&](const int32_t* a, int32_t n) {
      for (int32_t j = 0; j < n; ++j) u[j] = (uint16_t)a[j];
      u += n;
    };
    put16(F.clause_lits, F.ncl);
    put16(F.card_lits, F.nkl);
    put16(F.card_bound, F.nk);
    put16(F.anchors, F.na);
    uint8_t* const b = reinterpret_cast<uint8_t*>(r + DP_H_SIZE);
    uint8_t* t = reinterpret_cast<uint8_t*>(u);
    std::memset(t, 0, (size_t)(b + at - t));
    t = b + at;
    for (int32_t i = 0; i < F.nc; ++i) *t++ = (uint8_t)(F.clause_off[i + 1] - F.clause_off[i]);
    for (int32_t k = 0; k < F.nk; ++k) *t++ = (uint8_t)(F.card_off[k + 1] - F.card_off[k]);
    std::memcpy(t, F.src, (size_t)F.nch);
    t += F.nch;
    std::memset(t, 0, (size_t)(reinterpret_cast<uint8_t*>(r + padded) - t));  // mask, then the padding
    for (int32_t k = 0; k < F.nk; ++k) t[F.card_id[k] >> 3] |= (uint8_t)(1u << (F.card_id[k] & 7));
    O.rec_len.push_back(padded);
    O.ivar.insert(O.ivar.end(), F.owner_v, F.owner_v + F.nid);
    O.icon.insert(O.icon.end(), F.owner_c, F.owner_c + F.nid);
    O.ident_len.push_back(F.nid);
    O.err.push_back(DP_LOWER_OK);
    O.msg.emplace_back();
    return true;
  }

  std::string_view str(int64_t i) const {
    return std::string_view(w.str_bytes + w.str_off[i], (size_t)(w.str_off[i + 1] - w.str_off[i]));
  }

  void lower_one(int32_t p, Work& W, Out& O) const {
    const int64_t v0 = w.prob_var_off[p], v1 = w.prob_var_off[p + 1];
    const int nv = (int)(v1 - v0);
    const uint64_t tag = W.tag_of(p, false);
    // pass 1: one literal per variable, reject duplicates (lit_mapping.go:50-57)
    W.names.clear();
    for (int i = 0; i < nv; ++i) {
      int64_t sid = w.var_id[v0 + i];
      bool dup;
      if (w.interned) {
        dup = W.st_tag[(size_t)sid] == tag;
        if (!dup) { W.st_tag[(size_t)sid] = tag; W.st_idx[(size_t)sid] = i; }
      } else {
        dup = !W.names.emplace(str(sid), i).second;
      }
      if (dup) {
        std::string_view s = str(sid);
        emit_error(O, DP_LOWER_DUPLICATE,
                   "duplicate identifier " + go_quote(s.data(), s.size()) + " in input");
        return;
      }
    }
    auto lit_of = [&](int64_t sid) -> int32_t {  // LitOf, lit_mapping.go:81-88
      int32_t v = -1;
      if (w.interned) {
        if (W.st_tag[(size_t)sid] == tag) v = W.st_idx[(size_t)sid];
      } else {
        auto it = W.names.find(str(sid));
        if (it != W.names.end()) v = it->second;
      }
      if (v < 0) {
        std::string_view s = str(sid);
        W.errs.push_back("variable " + go_quote(s.data(), s.size()) + " referenced but not provided");
      }
      return v;
    };

    Aig& aig = W.aig;
    aig.reset(nv);
    W.key_ident.reset();
    W.owner_v.clear(); W.owner_c.clear();
    W.clause_off.assign(1, 0); W.clause_lits.clear(); W.clause_id.clear();
    W.card_off.assign(1, 0); W.card_lits.clear(); W.card_bound.clear(); W.card_id.clear();
    W.errs.clear();
    W.naux = nv;

    // pass 2: Apply every constraint (lit_mapping.go:59-74)
    for (int vi = 0; vi < nv; ++vi) {
      const int64_t c0 = w.var_con_off[v0 + vi], c1 = w.var_con_off[v0 + vi + 1];
      for (int64_t c = c0; c < c1; ++c) {
        const int ci = (int)(c - c0);
        const int32_t kind = w.con_kind[c];
        const int64_t a0 = w.con_arg_off[c], a1 = w.con_arg_off[c + 1];
        bool bad = false;
        int32_t m = kF;
        switch (kind) {
          case DP_MANDATORY: m = Aig::input(vi); break;
          case DP_PROHIBITED: m = Aig::input(vi) ^ 1; break;
          case DP_DEPENDENCY:
            m = Aig::input(vi) ^ 1;
            for (int64_t a = a0; a < a1; ++a) {
              int32_t d = lit_of(w.con_arg[a]);
              if (d < 0) { bad = true; continue; }
              m = aig.Or(m, Aig::input(d));
            }
            break;
          case DP_CONFLICT: {
            int32_t t = lit_of(w.con_arg[a0]);
            if (t < 0) bad = true;
            else m = aig.Or(Aig::input(vi) ^ 1, Aig::input(t) ^ 1);
            break;
          }
          case DP_ATMOST: {
            W.ms.clear();
            for (int64_t a = a0; a < a1; ++a) {
              int32_t d = lit_of(w.con_arg[a]);
              if (d < 0) { bad = true; continue; }
              W.ms.push_back(Aig::input(d));
            }
            if (!bad) m = leq(aig, W, w.con_n[c]);
            break;
          }
        }
        if (bad || !W.errs.empty() || m == kT) continue;
        int32_t* slot = W.key_ident.find_slot((uint64_t)(uint32_t)m);
        if (!slot) {
          int32_t ident = (int32_t)W.owner_v.size();
          W.key_ident.insert((uint64_t)(uint32_t)m, ident);
          W.owner_v.push_back(vi);
          W.owner_c.push_back(ci);
          emit_rows(W, m, nv, kind, vi, w.con_n[c], a0, a1, ident);
        } else {
          W.owner_v[*slot] = vi;  // last writer wins, lit_mapping.go:69-72
          W.owner_c[*slot] = ci;
        }
      }
    }
    if (!W.errs.empty()) {
      std::string msg = std::to_string(W.errs.size()) + " errors encountered: ";
      for (size_t i = 0; i < W.errs.size(); ++i) {
        if (i) msg += ", ";
        msg += W.errs[i];
      }
      emit_error(O, DP_LOWER_LOOKUP, msg);
      return;
    }
    // choices in constraint order (search.go:59-69) and anchors (lit_mapping.go:163-174)
    W.var_choice_off.assign(1, 0); W.choice_off.assign(1, 0); W.choice_lits.clear(); W.anchors.clear();
    for (int vi = 0; vi < nv; ++vi) {
      const int64_t c0 = w.var_con_off[v0 + vi], c1 = w.var_con_off[v0 + vi + 1];
      bool anchor = false;
      for (int64_t c = c0; c < c1; ++c) {
        if (w.con_kind[c] == DP_MANDATORY) anchor = true;
        if (w.con_kind[c] == DP_DEPENDENCY && w.con_arg_off[c + 1] > w.con_arg_off[c]) {
          for (int64_t a = w.con_arg_off[c]; a < w.con_arg_off[c + 1]; ++a)
            W.choice_lits.push_back(lit_of(w.con_arg[a]));
          W.choice_off.push_back((int32_t)W.choice_lits.size());
        }
      }
      W.var_choice_off.push_back((int32_t)W.choice_off.size() - 1);
      if (anchor) W.anchors.push_back(vi);
    }
    W.var_choice_off.resize((size_t)W.naux + 1, W.var_choice_off.back());  // auxiliaries: no choices
    const size_t base = O.nrec;
    emit_record(W, O, W.naux, W.naux > nv ? nv : 0);
    narrow_last(O, base);
  }

  // lower_one's exact result without the And-inverter graph, from the
  // canonical keys above.  Returns 1 (record emitted), 0 (the keys cannot
  // decide: nothing emitted, lower_one must run) or -1 (malformed problem).
  // The problem's own arrays are validated on the way (problem_ok's checks).
  // Arrays are raw buffers sized from the problem's counts: a problem with C
  // constraints and A arguments has at most C rows, A + C clause literals, A
  // AtMost positions and A choice literals.
  int lower_fast(int32_t p, Work& W, Out& O) const {
    if (!w.interned) return 0;
    const int64_t v0 = w.prob_var_off[p], v1 = w.prob_var_off[p + 1];
    const int nv = (int)(v1 - v0);
    if (nv >= (1 << 28)) return 0;
    const uint64_t nstr = (uint64_t)w.n_strs;
    const int64_t* const var_id = w.var_id;
    const int64_t* const var_con_off = w.var_con_off;
    const int32_t* const con_kind = w.con_kind;
    const int32_t* const con_n = w.con_n;
    const int64_t* const con_arg_off = w.con_arg_off;
    const int64_t* const con_arg = w.con_arg;
    // this path's stamps are its own (lower_one may follow)
    uint64_t* const fst = W.fst.data();
    const uint64_t stamp = (uint64_t)W.next_fstamp() << 32;
    for (int i = 0; i < nv; ++i) {
      const uint64_t sid = (uint64_t)var_id[v0 + i];
      if (sid >= nstr || var_con_off[v0 + i + 1] < var_con_off[v0 + i]) return -1;
      if ((fst[sid] & ~0xffffffffULL) == stamp) return 0;  // a duplicate: lower_one reports it
      fst[sid] = stamp | (uint32_t)i;
    }
    const int64_t cb = nv ? var_con_off[v0] : 0, ce = nv ? var_con_off[v1] : 0;
    const int64_t C = ce - cb, A = nv ? con_arg_off[ce] - con_arg_off[cb] : 0;
    if (A < 0) return -1;
    // var of string id sid, -1 if not a variable of this problem, -2 if out of range
    auto var = [&](int64_t sid) -> int32_t {
      if ((uint64_t)sid >= nstr) return -2;
      const uint64_t e = fst[(size_t)sid];
      return (e & ~0xffffffffULL) == stamp ? (int32_t)(uint32_t)e : -1;
    };
    Fast& F = W.fast;
    F.reset((size_t)nv, (size_t)C, (size_t)A);
    W.fkey.reset();
    // the record's counters and arrays in locals: stores through the int32
    // arrays could alias F's int32 counters, which would then be reloaded
    // and stored around every element
    int32_t nc = 0, ncl = 0, nk = 0, nkl = 0, nch = 0, nchl = 0, na = 0, nid = 0;
    bool src_ok = true;
    int32_t* const clause_off = F.clause_off;
    int32_t* const clause_lits = F.clause_lits;
    int32_t* const clause_id = F.clause_id;
    int32_t* const card_off = F.card_off;
    int32_t* const card_lits = F.card_lits;
    int32_t* const card_bound = F.card_bound;
    int32_t* const card_id = F.card_id;
    int32_t* const var_choice_off = F.var_choice_off;
    int32_t* const choice_off = F.choice_off;
    int32_t* const choice_lits = F.choice_lits;
    int32_t* const anchors = F.anchors;
    int32_t* const owner_v = F.owner_v;
    int32_t* const owner_c = F.owner_c;
    int32_t* const first_s = F.first_s;
    int32_t* const list_id = F.list_id;
    int64_t* const first_c = F.first_c;
    uint8_t* const src = F.src;
    auto close_clause = [&](int32_t id) {
      clause_id[nc] = id;
      clause_off[++nc] = ncl;
    };
    for (int vi = 0; vi < nv; ++vi) {
      const int64_t c0 = var_con_off[v0 + vi], c1 = var_con_off[v0 + vi + 1];
      bool anchor = false;
      for (int64_t c = c0; c < c1; ++c) {
        const int32_t kind = con_kind[c];
        const int64_t a0 = con_arg_off[c], a1 = con_arg_off[c + 1];
        if (a1 < a0) return -1;
        uint64_t key = 0;
        bool taut = false, hashed = false;
        int32_t* seq = F.seq;
        int32_t ns = 0;
        const int ci = (int)(c - c0);
        if (kind == DP_DEPENDENCY && a1 > a0) {
          seq = choice_lits + nchl;  // the arguments are the Order() list, search.go:59-69
          for (int64_t a = a0; a < a1; ++a) {
            const int32_t d = var(con_arg[a]);
            if (d < 0) return d == -2 ? -1 : 0;
            seq[ns++] = d;
          }
          const int32_t k = nch;  // this constraint's choice list
          nchl += ns;
          choice_off[++nch] = nchl;
          if (seq[0] == vi) {  // Or(!x_s, x_s) = T: a list without a row
            list_id[k] = -1;
            src_ok = false;
            continue;
          }
          // K_DEP: only a Dependency of the same subject over the same
          // candidate sequence builds the same Or chain, and a variable's
          // constraints are lowered together, so the term is known iff an
          // earlier list of this subject equals this one (its first
          // writer's: the earliest such list)
          int32_t k0 = var_choice_off[vi];
          for (; k0 < k; ++k0) {
            if (list_id[k0] < 0) continue;
            const int32_t b0 = choice_off[k0];
            if (choice_off[k0 + 1] - b0 == ns && std::equal(seq, seq + ns, choice_lits + b0)) break;
          }
          if (k0 < k) {
            const int32_t id = list_id[k0];
            list_id[k] = id;
            owner_v[id] = vi;  // last writer wins, lit_mapping.go:69-72
            owner_c[id] = ci;
            // a repeat of the list that took the row (choice_sources: the
            // nearest earlier list of the subject with this content and a row)
            if (k - k0 > 255) src_ok = false;
            else src[k] = (uint8_t)(k - k0);
            continue;
          }
          const int32_t id = nid++;
          list_id[k] = id;
          owner_v[id] = vi;
          owner_c[id] = ci;
          first_c[id] = c;
          first_s[id] = vi;
          // the row (!s, d1..dn), each candidate once; none when s recurs (T)
          const int32_t start = ncl;
          clause_lits[ncl++] = 2 * vi + 1;
          bool tautology = false;
          for (int32_t j = 0; j < ns; ++j) {
            const int32_t d = seq[j];
            if (d == vi) { tautology = true; break; }
            bool seen = false;
            for (int32_t q = start + 1; q < ncl; ++q) seen |= clause_lits[q] == 2 * d;
            if (!seen) clause_lits[ncl++] = 2 * d;
          }
          if (tautology) {
            ncl = start;
            src_ok = false;  // a list without a row
          } else {
            src_ok &= ncl - start == ns + 1;  // a repeated candidate: the row is shorter than the list
            close_clause(id);
          }
          src[k] = 0;
          continue;
        }
        switch (kind) {
          case DP_MANDATORY:
            if (a1 != a0) return -1;
            key = key1(K_POS, (uint32_t)vi);
            anchor = true;
            break;
          case DP_PROHIBITED:
            if (a1 != a0) return -1;
            key = key1(K_NEG, (uint32_t)vi);
            break;
          case DP_DEPENDENCY:  // without candidates: !x_s
            key = key1(K_NEG, (uint32_t)vi);
            break;
          case DP_CONFLICT: {
            if (a1 - a0 != 1) return -1;
            const int32_t t = var(con_arg[a0]);
            if (t < 0) return t == -2 ? -1 : 0;
            seq[ns++] = t;
            key = t == vi ? key1(K_NEG, (uint32_t)vi) : key2(K_CONF, (uint32_t)vi, (uint32_t)t);
            break;
          }
          case DP_ATMOST: {
            const int64_t N = a1 - a0;
            const int32_t n = con_n[c];
            for (int64_t a = a0; a < a1; ++a) {
              const int32_t d = var(con_arg[a]);
              if (d < 0) return d == -2 ? -1 : 0;
              seq[ns++] = d;
            }
            if (n < 0) { key = key1(K_F, 0); break; }
            if (n >= N) { taut = true; break; }
            int32_t* srt = F.seq2;
            // insertion sort (AtMost rows are short)
            for (int32_t j = 0; j < ns; ++j) {
              const int32_t x = seq[j];
              int32_t q = j;
              for (; q > 0 && srt[q - 1] > x; --q) srt[q] = srt[q - 1];
              srt[q] = x;
            }
            for (int32_t j = 1; j < ns; ++j)
              if (srt[j] == srt[j - 1]) return 0;  // multiplicity: exact path
            if (N == 1) key = key1(K_NEG, (uint32_t)seq[0]);
            else if (N == 2) key = key2(n == 0 ? K_NOR : K_CONF, (uint32_t)seq[0], (uint32_t)seq[1]);
            else {
              uint64_t h = hmix(0x63617264ULL, (uint64_t)n);
              for (int32_t j = 0; j < ns; ++j) h = hmix(h, (uint64_t)srt[j]);
              key = keyh(K_CARD, h);
              hashed = true;
            }
            break;
          }
          default:
            return -1;
        }
        if (taut) continue;
        int32_t* slot = W.fkey.find_or_insert(key, nid);
        if (*slot != nid) {  // a known term
          const int32_t id = *slot;
          if (hashed && !same_term(first_c, first_s, id, c, vi, seq, ns, var)) return 0;
          owner_v[id] = vi;  // last writer wins, lit_mapping.go:69-72
          owner_c[id] = ci;
          continue;
        }
        const int32_t id = nid++;
        owner_v[id] = vi;
        owner_c[id] = ci;
        first_c[id] = c;
        first_s[id] = vi;
        // the rows of a new identity, from its first writer (emit_rows)
        const uint64_t tg = key >> 60;
        if (tg == K_F) {
          close_clause(id);
        } else if (tg == K_POS || tg == K_NEG) {
          clause_lits[ncl++] = 2 * (int32_t)(key & 0x3fffffff) + (tg == K_NEG);
          close_clause(id);
        } else if (kind == DP_CONFLICT) {
          clause_lits[ncl++] = 2 * vi + 1;
          clause_lits[ncl++] = 2 * seq[0] + 1;
          close_clause(id);
        } else {  // AtMost over distinct variables
          std::copy(seq, seq + ns, card_lits + nkl);
          nkl += ns;
          card_off[++nk] = nkl;
          card_bound[nk - 1] = con_n[c];
          card_id[nk - 1] = id;
        }
      }
      var_choice_off[vi + 1] = nch;
      if (anchor) anchors[na++] = vi;
    }
    F.nc = nc; F.ncl = ncl; F.nk = nk; F.nkl = nkl; F.nch = nch; F.nchl = nchl; F.na = na; F.nid = nid;
    F.src_ok = src_ok;
    if (emit_p16d(F, O, nv)) return 1;
    const size_t base = O.nrec;
    emit_fast(F, O, nv);
    narrow_last(O, base, src_ok ? src : nullptr);
    return 1;
  }

  // The record of the fast path (the layout emit_record writes).
  static void emit_fast(const Fast& F, Out& O, int nv) {
    int32_t hdr[DP_H_SIZE] = {0};
    hdr[DP_H_MAGIC] = DP_REC_MAGIC;
    hdr[DP_H_NV] = nv;
    hdr[DP_H_NC] = F.nc;
    hdr[DP_H_NK] = F.nk;
    hdr[DP_H_NCH] = F.nch;
    hdr[DP_H_NA] = F.na;
    hdr[DP_H_NID] = F.nid;
    hdr[DP_H_NCL] = F.ncl;
    hdr[DP_H_NKL] = F.nkl;
    hdr[DP_H_NCHL] = F.nchl;
    const dp_rec_layout L = dp_rec_layout_of(hdr);
    hdr[DP_H_WORDS] = L.words;
    int32_t* r = O.extend((size_t)L.words);
    auto put = [&](int32_t at, const int32_t* src, int32_t n) { std::memcpy(r + at, src, (size_t)n * 4); };
    std::memcpy(r, hdr, sizeof hdr);
    put(L.clause_off, F.clause_off, F.nc + 1);
    put(L.clause_lits, F.clause_lits, F.ncl);
    put(L.clause_id, F.clause_id, F.nc);
    put(L.card_off, F.card_off, F.nk + 1);
    put(L.card_lits, F.card_lits, F.nkl);
    put(L.card_bound, F.card_bound, F.nk);
    put(L.card_id, F.card_id, F.nk);
    put(L.var_choice_off, F.var_choice_off, nv + 1);
    put(L.choice_off, F.choice_off, F.nch + 1);
    put(L.choice_lits, F.choice_lits, F.nchl);
    put(L.anchors, F.anchors, F.na);
    O.rec_len.push_back(L.words);
    O.ivar.insert(O.ivar.end(), F.owner_v, F.owner_v + F.nid);
    O.icon.insert(O.icon.end(), F.owner_c, F.owner_c + F.nid);
    O.ident_len.push_back(F.nid);
    O.err.push_back(DP_LOWER_OK);
    O.msg.emplace_back();
  }

  // Is the term of constraint c on subject s (a hashed key, its arguments
  // resolved in seq[0..ns)) the one of identity id's first writer?  Same
  // kind, subject and argument sequence (and bound) build the same term.
  template <class Var>
  bool same_term(const int64_t* first_c, const int32_t* first_s, int32_t id, int64_t c, int s, const int32_t* seq,
                 int32_t ns, const Var& var) const {
    const int64_t f = first_c[id];
    if (w.con_kind[f] != w.con_kind[c]) return false;
    if (w.con_kind[c] == DP_DEPENDENCY && first_s[id] != s) return false;
    if (w.con_kind[c] == DP_ATMOST && w.con_n[f] != w.con_n[c]) return false;
    const int64_t a0 = w.con_arg_off[f], a1 = w.con_arg_off[f + 1];
    if (a1 - a0 != (int64_t)ns) return false;
    for (int64_t a = a0; a < a1; ++a)
      if (var(w.con_arg[a]) != seq[a - a0]) return false;
    return true;
  }

  // CardSort(ms).Leq(n): the network is built before Leq reads it, whatever
  // n (gini's order, constraints.go:180-186), so an AtMost folded to a
  // constant still adds its gates to the graph (the nodes later networks
  // share and number after).
  static int32_t leq(Aig& aig, Work& W, int32_t n) {
    const int N = (int)W.ms.size();
    int p = 1;
    while (p < N) p <<= 1;
    W.sorted.assign(W.ms.begin(), W.ms.end());
    W.sorted.resize((size_t)p, kF);
    for (auto& pr : batcher(p)) {
      int32_t a = W.sorted[(size_t)pr.first], b = W.sorted[(size_t)pr.second];
      int32_t hi = aig.Or(a, b), lo = aig.And(a, b);
      W.sorted[(size_t)pr.first] = hi;
      W.sorted[(size_t)pr.second] = lo;
    }
    if (n < 0) return kF;
    if (n >= N) return kT;
    return W.sorted[(size_t)n] ^ 1;
  }

  // Rows of a new identity, from the semantics of its first writer.
  void emit_rows(Work& W, int32_t m, int nv, int32_t kind, int s, int32_t n, int64_t a0,
                 int64_t a1, int32_t ident) const {
    auto close_clause = [&]() {
      W.clause_off.push_back((int32_t)W.clause_lits.size());
      W.clause_id.push_back(ident);
    };
    if (m == kF) { close_clause(); return; }  // empty clause: always conflicting
    int32_t node = m >> 1;
    if (node >= 1 && node <= nv) {  // an input literal: unit clause
      W.clause_lits.push_back(2 * (node - 1) + (m & 1));
      close_clause();
      return;
    }
    auto var_of = [&](int64_t a) -> int32_t {
      int64_t sid = w.con_arg[a];
      if (w.interned) return W.st_idx[(size_t)sid];
      return W.names.find(str(sid))->second;
    };
    if (kind == DP_DEPENDENCY) {
      size_t start = W.clause_lits.size();
      W.clause_lits.push_back(2 * s + 1);
      for (int64_t a = a0; a < a1; ++a) {
        int32_t l = 2 * var_of(a);
        if (l == 2 * s) { W.clause_lits.resize(start); return; }  // tautology: no row
        bool seen = false;
        for (size_t j = start; j < W.clause_lits.size(); ++j) seen |= W.clause_lits[j] == l;
        if (!seen) W.clause_lits.push_back(l);
      }
      close_clause();
    } else if (kind == DP_CONFLICT) {
      W.clause_lits.push_back(2 * s + 1);
      W.clause_lits.push_back(2 * var_of(a0) + 1);
      close_clause();
    } else if (kind == DP_ATMOST) {
      W.order.clear(); W.mult.clear();
      for (int64_t a = a0; a < a1; ++a) {
        int32_t v = var_of(a);
        size_t j = 0;
        while (j < W.order.size() && W.order[j] != v) ++j;
        if (j == W.order.size()) { W.order.push_back(v); W.mult.push_back(0); }
        W.mult[j]++;
      }
      if ((int64_t)W.order.size() < a1 - a0) {  // a variable listed more than once
        network_rows(W, m, nv, ident);
        return;
      }
      for (size_t j = 0; j < W.order.size(); ++j)
        for (int t = 0; t < W.mult[j]; ++t) W.card_lits.push_back(W.order[j]);
      W.card_off.push_back((int32_t)W.card_lits.size());
      W.card_bound.push_back(n);
      W.card_id.push_back(ident);
    }
  }

  static void emit_error(Out& O, int32_t code, const std::string& msg) {
    // an nv = 0 record: header + the four one-entry offset arrays
    int32_t hdr[DP_H_SIZE + 4] = {0};
    hdr[DP_H_MAGIC] = DP_REC_MAGIC;
    hdr[DP_H_WORDS] = dp_rec_layout_of(hdr).words;
    std::memcpy(O.extend((size_t)hdr[DP_H_WORDS]), hdr, 4 * (size_t)hdr[DP_H_WORDS]);
    O.rec_len.push_back(hdr[DP_H_WORDS]);
    O.ident_len.push_back(0);
    O.err.push_back(code);
    O.msg.push_back(msg);
  }

  // AtMost(n; ids) listing a variable more than once: the rows of gini's own
  // encoding, CardSort(ms).Leq(n) (constraints.go:180-186), because unit
  // propagation over a counting row is strictly stronger there (DESIGN.md
  // §3.1).  Every And gate in the cone of m becomes an auxiliary variable
  // (after the input's variables, in ascending node order) with its three
  // Tseitin rows (~g a) (~g b) (g ~a ~b); then the unit row (m).  Every row
  // carries the AtMost's identity (oracle/lower_ref.py _network_rows).
  static void network_rows(Work& W, int32_t m, int nv, int32_t ident) {
    const Aig& aig = W.aig;
    const int32_t first = nv + 1;  // the first gate's node
    W.vis.assign((size_t)(aig.next_node - first), 0);
    W.cone.clear();
    W.walk.assign(1, m >> 1);
    while (!W.walk.empty()) {
      const int32_t node = W.walk.back();
      W.walk.pop_back();
      if (node < first || W.vis[(size_t)(node - first)]) continue;
      W.vis[(size_t)(node - first)] = 1;
      W.cone.push_back(node);
      const uint64_t key = aig.fanin[(size_t)(node - first)];
      W.walk.push_back((int32_t)(key >> 32) >> 1);
      W.walk.push_back((int32_t)(uint32_t)key >> 1);
    }
    std::sort(W.cone.begin(), W.cone.end());
    const int32_t base = W.naux;
    W.naux += (int32_t)W.cone.size();
    auto lit = [&](int32_t x) -> int32_t {  // AIG literal -> record literal
      const int32_t node = x >> 1;
      const int32_t v = node < first ? node - 1
                                     : base + (int32_t)(std::lower_bound(W.cone.begin(), W.cone.end(), node) -
                                                        W.cone.begin());
      return 2 * v + (x & 1);
    };
    auto row = [&](std::initializer_list<int32_t> ls) {
      for (int32_t l : ls) W.clause_lits.push_back(l);
      W.clause_off.push_back((int32_t)W.clause_lits.size());
      W.clause_id.push_back(ident);
    };
    for (const int32_t node : W.cone) {
      const uint64_t key = aig.fanin[(size_t)(node - first)];
      const int32_t g = lit(2 * node), a = lit((int32_t)(key >> 32)), b = lit((int32_t)(uint32_t)key);
      row({g ^ 1, a});
      row({g ^ 1, b});
      row({g, a ^ 1, b ^ 1});
    }
    row({lit(m)});
  }

  static void emit_record(Work& W, Out& O, int nv, int nvu = 0) {
    const int32_t nc = (int32_t)W.clause_id.size(), nk = (int32_t)W.card_id.size();
    const int32_t nch = (int32_t)W.choice_off.size() - 1;
    int32_t hdr[DP_H_SIZE] = {0};
    hdr[DP_H_MAGIC] = DP_REC_MAGIC;
    hdr[DP_H_NV] = nv;
    hdr[DP_H_NC] = nc;
    hdr[DP_H_NK] = nk;
    hdr[DP_H_NCH] = nch;
    hdr[DP_H_NA] = (int32_t)W.anchors.size();
    hdr[DP_H_NID] = (int32_t)W.owner_v.size();
    hdr[DP_H_NCL] = (int32_t)W.clause_lits.size();
    hdr[DP_H_NKL] = (int32_t)W.card_lits.size();
    hdr[DP_H_NCHL] = (int32_t)W.choice_lits.size();
    hdr[DP_H_NVU] = nvu;
    dp_rec_layout L = dp_rec_layout_of(hdr);
    hdr[DP_H_WORDS] = L.words;
    size_t base = O.nrec;
    std::memcpy(O.extend(DP_H_SIZE), hdr, 4 * DP_H_SIZE);
    auto app = [&](const std::vector<int32_t>& v) {
      if (!v.empty()) std::memcpy(O.extend(v.size()), v.data(), 4 * v.size());
    };
    app(W.clause_off); app(W.clause_lits); app(W.clause_id);
    app(W.card_off); app(W.card_lits); app(W.card_bound); app(W.card_id);
    app(W.var_choice_off); app(W.choice_off); app(W.choice_lits); app(W.anchors);
    O.rec_len.push_back((int64_t)(O.nrec - base));
    O.ivar.insert(O.ivar.end(), W.owner_v.begin(), W.owner_v.end());
    O.icon.insert(O.icon.end(), W.owner_c.begin(), W.owner_c.end());
    O.ident_len.push_back((int64_t)W.owner_v.size());
    O.err.push_back(DP_LOWER_OK);
    O.msg.emplace_back();
  }
};

}  // namespace
}  // namespace dp

// The records (and identity arrays) of a dp_lowered: grown, never shrunk,
// contents not preserved across a resize (every call rewrites them);
// page-locked when asked and a HIP device is present (dp_submit then copies
// the records to the device as they are, and dp_lower_device copies into
// them by DMA), else ordinary 64-byte aligned memory.
template <class T>
struct HostStore {
  T* p = nullptr;
  size_t n = 0, cap = 0;
  bool pinned = false;
  void resize(size_t m, bool want_pinned) {
    if (m > cap || want_pinned != pinned) {
      release();
      const size_t c = std::max<size_t>(m + m / 8, 1024);
      void* q = want_pinned ? dp::pinned_alloc(sizeof(T) * c) : nullptr;
      pinned = q != nullptr;
      if (!q) q = std::aligned_alloc(64, (sizeof(T) * c + 63) & ~(size_t)63);
      if (!q) throw std::bad_alloc();
      p = static_cast<T*>(q);
      cap = c;
    }
    n = m;
  }
  T* data() { return p; }
  const T* data() const { return p; }
  size_t size() const { return n; }
  T* begin() { return p; }
  void release() {
    if (p) pinned ? dp::pinned_free(p) : std::free(p);
    p = nullptr;
    cap = n = 0;
    pinned = false;
  }
  void swap(HostStore& o) {
    std::swap(p, o.p);
    std::swap(n, o.n);
    std::swap(cap, o.cap);
    std::swap(pinned, o.pinned);
  }
  ~HostStore() { release(); }
};
using RecStore = HostStore<int32_t>;

struct dp_lowered {
  int32_t n = 0;
  std::vector<int64_t> rec_off, ident_off;
  RecStore rec;
  HostStore<int32_t> ivar, icon;
  std::vector<int32_t> err;
  std::vector<std::string> msg;
  // scratch kept across dp_lower_into calls (once grown, no allocation or
  // page fault per call): per pool thread, and chunk c's slices of outs[t]
  std::vector<dp::Work> work;
  std::vector<dp::Out> outs;
  struct Piece {
    int t;
    size_t r0, r1, i0, i1, q0, q1;
  };
  std::vector<Piece> pieces;
  std::vector<size_t> at_rec, at_id, at_p;
  std::atomic<int64_t> n_exact{0};  // problems the last call lowered through the full AIG
  // dp_lower_device's problems lowered on the host (dp::lowered_splice):
  // their own result, and the spliced arrays before they are swapped in
  std::unique_ptr<dp_lowered> sub;
  RecStore rec2;
  HostStore<int32_t> ivar2, icon2;
  std::vector<int64_t> ro2, io2;
  std::vector<int32_t> src2;
};

extern "C" {

const char* dp_last_global_error(void) { return dp::g_err.c_str(); }

// The batch-level shape of a wire batch (serial, O(problems)); each problem's
// own arrays are checked by problem_ok on the lowering threads.  The offsets
// are absolute: a batch may be a problem range of a larger one's arrays
// (prob_var_off pointing into its offsets; include/deppy_hip.h dp_wire).
static bool wire_ok(const dp_wire* w) {
  if (!w || w->n_problems < 0 || !w->prob_var_off) return false;
  if (w->n_problems == 0) return true;
  const int64_t v0 = w->prob_var_off[0], nvars = w->prob_var_off[w->n_problems];
  if (v0 < 0) return false;
  for (int32_t p = 0; p < w->n_problems; ++p)
    if (w->prob_var_off[p + 1] < w->prob_var_off[p]) return false;
  if (nvars > v0 && (!w->var_id || !w->var_con_off || w->var_con_off[v0] < 0)) return false;
  if (nvars > v0 && w->var_con_off[nvars] > w->var_con_off[v0] &&
      (!w->con_kind || !w->con_arg_off || w->con_arg_off[w->var_con_off[v0]] < 0))
    return false;
  return true;
}

// Problem p's variables, constraints and arguments are well formed.
static bool problem_ok(const dp_wire* w, int32_t p) {
  const int64_t v0 = w->prob_var_off[p], v1 = w->prob_var_off[p + 1];
  for (int64_t v = v0; v < v1; ++v) {
    if (w->var_con_off[v + 1] < w->var_con_off[v]) return false;
    if (w->var_id[v] < 0 || w->var_id[v] >= w->n_strs) return false;
  }
  if (v1 == v0) return true;
  for (int64_t c = w->var_con_off[v0]; c < w->var_con_off[v1]; ++c) {
    int32_t k = w->con_kind[c];
    if (k < DP_MANDATORY || k > DP_ATMOST) return false;
    int64_t na = w->con_arg_off[c + 1] - w->con_arg_off[c];
    if (na < 0) return false;
    if (k == DP_CONFLICT && na != 1) return false;
    if ((k == DP_MANDATORY || k == DP_PROHIBITED) && na != 0) return false;
    for (int64_t a = w->con_arg_off[c]; a < w->con_arg_off[c + 1]; ++a)
      if (w->con_arg[a] < 0 || w->con_arg[a] >= w->n_strs) return false;
  }
  return true;
}

int dp_lower(const dp_wire* wire, dp_lowered** out) {
  if (!out) return -1;
  auto* lw = new dp_lowered;
  if (dp_lower_into(wire, 0, lw) != 0) {
    delete lw;
    return -1;
  }
  *out = lw;
  return 0;
}

int dp_lower_into(const dp_wire* wire, int32_t flags, dp_lowered* lw) {
  if (!lw || !wire_ok(wire)) {
    dp::set_global_error("dp_lower: malformed wire batch");
    return -1;
  }
  const int32_t P = wire->n_problems;
  // DEPPY_LOWER_EXACT=1: every problem through the full AIG (tests, A/B)
  const char* ex = std::getenv("DEPPY_LOWER_EXACT");
  const bool exact = ex && *ex && *ex != '0';
  dp::Pool& pool = dp::host_pool();
  int nt = pool.size();
  // threads by work (constraint arguments), chunks small enough to balance
  const int64_t work = P ? wire->con_arg_off[wire->var_con_off[wire->prob_var_off[P]]] -
                               wire->con_arg_off[wire->var_con_off[wire->prob_var_off[0]]]
                         : 0;
  if (work < 200000) nt = 1;
  const int32_t chunk = (int32_t)std::max<int64_t>(1, std::min<int64_t>(64, P / (8 * (int64_t)nt)));
  const int32_t nchunks = (P + chunk - 1) / chunk;
  if ((int)lw->work.size() < pool.size()) {
    lw->work.resize((size_t)pool.size());
    lw->outs.resize((size_t)pool.size());
  }
  for (auto& W : lw->work) {
    ++W.gen;
    if (wire->interned && W.st_tag.size() < (size_t)wire->n_strs) {
      W.st_tag.resize((size_t)wire->n_strs, 0);
      W.st_idx.resize((size_t)wire->n_strs, 0);
      W.fst.resize((size_t)wire->n_strs, 0);
    }
  }
  for (auto& O : lw->outs) {
    O.nrec = 0; O.rec_len.clear(); O.ivar.clear(); O.icon.clear();
    O.ident_len.clear(); O.err.clear(); O.msg.clear();
  }
  lw->pieces.resize((size_t)nchunks);
  lw->n_exact.store(0);
  const char* hw = std::getenv("DEPPY_HOST_WATCHES");
  dp::Lowerer L(*wire, (flags & DP_LOWER_NARROW) != 0,
                (flags & (DP_LOWER_NARROW | DP_LOWER_PACKED)) == (DP_LOWER_NARROW | DP_LOWER_PACKED),
                hw && *hw && *hw != '0', (flags & DP_LOWER_NO_P8) == 0);
  std::atomic<bool> bad{false};
  auto lower_chunk = [&](int64_t c, int t) {
    dp::Work& W = lw->work[(size_t)t];
    dp::Out& O = lw->outs[(size_t)t];
    auto& pc = lw->pieces[(size_t)c];
    pc.t = t;
    pc.r0 = O.nrec; pc.i0 = O.ivar.size(); pc.q0 = O.rec_len.size();
    for (int32_t p = (int32_t)c * chunk; p < std::min<int32_t>(P, ((int32_t)c + 1) * chunk); ++p)
    {
      const int r = exact ? 0 : L.lower_fast(p, W, O);
      if (r < 0 || (r == 0 && !problem_ok(wire, p))) {
        bad.store(true, std::memory_order_relaxed);
        return;
      }
      if (r == 0) {
        L.lower_one(p, W, O);
        lw->n_exact.fetch_add(1, std::memory_order_relaxed);
      }
    }
    pc.r1 = O.nrec; pc.i1 = O.ivar.size(); pc.q1 = O.rec_len.size();
  };
  if (nt == 1)
    for (int32_t c = 0; c < nchunks; ++c) lower_chunk(c, 0);
  else
    pool.run(nchunks, lower_chunk, 1);
  if (bad.load()) {
    lw->n = 0;
    lw->rec_off.assign(1, 0);
    lw->ident_off.assign(1, 0);
    dp::set_global_error("dp_lower: malformed wire batch");
    return -1;
  }
  // pieces -> one batch: offsets serially, the copies in parallel
  lw->n = P;
  auto& ar = lw->at_rec;
  auto& ai = lw->at_id;
  auto& ap = lw->at_p;
  ar.assign((size_t)nchunks + 1, 0); ai.assign((size_t)nchunks + 1, 0); ap.assign((size_t)nchunks + 1, 0);
  for (int32_t c = 0; c < nchunks; ++c) {
    const auto& pc = lw->pieces[(size_t)c];
    ar[(size_t)c + 1] = ar[(size_t)c] + (pc.r1 - pc.r0);
    ai[(size_t)c + 1] = ai[(size_t)c] + (pc.i1 - pc.i0);
    ap[(size_t)c + 1] = ap[(size_t)c] + (pc.q1 - pc.q0);
  }
  lw->rec.resize(ar.back(), (flags & DP_LOWER_PINNED) != 0);
  lw->ivar.resize(ai.back(), (flags & DP_LOWER_PINNED) != 0);
  lw->icon.resize(ai.back(), (flags & DP_LOWER_PINNED) != 0);
  lw->rec_off.resize((size_t)P + 1);
  lw->ident_off.resize((size_t)P + 1);
  lw->err.resize((size_t)P);
  lw->msg.resize((size_t)P);
  lw->rec_off[0] = lw->ident_off[0] = 0;
  auto merge = [&](int64_t c) {
    const auto& pc = lw->pieces[(size_t)c];
    dp::Out& o = lw->outs[(size_t)pc.t];
    std::copy(o.rec.begin() + (int64_t)pc.r0, o.rec.begin() + (int64_t)pc.r1, lw->rec.p + ar[(size_t)c]);
    std::copy(o.ivar.begin() + (int64_t)pc.i0, o.ivar.begin() + (int64_t)pc.i1, lw->ivar.begin() + (int64_t)ai[(size_t)c]);
    std::copy(o.icon.begin() + (int64_t)pc.i0, o.icon.begin() + (int64_t)pc.i1, lw->icon.begin() + (int64_t)ai[(size_t)c]);
    int64_t r = (int64_t)ar[(size_t)c], d = (int64_t)ai[(size_t)c];
    for (size_t q = pc.q0; q < pc.q1; ++q) {
      const size_t p = ap[(size_t)c] + (q - pc.q0);
      r += o.rec_len[q];
      d += o.ident_len[q];
      lw->rec_off[p + 1] = r;
      lw->ident_off[p + 1] = d;
      lw->err[p] = o.err[q];
      if (o.err[q]) lw->msg[p] = std::move(o.msg[q]);
      else if (!lw->msg[p].empty()) lw->msg[p].clear();
    }
  };
  if (nt == 1)
    for (int32_t c = 0; c < nchunks; ++c) merge(c);
  else
    pool.run(nchunks, std::function<void(int64_t)>(merge), 1);
  return 0;
}

}  // extern "C"

namespace dp {

// dp_lower_device's hand-over (lower_device.hip): lw sized for P problems,
// rec_words record words and n_ident identities, every problem without an
// error; the caller fills the arrays.
LoweredOut lowered_prepare(dp_lowered* lw, int32_t P, int64_t rec_words, int64_t n_ident, bool pinned) {
  lw->n = P;
  lw->n_exact.store(0);
  lw->rec.resize((size_t)rec_words, pinned);
  lw->ivar.resize((size_t)n_ident, pinned);
  lw->icon.resize((size_t)n_ident, pinned);
  lw->rec_off.resize((size_t)P + 1);
  lw->ident_off.resize((size_t)P + 1);
  lw->err.assign((size_t)P, DP_LOWER_OK);
  if (lw->msg.size() != (size_t)P) lw->msg.resize((size_t)P);
  for (auto& m : lw->msg)
    if (!m.empty()) m.clear();
  return {lw->rec_off.data(), lw->ident_off.data(), lw->rec.data(), lw->ivar.data(), lw->icon.data()};
}

// The problems `which` (ascending; lw gives them no record words and no
// identities) lowered on the host from `sub` (exactly those problems, in
// that order) and spliced into lw: records, identities and errors, as
// dp_lower_into gives them.  Returns 0, or -1 for a malformed problem.
int lowered_splice(dp_lowered* lw, const dp_wire* sub, int32_t flags, const int32_t* which, int32_t nw) {
  if (!lw->sub) lw->sub.reset(new dp_lowered);
  dp_lowered& t = *lw->sub;
  if (dp_lower_into(sub, flags & ~DP_LOWER_PINNED, &t) != 0) return -1;
  lw->n_exact.store(t.n_exact.load());
  const int32_t P = lw->n;
  const bool pinned = lw->rec.pinned;
  // the new offsets (serial, O(P)), then the copies on the host pool
  std::vector<int64_t>& ro = lw->rec_off;
  std::vector<int64_t>& io = lw->ident_off;
  std::vector<int64_t>& nro = lw->ro2;
  std::vector<int64_t>& nio = lw->io2;
  std::vector<int32_t>& src = lw->src2;  // problem -> its index in `which`, or -1
  nro.resize((size_t)P + 1);
  nio.resize((size_t)P + 1);
  src.assign((size_t)P, -1);
  nro[0] = nio[0] = 0;
  for (int32_t j = 0; j < nw; ++j) src[(size_t)which[j]] = j;
  for (int32_t p = 0; p < P; ++p) {
    const int32_t j = src[(size_t)p];
    nro[(size_t)p + 1] = nro[(size_t)p] + (j >= 0 ? t.rec_off[(size_t)j + 1] - t.rec_off[(size_t)j]
                                                    : ro[(size_t)p + 1] - ro[(size_t)p]);
    nio[(size_t)p + 1] = nio[(size_t)p] + (j >= 0 ? t.ident_off[(size_t)j + 1] - t.ident_off[(size_t)j]
                                                    : io[(size_t)p + 1] - io[(size_t)p]);
  }
  lw->rec2.resize((size_t)nro[(size_t)P], pinned);
  lw->ivar2.resize((size_t)nio[(size_t)P], pinned);
  lw->icon2.resize((size_t)nio[(size_t)P], pinned);
  dp::host_pool().run(P, std::function<void(int64_t)>([&](int64_t p) {
    const int32_t j = src[(size_t)p];
    const int32_t* r = j >= 0 ? t.rec.p + t.rec_off[(size_t)j] : lw->rec.p + ro[(size_t)p];
    const int32_t* iv = j >= 0 ? t.ivar.p + t.ident_off[(size_t)j] : lw->ivar.p + io[(size_t)p];
    const int32_t* ic = j >= 0 ? t.icon.p + t.ident_off[(size_t)j] : lw->icon.p + io[(size_t)p];
    std::copy(r, r + (nro[(size_t)p + 1] - nro[(size_t)p]), lw->rec2.p + nro[(size_t)p]);
    std::copy(iv, iv + (nio[(size_t)p + 1] - nio[(size_t)p]), lw->ivar2.p + nio[(size_t)p]);
    std::copy(ic, ic + (nio[(size_t)p + 1] - nio[(size_t)p]), lw->icon2.p + nio[(size_t)p]);
  }), 256);
  for (int32_t j = 0; j < nw; ++j) {
    lw->err[(size_t)which[j]] = t.err[(size_t)j];
    lw->msg[(size_t)which[j]] = t.msg[(size_t)j];
  }
  ro.swap(nro);
  io.swap(nio);
  lw->rec.swap(lw->rec2);
  lw->ivar.swap(lw->ivar2);
  lw->icon.swap(lw->icon2);
  return 0;
}

}  // namespace dp

extern "C" {

void dp_lowered_free(dp_lowered* lw) { delete lw; }
dp_lowered* dp_lowered_new(void) { return new dp_lowered; }
int32_t dp_lowered_num_problems(const dp_lowered* lw) { return lw->n; }
int64_t dp_lowered_exact_count(const dp_lowered* lw) { return lw->n_exact.load(); }
const int64_t* dp_lowered_rec_off(const dp_lowered* lw) { return lw->rec_off.data(); }
const int32_t* dp_lowered_rec(const dp_lowered* lw) { return lw->rec.p; }
int32_t dp_lowered_pinned(const dp_lowered* lw) { return lw->rec.pinned ? 1 : 0; }
const int64_t* dp_lowered_ident_off(const dp_lowered* lw) { return lw->ident_off.data(); }
const int32_t* dp_lowered_ident_var(const dp_lowered* lw) { return lw->ivar.data(); }
const int32_t* dp_lowered_ident_con(const dp_lowered* lw) { return lw->icon.data(); }
int32_t dp_lowered_error(const dp_lowered* lw, int32_t p, const char** msg) {
  if (p < 0 || p >= lw->n) return -1;
  if (msg) *msg = lw->msg[(size_t)p].c_str();
  return lw->err[(size_t)p];
}

int32_t dp_lowered_errors(const dp_lowered* lw, int32_t* err) {
  int32_t bad = 0;
  for (int32_t p = 0; p < lw->n; ++p) {
    err[p] = lw->err[(size_t)p];
    bad += err[p] != DP_LOWER_OK;
  }
  return bad;
}

int dp_rec_widen(const int32_t* rec, int64_t avail, int32_t* out) {
  if (!rec || !out || avail < DP_H_SIZE) return -1;
  if (rec[DP_H_MAGIC] != DP_REC_MAGIC) return -2;
  for (int i = DP_H_NV; i <= DP_H_NCHL; ++i)
    if (rec[i] < 0 || rec[i] > (1 << 28)) return -3;
  const int32_t fmt = rec[DP_H_FMT];
  if (fmt != DP_FMT_I32 && fmt != DP_FMT_U16 && !dp_fmt_packed(fmt) && fmt != DP_FMT_I32W) return -16;
  const dp_rec_layout L = dp_rec_layout_of(rec);
  if (L.words != rec[DP_H_WORDS] || ((fmt == DP_FMT_U16 || dp_fmt_packed(fmt)) && !dp_rec_fits16(rec))) return -4;
  if (dp_fmt_packed(fmt) && dp_p16_tail_bytes(rec) > DP_P16_TAIL_MAX) return -17;
  if (fmt == DP_FMT_P8D) {  // its DP_FMT_P16D record, then that one's int32 form
    static thread_local std::vector<int32_t> p16;
    const int e = dp::p8_to_p16d(rec, avail, p16);
    return e ? e : dp_rec_widen(p16.data(), (int64_t)p16.size(), out);
  }
  if (dp_rec_phys_words(rec) > avail) return -4;
  const int64_t words = rec[DP_H_WORDS];
  std::memcpy(out, rec, 4 * DP_H_SIZE);
  out[DP_H_FMT] = DP_FMT_I32;
  if (fmt == DP_FMT_I32 || fmt == DP_FMT_I32W) {
    std::memcpy(out + DP_H_SIZE, rec + DP_H_SIZE, 4 * (size_t)(words - DP_H_SIZE));
  } else if (fmt == DP_FMT_U16) {
    const uint16_t* u = reinterpret_cast<const uint16_t*>(rec + DP_H_SIZE);
    for (int64_t j = DP_H_SIZE; j < words; ++j) out[j] = u[j - DP_H_SIZE];
  } else {
    const uint16_t* u = reinterpret_cast<const uint16_t*>(rec + DP_H_SIZE);
    auto get16 = [&](int32_t off, int32_t n) {
      for (int32_t j = 0; j < n; ++j) out[off + j] = *u++;
    };
    get16(L.clause_lits, rec[DP_H_NCL]);
    get16(L.card_lits, rec[DP_H_NKL]);
    get16(L.card_bound, rec[DP_H_NK]);
    if (fmt == DP_FMT_P16) get16(L.choice_lits, rec[DP_H_NCHL]);
    get16(L.anchors, rec[DP_H_NA]);
    const uint8_t* t = reinterpret_cast<const uint8_t*>(rec + DP_H_SIZE) + dp_p16_tail_at(rec);
    auto get_lens = [&](int32_t off, int32_t n) {
      out[off] = 0;
      for (int32_t j = 0; j < n; ++j) out[off + j + 1] = out[off + j] + *t++;
    };
    get_lens(L.clause_off, rec[DP_H_NC]);
    get_lens(L.card_off, rec[DP_H_NK]);
    const uint8_t* srcs = t;
    if (fmt == DP_FMT_P16) {
      get_lens(L.var_choice_off, rec[DP_H_NV]);
      get_lens(L.choice_off, rec[DP_H_NCH]);
    } else {
      t += rec[DP_H_NCH];  // the lists' sources; the lists follow the identities
    }
    int32_t c0 = 0, c1 = 0;
    const int32_t nc = rec[DP_H_NC], nk = rec[DP_H_NK];
    for (int32_t i = 0; i < rec[DP_H_NID]; ++i) {
      if ((t[i >> 3] >> (i & 7)) & 1) {
        if (c1 == nk) return -18;
        out[L.card_id + c1++] = i;
      } else {
        if (c0 == nc) return -18;
        out[L.clause_id + c0++] = i;
      }
    }
    if (c0 != nc || c1 != nk) return -18;
    // DP_FMT_P16D: the lists from the rows (the clause literals are not
    // range-checked yet: implied_choices checks every index it derives)
    if (fmt == DP_FMT_P16D &&
        (out[L.clause_off + nc] != rec[DP_H_NCL] ||
         !dp::implied_choices(out + L.clause_off, out + L.clause_lits, nc, rec[DP_H_NV], rec[DP_H_NCH], rec[DP_H_NCHL],
                              srcs, out + L.var_choice_off, out + L.choice_off, out + L.choice_lits)))
      return -20;
  }
  return 0;
}

int dp_rec_validate(const int32_t* rec, int64_t words) {
  if (!rec || words < DP_H_SIZE) return -1;
  if (rec[DP_H_MAGIC] != DP_REC_MAGIC) return -2;
  if (rec[DP_H_FMT] == DP_FMT_I32W) {  // the watch lists' bounds, then the record's checks
    for (int i = DP_H_NV; i <= DP_H_NCHL; ++i)
      if (rec[i] < 0 || rec[i] > (1 << 28)) return -3;
    if (dp_rec_layout_of(rec).words != rec[DP_H_WORDS] || dp_rec_phys_words(rec) > words) return -4;
    const int64_t n2 = 2 * (int64_t)rec[DP_H_NV], cap = (int64_t)rec[DP_H_NCL] + rec[DP_H_NKL];
    const int32_t* wo = rec + rec[DP_H_WORDS];
    const int32_t* w = wo + n2 + 1;
    if (wo[0] != 0 || wo[n2] > cap) return -19;
    for (int64_t l = 0; l < n2; ++l)
      if (wo[l + 1] < wo[l]) return -19;
    const int64_t nrows = (int64_t)rec[DP_H_NC] + rec[DP_H_NK];
    for (int64_t j = 0; j < wo[n2]; ++j)
      if (w[j] < 0 || w[j] >= nrows) return -19;
    std::vector<int32_t> t(rec, rec + rec[DP_H_WORDS]);
    t[DP_H_FMT] = DP_FMT_I32;
    return dp_rec_validate(t.data(), (int64_t)t.size());
  }
  if (rec[DP_H_FMT] == DP_FMT_U16 || dp_fmt_packed(rec[DP_H_FMT])) {  // widen, then the int32 checks
    for (int i = DP_H_NV; i <= DP_H_NCHL; ++i)
      if (rec[i] < 0 || rec[i] > (1 << 28)) return -3;
    std::vector<int32_t> w((size_t)std::max<int32_t>(rec[DP_H_WORDS], DP_H_SIZE));
    const int e = dp_rec_widen(rec, words, w.data());
    if (e) return e;
    return dp_rec_validate(w.data(), (int64_t)w.size());
  }
  if (rec[DP_H_FMT] != DP_FMT_I32) return -16;
  for (int i = DP_H_NV; i <= DP_H_NCHL; ++i)
    if (rec[i] < 0) return -3;
  dp_rec_layout L = dp_rec_layout_of(rec);
  if (L.words != rec[DP_H_WORDS] || L.words > words) return -4;
  const int32_t nv = rec[DP_H_NV], nc = rec[DP_H_NC], nk = rec[DP_H_NK], nch = rec[DP_H_NCH];
  const int32_t nid = rec[DP_H_NID];
  if (rec[DP_H_NVU] < 0 || rec[DP_H_NVU] > nv) return -21;
  std::vector<int32_t> run_starts;
  auto mono = [&](int32_t off, int32_t n, int32_t total) {
    if (rec[off] != 0 || rec[off + n] != total) return false;
    for (int32_t i = 0; i < n; ++i)
      if (rec[off + i + 1] < rec[off + i]) return false;
    return true;
  };
  if (!mono(L.clause_off, nc, rec[DP_H_NCL])) return -5;
  if (!mono(L.card_off, nk, rec[DP_H_NKL])) return -6;
  if (!mono(L.var_choice_off, nv, nch)) return -7;
  if (!mono(L.choice_off, nch, rec[DP_H_NCHL])) return -8;
  for (int32_t j = 0; j < rec[DP_H_NCL]; ++j)
    if (rec[L.clause_lits + j] < 0 || rec[L.clause_lits + j] >= 2 * nv) return -9;
  for (int32_t r = 0; r < nc; ++r)
    if (rec[L.clause_id + r] < 0 || rec[L.clause_id + r] >= nid) return -10;
  for (int32_t k = 0; k < nk; ++k) {
    if (rec[L.card_id + k] < 0 || rec[L.card_id + k] >= nid) return -10;
    if (rec[L.card_bound + k] < 0) return -15;  // (lowering folds AtMost(n<0) into an empty clause)
    // duplicates of a variable must be consecutive (one run per variable):
    // the run starts of a row are distinct
    const int32_t a = rec[L.card_off + k], b = rec[L.card_off + k + 1];
    for (int32_t j = a; j < b; ++j) {
      int32_t v = rec[L.card_lits + j];
      if (v < 0 || v >= nv) return -11;
    }
    run_starts.clear();
    for (int32_t j = a; j < b; ++j)
      if (j == a || rec[L.card_lits + j - 1] != rec[L.card_lits + j]) run_starts.push_back(rec[L.card_lits + j]);
    std::sort(run_starts.begin(), run_starts.end());
    if (std::adjacent_find(run_starts.begin(), run_starts.end()) != run_starts.end()) return -12;
  }
  for (int32_t j = 0; j < rec[DP_H_NCHL]; ++j)
    if (rec[L.choice_lits + j] < 0 || rec[L.choice_lits + j] >= nv) return -13;
  for (int32_t i = 0; i < rec[DP_H_NA]; ++i)
    if (rec[L.anchors + i] < 0 || rec[L.anchors + i] >= nv) return -14;
  return 0;
}

}  // extern "C"

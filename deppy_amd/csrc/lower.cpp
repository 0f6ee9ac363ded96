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
#include <atomic>
#include <cstring>
#include <mutex>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include "common.hpp"

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
  std::vector<uint64_t> key;
  std::vector<int32_t> val;
  std::vector<uint32_t> gen;
  uint32_t cur = 1;
  size_t count = 0, mask = 0;
  FlatMap() { grow(1024); }
  void grow(size_t cap) {
    std::vector<uint64_t> k2(cap);
    std::vector<int32_t> v2(cap);
    std::vector<uint32_t> g2(cap, 0);
    const size_t m2 = cap - 1;
    for (size_t i = 0; i < key.size(); ++i)
      if (gen[i] == cur) {
        size_t h = hash(key[i]) & m2;
        while (g2[h] == cur) h = (h + 1) & m2;
        k2[h] = key[i]; v2[h] = val[i]; g2[h] = cur;
      }
    key.swap(k2); val.swap(v2); gen.swap(g2);
    mask = m2;
  }
  static size_t hash(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33;
    return (size_t)x;
  }
  void reset() {
    count = 0;
    if (++cur == 0) {  // generation wrap: clear for real
      std::fill(gen.begin(), gen.end(), 0u);
      cur = 1;
    }
  }
  // the value of k, or -1
  int32_t find(uint64_t k) const {
    for (size_t h = hash(k) & mask; gen[h] == cur; h = (h + 1) & mask)
      if (key[h] == k) return val[h];
    return -1;
  }
  // insert k -> v (k must be absent)
  void insert(uint64_t k, int32_t v) {
    if (2 * (count + 1) > key.size()) grow(2 * key.size());
    size_t h = hash(k) & mask;
    while (gen[h] == cur) h = (h + 1) & mask;
    key[h] = k; val[h] = v; gen[h] = cur;
    ++count;
  }
  int32_t* find_slot(uint64_t k) {
    for (size_t h = hash(k) & mask; gen[h] == cur; h = (h + 1) & mask)
      if (key[h] == k) return &val[h];
    return nullptr;
  }
};

// And-inverter graph with structural hashing (gini logic.C).
struct Aig {
  int32_t next_node = 1;
  FlatMap strash;
  void reset(int nv) {
    next_node = 1 + nv;
    strash.reset();
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

struct Out {  // per-thread output chunk
  std::vector<int32_t> rec;
  std::vector<int64_t> rec_len;  // per problem
  std::vector<int32_t> ivar, icon;
  std::vector<int64_t> ident_len;
  std::vector<int32_t> err;
  std::vector<std::string> msg;
};

struct Work {  // per-thread scratch
  Aig aig;
  std::vector<int64_t> stamp;  // interned path: string -> (tag << 32 | var)
  std::unordered_map<std::string_view, int32_t> names;
  FlatMap key_ident;  // gate literal -> identity
  std::vector<int32_t> owner_v, owner_c;
  std::vector<int32_t> clause_off, clause_lits, clause_id;
  std::vector<int32_t> card_off, card_lits, card_bound, card_id;
  std::vector<int32_t> var_choice_off, choice_off, choice_lits, anchors;
  std::vector<int32_t> ms, sorted, order, mult;
  std::vector<std::string> errs;
};

struct Lowerer {
  const dp_wire& w;
  explicit Lowerer(const dp_wire& wire) : w(wire) {}

  std::string_view str(int64_t i) const {
    return std::string_view(w.str_bytes + w.str_off[i], (size_t)(w.str_off[i + 1] - w.str_off[i]));
  }

  void lower_one(int32_t p, Work& W, Out& O) const {
    const int64_t v0 = w.prob_var_off[p], v1 = w.prob_var_off[p + 1];
    const int nv = (int)(v1 - v0);
    const int64_t tag = (int64_t)p + 1;
    // pass 1: one literal per variable, reject duplicates (lit_mapping.go:50-57)
    W.names.clear();
    for (int i = 0; i < nv; ++i) {
      int64_t sid = w.var_id[v0 + i];
      bool dup;
      if (w.interned) {
        int64_t& st = W.stamp[(size_t)sid];
        dup = (st >> 32) == tag;
        if (!dup) st = (tag << 32) | i;
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
        int64_t st = W.stamp[(size_t)sid];
        if ((st >> 32) == tag) v = (int32_t)(st & 0xffffffff);
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
    emit_record(W, O, nv);
  }

  static int32_t leq(Aig& aig, Work& W, int32_t n) {
    const int N = (int)W.ms.size();
    if (n < 0) return kF;
    if (n >= N) return kT;
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
      if (w.interned) return (int32_t)(W.stamp[(size_t)sid] & 0xffffffff);
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
    O.rec.insert(O.rec.end(), hdr, hdr + hdr[DP_H_WORDS]);
    O.rec_len.push_back(hdr[DP_H_WORDS]);
    O.ident_len.push_back(0);
    O.err.push_back(code);
    O.msg.push_back(msg);
  }

  static void emit_record(Work& W, Out& O, int nv) {
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
    dp_rec_layout L = dp_rec_layout_of(hdr);
    hdr[DP_H_WORDS] = L.words;
    size_t base = O.rec.size();
    O.rec.insert(O.rec.end(), hdr, hdr + DP_H_SIZE);
    auto app = [&](const std::vector<int32_t>& v) { O.rec.insert(O.rec.end(), v.begin(), v.end()); };
    app(W.clause_off); app(W.clause_lits); app(W.clause_id);
    app(W.card_off); app(W.card_lits); app(W.card_bound); app(W.card_id);
    app(W.var_choice_off); app(W.choice_off); app(W.choice_lits); app(W.anchors);
    O.rec_len.push_back((int64_t)(O.rec.size() - base));
    O.ivar.insert(O.ivar.end(), W.owner_v.begin(), W.owner_v.end());
    O.icon.insert(O.icon.end(), W.owner_c.begin(), W.owner_c.end());
    O.ident_len.push_back((int64_t)W.owner_v.size());
    O.err.push_back(DP_LOWER_OK);
    O.msg.emplace_back();
  }
};

}  // namespace
}  // namespace dp

struct dp_lowered {
  int32_t n = 0;
  std::vector<int64_t> rec_off, ident_off;
  std::vector<int32_t> rec, ivar, icon, err;
  std::vector<std::string> msg;
};

extern "C" {

const char* dp_last_global_error(void) { return dp::g_err.c_str(); }

static bool wire_ok(const dp_wire* w) {
  if (!w || w->n_problems < 0 || !w->prob_var_off) return false;
  if (w->n_problems == 0) return true;
  const int64_t nvars = w->prob_var_off[w->n_problems];
  if (w->prob_var_off[0] != 0) return false;
  for (int32_t p = 0; p < w->n_problems; ++p)
    if (w->prob_var_off[p + 1] < w->prob_var_off[p]) return false;
  if (nvars > 0 && (!w->var_id || !w->var_con_off)) return false;
  if (nvars == 0) return true;
  const int64_t ncons = w->var_con_off[nvars];
  for (int64_t v = 0; v < nvars; ++v) {
    if (w->var_con_off[v + 1] < w->var_con_off[v]) return false;
    if (w->var_id[v] < 0 || w->var_id[v] >= w->n_strs) return false;
  }
  for (int64_t c = 0; c < ncons; ++c) {
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
  if (!out || !wire_ok(wire)) {
    dp::set_global_error("dp_lower: malformed wire batch");
    return -1;
  }
  const int32_t P = wire->n_problems;
  unsigned hw = std::thread::hardware_concurrency();
  int nt = (int)std::min<unsigned>(hw ? hw : 1, 16);
  // threads by work (constraint arguments), chunks small enough to balance
  const int64_t work = P ? wire->con_arg_off[wire->var_con_off[wire->prob_var_off[P]]] : 0;
  if (work < 200000) nt = 1;
  const int32_t chunk = (int32_t)std::max<int64_t>(1, std::min<int64_t>(64, P / (8 * (int64_t)nt)));
  const int32_t nchunks = (P + chunk - 1) / chunk;
  std::vector<dp::Out> outs((size_t)std::max(nchunks, 1));
  dp::Lowerer L(*wire);
  std::atomic_int next{0};
  auto worker = [&]() {
    dp::Work W;
    if (wire->interned) W.stamp.assign((size_t)wire->n_strs, 0);
    for (;;) {
      int c = next.fetch_add(1);
      if (c >= nchunks) break;
      // fill a chunk in thread-local storage, then move it into place: the
      // Out headers of neighbouring chunks share cache lines
      dp::Out local;
      for (int32_t p = c * chunk; p < std::min(P, (c + 1) * chunk); ++p) L.lower_one(p, W, local);
      outs[(size_t)c] = std::move(local);
    }
  };
  if (nt == 1) worker();
  else {
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t) th.emplace_back(worker);
    for (auto& t : th) t.join();
  }
  auto* lw = new dp_lowered;
  lw->n = P;
  lw->rec_off.assign(1, 0);
  lw->ident_off.assign(1, 0);
  size_t tot = 0, toti = 0;
  for (auto& o : outs) { tot += o.rec.size(); toti += o.ivar.size(); }
  lw->rec.reserve(tot);
  lw->ivar.reserve(toti);
  lw->icon.reserve(toti);
  for (auto& o : outs) {
    for (size_t i = 0; i < o.rec_len.size(); ++i) {
      lw->rec_off.push_back(lw->rec_off.back() + o.rec_len[i]);
      lw->ident_off.push_back(lw->ident_off.back() + o.ident_len[i]);
    }
    lw->rec.insert(lw->rec.end(), o.rec.begin(), o.rec.end());
    lw->ivar.insert(lw->ivar.end(), o.ivar.begin(), o.ivar.end());
    lw->icon.insert(lw->icon.end(), o.icon.begin(), o.icon.end());
    lw->err.insert(lw->err.end(), o.err.begin(), o.err.end());
    for (auto& m : o.msg) lw->msg.push_back(std::move(m));
  }
  *out = lw;
  return 0;
}

void dp_lowered_free(dp_lowered* lw) { delete lw; }
int32_t dp_lowered_num_problems(const dp_lowered* lw) { return lw->n; }
const int64_t* dp_lowered_rec_off(const dp_lowered* lw) { return lw->rec_off.data(); }
const int32_t* dp_lowered_rec(const dp_lowered* lw) { return lw->rec.data(); }
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

int dp_rec_validate(const int32_t* rec, int64_t words) {
  if (!rec || words < DP_H_SIZE) return -1;
  if (rec[DP_H_MAGIC] != DP_REC_MAGIC) return -2;
  for (int i = DP_H_NV; i <= DP_H_NCHL; ++i)
    if (rec[i] < 0) return -3;
  dp_rec_layout L = dp_rec_layout_of(rec);
  if (L.words != rec[DP_H_WORDS] || L.words > words) return -4;
  const int32_t nv = rec[DP_H_NV], nc = rec[DP_H_NC], nk = rec[DP_H_NK], nch = rec[DP_H_NCH];
  const int32_t nid = rec[DP_H_NID];
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
    // duplicates of a variable must be consecutive (one run per variable)
    for (int32_t j = rec[L.card_off + k]; j < rec[L.card_off + k + 1]; ++j) {
      int32_t v = rec[L.card_lits + j];
      if (v < 0 || v >= nv) return -11;
      if (j > rec[L.card_off + k] && rec[L.card_lits + j - 1] != v)
        for (int32_t i = rec[L.card_off + k]; i < j - 1; ++i)
          if (rec[L.card_lits + i] == v) return -12;
    }
  }
  for (int32_t j = 0; j < rec[DP_H_NCHL]; ++j)
    if (rec[L.choice_lits + j] < 0 || rec[L.choice_lits + j] >= nv) return -13;
  for (int32_t i = 0; i < rec[DP_H_NA]; ++i)
    if (rec[L.anchors + i] < 0 || rec[L.anchors + i] >= nv) return -14;
  return 0;
}

}  // extern "C"

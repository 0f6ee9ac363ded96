/*
 * sat_oracle.c — CPU restatement of deppy's pkg/sat solve path.
 *
 * TEST INFRASTRUCTURE (see sat_oracle.h).  Plain C, single problem per call,
 * sequential.  The HIP kernel (deppy_amd/csrc/solve_kernel.hip) computes the
 * same function with one wavefront per problem; tests require bit-identical
 * status / installed set / core / steps.
 *
 * Semantics:
 *
 *  Unit propagation ("BCP", gini Test) is run in synchronous rounds: every row
 *  watched by a literal assigned in round t is evaluated against the
 *  assignment as it stood at the start of round t+1; implications are
 *  committed together.  The reason of a variable is the lowest row id that
 *  implied it; the reported conflict of a round is the lowest conflicting row,
 *  else the lowest variable implied both ways.  The fixpoint / conflict verdict
 *  equals any other unit-propagation schedule; fixing the schedule makes
 *  reasons (and therefore cores) deterministic.
 *
 *  AtMost rows propagate by counting (generalised arc consistency, the
 *  propagation strength of the sorting network gini.CardSort builds,
 *  constraints.go:180-186); a variable listed m times counts m.
 *
 *  Test(m)   = assume m, propagate; -1 conflict, 1 all variables assigned, else 0.
 *  Untest()  = truncate the trail to the scope mark; unit propagation of the
 *              learned rows decides the restored scope's result.
 *  Solve()   = complete search under the open scopes (dpll below); when it
 *              fails, the nogood of the guesses its refutation used is learned
 *              (gini keeps the clauses Solve learns).
 */
#include "sat_oracle.h"

#include "../include/deppy_hip.h"

#include <limits.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define INF INT32_MAX
#define R_DECISION (-1) /* assumption / guess / decision: no reason row */
#define R_EXTRA (-2)    /* epilogue cardinality bound over the extras    */

enum { CK_NONE = 0, CK_ROW, CK_VAR, CK_ASSUME, CK_EXTRA };

typedef struct {
  int nv, nc, nk, nch, na, nid, nrows;
  int nvu; /* the input's variables: nvu..nv-1 are an AtMost network's gates (DP_H_NVU) */
  const int32_t *clause_off, *clause_lits, *clause_id;
  const int32_t *card_off, *card_lits, *card_bound, *card_id;
  const int32_t *var_choice_off, *choice_off, *choice_lits, *anchors;
} prob_t;

typedef struct search_s search_t;

typedef struct {
  prob_t p;
  int32_t* wide; /* the int32 copy of a 16-bit-form record (widen), or NULL */
  /* watch lists: rows to evaluate when literal l becomes TRUE */
  int32_t *w_off, *w;
#ifdef ORACLE_TWL
  /* two-watched-literal lists (the kernel's DP_TWL_LDS variant): live end
   * of each list, watched positions per clause row, dynamic rows */
  int32_t *wend, *wpos;
  uint8_t* dyn;
#endif
  /* assignment */
  int8_t* val; /* 0 unassigned, 1 true, -1 false */
  int32_t *reason, *rnd, *trail;
  int32_t tlen, qhead, round;
  /* per-round implication scratch */
  int32_t *imp_pos, *imp_neg, *touched;
  int32_t ntouched;
  /* row filter (core refutations) */
  const uint8_t* enabled;
  /* epilogue cardinality bound over extras */
  int extra_mode, extra_w;
  uint8_t* is_extra;
  /* last conflict */
  int ck, c_row, c_var, c_rp, c_rn;
  /* budget */
  int64_t steps, budget;
  int budget_hit;
  /* conflict analysis */
  uint8_t *seen, *used;
  int32_t* work;
  int32_t nwork;
  int collect;
  /* search */
  uint8_t* inS;
  uint32_t* model;
  int model_valid;
  /* dpll decision stack */
  int32_t *d_lit, *d_mark;
  uint8_t* d_flip;
  /* learned nogoods of failed Solve() calls: rows nrows.. (see learn()) */
  int32_t *l_off, *l_lits;
  int32_t nl, lcap, learn_lo, collect_guess; /* rows below learn_lo are switched off */
  uint8_t* fg; /* guesses met by the refutation of the current Solve() */
  int32_t* dix;    /* decision index of a Solve() decision variable, else -1 */
  uint8_t* dset;   /* decisions met by the last conflict analysis */
  uint8_t* uacc; /* identities of the search's refutation (union over its analyses) */
  /* search trace (Tracer, search.go:173): event records, see oracle_solve_traced */
  int32_t* trace;
  int32_t trace_cap, trace_len, trace_stop;
} st_t;

#ifdef ORACLE_TWL
/* Round counters of the two-watched-literal variant (single-threaded use:
 * oracle_twl_stats): rounds, watch entries visited, 64-entry batches a
 * wavefront would take (one frontier literal: its list; several: their lists
 * flattened 64 literals at a time), two-watched row visits, watch moves, and
 * what the occurrence lists would have visited in the same rounds: entries
 * and batches (a list's capacity is its occurrence count). */
static long long g_twl_stats[7];
void oracle_twl_stats(long long* out, int reset) {
  for (int i = 0; i < 7; ++i) {
    out[i] = g_twl_stats[i];
    if (reset) g_twl_stats[i] = 0;
  }
}
#endif

/* learned-row store: at most L_MAX rows and nv+64 literals */
#define L_MAX 64

/* ------------------------------------------------------------------ */
/* record parsing + watch lists                                        */
/* ------------------------------------------------------------------ */

static void parse(prob_t* p, const int32_t* rec) {
  dp_rec_layout L = dp_rec_layout_of(rec);
  p->nv = rec[DP_H_NV];
  p->nc = rec[DP_H_NC];
  p->nk = rec[DP_H_NK];
  p->nch = rec[DP_H_NCH];
  p->na = rec[DP_H_NA];
  p->nid = rec[DP_H_NID];
  /* (clamped as the kernel's nvu_of: a record with NVU past nv reads no bit past nv) */
  p->nvu = rec[DP_H_NVU] > 0 && rec[DP_H_NVU] < p->nv ? rec[DP_H_NVU] : p->nv;
  p->nrows = p->nc + p->nk;
  p->clause_off = rec + L.clause_off;
  p->clause_lits = rec + L.clause_lits;
  p->clause_id = rec + L.clause_id;
  p->card_off = rec + L.card_off;
  p->card_lits = rec + L.card_lits;
  p->card_bound = rec + L.card_bound;
  p->card_id = rec + L.card_id;
  p->var_choice_off = rec + L.var_choice_off;
  p->choice_off = rec + L.choice_off;
  p->choice_lits = rec + L.choice_lits;
  p->anchors = rec + L.anchors;
}

static int row_ident(const prob_t* p, int r) {
  return r < p->nc ? p->clause_id[r] : r < p->nrows ? p->card_id[r - p->nc] : -1;
}

static void* xcalloc(size_t n, size_t sz) { return calloc(n ? n : 1, sz); }

/* A record in a 16-bit form widened to int32 words in *tmp (freed by the
 * caller); int32 records are returned as they are.  DP_FMT_U16: every body
 * word a uint16.  DP_FMT_P16 (include/deppy_hip.h): the uint16 arrays, then
 * byte lengths of the offsets arrays and the AtMost-identity bit mask (a
 * mask with the wrong number of set bits leaves the ids it cannot place 0;
 * records are validated before the oracle sees them).  DP_FMT_P16D: the same
 * without the choice lists, restated from the dependency rows by
 * implied_choices below. */
/* DP_FMT_P16D's choice lists (include/deppy_hip.h): dependency rows -- two
 * or more literals, the first negative, the rest positive -- in row order;
 * src[k] == 0: list k is the next one's variables after its first literal,
 * src[k] = d: list k repeats list k - d; var_choice_off counts the lists per
 * subject (the first literal's variable).  Records are validated before the
 * oracle sees them. */
static void implied_choices(const dp_rec_layout* L, const uint8_t* src, int32_t* o) {
  const int32_t nc = o[DP_H_NC], nv = o[DP_H_NV], nch = o[DP_H_NCH];
  int32_t* rowk = xcalloc((size_t)nch + 1, sizeof(int32_t));
  int32_t r = 0, n = 0, filled = 0;
  o[L->var_choice_off] = 0;
  o[L->choice_off] = 0;
  for (int32_t k = 0; k < nch; ++k) {
    int32_t row = -1;
    if (src[k] == 0) {
      for (; r < nc && row < 0; ++r) {
        const int32_t a = o[L->clause_off + r], b = o[L->clause_off + r + 1];
        int dep = b - a >= 2 && (o[L->clause_lits + a] & 1);
        for (int32_t j = a + 1; j < b && dep; ++j) dep = !(o[L->clause_lits + j] & 1);
        if (dep) row = r;
      }
    } else if (src[k] <= k) {
      row = rowk[k - src[k]];
    }
    rowk[k] = row;
    if (row < 0) break;
    const int32_t a = o[L->clause_off + row], b = o[L->clause_off + row + 1];
    const int32_t subj = o[L->clause_lits + a] >> 1;
    while (filled < subj && filled < nv) o[L->var_choice_off + ++filled] = k;
    for (int32_t j = a + 1; j < b && n < o[DP_H_NCHL]; ++j) o[L->choice_lits + n++] = o[L->clause_lits + j] >> 1;
    o[L->choice_off + k + 1] = n;
  }
  while (filled < nv) o[L->var_choice_off + ++filled] = nch;
  free(rowk);
}

/* DP_FMT_P8D (include/deppy_hip.h) into the int32 record o (header copied):
 * the 8-bit variables with their sign and bit-8 planes, the byte or nibble
 * lengths, the nonzero list sources and the identity mask, read in the
 * order the format lists them; then the lists as DP_FMT_P16D's. */
static int p8_bit(const uint8_t* b, int64_t at, int64_t j) { return (b[at + (j >> 3)] >> (j & 7)) & 1; }
static void widen_p8(const int32_t* rec, int32_t* o) {
  const dp_rec_layout L = dp_rec_layout_of(rec);
  const int32_t f = rec[DP_H_P8] & 0xff;
  const int32_t ncl = rec[DP_H_NCL], nkl = rec[DP_H_NKL], na = rec[DP_H_NA], nk = rec[DP_H_NK];
  const int32_t nc = rec[DP_H_NC], nch = rec[DP_H_NCH], nid = rec[DP_H_NID];
  const uint8_t* b = (const uint8_t*)(rec + DP_H_SIZE);
  int64_t at = 0;
  const int64_t cv = at; at += ncl;
  const int64_t kv = at; at += nkl;
  const int64_t av = at; at += na;
  const int64_t kb = at; at += (f & DP_P8_B1) ? 0 : nk;
  const int64_t neg = at; at += (ncl + 7) / 8;
  int64_t chi = -1, khi = -1, ahi = -1;
  if (f & DP_P8_HI) {
    chi = at; at += (ncl + 7) / 8;
    khi = at; at += (nkl + 7) / 8;
    ahi = at; at += (na + 7) / 8;
  }
  for (int32_t j = 0; j < ncl; ++j)
    o[L.clause_lits + j] = 2 * (b[cv + j] + (chi >= 0 ? 256 * p8_bit(b, chi, j) : 0)) + p8_bit(b, neg, j);
  for (int32_t j = 0; j < nkl; ++j) o[L.card_lits + j] = b[kv + j] + (khi >= 0 ? 256 * p8_bit(b, khi, j) : 0);
  for (int32_t i = 0; i < na; ++i) o[L.anchors + i] = b[av + i] + (ahi >= 0 ? 256 * p8_bit(b, ahi, i) : 0);
  for (int32_t k = 0; k < nk; ++k) o[L.card_bound + k] = (f & DP_P8_B1) ? 1 : b[kb + k];
  const int32_t offs[2] = {L.clause_off, L.card_off}, ns[2] = {nc, nk};
  int64_t i = 0;
  for (int a = 0; a < 2; ++a) {
    o[offs[a]] = 0;
    for (int32_t j = 0; j < ns[a]; ++j, ++i) {
      const int len = (f & DP_P8_NIB) ? (b[at + i / 2] >> (4 * (i % 2))) & 15 : b[at + i];
      o[offs[a] + j + 1] = o[offs[a] + j] + len;
    }
  }
  at += (f & DP_P8_NIB) ? (nc + nk + 1) / 2 : nc + nk;
  const int64_t snz = at;
  at += (nch + 7) / 8;
  uint8_t* src = xcalloc((size_t)nch + 1, 1);
  for (int32_t k = 0; k < nch; ++k)
    if (p8_bit(b, snz, k)) src[k] = b[at++];
  int32_t c0 = 0, c1 = 0;
  for (int32_t id = 0; id < nid; ++id) {
    if (p8_bit(b, at, id)) {
      if (c1 < nk) o[L.card_id + c1++] = id;
    } else if (c0 < nc) {
      o[L.clause_id + c0++] = id;
    }
  }
  implied_choices(&L, src, o);
  free(src);
}

static const int32_t* widen(const int32_t* rec, int32_t** tmp) {
  *tmp = NULL;
  const int32_t fmt = rec[DP_H_FMT];
  if (fmt == DP_FMT_P8D) {
    int32_t* o = xcalloc((size_t)rec[DP_H_WORDS], sizeof(int32_t));
    memcpy(o, rec, DP_H_SIZE * sizeof(int32_t));
    o[DP_H_FMT] = DP_FMT_I32;
    o[DP_H_P8] = 0;
    widen_p8(rec, o);
    *tmp = o;
    return o;
  }
  if (fmt != DP_FMT_U16 && fmt != DP_FMT_P16 && fmt != DP_FMT_P16D) return rec;
  int32_t w = rec[DP_H_WORDS];
  int32_t* o = xcalloc((size_t)w, sizeof(int32_t));
  memcpy(o, rec, DP_H_SIZE * sizeof(int32_t));
  o[DP_H_FMT] = DP_FMT_I32;
  const uint16_t* u = (const uint16_t*)(rec + DP_H_SIZE);
  if (rec[DP_H_FMT] == DP_FMT_U16) {
    for (int32_t j = DP_H_SIZE; j < w; ++j) o[j] = u[j - DP_H_SIZE];
  } else {
    const dp_rec_layout L = dp_rec_layout_of(rec);
    const int32_t nc = rec[DP_H_NC], nk = rec[DP_H_NK];
    const int derived = fmt == DP_FMT_P16D;
    const int32_t n16[5] = {rec[DP_H_NCL], rec[DP_H_NKL], nk, derived ? 0 : rec[DP_H_NCHL], rec[DP_H_NA]};
    const int32_t at16[5] = {L.clause_lits, L.card_lits, L.card_bound, L.choice_lits, L.anchors};
    for (int a = 0; a < 5; ++a)
      for (int32_t j = 0; j < n16[a]; ++j) o[at16[a] + j] = *u++;
    const uint8_t* t = (const uint8_t*)(rec + DP_H_SIZE) + dp_p16_tail_at(rec);
    const int32_t nl[4] = {nc, nk, rec[DP_H_NV], rec[DP_H_NCH]};
    const int32_t atl[4] = {L.clause_off, L.card_off, L.var_choice_off, L.choice_off};
    for (int a = 0; a < (derived ? 2 : 4); ++a) {
      o[atl[a]] = 0;
      for (int32_t j = 0; j < nl[a]; ++j) o[atl[a] + j + 1] = o[atl[a] + j] + *t++;
    }
    const uint8_t* src = t;
    if (derived) t += rec[DP_H_NCH];
    int32_t c0 = 0, c1 = 0;
    for (int32_t i = 0; i < rec[DP_H_NID]; ++i) {
      if ((t[i >> 3] >> (i & 7)) & 1) {
        if (c1 < nk) o[L.card_id + c1++] = i;
      } else if (c0 < nc) {
        o[L.clause_id + c0++] = i;
      }
    }
    if (derived) implied_choices(&L, src, o);
  }
  *tmp = o;
  return o;
}

static int st_init(st_t* s, const int32_t* rec) {
  memset(s, 0, sizeof(*s));
  rec = widen(rec, &s->wide);
  parse(&s->p, rec);
  const prob_t* p = &s->p;
  int nl = 2 * p->nv;
  s->w_off = xcalloc((size_t)nl + 1, sizeof(int32_t));
  /* count: clause literal x in row r -> watched by ~x; card var v -> by +v */
  for (int r = 0; r < p->nc; ++r)
    for (int j = p->clause_off[r]; j < p->clause_off[r + 1]; ++j) s->w_off[(p->clause_lits[j] ^ 1) + 1]++;
  for (int k = 0; k < p->nk; ++k)
    for (int j = p->card_off[k]; j < p->card_off[k + 1]; ++j) s->w_off[2 * p->card_lits[j] + 1]++;
  for (int l = 0; l < nl; ++l) s->w_off[l + 1] += s->w_off[l];
  s->w = xcalloc((size_t)s->w_off[nl], sizeof(int32_t));
  int32_t* cur = xcalloc((size_t)nl, sizeof(int32_t));
  for (int l = 0; l < nl; ++l) cur[l] = s->w_off[l];
#ifdef ORACLE_TWL
  /* a clause row of 3..254 literals sits in the lists of its positions 0 and
   * 1 only (entry r | slot << 30); shorter and longer rows in every one */
  s->dyn = xcalloc((size_t)p->nc, 1);
  s->wpos = xcalloc((size_t)p->nc * 2, sizeof(int32_t));
  for (int r = 0; r < p->nc; ++r) {
    const int a = p->clause_off[r], len = p->clause_off[r + 1] - a;
    s->dyn[r] = len >= 3 && len <= 254;
    if (s->dyn[r]) {
      s->wpos[2 * r] = 0;
      s->wpos[2 * r + 1] = 1;
      s->w[cur[p->clause_lits[a] ^ 1]++] = r;
      s->w[cur[p->clause_lits[a + 1] ^ 1]++] = r | (1 << 30);
    } else {
      for (int j = a; j < a + len; ++j) s->w[cur[p->clause_lits[j] ^ 1]++] = r;
    }
  }
#else
  for (int r = 0; r < p->nc; ++r)
    for (int j = p->clause_off[r]; j < p->clause_off[r + 1]; ++j) s->w[cur[p->clause_lits[j] ^ 1]++] = r;
#endif
  for (int k = 0; k < p->nk; ++k)
    for (int j = p->card_off[k]; j < p->card_off[k + 1]; ++j) s->w[cur[2 * p->card_lits[j]]++] = p->nc + k;
#ifdef ORACLE_TWL
  s->wend = cur;
#else
  free(cur);
#endif
  int nv = p->nv;
  s->val = xcalloc((size_t)nv, 1);
  s->reason = xcalloc((size_t)nv, sizeof(int32_t));
  s->rnd = xcalloc((size_t)nv, sizeof(int32_t));
  s->trail = xcalloc((size_t)nv, sizeof(int32_t));
  s->imp_pos = xcalloc((size_t)nv, sizeof(int32_t));
  s->imp_neg = xcalloc((size_t)nv, sizeof(int32_t));
  s->touched = xcalloc((size_t)nv, sizeof(int32_t));
  for (int v = 0; v < nv; ++v) s->imp_pos[v] = s->imp_neg[v] = INF;
  s->is_extra = xcalloc((size_t)nv, 1);
  s->seen = xcalloc((size_t)nv, 1);
  s->used = xcalloc((size_t)p->nid, 1);
  s->uacc = xcalloc((size_t)p->nid + 1, 1);
  s->work = xcalloc((size_t)nv, sizeof(int32_t));
  s->inS = xcalloc((size_t)nv, 1);
  s->model = xcalloc((size_t)(nv + 31) / 32, sizeof(uint32_t));
  s->d_lit = xcalloc((size_t)nv, sizeof(int32_t));
  s->d_mark = xcalloc((size_t)nv, sizeof(int32_t));
  s->d_flip = xcalloc((size_t)nv, 1);
  s->lcap = nv + 64;
  s->l_off = xcalloc(L_MAX + 1, sizeof(int32_t));
  s->l_lits = xcalloc((size_t)s->lcap, sizeof(int32_t));
  s->fg = xcalloc((size_t)nv, 1);
  s->dix = xcalloc((size_t)nv, sizeof(int32_t));
  s->dset = xcalloc((size_t)nv + 1, 1);
  s->learn_lo = 0;
  return 0;
}

static void st_free(st_t* s) {
  free(s->wide);
#ifdef ORACLE_TWL
  free(s->wend); free(s->wpos); free(s->dyn);
#endif
  free(s->w_off); free(s->w); free(s->val); free(s->reason); free(s->rnd); free(s->trail);
  free(s->imp_pos); free(s->imp_neg); free(s->touched); free(s->is_extra); free(s->seen);
  free(s->used); free(s->uacc); free(s->work); free(s->inS); free(s->model); free(s->d_lit); free(s->d_mark);
  free(s->d_flip); free(s->l_off); free(s->l_lits); free(s->fg); free(s->dix); free(s->dset);
}

/* ------------------------------------------------------------------ */
/* unit propagation                                                    */
/* ------------------------------------------------------------------ */

static inline int row_on(const st_t* s, int r) {
  return !s->enabled || s->enabled[row_ident(&s->p, r)];
}

static inline int lit_val(const st_t* s, int l) {
  int x = s->val[l >> 1];
  return (l & 1) ? -x : x;
}

static inline void note(st_t* s, int l, int r) {
  int v = l >> 1;
  if (s->imp_pos[v] == INF && s->imp_neg[v] == INF) s->touched[s->ntouched++] = v;
  if (l & 1) {
    if (r < s->imp_neg[v]) s->imp_neg[v] = r;
  } else {
    if (r < s->imp_pos[v]) s->imp_pos[v] = r;
  }
}

/* Evaluate one row against the current assignment (start-of-round snapshot:
 * nothing is committed while a round is being evaluated). */
static void eval_clause(st_t* s, int r, const int32_t* lits, int a, int b, int* crow) {
  int nun = 0, ul = -1;
  for (int j = a; j < b; ++j) {
    int x = lit_val(s, lits[j]);
    if (x > 0) return; /* satisfied */
    if (x == 0) { ++nun; ul = lits[j]; }
  }
  if (nun == 0) { if (r < *crow) *crow = r; }
  else if (nun == 1) note(s, ul, r);
}

static void eval_row(st_t* s, int r, int* crow) {
  const prob_t* p = &s->p;
  if (r < p->nc) {
    eval_clause(s, r, p->clause_lits, p->clause_off[r], p->clause_off[r + 1], crow);
  } else if (r >= p->nrows) {
    int j = r - p->nrows;
    eval_clause(s, r, s->l_lits, s->l_off[j], s->l_off[j + 1], crow);
  } else {
    int k = r - p->nc, a = p->card_off[k], b = p->card_off[k + 1], cnt = 0, nun = 0;
    for (int j = a; j < b; ++j) {
      int x = s->val[p->card_lits[j]];
      cnt += (x > 0);
      nun += (x == 0);
    }
    int bound = p->card_bound[k];
    if (cnt > bound) { if (r < *crow) *crow = r; }
    else if (nun > 0) {
      /* a variable repeated m times is a run of m equal positions; it is
       * forced false once cnt + m exceeds the bound */
      for (int j = a; j < b;) {
        int v = p->card_lits[j], e = j + 1;
        while (e < b && p->card_lits[e] == v) ++e;
        if (s->val[v] == 0 && cnt + (e - j) > bound) note(s, 2 * v + 1, r);
        j = e;
      }
    }
  }
}

static inline void assign(st_t* s, int l, int reason, int rd) {
  int v = l >> 1;
  s->val[v] = (l & 1) ? -1 : 1;
  s->reason[v] = reason;
  s->rnd[v] = rd;
  s->dix[v] = -1;
  s->trail[s->tlen++] = l;
}

static void clear_touched(st_t* s) {
  for (int i = 0; i < s->ntouched; ++i) s->imp_pos[s->touched[i]] = s->imp_neg[s->touched[i]] = INF;
  s->ntouched = 0;
}

/* Commit the implications of round rd, or report its conflict. */
static int finish_round(st_t* s, int rd, int crow) {
  if (crow != INF) {
    clear_touched(s);
    s->ck = CK_ROW; s->c_row = crow;
    return -1;
  }
  int cvar = INF;
  for (int i = 0; i < s->ntouched; ++i) {
    int v = s->touched[i];
    if (s->imp_pos[v] != INF && s->imp_neg[v] != INF && v < cvar) cvar = v;
  }
  if (cvar != INF) {
    s->ck = CK_VAR; s->c_var = cvar; s->c_rp = s->imp_pos[cvar]; s->c_rn = s->imp_neg[cvar];
    s->c_row = rd; /* round of the conflict, bounds card antecedents */
    clear_touched(s);
    return -1;
  }
  for (int i = 0; i < s->ntouched; ++i) {
    int v = s->touched[i];
    if (s->imp_pos[v] != INF) assign(s, 2 * v, s->imp_pos[v], rd);
    else assign(s, 2 * v + 1, s->imp_neg[v], rd);
  }
  clear_touched(s);
  return 0;
}

/* Epilogue bound "at most extra_w of the extras are true" (the Leq(w)
 * assumption over CardinalityConstrainer, solve.go:105-107). */
static int extra_check(st_t* s) {
  int cnt = 0, nun = 0;
  for (int v = 0; v < s->p.nv; ++v)
    if (s->is_extra[v]) { cnt += (s->val[v] > 0); nun += (s->val[v] == 0); }
  if (cnt > s->extra_w) { s->ck = CK_EXTRA; return -1; }
  if (cnt == s->extra_w && nun > 0) {
    int rd = ++s->round;
    for (int v = 0; v < s->p.nv; ++v)
      if (s->is_extra[v] && s->val[v] == 0) assign(s, 2 * v + 1, R_EXTRA, rd);
    return 1;
  }
  return 0;
}

/* Learned rows are evaluated in every round (they are few); a core
 * refutation switches off the rows learned before it (learn_lo). */
static void eval_learned(st_t* s, int* crow) {
  for (int j = s->learn_lo; j < s->nl; ++j) eval_row(s, s->p.nrows + j, crow);
}

#ifdef ORACLE_TWL
/* The kernel's two-watched-literal visit (solve_kernel.hpp twl_row) of
 * dynamic clause row r through slot k, whose literal a round falsified:
 * nothing when the other watch is true; else the row's outcome exactly as
 * eval_clause gives it, and slot k moves to N[k] (both watches false) or to
 * the first of N that is not the other watch, N being the row's first two
 * non-false positions.  Returns 1 to keep the entry in its list. */
static int twl_visit(st_t* s, int r, int k, int* crow) {
  const prob_t* p = &s->p;
  const int32_t* L = p->clause_lits;
  const int a = p->clause_off[r], b = p->clause_off[r + 1];
  const int po = s->wpos[2 * r + 1 - k];
  const int vo = lit_val(s, L[a + po]);
  g_twl_stats[3]++;
  if (vo > 0) return 1;
  int n0 = -1, n1 = -1;
  for (int j = a; j < b && n1 < 0; ++j)
    if (lit_val(s, L[j]) >= 0) {
      if (n0 < 0) n0 = j - a;
      else n1 = j - a;
    }
  if (n1 < 0) {
    if (n0 < 0) { if (r < *crow) *crow = r; }
    else if (lit_val(s, L[a + n0]) == 0) note(s, L[a + n0], r);
  }
  const int q = vo < 0 ? (k ? n1 : n0) : (n0 != po ? n0 : n1);
  if (q < 0) return 1;
  s->wpos[2 * r + k] = q;
  const int li = L[a + q] ^ 1;
  s->w[s->wend[li]++] = r | (k << 30);
  g_twl_stats[4]++;
  return 0;
}
#endif

static int propagate(st_t* s) {
  for (;;) {
    if (s->qhead == s->tlen) {
      if (s->extra_mode) {
        int r = extra_check(s);
        if (r < 0) return -1;
        if (r > 0) continue;
      }
      return s->tlen == s->p.nv ? 1 : 0;
    }
    int lo = s->qhead, hi = s->tlen, rd = ++s->round, crow = INF;
    s->qhead = hi;
#ifdef ORACLE_TWL
    g_twl_stats[0]++;
    for (int c = lo; c < hi; c += 64) {
      int t = 0, o = 0;
      for (int i = c; i < hi && i < c + 64; ++i) {
        t += s->wend[s->trail[i]] - s->w_off[s->trail[i]];
        o += s->w_off[s->trail[i] + 1] - s->w_off[s->trail[i]];
      }
      g_twl_stats[2] += (t + 63) / 64;
      g_twl_stats[5] += o;
      g_twl_stats[6] += (o + 63) / 64;
    }
    for (int i = lo; i < hi; ++i) {
      const int l = s->trail[i], e = s->wend[l];
      int at = s->w_off[l];
      for (int k = s->w_off[l]; k < e; ++k) {
        const int ent = s->w[k], r = ent & ~(1 << 30);
        int keep = 1;
        g_twl_stats[1]++;
        if (row_on(s, r)) {
          if (r < s->p.nc && s->dyn[r]) keep = twl_visit(s, r, ent >> 30, &crow);
          else eval_row(s, r, &crow);
        }
        if (keep) s->w[at++] = ent;
      }
      s->wend[l] = at;
    }
#else
    for (int i = lo; i < hi; ++i) {
      int l = s->trail[i];
      for (int k = s->w_off[l]; k < s->w_off[l + 1]; ++k)
        if (row_on(s, s->w[k])) eval_row(s, s->w[k], &crow);
    }
#endif
    eval_learned(s, &crow);
    if (finish_round(s, rd, crow) < 0) return -1;
  }
}

/* The base scope (solve.go:63-79): every constraint row is hard and every
 * anchor is assumed; one round evaluates every (enabled) row. */
static int base_propagate(st_t* s) {
  int rd = ++s->round, crow = INF;
  for (int r = 0; r < s->p.nrows; ++r)
    if (row_on(s, r)) eval_row(s, r, &crow);
  eval_learned(s, &crow);
  if (finish_round(s, rd, crow) < 0) return -1;
  return propagate(s);
}

static void truncate_to(st_t* s, int mark) {
  while (s->tlen > mark) s->val[s->trail[--s->tlen] >> 1] = 0;
  s->qhead = s->tlen;
}

/* gini Untest(): close the scope and report the restored scope's consistency
 * under unit propagation, learned rows included (search.go:84). */
static int untest_to(st_t* s, int mark) {
  truncate_to(s, mark);
  if (s->nl > s->learn_lo) {
    int rd = ++s->round, crow = INF;
    eval_learned(s, &crow);
    if (finish_round(s, rd, crow) < 0) return -1;
    return propagate(s);
  }
  return s->tlen == s->p.nv ? 1 : 0;
}

/* gini Assume(m) + Test(): one scope, one BCP. */
static int test_assume(st_t* s, int l) {
  s->steps++;
  int x = lit_val(s, l);
  if (x > 0) return propagate(s);
  if (x < 0) { s->ck = CK_ASSUME; s->c_var = l >> 1; return -1; }
  assign(s, l, R_DECISION, ++s->round);
  return propagate(s);
}

/* ------------------------------------------------------------------ */
/* conflict analysis: identities of the rows a conflict depends on     */
/* ------------------------------------------------------------------ */

static void push_ante(st_t* s, int r, int u, int bound_rd) {
  const prob_t* p = &s->p;
  if (r < 0) return;
  if (r < p->nc || r >= p->nrows) {
    const int32_t* lits = p->clause_lits;
    int a, b;
    if (r < p->nc) { a = p->clause_off[r]; b = p->clause_off[r + 1]; s->used[p->clause_id[r]] = 1; }
    else { lits = s->l_lits; a = s->l_off[r - p->nrows]; b = s->l_off[r - p->nrows + 1]; }
    for (int j = a; j < b; ++j) {
      int v = lits[j] >> 1;
      if (v != u && !s->seen[v]) { s->seen[v] = 1; s->work[s->nwork++] = v; }
    }
  } else {
    s->used[p->card_id[r - p->nc]] = 1;
    int k = r - p->nc;
    for (int j = p->card_off[k]; j < p->card_off[k + 1]; ++j) {
      int v = p->card_lits[j];
      if (v != u && s->val[v] > 0 && s->rnd[v] < bound_rd && !s->seen[v]) {
        s->seen[v] = 1; s->work[s->nwork++] = v;
      }
    }
  }
}

/* antecedents of the epilogue bound: the extras already true */
static void push_extra(st_t* s, int u, int bound_rd) {
  for (int v = 0; v < s->p.nv; ++v)
    if (v != u && s->is_extra[v] && s->val[v] > 0 && s->rnd[v] < bound_rd && !s->seen[v]) {
      s->seen[v] = 1; s->work[s->nwork++] = v;
    }
}

/* Walk the implication graph back from the last conflict.  Marks the
 * identities of every row used (used[]), the Solve() decisions reached
 * (dset[] by decision index) and, when collecting, the guesses reached (fg[]). */
static void analyze(st_t* s) {
  s->nwork = 0;
  if (s->ck == CK_ROW) push_ante(s, s->c_row, -1, INF);
  else if (s->ck == CK_VAR) {
    push_ante(s, s->c_rp, s->c_var, s->c_row);
    push_ante(s, s->c_rn, s->c_var, s->c_row);
  } else if (s->ck == CK_EXTRA) push_extra(s, -1, INF);
  else if (s->ck == CK_ASSUME) {  /* the assumed literal is false: its variable's reasons */
    s->seen[s->c_var] = 1;
    s->work[s->nwork++] = s->c_var;
  } else return;
  for (int i = 0; i < s->nwork; ++i) {
    int u = s->work[i];
    int r = s->reason[u];
    if (r >= 0) push_ante(s, r, u, s->rnd[u]);
    else if (r == R_EXTRA) push_extra(s, u, s->rnd[u]);
    else if (s->dix[u] >= 0) s->dset[s->dix[u]] = 1;
    else if (s->collect_guess && s->inS[u]) s->fg[u] = 1;
  }
  for (int i = 0; i < s->nwork; ++i) s->seen[s->work[i]] = 0;
}

/* ------------------------------------------------------------------ */
/* Solve(): complete search under the open scopes                      */
/* ------------------------------------------------------------------ */

/* Decision literal: the first positive, unassigned literal of the lowest
 * clause row that the all-false completion of the current assignment
 * violates; -1 if that completion is a model. */
static int first_violated(const st_t* s) {
  const prob_t* p = &s->p;
  for (int c = 0; c < p->nc; ++c) {
    if (!row_on(s, c)) continue;
    int viol = 1, fu = -1;
    for (int j = p->clause_off[c]; j < p->clause_off[c + 1]; ++j) {
      int l = p->clause_lits[j], x = s->val[l >> 1];
      if (l & 1) { if (x != 1) { viol = 0; break; } }
      else {
        if (x == 1) { viol = 0; break; }
        if (x == 0 && fu < 0) fu = l;
      }
    }
    if (viol) return fu;
  }
  return -1;
}

static void save_model(st_t* s) {
  int nw = (s->p.nv + 31) / 32;
  memset(s->model, 0, (size_t)nw * 4);
  for (int v = 0; v < s->p.nv; ++v)
    if (s->val[v] > 0) s->model[v >> 5] |= 1u << (v & 31);
  s->model_valid = 1;
}

enum { R_SAT = 1, R_UNSAT = -1, R_BUDGET = 2 };

/* Solve(): CDCL from a consistent fixpoint.  Decision: the preferred
 * (first unassigned) candidate of the first dependency row the all-false
 * completion violates, set true.  A conflict learns the nogood of the
 * decisions its analysis reaches (ascending decision order), backjumps to the
 * second-highest of them and asserts the negation of the highest.  Learned
 * rows live until this call returns; when their store is full the conflict is
 * resolved by flipping the last unflipped decision instead (plain DPLL).
 * On SAT the model is saved; the trail is restored to `root` either way. */
static int dpll(st_t* s) {
  const int root = s->tlen, nl0 = s->nl;
  int nd = 0, r;
  for (;;) {
    int l = first_violated(s);
    if (l < 0) { save_model(s); r = R_SAT; break; }
    if (++s->steps > s->budget) { s->budget_hit = 1; r = R_BUDGET; break; }
    s->d_lit[nd] = l; s->d_mark[nd] = s->tlen; s->d_flip[nd] = 0;
    assign(s, l, R_DECISION, ++s->round);
    s->dix[l >> 1] = nd++;
    int res = propagate(s);
    while (res < 0) {
      memset(s->dset, 0, (size_t)nd);
      analyze(s);
      int h = -1, b = -1, n = 0;
      for (int i = 0; i < nd; ++i)
        if (s->dset[i]) { b = h; h = i; ++n; }
      if (h < 0) { r = R_UNSAT; goto done; }
      if (++s->steps > s->budget) { s->budget_hit = 1; r = R_BUDGET; goto done; }
      if (s->nl < L_MAX && s->l_off[s->nl] + n <= s->lcap) {
        int at = s->l_off[s->nl];
        for (int i = 0; i < nd; ++i)
          if (s->dset[i]) s->l_lits[at++] = s->d_lit[i] ^ 1;
        s->l_off[++s->nl] = at;
        nd = b + 1;
        truncate_to(s, s->d_mark[nd]);
        assign(s, s->d_lit[h] ^ 1, s->p.nrows + s->nl - 1, ++s->round);
      } else {
        while (nd > 0 && s->d_flip[nd - 1]) --nd;
        if (nd == 0) { r = R_UNSAT; goto done; }
        truncate_to(s, s->d_mark[nd - 1]);
        s->d_flip[nd - 1] = 1;
        assign(s, s->d_lit[nd - 1] ^ 1, R_DECISION, ++s->round);
        s->dix[s->d_lit[nd - 1] >> 1] = nd - 1;
      }
      res = propagate(s);
    }
  }
done:
  truncate_to(s, root);
  s->nl = nl0;
  return r;
}

/* ------------------------------------------------------------------ */
/* search.Do (pkg/sat/search.go:158-203) over a pluggable inter.S       */
/* ------------------------------------------------------------------ */

typedef struct {
  int (*test)(void* u, st_t* s, int lit); /* Assume(lit) + Test() */
  int (*untest)(void* u, st_t* s, int mark);
  int (*solve)(void* u, st_t* s);
  void* u;
} backend_t;

typedef struct { int32_t list, idx; } choice_t; /* list>=0: choice row; <0: anchor ~list */
typedef struct { int32_t list, idx, m, children, mark; } guess_t;

struct search_s {
  choice_t* dq;
  int cap, head, n;
  guess_t* g;
  int ng;
  int result;
  int class_b, solve_unsat, last_solve;
  int final_from_solve; /* the last failure came from Solve() (else Test/Untest) */
};

static inline int list_len(const prob_t* p, int list) {
  return list < 0 ? 1 : p->choice_off[list + 1] - p->choice_off[list];
}
static inline int list_at(const prob_t* p, int list, int i) {
  return list < 0 ? ~list : p->choice_lits[p->choice_off[list] + i];
}

static void dq_push_back(search_t* h, choice_t c) { h->dq[(h->head + h->n++) % h->cap] = c; }
static void dq_push_front(search_t* h, choice_t c) {
  h->head = (h->head + h->cap - 1) % h->cap;
  h->dq[h->head] = c;
  h->n++;
}
static choice_t dq_pop_front(search_t* h) {
  choice_t c = h->dq[h->head];
  h->head = (h->head + 1) % h->cap;
  h->n--;
  return c;
}
static void dq_pop_back(search_t* h) { h->n--; }

/* PushGuess, search.go:34-77 */
static void push_guess(search_t* h, st_t* s, const backend_t* be) {
  const prob_t* p = &s->p;
  choice_t c = dq_pop_front(h);
  int len = list_len(p, c.list);
  guess_t g = {c.list, c.idx, -1, 0, s->tlen};
  if (c.idx < len) g.m = list_at(p, c.list, c.idx);
  int any = 0;
  for (int i = 0; i < len; ++i)
    if (s->inS[list_at(p, c.list, i)]) { any = 1; break; }
  if (any) g.m = -1;
  else if (c.idx >= len) h->class_b = 1; /* exhausted choice, SURVEY.md A.6.3 */
  h->g[h->ng++] = g;
  if (g.m < 0) return;
  for (int r = p->var_choice_off[g.m]; r < p->var_choice_off[g.m + 1]; ++r) {
    h->g[h->ng - 1].children++;
    dq_push_back(h, (choice_t){r, 0});
  }
  s->inS[g.m] = 1;
  h->result = be->test(be->u, s, 2 * g.m);
  h->last_solve = 0;
}

/* PopGuess, search.go:79-98 */
static void pop_guess(search_t* h, st_t* s, const backend_t* be) {
  guess_t g = h->g[--h->ng];
  if (g.m >= 0) {
    s->inS[g.m] = 0;
    h->result = be->untest(be->u, s, g.mark);
    h->last_solve = 0;
  }
  for (int i = 0; i < g.children; ++i) dq_pop_back(h);
  dq_push_front(h, (choice_t){g.list, g.idx + (g.m >= 0)});
}

/* Tracer.Trace(SearchPosition) at an unsatisfiable search step (search.go:173).
 * Variables(): the guessed variables, stack order (search.go:205-213).
 * Conflicts(): restated as the identities the failure's conflict analysis
 * reaches, ascending -- for a failed Test/Untest the analysis of its BCP
 * conflict, for a failed Solve() the union over its refutation's analyses
 * (gini's Why, lit_mapping.go:198-207; the reference only logs traces,
 * solve_test.go:302-353, so their content is parity-unpinned).
 * Record: [n, variables..., m, identities...]; an event that does not fit the
 * remaining capacity stops the trace (DP_F_TRACE_TRUNCATED). */
static void trace_event(search_t* h, st_t* s, int from_solve);

/* Do, search.go:158-203.  Returns the result; leaves the guessed variables of
 * the final stack (search.Lits()) in lits[0..*nlits) and pops every guess. */
static int search_do(search_t* h, st_t* s, const backend_t* be, int32_t* lits, int32_t* nlits) {
  const prob_t* p = &s->p;
  h->cap = p->na + p->nch + 2;
  h->dq = xcalloc((size_t)h->cap, sizeof(choice_t));
  h->g = xcalloc((size_t)h->cap, sizeof(guess_t));
  h->head = h->n = h->ng = 0;
  h->result = 0;
  for (int i = 0; i < p->na; ++i) dq_push_back(h, (choice_t){~p->anchors[i], 0});
  /* used[] collects the identities of every conflict analysis of the
   * search's Solve() calls: the derivations of its learned nogoods, and so
   * (with the final root conflict, analysed by the caller) an unsatisfiable
   * identity set when the search fails.  With tracing, used[] holds the
   * current step's identities and uacc[] the rest of the union. */
  memset(s->used, 0, (size_t)p->nid);
  memset(s->uacc, 0, (size_t)p->nid);
  int from_solve = 0;
  for (;;) {
    if (h->n == 0 && h->result == 0) {
      if (s->trace) {
        for (int i = 0; i < p->nid; ++i) s->uacc[i] |= s->used[i];
        memset(s->used, 0, (size_t)p->nid);
      }
      h->result = be->solve(be->u, s);
      h->last_solve = (h->result == 1);
      from_solve = 1;
      if (h->result == R_BUDGET) break;
      if (h->result < 0) h->solve_unsat = 1;
    }
    if (h->result < 0) {
      if (s->trace) trace_event(h, s, from_solve);  /* h.tracer.Trace(h), search.go:173 */
      if (h->ng == 0) break;
      pop_guess(h, s, be);
      from_solve = 0;
      continue;
    }
    if (h->n == 0) break;
    push_guess(h, s, be);
    from_solve = 0;
    if (s->budget_hit) { h->result = R_BUDGET; break; }
  }
  h->final_from_solve = from_solve;
  for (int i = 0; i < p->nid; ++i) s->used[i] |= s->uacc[i];
  /* Value() after a Test()==1 ending reads the full assignment of that scope */
  if (h->result == 1 && !h->last_solve) save_model(s);
  int k = 0;
  for (int i = 0; i < h->ng; ++i)
    if (h->g[i].m >= 0) lits[k++] = h->g[i].m;
  *nlits = k;
  int result = h->result;
  if (result != R_BUDGET)
    while (h->ng > 0) pop_guess(h, s, be);
  free(h->dq);
  free(h->g);
  return result;
}

static void trace_event(search_t* h, st_t* s, int from_solve) {
  if (s->trace_stop) return;
  const prob_t* p = &s->p;
  if (!from_solve) {  /* a trace-only analysis: kept out of the union */
    for (int i = 0; i < p->nid; ++i) s->uacc[i] |= s->used[i];
    memset(s->used, 0, (size_t)p->nid);
    analyze(s);
  }
  int ng = 0, ni = 0;
  for (int i = 0; i < h->ng; ++i) ng += h->g[i].m >= 0;
  for (int i = 0; i < p->nid; ++i) ni += s->used[i];
  if (s->trace_len + 2 + ng + ni > s->trace_cap) {
    s->trace_stop = 1;
    if (!from_solve) memset(s->used, 0, (size_t)p->nid);
    return;
  }
  int32_t* o = s->trace + s->trace_len;
  *o++ = ng;
  for (int i = 0; i < h->ng; ++i)
    if (h->g[i].m >= 0) *o++ = h->g[i].m;
  *o++ = ni;
  for (int i = 0; i < p->nid; ++i)
    if (s->used[i]) *o++ = i;
  s->trace_len += 2 + ng + ni;
  if (!from_solve) memset(s->used, 0, (size_t)p->nid);
}

/* the real backend: our BCP */
static int be_test(void* u, st_t* s, int lit) {
  (void)u;
  if (s->steps + 1 > s->budget) { s->budget_hit = 1; return 0; }
  return test_assume(s, lit);
}
static int be_untest(void* u, st_t* s, int mark) {
  (void)u;
  return untest_to(s, mark);
}

/* A failed Solve() leaves gini with learned clauses that make every scope
 * still holding the refuted guesses inconsistent (search_test.go:50 scripts
 * such Untest() == -1 returns).  Restated: the refutation's conflict analyses
 * collect the guesses they reach; their nogood becomes a learned row. */
static void learn(st_t* s) {
  int n = 0;
  for (int v = 0; v < s->p.nv; ++v) n += s->fg[v];
  if (s->nl >= L_MAX || s->l_off[s->nl] + n > s->lcap) return;
  int at = s->l_off[s->nl];
  for (int v = 0; v < s->p.nv; ++v)
    if (s->fg[v]) s->l_lits[at++] = 2 * v + 1;
  s->l_off[++s->nl] = at;
}

static int be_solve(void* u, st_t* s) {
  (void)u;
  memset(s->fg, 0, (size_t)s->p.nv);
  s->collect_guess = 1;
  int r = dpll(s);
  s->collect_guess = 0;
  if (r == R_SAT) return 1;
  if (r == R_UNSAT) {
    learn(s);
    return -1;
  }
  return R_BUDGET;
}

/* ------------------------------------------------------------------ */
/* NotSatisfiable: deletion-minimal core over identities               */
/* ------------------------------------------------------------------ */

static void reset_all(st_t* s) {
  truncate_to(s, 0);
  s->tlen = s->qhead = 0;
}

/* Complete refutation of the enabled identities; on UNSAT s->used holds the
 * identities of every conflict the refutation met. */
static int refute(st_t* s, const uint8_t* en) {
  reset_all(s);
  /* the search's learned rows are not part of the base formula; the rows
   * this refutation's own Solve() learns are (they prune its search) */
  const int lo = s->learn_lo;
  s->learn_lo = s->nl;
  s->enabled = en;
  memset(s->used, 0, (size_t)s->p.nid);
  s->collect = 1;
  int r;
  if (base_propagate(s) < 0) { analyze(s); r = R_UNSAT; }
  else r = dpll(s);
  s->collect = 0;
  reset_all(s);
  s->enabled = NULL;
  s->learn_lo = lo;
  return r;
}

/* Recursive model rotation (Marques-Silva & Lynce's MUS technique), the walk
 * the kernel makes (solve_kernel.hpp Group::rotate).  A refutation of K \ {c}
 * that finds a model m proves c necessary: m satisfies every identity of K
 * but c.  Flipping one variable of c's row in m and leaving exactly one
 * other identity c' of K violated proves c' necessary the same way, without
 * a refutation; the walk continues from that model.  Only identities that
 * own exactly one row are rotated (their row holds every flipped variable,
 * so the rows that can change are the flipped variable's occurrences).
 * Depth first, positions of the row in order, an explicit stack of at most
 * ROT_DEPTH frames (a necessary identity found below it is marked, not
 * explored).  Criticality only grows as K shrinks (a subset of a satisfiable
 * set is satisfiable), so the deletion pass below ends on the same core as
 * without rotation; only the refutations it skips (and their steps) go. */
enum { ROT_DEPTH = 32 };

static int mval(const uint32_t* m, int v) { return (int)((m[v >> 5] >> (v & 31)) & 1u); }

/* Is row r violated by the total assignment m? */
static int row_violated(const prob_t* p, const uint32_t* m, int r) {
  if (r < p->nc) {
    for (int j = p->clause_off[r]; j < p->clause_off[r + 1]; ++j) {
      const int l = p->clause_lits[j];
      if (mval(m, l >> 1) != (l & 1)) return 0; /* a true literal */
    }
    return 1;
  }
  const int k = r - p->nc;
  int cnt = 0;
  for (int j = p->card_off[k]; j < p->card_off[k + 1]; ++j) cnt += mval(m, p->card_lits[j]);
  return cnt > p->card_bound[k];
}

/* The single row of identity c, or -1 (none, or several). */
static int single_row(const prob_t* p, int c) {
  int row = -1, n = 0;
  for (int r = 0; r < p->nrows; ++r)
    if (row_ident(p, r) == c && n++ == 0) row = r;
  return n == 1 ? row : -1;
}

typedef struct {
  int32_t *off, *rows; /* rows holding variable v: rows[off[v] .. off[v + 1]) */
} occ_t;

static void occ_build(const prob_t* p, occ_t* o) {
  o->off = xcalloc((size_t)p->nv + 1, sizeof(int32_t));
  int32_t* last = xcalloc((size_t)p->nv, sizeof(int32_t));
  for (int v = 0; v < p->nv; ++v) last[v] = -1;
  for (int pass = 0; pass < 2; ++pass) {
    for (int v = 0; v < p->nv; ++v) last[v] = -1;
    for (int r = 0; r < p->nrows; ++r) {
      const int a = r < p->nc ? p->clause_off[r] : p->card_off[r - p->nc];
      const int b = r < p->nc ? p->clause_off[r + 1] : p->card_off[r - p->nc + 1];
      for (int j = a; j < b; ++j) {
        const int v = r < p->nc ? p->clause_lits[j] >> 1 : p->card_lits[j];
        if (last[v] == r) continue;
        last[v] = r;
        if (pass == 0) o->off[v + 1]++;
        else o->rows[o->off[v]++] = r;
      }
    }
    if (pass == 0) {
      for (int v = 0; v < p->nv; ++v) o->off[v + 1] += o->off[v];
      o->rows = xcalloc((size_t)o->off[p->nv], sizeof(int32_t));
    } else {
      for (int v = p->nv; v > 0; --v) o->off[v] = o->off[v - 1];
      o->off[0] = 0;
    }
  }
  free(last);
}

/* m (a model of K \ {c0}) rotated from identity c0; crit marks the
 * identities proven necessary. */
static void rotate(const prob_t* p, const occ_t* o, uint32_t* m, int c0, const uint8_t* K, uint8_t* crit) {
  int fc[ROT_DEPTH], fr[ROT_DEPTH], ft[ROT_DEPTH], d = 0;
  const int r0 = single_row(p, c0);
  if (r0 < 0) return;
  fc[0] = c0; fr[0] = r0; ft[0] = 0; d = 1;
  while (d > 0) {
    const int r = fr[d - 1], t = ft[d - 1];
    const int a = r < p->nc ? p->clause_off[r] : p->card_off[r - p->nc];
    const int b = r < p->nc ? p->clause_off[r + 1] : p->card_off[r - p->nc + 1];
    if (a + t >= b) { /* frame done: undo the flip that opened it */
      if (--d > 0) {
        const int pr = fr[d - 1], pj = (pr < p->nc ? p->clause_off[pr] : p->card_off[pr - p->nc]) + ft[d - 1] - 1;
        const int pv = pr < p->nc ? p->clause_lits[pj] >> 1 : p->card_lits[pj];
        m[pv >> 5] ^= 1u << (pv & 31);
      }
      continue;
    }
    ft[d - 1] = t + 1;
    const int v = r < p->nc ? p->clause_lits[a + t] >> 1 : p->card_lits[a + t];
    m[v >> 5] ^= 1u << (v & 31);
    /* the violated identities of K among the rows holding v (the others
     * keep their values): exactly one, not the frame's own? */
    int lo = INT32_MAX, hi = -1;
    for (int q = o->off[v]; q < o->off[v + 1]; ++q) {
      const int rr = o->rows[q], id = row_ident(p, rr);
      if (!K[id] || !row_violated(p, m, rr)) continue;
      lo = id < lo ? id : lo;
      hi = id > hi ? id : hi;
    }
    const int c = fc[d - 1];
    int opened = 0;
    if (lo == hi && lo != c && !crit[lo]) {
      crit[lo] = 1;
      const int rn = single_row(p, lo);
      if (d < ROT_DEPTH && rn >= 0) { /* continue from this model (v stays flipped) */
        fc[d] = lo; fr[d] = rn; ft[d] = 0; ++d;
        opened = 1;
      }
    }
    if (!opened) m[v >> 5] ^= 1u << (v & 31);
  }
}

static int core_extract(st_t* s, int32_t* core, int32_t* flags) {
  int nid = s->p.nid, len = 0;
  uint8_t* K = xcalloc((size_t)nid, 1);
  uint8_t* K2 = xcalloc((size_t)nid, 1);
  uint8_t* crit = xcalloc((size_t)nid, 1);
  const int nw = (s->p.nv + 31) / 32;
  uint32_t* m = xcalloc((size_t)nw + 1, 4);
  occ_t occ = {NULL, NULL};
  int64_t saved_steps = s->steps;
  s->steps = 0; /* the explanation has its own budget */
  /* start from the identities of the solve's own refutation (used[]: the
   * base conflict, or the search's union), an unsatisfiable set: no fresh
   * refutation of the whole catalog */
  memcpy(K, s->used, (size_t)nid);
  int any = 0;
  for (int id = 0; id < nid; ++id) any |= K[id];
  int r = any ? R_UNSAT : R_BUDGET;
  if (r == R_UNSAT) {
    for (int id = 0; id < nid; ++id) {
      if (!K[id] || crit[id]) continue; /* (a necessary identity stays) */
      memcpy(K2, K, (size_t)nid);
      K2[id] = 0;
      r = refute(s, K2);
      if (r == R_UNSAT) memcpy(K, s->used, (size_t)nid);
      else if (r == R_BUDGET) { *flags |= DP_F_CORE_BUDGET; break; }
      else { /* a model of K \ {id}: id is necessary, and rotation finds others */
        crit[id] = 1;
        if (!occ.off) occ_build(&s->p, &occ);
        memcpy(m, s->model, (size_t)nw * 4);
        rotate(&s->p, &occ, m, id, K, crit);
      }
    }
    for (int id = 0; id < nid; ++id)
      if (K[id]) core[len++] = id;
  } else {
    *flags |= DP_F_CORE_BUDGET; /* verdict stands; explanation empty */
  }
  s->budget_hit = 0;
  s->steps += saved_steps;
  free(K);
  free(K2);
  free(crit);
  free(m);
  free(occ.off);
  free(occ.rows);
  return len;
}

/* ------------------------------------------------------------------ */
/* SAT epilogue, solve.go:86-110                                        */
/* ------------------------------------------------------------------ */

static int epilogue(st_t* s, int32_t* flags, uint32_t* installed) {
  const prob_t* p = &s->p;
  /* the extras, the fixed variables and the installed set are the input's
   * variables only (litMap.Variables, solve.go:88-96); the network's gates
   * stay free */
  int nv = p->nvu, ne = 0;
  int nw = (p->nv + 31) / 32;
  for (int v = 0; v < p->nv; ++v) s->is_extra[v] = 0;
  for (int v = 0; v < nv; ++v) {
    int mv = (s->model[v >> 5] >> (v & 31)) & 1;
    s->is_extra[v] = (uint8_t)(!s->inS[v] && mv);
    ne += s->is_extra[v];
  }
  if (ne == 0) {
    memset(installed, 0, (size_t)nw * 4);
    for (int v = 0; v < nv; ++v)
      if (s->inS[v]) installed[v >> 5] |= 1u << (v & 31);
    return DP_SAT;
  }
  *flags |= DP_F_EPILOGUE;
  /* Untest the base, re-assume constraints + aset + excluded (solve.go:99-104) */
  reset_all(s);
  if (base_propagate(s) < 0) return DP_ERROR;
  int rd = ++s->round;
  for (int v = 0; v < nv; ++v) {
    if (s->is_extra[v]) continue;
    int want = s->inS[v] ? 1 : -1;
    if (s->val[v] == -want) return DP_ERROR;
    if (s->val[v] == 0) assign(s, 2 * v + (want < 0), R_DECISION, rd);
  }
  if (propagate(s) < 0) return DP_ERROR;
  int mark = s->tlen, f = 0;
  for (int v = 0; v < nv; ++v) f += s->is_extra[v] && s->val[v] > 0;
  s->extra_mode = 1;
  for (int w = f; w <= ne; ++w) {
    truncate_to(s, mark);
    s->extra_w = w;
    if (propagate(s) < 0) continue;
    int r = dpll(s);
    if (r == R_SAT) {
      s->extra_mode = 0;
      memset(installed, 0, (size_t)nw * 4);
      for (int v = 0; v < nv; ++v)
        if ((s->model[v >> 5] >> (v & 31)) & 1) installed[v >> 5] |= 1u << (v & 31);
      return DP_SAT;
    }
    if (r == R_BUDGET) { s->extra_mode = 0; return DP_INCOMPLETE; }
  }
  s->extra_mode = 0;
  return DP_ERROR; /* "unexpected internal error", solve.go:113 */
}

/* ------------------------------------------------------------------ */
/* solver.Solve, solve.go:53-119                                        */
/* ------------------------------------------------------------------ */

int oracle_solve(const int32_t* rec, int64_t budget, int32_t* flags, uint32_t* installed,
                 int32_t* core, int32_t* core_len, int64_t* steps) {
  return oracle_solve_traced(rec, budget, flags, installed, core, core_len, steps, NULL, 0, NULL);
}

int oracle_solve_traced(const int32_t* rec, int64_t budget, int32_t* flags, uint32_t* installed,
                        int32_t* core, int32_t* core_len, int64_t* steps, int32_t* trace,
                        int32_t trace_cap, int32_t* trace_len) {
  st_t s;
  st_init(&s, rec);
  s.budget = budget > 0 ? budget : (1 << 16);
  s.trace = trace;
  s.trace_cap = trace_cap;
  int nv = s.p.nv, nw = (nv + 31) / 32;
  *flags = 0;
  *core_len = 0;
  memset(installed, 0, (size_t)nw * 4);
  int status;
  int base = base_propagate(&s);
  if (base < 0) {
    *flags |= DP_F_BASE_UNSAT;
    status = DP_UNSAT;
    memset(s.used, 0, (size_t)s.p.nid);
    analyze(&s); /* the base conflict's identities start the explanation */
  } else if (base == 1) {
    *flags |= DP_F_SEARCH_SKIPPED;
    save_model(&s);
    status = epilogue(&s, flags, installed);
  } else {
    search_t h;
    memset(&h, 0, sizeof(h));
    backend_t be = {be_test, be_untest, be_solve, NULL};
    int32_t* lits = xcalloc((size_t)nv, sizeof(int32_t));
    int32_t nl = 0;
    int r = search_do(&h, &s, &be, lits, &nl);
    if (h.class_b) *flags |= DP_F_CLASS_B;
    if (h.solve_unsat) *flags |= DP_F_SOLVE_UNSAT;
    if (r == R_BUDGET) {
      *flags |= DP_F_BUDGET;
      status = DP_INCOMPLETE;
    } else if (r < 0) {
      status = DP_UNSAT;
      if (!h.final_from_solve) analyze(&s); /* the final root conflict (an Untest) */
    } else {
      memset(s.inS, 0, (size_t)nv);
      for (int i = 0; i < nl; ++i) s.inS[lits[i]] = 1;
      status = epilogue(&s, flags, installed);
      if (status == DP_INCOMPLETE) *flags |= DP_F_BUDGET;
    }
    free(lits);
  }
  if (status == DP_UNSAT) *core_len = core_extract(&s, core, flags);
  if (steps) *steps = s.steps;
  if (trace_len) *trace_len = s.trace_len;
  if (s.trace_stop) *flags |= DP_F_TRACE_TRUNCATED;
  st_free(&s);
  return status;
}

int oracle_refute(const int32_t* rec, const uint8_t* enabled, int64_t budget) {
  st_t s;
  st_init(&s, rec);
  s.budget = budget > 0 ? budget : (1 << 20);
  int r = refute(&s, enabled);
  st_free(&s);
  return r == R_UNSAT ? -1 : (r == R_SAT ? 1 : 0);
}

/* ------------------------------------------------------------------ */
/* scripted backend (FakeS)                                            */
/* ------------------------------------------------------------------ */

typedef struct {
  const int32_t *tr, *ur;
  int nt, nu, it, iu, depth;
} script_t;

static int sc_test(void* u, st_t* s, int lit) {
  (void)s; (void)lit;
  script_t* c = u;
  c->depth++;
  int r = c->it < c->nt ? c->tr[c->it] : 0;
  c->it++;
  return r;
}
static int sc_untest(void* u, st_t* s, int mark) {
  (void)s; (void)mark;
  script_t* c = u;
  c->depth--;
  int r = c->iu < c->nu ? c->ur[c->iu] : 0;
  c->iu++;
  return r;
}
static int sc_solve(void* u, st_t* s) { (void)u; (void)s; return 0; }

int oracle_search_scripted(const int32_t* rec, const int32_t* test_ret, int32_t n_test,
                           const int32_t* untest_ret, int32_t n_untest, int32_t* out_result,
                           int32_t* out_lits, int32_t* out_nlits, int32_t* out_depth) {
  st_t s;
  st_init(&s, rec);
  s.budget = 1 << 20;
  script_t sc = {test_ret, untest_ret, n_test, n_untest, 0, 0, 0};
  backend_t be = {sc_test, sc_untest, sc_solve, &sc};
  search_t h;
  memset(&h, 0, sizeof(h));
  *out_result = search_do(&h, &s, &be, out_lits, out_nlits);
  *out_depth = sc.depth;
  st_free(&s);
  return 0;
}

/* ------------------------------------------------------------------ */
/* batch (CPU baseline)                                                 */
/* ------------------------------------------------------------------ */

typedef struct {
  int32_t n;
  const int64_t* rec_off;
  const int32_t* rec;
  int64_t budget;
  int8_t* status;
  int32_t* flags;
  uint32_t* installed;
  const int64_t* inst_off;
  int32_t* core;
  const int64_t* core_off;
  int32_t* core_len;
  int64_t* steps;
  int32_t* trace; /* NULL: no tracing; else trace_cap words per problem */
  int32_t trace_cap;
  int32_t* trace_len;
  int32_t next; /* shared work counter */
  pthread_mutex_t mu;
} batch_t;

static void* batch_worker(void* arg) {
  batch_t* b = arg;
  for (;;) {
    pthread_mutex_lock(&b->mu);
    int i0 = b->next;
    b->next += 16;
    pthread_mutex_unlock(&b->mu);
    if (i0 >= b->n) break;
    int i1 = i0 + 16 < b->n ? i0 + 16 : b->n;
    for (int i = i0; i < i1; ++i) {
      int64_t st = 0;
      b->status[i] = (int8_t)oracle_solve_traced(
          b->rec + b->rec_off[i], b->budget, &b->flags[i], b->installed + b->inst_off[i],
          b->core + b->core_off[i], &b->core_len[i], &st,
          b->trace ? b->trace + (int64_t)b->trace_cap * i : NULL, b->trace_cap,
          b->trace ? &b->trace_len[i] : NULL);
      if (b->steps) b->steps[i] = st;
    }
  }
  return NULL;
}

int oracle_solve_batch(int32_t n, const int64_t* rec_off, const int32_t* rec, int64_t budget,
                       int32_t nthreads, int8_t* status, int32_t* flags, uint32_t* installed,
                       const int64_t* inst_off, int32_t* core, const int64_t* core_off,
                       int32_t* core_len, int64_t* steps) {
  return oracle_solve_batch_traced(n, rec_off, rec, budget, nthreads, status, flags, installed,
                                   inst_off, core, core_off, core_len, steps, NULL, 0, NULL);
}

int oracle_solve_batch_traced(int32_t n, const int64_t* rec_off, const int32_t* rec,
                              int64_t budget, int32_t nthreads, int8_t* status, int32_t* flags,
                              uint32_t* installed, const int64_t* inst_off, int32_t* core,
                              const int64_t* core_off, int32_t* core_len, int64_t* steps,
                              int32_t* trace, int32_t trace_cap, int32_t* trace_len) {
  batch_t b = {n, rec_off, rec, budget, status, flags, installed, inst_off, core, core_off,
               core_len, steps, trace, trace_cap, trace_len, 0, PTHREAD_MUTEX_INITIALIZER};
  if (nthreads < 1) nthreads = 1;
  pthread_t* th = xcalloc((size_t)nthreads, sizeof(pthread_t));
  for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, batch_worker, &b);
  for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
  free(th);
  return 0;
}

/* Model check: every clause and card row satisfied by the installed set
 * (variables not installed are false).  Returns the first violated row, or -1. */
int oracle_check_model(const int32_t* rec, const uint32_t* installed) {
  prob_t p;
  int32_t* wide;
  rec = widen(rec, &wide);
  parse(&p, rec);
  for (int r = 0; r < p.nc; ++r) {
    int sat = 0;
    for (int j = p.clause_off[r]; j < p.clause_off[r + 1]; ++j) {
      int l = p.clause_lits[j], v = l >> 1;
      int x = (installed[v >> 5] >> (v & 31)) & 1;
      if (x != (l & 1)) { sat = 1; break; }
    }
    if (!sat) { free(wide); return r; }
  }
  for (int k = 0; k < p.nk; ++k) {
    int cnt = 0;
    for (int j = p.card_off[k]; j < p.card_off[k + 1]; ++j) {
      int v = p.card_lits[j];
      cnt += (installed[v >> 5] >> (v & 31)) & 1;
    }
    if (cnt > p.card_bound[k]) { free(wide); return p.nc + k; }
  }
  free(wide);
  return -1;
}

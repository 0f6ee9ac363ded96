/*
 * deppy_hip.h — C-ABI of the MI355X-native batched dependency-resolution engine.
 *
 * This is the drop-in boundary for the `pkg/sat` hot path of timflannagan/deppy.
 * The reference path is in-process Go:
 *
 *   sat.NewSolver(sat.WithInput(vars), sat.WithTracer(t))   pkg/sat/solve.go:121-146
 *   (Solver).Solve(ctx) ([]Variable, error)                  pkg/sat/solve.go:32-34, 53-119
 *
 * A Go caller (pkg/solver/solver.go:42-47) reaches this library through a thin
 * cgo shim.  Only plain pointers, sizes and int32/int64 arrays
 * cross the boundary; no Go pointers are retained and no torch types appear.
 *
 * Three layers, each usable on its own:
 *
 *   1. Wire format  (dp_wire)  — the reference's []Variable with its
 *      []Constraint lists, flattened into arrays of string-table indices.
 *      dp_lower() restates newLitMapping (pkg/sat/lit_mapping.go:40-77) and
 *      constraint Apply (pkg/sat/constraints.go:54-204) and produces...
 *
 *   2. Lowered records (one int32 record per problem, layout below) — the
 *      format the GPU consumes.  A caller that lowers on its own side (the
 *      survey's Go-side lowering) can hand records straight to...
 *
 *   3. dp_solve / dp_upload+dp_run+dp_download — batched resolution on one or
 *      more MI355X devices.  One wavefront solves one problem.
 *
 * Result statuses map onto the reference's return values:
 *   DP_SAT        -> ([]Variable in input order, nil)          solve.go:105-110, lit_mapping.go:176-184
 *   DP_UNSAT      -> (nil, NotSatisfiable{...})                solve.go:114-115, lit_mapping.go:198-207
 *   DP_INCOMPLETE -> (nil, ErrIncomplete)                       solve.go:14, 118
 *   DP_ERROR      -> (nil, <error>)                              solve.go:54-61, 113
 */
#ifndef DEPPY_HIP_H
#define DEPPY_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DP_ABI_VERSION 1

/* ------------------------------------------------------------------------ */
/* 1. Wire format                                                            */
/* ------------------------------------------------------------------------ */

/* Constraint kinds: pkg/sat/constraints.go:74 (Mandatory), :100 (Prohibited),
 * :138 (Dependency), :163 (Conflict), :199 (AtMost). */
enum dp_kind {
  DP_MANDATORY = 1,
  DP_PROHIBITED = 2,
  DP_DEPENDENCY = 3, /* args = candidate identifiers in preference order */
  DP_CONFLICT = 4,   /* args = exactly one identifier                    */
  DP_ATMOST = 5      /* args = identifiers; n = bound                     */
};

/* A batch of independent problems.  Every problem is the []Variable handed to
 * sat.WithInput (solve.go:133).  Identifiers are byte strings in a shared
 * string table; they are compared by bytes within one problem. */
/* Offsets are absolute indices into the arrays they point into, so a batch
 * may be a range of problems of a larger batch: prob_var_off pointing at
 * the range's first offset, every other array the larger batch's own (no
 * rebasing; prob_var_off[0] is then the range's first variable). */
typedef struct dp_wire {
  int32_t n_problems;
  const int64_t* prob_var_off; /* [n_problems+1] -> variables          */
  const int64_t* var_id;       /* [n_vars]   string index of Identifier  */
  const int64_t* var_con_off;  /* [n_vars+1] -> constraints             */
  const int32_t* con_kind;     /* [n_cons]   enum dp_kind               */
  const int32_t* con_n;        /* [n_cons]   AtMost bound (else ignored) */
  const int64_t* con_arg_off;  /* [n_cons+1] -> con_arg                  */
  const int64_t* con_arg;      /* [n_args]   string index               */
  int64_t n_strs;
  const int64_t* str_off;      /* [n_strs+1] -> str_bytes               */
  const char* str_bytes;
  int32_t interned; /* 1: equal bytes <=> equal string index (fast path) */
} dp_wire;

/* Per-problem lowering outcome (dp_lowered_error). */
enum dp_lower_err {
  DP_LOWER_OK = 0,
  DP_LOWER_DUPLICATE = 1, /* NewSolver error: DuplicateIdentifier, lit_mapping.go:12-16,52-54 */
  DP_LOWER_LOOKUP = 2     /* Solve error: "%d errors encountered: %s", lit_mapping.go:86,119-128 */
};

/* ------------------------------------------------------------------------ */
/* 2. Lowered record (one per problem, int32 words, problem-local indices)   */
/* ------------------------------------------------------------------------ */
/*
 *  Literal encoding: lit = 2*v + neg  (v = variable index in INPUT ORDER,
 *  neg = 1 for the negated literal).  Card / choice / anchor entries are
 *  plain variable indices.
 *
 *  Rows: clause rows 0..nc-1 then card rows nc..nc+nk-1 (one "row id" space).
 *  Every row carries an identity id in 0..nid-1.  An identity is one assumed
 *  constraint literal of the reference (constraints[m], lit_mapping.go:69-72):
 *  constraints whose gate literal coincides share one identity and one set of
 *  rows; NotSatisfiable reports identities.
 *
 *  header[DP_H_SIZE], then, in this order:
 *    clause_off[nc+1]      offsets into clause_lits (relative)
 *    clause_lits[ncl]
 *    clause_id[nc]
 *    card_off[nk+1]        offsets into card_lits (relative)
 *    card_lits[nkl]        variable indices, duplicates kept (multiplicity)
 *    card_bound[nk]        at most card_bound[k] of the positions are true
 *    card_id[nk]
 *    var_choice_off[nv+1]  choice rows of variable v: [var_choice_off[v], var_choice_off[v+1])
 *    choice_off[nch+1]     offsets into choice_lits (relative)
 *    choice_lits[nchl]     candidate variables in preference order (constraint.Order(), search.go:60-69)
 *    anchors[na]           variables with a Mandatory constraint, input order (lit_mapping.go:163-174)
 */
#define DP_REC_MAGIC 0x31525044 /* "DPR1" little-endian */
enum dp_rec_header {
  DP_H_MAGIC = 0,
  DP_H_NV = 1,
  DP_H_NC = 2,
  DP_H_NK = 3,
  DP_H_NCH = 4,
  DP_H_NA = 5,
  DP_H_NID = 6,
  DP_H_NCL = 7,
  DP_H_NKL = 8,
  DP_H_NCHL = 9,
  DP_H_WORDS = 10, /* total record length in int32 words, header included */
  /* 0, or the input's variable count when nv also counts auxiliary variables
   * nvu..nv-1: the gates of an AtMost that lists a variable more than once,
   * lowered as gini's sorting network (constraints.go:180-186) with its
   * Tseitin rows.  They have no choices, are never installed and are never
   * SAT-epilogue extras; 0 < nvu <= nv. */
  DP_H_NVU = 11,
  DP_H_SIZE = 16
};

/* Offsets (in int32 words from the record start) of each array. */
typedef struct dp_rec_layout {
  int32_t clause_off, clause_lits, clause_id;
  int32_t card_off, card_lits, card_bound, card_id;
  int32_t var_choice_off, choice_off, choice_lits, anchors;
  int32_t words;
} dp_rec_layout;

static inline dp_rec_layout dp_rec_layout_of(const int32_t* h) {
  dp_rec_layout L;
  int32_t o = DP_H_SIZE;
  L.clause_off = o;     o += h[DP_H_NC] + 1;
  L.clause_lits = o;    o += h[DP_H_NCL];
  L.clause_id = o;      o += h[DP_H_NC];
  L.card_off = o;       o += h[DP_H_NK] + 1;
  L.card_lits = o;      o += h[DP_H_NKL];
  L.card_bound = o;     o += h[DP_H_NK];
  L.card_id = o;        o += h[DP_H_NK];
  L.var_choice_off = o; o += h[DP_H_NV] + 1;
  L.choice_off = o;     o += h[DP_H_NCH] + 1;
  L.choice_lits = o;    o += h[DP_H_NCHL];
  L.anchors = o;        o += h[DP_H_NA];
  L.words = o;
  return L;
}

/* Header word DP_H_FMT selects the body's form.  DP_FMT_I32: every word after
 * the header is an int32 (DP_H_WORDS words in all).  DP_FMT_U16: every word
 * after the header is a uint16, two per int32 word (low half first), so the
 * record occupies dp_rec_phys_words() int32 words; this is the form the GPU
 * stages for one-wavefront problems, and dp_lower_into(DP_LOWER_NARROW)
 * emits it for every record that fits (dp_rec_fits16), so that staging is a
 * copy.  Offsets (rec_off) always count int32 words.
 *
 * DP_FMT_P16 (dp_lower_into DP_LOWER_PACKED): the 16-bit form with every
 * offsets array sent as byte lengths and the row identities as a bit mask,
 * about a fifth fewer bytes to cross PCIe than DP_FMT_U16.  After the header:
 *   uint16 clause_lits[ncl], card_lits[nkl], card_bound[nk], choice_lits[nchl],
 *          anchors[na]
 *   zero padding to a 16-byte boundary (from the body's start)
 *   uint8  clause_len[nc], card_len[nk], var_choice_len[nv], choice_len[nch]
 *          (the differences of the offsets arrays, each below 256)
 *   uint8  card_mask[(nid+7)/8]: bit i (LSB first) set iff identity i is an
 *          AtMost row's.  Every identity has exactly one row (nid == nc + nk)
 *          and each row kind lists its identities in ascending order, so
 *          clause_id is the clear bits in order and card_id the set ones.
 * The lengths and the mask together are at most DP_P16_TAIL_MAX bytes (the
 * kernel decodes them from one 16-byte load per lane).  DP_H_WORDS stays the
 * int32 form's length.  dp_rec_widen gives the int32 form of any record.
 *
 * DP_FMT_P16D: DP_FMT_P16 with the choice lists implied by the record's
 * dependency rows (dp_lower_into DP_LOWER_PACKED emits it when they are;
 * config 2's catalogs cross PCIe in about a third fewer bytes).  A
 * dependency row is a clause row of two or more literals whose first literal
 * is negative and every other one positive: Dependency(s; d1..dn) lowers to
 * (~s d1 .. dn), and no other constraint gives that shape.  src[k] == 0:
 * choice list k is the variables of the next dependency row (in row order)
 * after its first literal; src[k] = d > 0: list k repeats list k - d, which
 * took a row (a Dependency whose gate an earlier one of the same subject
 * already emitted).  Every dependency row is taken once; the lists'
 * subjects (first literal's variable) never decrease and var_choice_off
 * counts them per subject; nch and nchl are the header's.  After the header:
 *   uint16 clause_lits[ncl], card_lits[nkl], card_bound[nk], anchors[na]
 *   zero padding to a 16-byte boundary (from the body's start)
 *   uint8  clause_len[nc], card_len[nk], src[nch], card_mask[(nid+7)/8]
 *
 * DP_FMT_I32W: the int32 form followed by its watch lists, a form a problem
 * solved by a multi-wave workgroup may be staged in as it lies.  dp_lower_into
 * emits multi-wave records as DP_FMT_I32 (the device builds their watch
 * lists: in the solving workgroup up to 2048 variables, by grid-wide passes
 * before the launch above it); a caller that has the lists may send this form
 * instead, and the kernel checks their bounds:
 *   int32 w_off[2nv+1]  rows literal l wakes: w[w_off[l] .. w_off[l+1]) (the
 *                       clauses holding ~l; when l = 2v is positive, the
 *                       AtMost rows holding v, once each)
 *   int32 w[ncl+nkl]    row ids, ascending within a list (entries past
 *                       w_off[2nv] unused)
 * The kernel checks their bounds; that they list exactly those rows is the
 * producer's contract (dp_lower_into builds them). */
enum { DP_H_FMT = 13 };
enum { DP_FMT_I32 = 0, DP_FMT_U16 = 1, DP_FMT_P16 = 3, DP_FMT_I32W = 4, DP_FMT_P16D = 5, DP_FMT_P8D = 6 };
enum { DP_P16_TAIL_MAX = 1024 };

/* DP_FMT_P8D: DP_FMT_P16D with every variable in 8 bits plus bit planes, for
 * records of at most 512 variables (dp_lower_into DP_LOWER_PACKED emits it
 * where it applies; config 2's catalogs cross PCIe in about 45% fewer bytes
 * than DP_FMT_P16D).  Header word DP_H_P8 holds its flags (bits 0-7) and the
 * body's byte count (bits 8-31).  After the header,
 * byte-addressed from the body's start, no padding inside:
 *   uint8 clause_var[ncl]   the variable of each clause literal, low 8 bits
 *   uint8 card_var[nkl], anchor_var[na]                     (low 8 bits)
 *   uint8 card_bound[nk]    absent with DP_P8_B1 (every bound is 1)
 *   bits  clause_neg[ncl]   bit j (LSB first) set iff clause literal j is negative
 *   bits  clause_hi[ncl], card_hi[nkl], anchor_hi[na]
 *                           bit 8 of each variable; present only with DP_P8_HI
 *   lengths                 clause_len[nc] then card_len[nk], a byte each, or
 *                           with DP_P8_NIB a nibble each (low nibble first,
 *                           ceil((nc+nk)/2) bytes)
 *   bits  src_nz[nch]       bit k set iff DP_FMT_P16D's src[k] != 0
 *   uint8 src_val[...]      those src[k], in list order
 *   bits  card_mask[nid]    as DP_FMT_P16's
 * Each bit array is ceil(n/8) bytes.  A literal is 2 * variable + negative.
 * The record decodes to exactly DP_FMT_P16D's arrays (dp_rec_widen). */
enum { DP_H_P8 = 14 };
enum { DP_P8_B1 = 1, DP_P8_HI = 2, DP_P8_NIB = 4 };
enum { DP_P8_MAX_VARS = 512 };
static inline int64_t dp_p8_bits(int64_t n) { return (n + 7) >> 3; }
/* Byte offsets of DP_FMT_P8D's sections (from the body's start). */
typedef struct dp_p8_layout {
  int64_t cvar, kvar, avar, bound, neg, chi, khi, ahi, lens, srcnz, srcval, mask;
} dp_p8_layout;
static inline dp_p8_layout dp_p8_layout_of(const int32_t* h) {
  dp_p8_layout L;
  const int32_t f = h[DP_H_P8];
  const int64_t ncl = h[DP_H_NCL], nkl = h[DP_H_NKL], na = h[DP_H_NA], nk = h[DP_H_NK], nc = h[DP_H_NC];
  int64_t o = 0;
  L.cvar = o;  o += ncl;
  L.kvar = o;  o += nkl;
  L.avar = o;  o += na;
  L.bound = o; o += (f & DP_P8_B1) ? 0 : nk;
  L.neg = o;   o += dp_p8_bits(ncl);
  L.chi = o;   o += (f & DP_P8_HI) ? dp_p8_bits(ncl) : 0;
  L.khi = o;   o += (f & DP_P8_HI) ? dp_p8_bits(nkl) : 0;
  L.ahi = o;   o += (f & DP_P8_HI) ? dp_p8_bits(na) : 0;
  L.lens = o;  o += (f & DP_P8_NIB) ? (nc + nk + 1) / 2 : nc + nk;
  L.srcnz = o; o += dp_p8_bits(h[DP_H_NCH]);
  L.srcval = o;
  L.mask = -1; /* after the src values: their count is the popcount of src_nz */
  return L;
}

/* DP_FMT_P16 / DP_FMT_P16D (the packed forms): uint16 words before the
 * padding, byte offset of the lengths (from the body's start), and bytes of
 * lengths plus mask. */
static inline int dp_fmt_packed(int32_t fmt) { return fmt == DP_FMT_P16 || fmt == DP_FMT_P16D || fmt == DP_FMT_P8D; }
/* the packed forms whose choice lists are implied by the dependency rows */
static inline int dp_fmt_derived(int32_t fmt) { return fmt == DP_FMT_P16D || fmt == DP_FMT_P8D; }
static inline int64_t dp_p16_nu16(const int32_t* h) {
  return (int64_t)h[DP_H_NCL] + h[DP_H_NKL] + h[DP_H_NK] + h[DP_H_NA] +
         (dp_fmt_derived(h[DP_H_FMT]) ? 0 : h[DP_H_NCHL]);
}
static inline int64_t dp_p16_tail_at(const int32_t* h) { return (2 * dp_p16_nu16(h) + 15) & ~(int64_t)15; }
/* (DP_FMT_P8D: the DP_FMT_P16D tail its sections decode to) */
static inline int64_t dp_p16_tail_bytes(const int32_t* h) {
  return (int64_t)h[DP_H_NC] + h[DP_H_NK] + h[DP_H_NCH] + ((int64_t)h[DP_H_NID] + 7) / 8 +
         (dp_fmt_derived(h[DP_H_FMT]) ? 0 : (int64_t)h[DP_H_NV]);
}
/* DP_FMT_P8D body bytes up to the src values (their count is in the body:
 * the popcount of src_nz), and the whole body given that count. */
static inline int64_t dp_p8_body_bytes(const int32_t* h, int64_t n_src_val) {
  return dp_p8_layout_of(h).srcval + n_src_val + dp_p8_bits(h[DP_H_NID]);
}

/* Words of the record as it lies (for DP_FMT_P8D: header word DP_H_P8's
 * bits 8.. hold the body's byte count). */
static inline int64_t dp_rec_phys_words(const int32_t* h) {
  if (h[DP_H_FMT] == DP_FMT_U16) return DP_H_SIZE + ((int64_t)h[DP_H_WORDS] - DP_H_SIZE + 1) / 2;
  if (h[DP_H_FMT] == DP_FMT_P8D) return DP_H_SIZE + (((int64_t)((uint32_t)h[DP_H_P8] >> 8)) + 3) / 4;
  if (dp_fmt_packed(h[DP_H_FMT])) return DP_H_SIZE + (dp_p16_tail_at(h) + dp_p16_tail_bytes(h) + 3) / 4;
  if (h[DP_H_FMT] == DP_FMT_I32W)
    return (int64_t)h[DP_H_WORDS] + 2 * (int64_t)h[DP_H_NV] + 1 + h[DP_H_NCL] + h[DP_H_NKL];
  return (int64_t)h[DP_H_WORDS];
}

/* Does every index the record holds, and every value the solve stores per
 * variable or row, fit 16 bits (below the kernel's reserved reason codes)? */
static inline int dp_rec_fits16(const int32_t* h) {
  const int32_t nv = h[DP_H_NV];
  return h[DP_H_WORDS] < 65000 && nv < 16000 && h[DP_H_NID] < 65000 &&
         h[DP_H_NC] + h[DP_H_NK] + 64 + nv < 65000 && h[DP_H_NA] + h[DP_H_NCH] < 65000 &&
         h[DP_H_NCL] + h[DP_H_NKL] < 65000;
}

/* Validate one record of any form (bounds of every index).  Returns 0 if
 * well formed.  The solve checks every record the same way on the device, so
 * a malformed record yields DP_ERROR with DP_F_MALFORMED, never a fault. */
int dp_rec_validate(const int32_t* rec, int64_t words);
/* The int32 form (DP_FMT_I32, DP_H_WORDS words into out) of a record of any
 * form that occupies at most `avail` words.  Returns 0, or < 0 when the
 * header or a packed form's length / mask (or DP_FMT_P16D's implied choice
 * lists) is inconsistent. */
int dp_rec_widen(const int32_t* rec, int64_t avail, int32_t* out);

/* ------------------------------------------------------------------------ */
/* Lowering: wire -> records                                                  */
/* ------------------------------------------------------------------------ */

typedef struct dp_lowered dp_lowered; /* host-owned, opaque */

/* Lower a wire batch (restates newLitMapping, lit_mapping.go:40-77).  Never
 * fails per problem: DuplicateIdentifier / lookup errors are recorded per
 * problem (dp_lowered_error) and such problems get an empty record.
 * Returns 0, or -1 on malformed input (text in dp_last_global_error()). */
int dp_lower(const dp_wire* wire, dp_lowered** out);
/* dp_lower into an existing result, reusing its storage (a serving loop
 * lowers batch after batch without allocating).  flags: DP_LOWER_NARROW emits
 * every record that fits 16 bits in the DP_FMT_U16 form (the staged form:
 * half the bytes to write, to stage and to cross PCIe) and starts every
 * record on a 16-byte boundary (zero padding between records, counted in
 * rec_off); DP_LOWER_PINNED keeps the records in page-locked host memory
 * when a HIP device is present (dp_lowered_pinned).  A batch of both is
 * copied to the device by DMA from where it lies: dp_submit stages only
 * chunks that need another form.  DP_LOWER_PACKED (with DP_LOWER_NARROW)
 * emits the DP_FMT_P16 form for the records that allow it, the DP_FMT_U16
 * form for the other 16-bit ones.  With DP_LOWER_NARROW, records of problems
 * solved by multi-wave workgroups (too large for one wavefront's LDS image,
 * or beyond 16 bits) take the DP_FMT_I32W form.  Returns 0 or -1. */
/* DP_LOWER_PACKED emits DP_FMT_P8D for the DP_FMT_P16D records that allow
 * it; DP_LOWER_NO_P8 keeps them DP_FMT_P16D (tests, A/B). */
enum { DP_LOWER_NARROW = 1, DP_LOWER_PINNED = 2, DP_LOWER_PACKED = 4, DP_LOWER_NO_P8 = 8 };
int dp_lower_into(const dp_wire* wire, int32_t flags, dp_lowered* lw);
dp_lowered* dp_lowered_new(void); /* an empty result for dp_lower_into */
void dp_lowered_free(dp_lowered* lw);
int32_t dp_lowered_pinned(const dp_lowered* lw); /* 1: the records are page-locked */
int32_t dp_lowered_num_problems(const dp_lowered* lw);
/* Problems of the last lowering that went through the full And-inverter
 * graph instead of the canonical identity keys (measurement; lower.cpp). */
int64_t dp_lowered_exact_count(const dp_lowered* lw);
const int64_t* dp_lowered_rec_off(const dp_lowered* lw); /* [P+1] */
const int32_t* dp_lowered_rec(const dp_lowered* lw);
/* Identity -> reported AppliedConstraint (last writer, lit_mapping.go:69-72):
 * ident_var[ident_off[p] + i] = variable index, ident_con[...] = index of the
 * constraint in that variable's Constraints(). */
const int64_t* dp_lowered_ident_off(const dp_lowered* lw); /* [P+1] */
const int32_t* dp_lowered_ident_var(const dp_lowered* lw);
const int32_t* dp_lowered_ident_con(const dp_lowered* lw);
/* enum dp_lower_err; *msg (may be NULL) receives the reference's error text. */
int32_t dp_lowered_error(const dp_lowered* lw, int32_t p, const char** msg);
/* Every problem's enum dp_lower_err at once (err[n_problems]); returns the
 * number of problems with an error (fetch their text with dp_lowered_error). */
int32_t dp_lowered_errors(const dp_lowered* lw, int32_t* err);

/* ------------------------------------------------------------------------ */
/* Lowering on the device: compact wire -> records                          */
/* ------------------------------------------------------------------------ */
/* The compact wire: dp_wire's content in about 30-45% of its bytes, the form
 * that crosses PCIe to the device lowering.  Always interned (equal string
 * index <=> equal identifier).  Per problem, absolute offsets of its first
 * variable, constraint and argument; per variable and per constraint a
 * 16-bit count instead of an offset; a constraint's kind and AtMost bound in
 * one word.  Problem p's constraints are the counts of its variables in
 * order (their sum is prob_con_off[p+1] - prob_con_off[p]), and likewise its
 * arguments.  The string table is read only for error texts. */
typedef struct dp_wire32 {
  int32_t n_problems;
  const int32_t* prob_var_off;  /* [n_problems+1] -> variables            */
  const int32_t* prob_con_off;  /* [n_problems+1] -> constraints          */
  const int32_t* prob_arg_off;  /* [n_problems+1] -> arguments            */
  const int32_t* var_id;        /* [n_vars]  string index of Identifier
                                   (NULL when var_id16 is given)          */
  const uint16_t* var_ncon;     /* [n_vars]  constraints of the variable   */
  const int32_t* con_kn;        /* [n_cons]  enum dp_kind | bound << 3 (the
                                   AtMost bound, arithmetic shift)        */
  const uint16_t* con_nargs;    /* [n_cons]  arguments of the constraint   */
  const int32_t* con_arg;       /* [n_args]  string index (NULL when
                                   con_arg16 is given)                    */
  /* With at most 65,536 strings, the string indices in 16 bits instead
   * (about a third fewer bytes on config 2); both or neither. */
  const uint16_t* var_id16;     /* [n_vars]                                */
  const uint16_t* con_arg16;    /* [n_args]                                */
  int64_t n_strs;
  const int64_t* str_off;       /* [n_strs+1] -> str_bytes (error texts)   */
  const char* str_bytes;
} dp_wire32;

/* The device lowering of a context's first device: a stream, device buffers
 * and page-locked staging of its own, grown on demand and reused by every
 * call (a serving loop keeps one).  NULL on failure (dp_last_error(ctx)). */
typedef struct dp_ctx dp_ctx;
typedef struct dp_dlower dp_dlower;
dp_dlower* dp_dlower_new(dp_ctx* ctx);
void dp_dlower_free(dp_dlower* d);
/* dp_lower_into on the GPU: the same dp_lowered, byte for byte, for flags
 * DP_LOWER_NARROW | DP_LOWER_PACKED (| DP_LOWER_PINNED).  One wavefront per
 * problem runs the canonical-key lowering (lower.cpp lower_fast) in LDS and
 * writes the DP_FMT_P8D record; a problem it does not take (one the keys
 * cannot decide, an error to report, a record in another form, past the
 * kernel's sizes) is flagged and lowered on the host pool, and its record is
 * spliced in.  Other flags lower every problem on the host.  Synchronous.
 * Returns 0, or -1 (text in dp_last_global_error()). */
int dp_lower_device(dp_dlower* d, const dp_wire32* wire, int32_t flags, dp_lowered* lw);
/* Problems of the last dp_lower_device call lowered on the host. */
int64_t dp_dlower_host_count(const dp_dlower* d);
/* Page-locked host memory for wire batches (the H2D copy then runs by DMA
 * from where they lie).  NULL without a device. */
void* dp_host_alloc(int64_t bytes);
void dp_host_free(void* p);

/* ------------------------------------------------------------------------ */
/* 3. Solving                                                                 */
/* ------------------------------------------------------------------------ */

enum dp_status { DP_SAT = 1, DP_UNSAT = -1, DP_INCOMPLETE = 0, DP_ERROR = -2 };

/* Per-problem flag bits (class mix). */
enum dp_flag {
  DP_F_SEARCH_SKIPPED = 1 << 0, /* base Test returned 1 (solve.go:80)                  */
  DP_F_CLASS_B = 1 << 1,        /* an exhausted choice was guessed (A.6.3): gini-unpinned */
  DP_F_SOLVE_UNSAT = 1 << 2,    /* search Solve() returned -1 at least once              */
  DP_F_EPILOGUE = 1 << 3,       /* SAT epilogue had extras to minimise (solve.go:86-110) */
  DP_F_BASE_UNSAT = 1 << 4,     /* base Test returned -1                                 */
  DP_F_CORE_BUDGET = 1 << 5,    /* core not fully minimised within the step budget        */
  DP_F_BUDGET = 1 << 6,         /* step budget exhausted -> DP_INCOMPLETE                 */
  DP_F_TOO_LARGE = 1 << 7,      /* record does not fit the device path                    */
  DP_F_TRACE_TRUNCATED = 1 << 8, /* search trace stopped: an event exceeded the capacity  */
  DP_F_MALFORMED = 1 << 9        /* the record failed dp_rec_validate's checks (DP_ERROR) */
};

typedef struct dp_opts {
  int32_t first_device; /* HIP device ordinal of the first device used     */
  int32_t n_devices;    /* 0 = every visible device from first_device       */
  int64_t step_budget;  /* per-problem budget (BCP invocations); 0 = default */
  int32_t flags;        /* enum dp_opt_flag bits, normally 0                 */
} dp_opts;

/* Placement overrides (testing and measurement): by default a problem whose
 * 16-bit working set is small is solved by one wavefront out of LDS, a
 * mid-size one (up to a CU's LDS) by one multi-wave workgroup out of LDS,
 * and a larger one by one multi-wave workgroup reading its record from HBM
 * (per-variable state in LDS when it fits, else in HBM).  These flags send
 * every problem to one of the multi-wave paths. */
enum dp_opt_flag {
  DP_OPT_FORCE_GROUP = 1 << 0, /* every problem: multi-wave workgroup */
  DP_OPT_FORCE_HBM = 1 << 1,   /* every problem: multi-wave workgroup, state in HBM */
  DP_OPT_FORCE_MID = 1 << 2,   /* every problem: 4-wave workgroup (the mid-size path) */
  DP_OPT_TINY_TABLE = 1 << 3,  /* test: 4-slot round tables in the multi-wave modes, so rounds
                                  overflow them and are redone on the HBM arrays */
  DP_OPT_FORCE_LDSG = 1 << 4,  /* every problem whose 16-bit image fits a CU's LDS: the
                                  multi-wave all-LDS workgroup (M_LDSG) */
  DP_OPT_SHARE_ORDINAL = 1 << 5 /* test: the context's n_devices logical devices all run on
                                  first_device's GPU (each with its own submitting thread,
                                  host pool, lanes and streams), so the multi-device
                                  dispatcher -- chunk cut, per-device workers, dp_partition
                                  and result stitching -- runs on a one-GPU machine */
};

typedef struct dp_ctx dp_ctx;

/* Host-side batch of lowered records (caller memory, not retained). */
typedef struct dp_batch {
  int32_t n_problems;
  const int64_t* rec_off; /* [n_problems+1] word offsets into rec */
  const int32_t* rec;
} dp_batch;

/* Caller-allocated results.  Sizes come from dp_result_layout(). */
typedef struct dp_result {
  int8_t* status;            /* [P] enum dp_status                                  */
  int32_t* flags;            /* [P] enum dp_flag bits                               */
  uint32_t* installed;       /* bitmap, ceil(nv/32) words per problem (input order) */
  const int64_t* inst_off;   /* [P+1] word offsets into installed                   */
  int32_t* core;             /* identities of the NotSatisfiable explanation        */
  const int64_t* core_off;   /* [P+1] capacity offsets (nid per problem)            */
  int32_t* core_len;         /* [P]                                                 */
  int64_t* steps;            /* [P] BCP invocations used (may be NULL)              */
} dp_result;

/* Fill inst_off[P+1] and core_off[P+1] for a batch.  Returns 0 or -1. */
int dp_result_layout(const dp_batch* b, int64_t* inst_off, int64_t* core_off);

/* Create a context bound to MI355X device(s).  Returns NULL when no usable
 * gfx950 device exists (text in dp_last_global_error()); there is no CPU path. */
dp_ctx* dp_create(const dp_opts* opts);
void dp_destroy(dp_ctx* ctx);
const char* dp_last_error(const dp_ctx* ctx);
const char* dp_last_global_error(void);
int32_t dp_num_devices(const dp_ctx* ctx);
/* Pipeline chunk slots (lanes) per device: two per lane stream.  One lane
 * stream per hardware queue the HIP runtime opened, at most 8: HIP opens
 * GPU_MAX_HW_QUEUES queues (4 when it is not set) once, when it initialises.
 * The bindings raise that setting to 8 before HIP starts and pass the count
 * HIP actually runs with in DEPPY_HW_QUEUES (the setting no longer takes
 * effect once something else initialised HIP); without them the setting is
 * used.  DEPPY_STREAMS overrides.  A serving loop keeps this many chunks in
 * flight per device. */
int32_t dp_lanes(const dp_ctx* ctx);

/* Synchronous batch solve, host memory to host memory: the batched form of
 * (Solver).Solve (solve.go:53-119), which the reference also calls on host
 * memory.  Returns 0, or a negative whole-batch error (text in
 * dp_last_error); per-problem outcomes in res.  The results equal dp_submit +
 * dp_job_wait's.  A small batch of one-wavefront problems (up to 16, the
 * reference's one problem per Solve) takes a latency path on the calling
 * thread: the kernel reads the staged records from mapped pinned memory and
 * writes the results back into it, and completion is polled. */
int dp_solve(dp_ctx* ctx, const dp_batch* b, dp_result* res);

/* Asynchronous host-to-host solve (serving loops; no reference counterpart:
 * the reference solves one problem per call).  dp_submit cuts the batch into
 * chunks (at least one per device) and queues them to the devices' submitting
 * threads, one host thread per device, then returns at once.  Each thread
 * plans and stages its chunks into its lanes' pinned buffers (or DMAs
 * page-locked records as they lie) and enqueues copy and solve on the lane's
 * stream, and delivers finished chunks into res.  b's arrays (the records and
 * rec_off) and res must stay valid and unchanged until dp_job_wait(job)
 * returns, which blocks until every chunk is delivered and frees the job.
 * Several jobs may be in flight, from any number of caller threads. */
typedef struct dp_job dp_job;
int dp_submit(dp_ctx* ctx, const dp_batch* b, dp_result* res, dp_job** job);
int dp_job_wait(dp_ctx* ctx, dp_job* job);

/* Counters of the host-to-host path since the last reset (measurement). */
typedef struct dp_stats {
  int64_t problems;  /* problems staged by dp_submit / dp_solve              */
  int64_t chunks;    /* pipeline chunks                                      */
  int64_t launches;  /* solve kernel launches (all paths)                    */
  double kernel_ms;  /* sum over chunks of their kernels' device time (HIP
                        events on the chunk's stream, around its launches)   */
  int64_t h2d_bytes; /* bytes copied host -> device                          */
  int64_t d2h_bytes; /* bytes copied device -> host                          */
  int64_t rec_bytes; /* record image bytes the kernels read (dp_device_bytes) */
  double stage_ms;   /* host: staging records into pinned memory and writing
                        the chunk tables (after planning)                    */
  double plan_ms;    /* host: planning the launches (header pass, buckets)   */
  double wait_ms;    /* host: blocked on a chunk's completion                 */
  double scatter_ms; /* host: results -> the caller's dp_result              */
  int64_t direct_chunks; /* chunks copied from the caller's page-locked
                            records without staging (DP_LOWER_PINNED)        */
  int64_t bcp_bytes; /* bytes unit propagation read (watch entries, row
                        offsets, row literals and their values), summed over
                        the problems (SURVEY.md 8(d) "BCP-visited bytes")    */
  int64_t allocs;    /* host-side allocations dp_submit made (device / pinned
                        buffers, planning storage).  The first chunk of a
                        batch shape grows every lane of its device, so a
                        serving loop's steady state makes none               */
  int64_t placed[5];          /* problems solved per placement (enum dp_place) */
  int64_t placed_launches[5]; /* solve kernel launches per placement          */
} dp_stats;
int dp_get_stats(dp_ctx* ctx, dp_stats* out, int32_t reset);
/* The share of dp_get_stats that logical device `device` (0 .. dp_num_devices
 * - 1) ran through its submitting thread: its chunks, launches, kernel time
 * and bytes (the pipeline's per-device split of a batch).  dp_get_stats with
 * reset also resets these. */
int dp_get_device_stats(dp_ctx* ctx, int32_t device, dp_stats* out, int32_t reset);

/* Device-resident form (benchmarks, pipelines): the batch is partitioned over
 * the context's devices and copied once; dp_run solves it in place. */
typedef struct dp_resident dp_resident;
int dp_upload(dp_ctx* ctx, const dp_batch* b, dp_resident** out);
int dp_run(dp_ctx* ctx, dp_resident* r);           /* launch + wait; results stay in HBM */
/* Asynchronous form of dp_run for pipelines: dp_launch enqueues the solve and
 * returns; dp_wait blocks until it finished.  Launches of different residents
 * in flight run concurrently (each takes the next of eight per-device chunk
 * slots, two on each of four streams, one stream per hardware queue).
 * dp_launch on a resident still in flight waits for
 * it first; dp_download and dp_resident_free wait as well. */
int dp_launch(dp_ctx* ctx, dp_resident* r);
int dp_wait(dp_ctx* ctx, dp_resident* r);
int dp_download(dp_ctx* ctx, dp_resident* r, dp_result* res);
void dp_resident_free(dp_ctx* ctx, dp_resident* r);
/* Search trace (WithTracer, solve.go:141-146; Tracer.Trace at every
 * unsatisfiable search step, search.go:173).  dp_upload_traced reserves
 * trace_cap int32 words per problem; the solve writes one event record per
 * step: [n, variable indices of the guesses in stack order (SearchPosition
 * .Variables(), search.go:205-213), m, identity ids ascending (.Conflicts(),
 * search.go:215-217)].  An event that does not fit stops the problem's trace
 * and sets DP_F_TRACE_TRUNCATED.  dp_download_trace fills trace[P*trace_cap]
 * (problem p at p*trace_cap) and trace_len[P] (words written). */
int dp_upload_traced(dp_ctx* ctx, const dp_batch* b, int32_t trace_cap, dp_resident** out);
int dp_download_trace(dp_ctx* ctx, dp_resident* r, int32_t* trace, int32_t* trace_len);
int dp_solve_traced(dp_ctx* ctx, const dp_batch* b, int32_t trace_cap, dp_result* res,
                    int32_t* trace, int32_t* trace_len);

/* Measurement helper (no reference counterpart): bytes of the batch as the
 * device stores it.  rec_bytes = the record images the kernels read (the
 * compulsory input of SURVEY §8(d)): on the LDS path the 16-bit form (a
 * DP_FMT_P16 record as it is, else 64 header bytes + 2 per word; the kernel
 * builds the watch lists itself), on the multi-wave paths the int32 form
 * (watch lists are derived data and not counted, wherever they are built).
 * img_bytes = the staged copies as
 * they cross PCIe when staged (16-byte aligned).  opt_flags as
 * dp_opts.flags.  Returns 0 or -1. */
int dp_device_bytes(const dp_batch* b, int32_t opt_flags, int64_t* rec_bytes, int64_t* img_bytes);

/* Host-only test hooks (no device, no reference counterpart): the chunking,
 * staging and result stitching of dp_submit, run on the CPU.
 *   dp_stage_roundtrip: plans b in chunks as dp_submit does (chunk_problems /
 *     chunk_bytes; 0 = defaults), stages every chunk, and widens the staged
 *     copies back into out_rec (same offsets as b->rec): a round trip that
 *     reproduces every record except AtMost bounds over their row length,
 *     which are staged as the row length (out_rec NULL: stage only, for
 *     timing).  chunk_first[] receives the first
 *     problem of each chunk (cap entries at most).  Returns the number of
 *     chunks, or -1 for a malformed record.
 *   dp_stitch_selftest: for every chunk, fills the chunk's output region with
 *     synthetic results of problem p (status, flags, steps, installed words
 *     and a core, all functions of p) at pool positions in reverse claim
 *     order, then scatters them into res like a finished chunk.  Returns the
 *     number of chunks or -1.
 *   dp_partition: the contiguous per-device slices of a resident batch,
 *     balanced by record words: cut[nd+1]. */
int dp_stage_roundtrip(const dp_batch* b, int32_t opt_flags, int32_t chunk_problems, int64_t chunk_bytes,
                       int32_t* out_rec, int32_t* chunk_first, int32_t cap);
int dp_stitch_selftest(const dp_batch* b, int32_t chunk_problems, dp_result* res);
int dp_partition(const int64_t* rec_off, int32_t n_problems, int32_t nd, int32_t* cut);
/*   dp_plan_placements: the placement dp_submit plans for each problem of b
 *     as one chunk (enum dp_place, or DP_PLACE_MALFORMED / DP_PLACE_TOO_LARGE)
 *     into place[n_problems].  Returns 0 or -1. */
enum dp_place {
  DP_PLACE_LDS = 0,    /* one wavefront, record and working set in LDS          */
  DP_PLACE_SPLIT = 1,  /* 8-wave workgroup, per-variable and round state in LDS */
  DP_PLACE_HBM = 2,    /* 8-wave workgroup, working set in HBM                   */
  DP_PLACE_SPLIT4 = 3, /* 4-wave workgroup, as DP_PLACE_SPLIT                    */
  DP_PLACE_LDSG = 4,   /* 4-wave workgroup, the one-wavefront image all in LDS   */
  DP_PLACE_MALFORMED = -1,
  DP_PLACE_TOO_LARGE = -2
};
int dp_plan_placements(const dp_batch* b, int32_t opt_flags, int8_t* place);
/*   dp_plan_order: the launch order dp_submit plans for b as one chunk:
 *     order[] (the problems, skipped ones left out, in workgroup order:
 *     launch after launch) and launch_first[] (each launch's first index
 *     into order; up to 21 launches).  Returns the number of launches or -1. */
int dp_plan_order(const dp_batch* b, int32_t opt_flags, int32_t* order, int32_t* launch_first);

/* Device time of the solve kernel(s) of the last waited launch (dp_run,
 * dp_wait, dp_solve), measured with HIP events on its stream (max over devices). */
int dp_last_kernel_ms(const dp_ctx* ctx, double* ms);

/* ------------------------------------------------------------------------ */
/* Synthetic catalogs (SURVEY.md §8(d) generator; bench/test tooling)         */
/* ------------------------------------------------------------------------ */

/* Configurations of BASELINE.json: 2 = ~200-entity catalogs, 3 = small
 * (P~U{4..12}), 4 = OLM-scale (P=5000, V~55k, deep chains), 5 = mixed-size
 * UNSAT-heavy; 6 = the distribution of the reference's BenchmarkInput
 * (pkg/sat/bench_test.go:10-64: 256 variables, 10% Mandatory, 15% one
 * Dependency of 1-5 candidates, 5% 1-2 Conflicts).  seed_i = base_seed + i. */
typedef struct dp_gen dp_gen; /* owns a dp_wire and its arrays */
dp_gen* dp_gen_catalogs(int32_t config, int32_t n_problems, uint64_t base_seed);
const dp_wire* dp_gen_wire(const dp_gen* g);
void dp_gen_free(dp_gen* g);

/* Build provenance: "sources=<digest> arch=gfx950", the digest (sha256,
 * 16 hex digits) of every source, header and compile flag the library was
 * built from (deppy_amd/build.py sources_digest).  No reference counterpart:
 * the binding compares it with the tree it runs from and refuses a stale
 * library. */
const char* dp_build_info(void);

#ifdef __cplusplus
}
#endif
#endif /* DEPPY_HIP_H */

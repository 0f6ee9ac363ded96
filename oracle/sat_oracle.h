/*
 * sat_oracle.h — CPU restatement of the deppy pkg/sat hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library, and only as the checker
 * (or the reported CPU baseline).  The product path (deppy_amd/, libdeppy_hip)
 * never links or calls it.
 *
 * It consumes the lowered record format of include/deppy_hip.h and restates:
 *   - base scope + Test/Untest        pkg/sat/solve.go:63-79, search.go:75-76,84
 *   - the preference search           pkg/sat/search.go:34-203
 *   - Solve() under scopes            search.go:167-169 (gini contract)
 *   - SAT epilogue                    pkg/sat/solve.go:86-110, lit_mapping.go:147-184
 *   - UNSAT explanation               solve.go:114-115, lit_mapping.go:198-207
 * Parity pinning: tests/golden (TestSolve, TestSearch, error strings, README);
 * see DESIGN.md §Oracle.
 */
#ifndef DEPPY_SAT_ORACLE_H
#define DEPPY_SAT_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* Solve one lowered record.  installed: ceil(nv/32) words; core: nid words.
 * Returns status (1 SAT, -1 UNSAT, 0 INCOMPLETE, -2 ERROR). */
int oracle_solve(const int32_t* rec, int64_t budget, int32_t* flags, uint32_t* installed,
                 int32_t* core, int32_t* core_len, int64_t* steps);

/* oracle_solve with the search trace (Tracer, search.go:173): trace_cap
 * int32 words of event records [n, variables..., m, identities...], one per
 * unsatisfiable search step; *trace_len = words written; an event that does
 * not fit stops the trace and sets DP_F_TRACE_TRUNCATED. */
int oracle_solve_traced(const int32_t* rec, int64_t budget, int32_t* flags, uint32_t* installed,
                        int32_t* core, int32_t* core_len, int64_t* steps, int32_t* trace,
                        int32_t trace_cap, int32_t* trace_len);

/* Batch forms on nthreads host threads (the CPU baseline). */
int oracle_solve_batch(int32_t n, const int64_t* rec_off, const int32_t* rec, int64_t budget,
                       int32_t nthreads, int8_t* status, int32_t* flags, uint32_t* installed,
                       const int64_t* inst_off, int32_t* core, const int64_t* core_off,
                       int32_t* core_len, int64_t* steps);
int oracle_solve_batch_traced(int32_t n, const int64_t* rec_off, const int32_t* rec,
                              int64_t budget, int32_t nthreads, int8_t* status, int32_t* flags,
                              uint32_t* installed, const int64_t* inst_off, int32_t* core,
                              const int64_t* core_off, int32_t* core_len, int64_t* steps,
                              int32_t* trace, int32_t trace_cap, int32_t* trace_len);

/* search.Do with a scripted inter.S (the counterfeiter FakeS of
 * pkg/sat/zz_search_test.go): Test()/Untest() return the scripted values in
 * call order and 0 once the script runs out; Solve() returns 0.
 * out_lits receives the guessed variables (search.Lits()), out_depth the
 * Test-minus-Untest balance (search_test.go:14-29). */
int oracle_search_scripted(const int32_t* rec, const int32_t* test_ret, int32_t n_test,
                           const int32_t* untest_ret, int32_t n_untest, int32_t* out_result,
                           int32_t* out_lits, int32_t* out_nlits, int32_t* out_depth);

/* Unit propagation over the rows of the identities enabled in `enabled`
 * (nid bytes; NULL = all) from the empty assignment.  Returns -1 on a
 * conflict, else 0/1; used to verify cores (re-solve the core alone). */
int oracle_refute(const int32_t* rec, const uint8_t* enabled, int64_t budget);

/* -1 if the installed set satisfies every row, else the first violated row. */
int oracle_check_model(const int32_t* rec, const uint32_t* installed);

#ifdef __cplusplus
}
#endif
#endif

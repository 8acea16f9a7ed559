/*
 * pgmhip.h — C-ABI of the MI355X (gfx950) discrete-factor engine.
 *
 * Plain C types only (pointers, sizes, fixed-layout structs); no torch and no
 * HIP types cross this boundary (streams travel as opaque `void*`).  Every
 * entry point returns an int status: PGM_OK (0) or a negative PGM_E* code; the
 * thread-local message of the last failure is read with pgm_last_error().  No
 * C++ exception crosses the ABI.  The Python binding is ctypes
 * (pgmpy_amd/_native.py); INTEGRATION.md shows the stub a pgmpy maintainer adds
 * to pgmpy/utils/compat_fns.py to bind it.
 *
 * The reference (pgmpy 1.0.0, /root/reference) is pure Python: every entry
 * point below replaces a numpy / opt_einsum call site, cited per function.
 *
 * Data layout: factor values are fp64 (pgmpy/global_vars.py:38 DTYPE
 * "float64") addressed through per-dimension element strides, so a C-order
 * DiscreteFactor (pgmpy/factors/discrete/DiscreteFactor.py:122, last variable
 * fastest), a broadcast operand (stride 0), a transposed view, and a batch of
 * evidence rows (one extra loop dimension, "batch-innermost" stride 1) are all
 * the same descriptor.  Evidence is column-major uint8 state codes
 * codes[col * ld + row] (code 255 = not observed).
 */
#ifndef PGMHIP_H
#define PGMHIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes (Python maps them to the exception pgmpy raises for the same misuse) */
#define PGM_OK 0
#define PGM_EINVAL (-1)  /* ValueError  */
#define PGM_EINDEX (-2)  /* IndexError  (state code >= cardinality)      */
#define PGM_ENOMEM (-3)  /* MemoryError */
#define PGM_EDEVICE (-4) /* RuntimeError: HIP runtime failure / no device */

#define PGM_MAX_DIMS 32     /* loop dims accepted per side before coalescing */
#define PGM_EV_MISSING 255  /* evidence code meaning "not observed" */

/* ---------------------------------------------------------------- runtime */
int pgm_version(void);                         /* ABI version (PGM_OK-free: returns the number) */
int pgm_last_error(char *buf, size_t len);     /* copies the thread-local message */
int pgm_device_count(int *n);
int pgm_set_device(int device);
int pgm_alloc(void **ptr, size_t bytes);
int pgm_free(void *ptr);
int pgm_memcpy_h2d(void *dst, const void *src, size_t bytes, void *stream);
int pgm_memcpy_d2h(void *dst, const void *src, size_t bytes, void *stream);  /* synchronises the stream */
/* stream-ordered D2H without the synchronize (graph-capturable; dst pinned host memory) */
int pgm_memcpy_d2h_async(void *dst, const void *src, size_t bytes, void *stream);
int pgm_memcpy_d2d(void *dst, const void *src, size_t bytes, void *stream);
int pgm_memset(void *dst, int value, size_t bytes, void *stream);
/* host memory that kernels read and write directly (pinned, mapped, coherent / fine-grained; zeroed):
 * a single query's evidence codes and result, so its captured graph needs no copy nodes */
int pgm_host_alloc(void **ptr, size_t bytes);
int pgm_host_free(void *ptr);
int pgm_stream_sync(void *stream);
/* the same wait by polling (no blocking wait's wake-up latency; a host core spins meanwhile): the single
 * query path (VariableElimination.query, ExactInference.py:246-440) waits for its one graph launch this way */
int pgm_stream_sync_spin(void *stream);
/* HIP events, for timing a kernel on the stream it runs on (bench.py) */
int pgm_event_create(void **ev);
int pgm_event_destroy(void *ev);
int pgm_event_record(void *ev, void *stream);
int pgm_event_elapsed_ms(void *start, void *stop, float *ms);

/* ---------------------------------------------------------------- contract
 * The one generic kernel behind DiscreteFactor.product / sum / divide /
 * marginalize / maximize / normalize and every pairwise step of the
 * sum-product contraction:
 *
 *   C[keep] = REDUCE_{red} COMBINE(A[keep, red], B[keep, red])
 *
 * keep dims are the output loop (outermost first; C is written at keep_sc
 * strides), red dims are summed (PGM_RED_SUM) or max-ed (PGM_RED_MAX) away.
 * Replaces:
 *   product      np.einsum(A, ia, B, ib, union)    DiscreteFactor.py:771-777
 *   marginalize  np.einsum(A, range(n), keep)      DiscreteFactor.py:408
 *   maximize     np.max(A, axis)                   DiscreteFactor.py:480 (compat_fns.py:53-60)
 *   sum          A + B (broadcast)                 DiscreteFactor.py:712
 *   divide       A / B, NaN -> 0                   DiscreteFactor.py:859-863
 *   normalize    A / A.sum()                       DiscreteFactor.py:530 (two calls: SUM, then DIV_RAW)
 *   one pairwise tensordot/einsum step of opt_einsum.contract(..., "greedy")
 *                                                  ExactInference.py:404-406, factors/base.py:106
 */
enum pgm_combine {
  PGM_COMBINE_MUL = 0,     /* A*B                                   */
  PGM_COMBINE_ADD = 1,     /* A+B                                   */
  PGM_COMBINE_DIV = 2,     /* A/B with NaN -> 0 (factor division)   */
  PGM_COMBINE_COPY = 3,    /* A (B unused)                          */
  PGM_COMBINE_DIV_RAW = 4  /* A/B, IEEE (0/0 = NaN, as normalize)   */
};
enum pgm_reduce { PGM_RED_NONE = 0, PGM_RED_SUM = 1, PGM_RED_MAX = 2 };

typedef struct {
  int32_t combine; /* enum pgm_combine */
  int32_t reduce;  /* enum pgm_reduce  */
  int32_t n_keep;
  int32_t n_red;
  int64_t keep_card[PGM_MAX_DIMS];
  int64_t keep_sa[PGM_MAX_DIMS];
  int64_t keep_sb[PGM_MAX_DIMS];
  int64_t keep_sc[PGM_MAX_DIMS];
  int64_t red_card[PGM_MAX_DIMS];
  int64_t red_sa[PGM_MAX_DIMS];
  int64_t red_sb[PGM_MAX_DIMS];
} pgm_contract_desc;

/* bytes of device workspace pgm_contract needs for this descriptor (0 = none) */
int pgm_contract_workspace(const pgm_contract_desc *d, size_t *bytes);
int pgm_contract(const pgm_contract_desc *d, const double *A, const double *B, double *C,
                 void *workspace, size_t workspace_bytes, void *stream);

/* ---------------------------------------------------------------- n-ary product
 * C[keep] = prod_i X_i[keep . keep_s[i]]  (up to PGM_PRODN_MAX_OPS broadcast operands).
 * factor_product's left fold of __mul__ (pgmpy/factors/base.py:20-66) in one pass, and the
 * batched-BP clique update beta = psi x findings x prod(child messages) written once instead of
 * once per incoming message (ExactInference.py:798-802).  ops is a HOST array of device pointers.
 */
#define PGM_PRODN_MAX_OPS 8
enum pgm_prodn_kind {
  PGM_PRODN_MUL = 0,   /* prod *= X_i                                                    */
  PGM_PRODN_RATIO = 1, /* prod *= X_i / X_{i+1}, NaN -> 0 (sepset update sigma / mu,     */
  PGM_PRODN_DEN = 2,   /*   ExactInference.py:798-802 + DiscreteFactor.py:859-863)       */
  PGM_PRODN_MDIV = 3   /* pgm_product_n_marginal only: prod *= X_i like MUL, and the marginal M is
                          stored divided by X_i (0/0 -> 0) — X_i must not vary over the entries M sums
                          (a child's message mu on its separator: M = sigma' / mu, the child's update
                          ratio, ExactInference.py:798-802).  At most one per call; other calls:
                          PGM_EINVAL */
};
typedef struct {
  int32_t n_ops;
  int32_t n_keep;
  int32_t op_kind[PGM_PRODN_MAX_OPS];
  int64_t keep_card[PGM_MAX_DIMS];
  int64_t keep_sc[PGM_MAX_DIMS];
  int64_t keep_s[PGM_PRODN_MAX_OPS][PGM_MAX_DIMS];
} pgm_productn_desc;

int pgm_product_n(const pgm_productn_desc *d, const double *const *ops, double *C, void *stream);

/* r06: an n-ary contraction, C[keep] = REDUCE over red of prod_t X_t[keep . keep_s[t] + red . red_s[t]]
 * (up to PGM_PRODN_MAX_OPS operands, reduce PGM_RED_SUM or PGM_RED_MAX), as a JOB of a batch only
 * (pgm_batch_add_contract_n): several consecutive pairwise steps of a contraction path
 * (ExactInference.py:404-406, opt_einsum's pairwise tensordots) in one job of one launch, so the
 * compiled path has fewer dependency levels.  A batch holding one runs only as its specialised kernel
 * (pgm_batch_specialise); pgm_batch_run refuses it (PGM_EINVAL).  Products are rounded before they are
 * summed, operands multiplied in order (a left fold, as factor_product). */
typedef struct {
  int32_t n_ops;
  int32_t reduce;
  int32_t n_keep;
  int32_t n_red;
  int64_t keep_card[PGM_MAX_DIMS];
  int64_t keep_sc[PGM_MAX_DIMS];
  int64_t keep_s[PGM_PRODN_MAX_OPS][PGM_MAX_DIMS];
  int64_t red_card[PGM_MAX_DIMS];
  int64_t red_s[PGM_PRODN_MAX_OPS][PGM_MAX_DIMS];
} pgm_contractn_desc;

/* The same product and, in the same pass, M = reduce(C) over the keep dims with marg_s == 0
 * (marg_s[i]: stride of keep dim i in M; the last keep dim, the evidence rows, must have stride 1
 * in C and M).  Batched-BP collect (a clique belief and its message to the parent,
 * ExactInference.py:784-802) and distribute (beta_c *= sigma'/mu in place, C may alias operand 0,
 * with the marginal onto a child separator) read each clique once.  reduce: PGM_RED_SUM or
 * PGM_RED_MAX (max-calibration).  Only shapes with pgm_product_n_marginal_ok() == 1 run fused
 * (<= 4 operands, rows innermost with an even count >= 64, <= 512 reduced states per kept state,
 * enough kept states to fill the chip); others return PGM_EINVAL without launching and the caller
 * runs pgm_product_n + pgm_contract.  C == NULL computes M alone (the strides of C still describe
 * the product's index space): a batched-BP collect message without writing the clique belief, which
 * the distribute pass then writes once. */
int pgm_product_n_marginal_ok(const pgm_productn_desc *d, const double *const *ops, const double *C,
                              const int64_t *marg_s, const double *M);
int pgm_product_n_marginal(const pgm_productn_desc *d, const double *const *ops, double *C,
                           const int64_t *marg_s, int32_t reduce, double *M, void *stream);

/* The same fused step bound to its pointers with the plan compiled in (hipRTC, gfx950): kept /
 * reduced index spaces, strides and operand kinds as literals, the reduced entries as unrolled loops.
 * *bound = NULL (PGM_OK) when the generic kernel should run instead (clique below the size threshold,
 * or PGM_PM_JIT=0 / PGM_NO_JIT set, or the compile failed); the same shape errors as
 * pgm_product_n_marginal otherwise.  pgm_pm_bound_run launches it on stream (capturable in a
 * graph); the pointers must stay valid until pgm_pm_bound_destroy.  Replaces the per-step
 * DiscreteFactor.product / marginalize pair of a batched calibration (ExactInference.py:784-802). */
int pgm_product_n_marginal_bind(const pgm_productn_desc *d, const double *const *ops, double *C,
                                const int64_t *marg_s, int32_t reduce, double *M, void **bound);
/* pgm_product_n as a bound specialised step (no marginal; every dim kept), mergeable with the other
 * bound steps of its level (pgm_pm_merge); *bound = NULL when the shape is not one the fused
 * kernel handles (rows innermost, even, >= 64) or is too small. */
int pgm_product_n_bind(const pgm_productn_desc *d, const double *const *ops, double *C, void **bound);

/* Two marginals of the same product in ONE pass (nothing else stored), as a bound specialised step
 * (mergeable): M1 over the keep dims with marg_s1 != 0, M2 likewise with marg_s2 (rows last, stride 1
 * in both).  A batched-BP parent's sigma' onto two child scopes from its operands
 * (ExactInference.py:784-797: each sigma is a marginalize of the same belief).  *bound = NULL when
 * the shapes are outside the pass's limits (<= 32 accumulators, <= 512 unrolled states); then run two
 * marginal passes. */
int pgm_product_n_marginals_bind(const pgm_productn_desc *d, const double *const *ops, const int64_t *marg_s1,
                                 double *M1, const int64_t *marg_s2, double *M2, int32_t reduce, void **bound);

/* The generated kernel source for the same arguments (no compile, no GPU): returns its length (0
 * when the generic kernel would run), copies at most len-1 bytes + NUL into buf.  Inspection and
 * host-side tests. */
int pgm_product_n_marginal_source(const pgm_productn_desc *d, const double *const *ops, double *C,
                                  const int64_t *marg_s, int32_t reduce, double *M, char *buf, size_t len);
/* Compile (hipRTC, distinct sources, optionally on parallel threads, code-object disk cache) and load the kernels
 * of bound / merged steps that are not loaded yet; a bound step not prepared compiles at its first
 * run.  Call before graph capture. */
int pgm_pm_prepare(void *const *bounds, int32_t n);
/* The generated source of a bound / merged step (its length; at most len-1 bytes + NUL copied). */
int pgm_pm_bound_source(void *bound, char *buf, size_t len);
int pgm_pm_bound_run(void *bound, void *stream);
/* Several bound steps with no dependence between them (one level of a batched-BP sweep) as ONE
 * launch: a kernel whose block ranges run the steps' bodies.  *merged = NULL (PGM_OK) when the merge
 * is not possible (grid too large, compile failed): launch the steps separately.  The inputs stay
 * valid and owned by the caller; destroy the merged handle with pgm_pm_bound_destroy. */
int pgm_pm_merge(void *const *bounds, int32_t n, void **merged);
int pgm_pm_bound_destroy(void *bound);

/* ---------------------------------------------------------------- dense pairwise step (FP64 MFMA)
 * C[b, m, n] = sum_k A[b, m, k] * B[b, k, n] where each index is a GROUP of variables laid out in
 * any order inside its tensor: the element offsets come from a DEVICE int64 table,
 *   offsets = [A_b (batch) | B_b (batch) | C_b (batch) | A_m (m) | C_m (m) | A_k (k) | B_k (k) |
 *              B_n (n) | C_n (n)]
 * so A is read at A[A_b[b] + A_m[m] + A_k[k]] and C written at C[C_b[b] + C_m[m] + C_n[n]].
 * These are the greedy contraction's pairwise steps that are genuine GEMMs — the two factors
 * share summed-out variables (k), each keeps its own (m, n), shared kept variables batch (b) —
 * as in the tensordot/BLAS calls opt_einsum makes for opt_einsum.contract(..., "greedy")
 * (pgmpy/inference/ExactInference.py:404-406, pgmpy/factors/base.py:106).  Exact fp64 products
 * (v_mfma_f64_16x16x4_f64); the k-summation order differs from a sequential loop.
 */
typedef struct {
  int64_t batch, m, n, k;
  const int64_t *offsets; /* device, 3*batch + 2*m + 2*k + 2*n entries */
  int64_t stride[9];      /* per table part: >= 0 -> offset = index * stride (table not read), -1 -> table */
  int32_t lane_order;     /* hint for table groups: bit 0 = consecutive m are adjacent in A, bit 1 = consecutive
                             k are adjacent in B (tile loads then run along that axis); strided groups are
                             detected from the strides */
  int32_t _pad;
} pgm_gemm_desc;

int pgm_gemm(const pgm_gemm_desc *d, const double *A, const double *B, double *C, void *stream);

/* Evidence ingestion: per-column int8 category indices raw[col * ld_raw + row]
 * (pandas Categorical codes / Arrow dictionary indices, -1 = NaN) -> uint8 state codes
 * out[col * ld_out + row] through a per-column LUT lut[col * lut_stride + category] (254 marks a
 * category that is not a state name: err_flag is set), 255 for NaN.  When row_key is given (zeroed
 * by the caller, with row_nmiss), row_key[row] ^= col_key[col] and row_nmiss[row] += 1 for every
 * missing column: the row's evidence-pattern key, from which predict() groups rows.  When row_hash
 * is given (zeroed, 2 x uint64 per row) it receives a 128-bit hash of the row's codes (predict's
 * de-duplication of identical rows, DiscreteBayesianNetwork.py:867-870).  Replaces the
 * per-cell state-name lookups of the reference (state_name.py:71-84 via DiscreteFactor.py:589-597,
 * called per row from DiscreteBayesianNetwork.py:871-878 / :974-979). */
int pgm_codes_remap(const int8_t *raw, int64_t ld_raw, int32_t n_cols, int64_t n_rows, const uint8_t *lut,
                    int32_t lut_stride, const uint64_t *col_key, uint8_t *out, int64_t ld_out, uint64_t *row_key,
                    uint32_t *row_nmiss, uint64_t *row_hash, int32_t *err_flag, void *stream);

/* predict(stochastic=True): for each output row r, numpy's Generator.choice over the joint column
 * joint[i * ld + group[r]] (i < P): cdf = cumsum(p); cdf /= cdf[-1]; out_idx[r] = searchsorted(cdf,
 * u[r], "right") (DiscreteFactor.sample, DiscreteFactor.py:868-912, called per unique evidence row at
 * DiscreteBayesianNetwork.py:889-892).  u: the uniforms of the reference's seeded stream. */
int pgm_sample_joint(const double *joint, int64_t ld, int64_t P, const int32_t *group, const double *u, int64_t n,
                     int32_t *out_idx, void *stream);

/* ---------------------------------------------------------------- evidence column select
 * out[j * n_rows + r] = codes[cols[j] * ld + row0 + r]: copies the evidence columns a compiled
 * plan reads into its own fixed buffer (so the captured graph never sees caller pointers).
 * cols is a DEVICE int32 array of n_cols column indices. */
int pgm_codes_select(const uint8_t *codes, int64_t ld, int64_t row0, const int32_t *cols, int32_t n_cols,
                     int64_t n_rows, uint8_t *out, void *stream);

/* ---------------------------------------------------------------- HIP graphs
 * Capture every launch issued on `stream` between begin and end into an executable graph, then
 * replay it with one launch (compiled BP schedules, fixed-shape contraction plans).  The stream
 * must not be the legacy default stream. */
int pgm_graph_capture_begin(void *stream);
int pgm_graph_capture_end(void *stream, void **graph_exec);
int pgm_graph_launch(void *graph_exec, void *stream);
int pgm_graph_destroy(void *graph_exec);

/* ---------------------------------------------------------------- evidence gather
 * Batched DiscreteFactor.reduce: one evidence row per value of the batch
 * loop dim; the reduced variables' states come from the per-row codes.
 *   C[keep] = A[keep_sa . keep + sum_j codes[ev_col[j]*ld + row] * ev_stride[j]]
 * Replaces basic indexing values[tuple(slice_)] (DiscreteFactor.py:614;
 * the greedy path's per-factor slice ExactInference.py:352-365,385).
 * A code >= ev_card[j] sets *err_flag (-> IndexError, test_Factor.py:555-565);
 * PGM_EV_MISSING is rejected the same way (the plan must not gather it).
 */
typedef struct {
  int32_t n_keep;
  int32_t n_ev;
  int32_t batch_dim; /* index into keep dims that enumerates rows (-1: row 0 only) */
  int32_t _pad;
  int64_t ld;        /* leading dimension of codes (rows per column) */
  int64_t row0;      /* first row of this call (sharding offset) */
  int64_t keep_card[PGM_MAX_DIMS];
  int64_t keep_sa[PGM_MAX_DIMS];
  int64_t keep_sc[PGM_MAX_DIMS];
  int64_t ev_col[PGM_MAX_DIMS];
  int64_t ev_stride[PGM_MAX_DIMS];
  int64_t ev_card[PGM_MAX_DIMS];
} pgm_gather_desc;

int pgm_gather(const pgm_gather_desc *d, const double *A, const uint8_t *codes, double *C,
               int32_t *err_flag, void *stream);

/* 0/1 evidence indicator (BP findings):
 * out[k*s_state + r*s_row] = (codes[r] == k) or 1 when codes[r] == PGM_EV_MISSING */
int pgm_indicator(const uint8_t *codes, int64_t n_rows, int64_t card, double *out, int64_t s_state,
                  int64_t s_row, int32_t *err_flag, void *stream);

/* ---------------------------------------------------------------- argmax
 * First-flat-index argmax per row (np.argmax semantics incl. NaN-first):
 * replaces compat_fns.argmax (compat_fns.py:70-74) in map_query
 * (ExactInference.py:616).  idx[r] = argmax_i X[r*s_row + i*s_elem], written to
 * out_idx (int64) and/or out_idx32 (int32); either may be NULL. */
int pgm_argmax(const double *X, int64_t n_rows, int64_t row_len, int64_t s_row, int64_t s_elem,
               int64_t *out_idx, int32_t *out_idx32, void *stream);

/* ---------------------------------------------------------------- batched small jobs
 * Many INDEPENDENT small contractions / evidence gathers run as one launch (one level of a
 * compiled greedy contraction path, ExactInference.py:404-406: every step whose inputs are ready;
 * or all of a plan's per-factor evidence slices, ExactInference.py:352-365).  Jobs are planned on
 * add (same descriptors and checks as pgm_contract / pgm_gather; contractions run in flat mode
 * without split-K), uploaded once by finalize, and replayed by run (graph-capturable).  The
 * caller guarantees that no job reads another job's output. */
int pgm_batch_create(void **handle);
int pgm_batch_add_contract(void *handle, const pgm_contract_desc *d, const double *A, const double *B, double *C);
int pgm_batch_add_gather(void *handle, const pgm_gather_desc *d, const double *A, const uint8_t *codes, double *C,
                         int32_t *err_flag);
/* an n-ary product job (pgm_product_n's descriptor and checks; flat mode): batched BP runs every
 * small clique / separator product of one dependency level of the calibration as one launch */
int pgm_batch_add_product_n(void *handle, const pgm_productn_desc *d, const double *const *ops, double *C);
/* r06: an n-ary contraction job (pgm_contractn_desc; ops: a HOST array of n_ops device pointers). */
int pgm_batch_add_contract_n(void *batch, const pgm_contractn_desc *d, const double *const *ops, double *C);
/* a findings-indicator job (pgm_indicator's arguments): all of a BP sweep's findings in one launch */
int pgm_batch_add_indicator(void *handle, const uint8_t *codes, int64_t n_rows, int64_t card, double *out,
                            int64_t s_state, int64_t s_row, int32_t *err_flag);
/* Single-workgroup levelled batch (mode PGM_BATCH_ONE_WORKGROUP, set before the first job): jobs added
 * after pgm_batch_add_level belong to the next level and may read earlier levels' outputs.  run
 * launches ONE 1,024-thread workgroup that stages every job descriptor, the block map and the level
 * table in LDS and executes each level's blocks (four 256-thread virtual blocks at a time) with a
 * workgroup barrier between levels (no grid barrier, no cache maintenance: producer and consumer are
 * the same workgroup) — for chains of tiny dependent levels (the last levels of a contraction path
 * down to the query marginal and its normalisation, ExactInference.py:404-421), whose
 * one-launch-per-level cost is all launch latency.  Contraction jobs only, tables <= 48 KB
 * (finalize: PGM_EINVAL otherwise).  pgm_batch_add_level needs this mode (PGM_EINVAL in the default
 * PGM_BATCH_GRID mode: one level, one launch).  ABI 20 removed the persistent grid-barrier form
 * (measured slower than one launch per level, r03) and pgm_batch_info. */
int pgm_batch_add_level(void *handle);
enum { PGM_BATCH_GRID = 0, PGM_BATCH_ONE_WORKGROUP = 1 };
int pgm_batch_set_mode(void *handle, int32_t mode);
/* blocks (256-thread workgroups) the jobs added so far occupy; the levelled single-workgroup kernel
 * runs them four at a time, so callers keep it to levels of a few blocks */
int pgm_batch_blocks(void *handle, int64_t *blocks);
int pgm_batch_finalize(void *handle);
int pgm_batch_run(void *handle, void *stream);
/* The finalized batch (contraction jobs only, either mode) as ONE plan-specialised kernel (hipRTC,
 * cached by source like the fused BP steps): each job's output decode, strides, reduction walk and
 * lanes per output are literals and a block finds its job from literal block ranges, so no block map
 * or descriptor is read (C1 / C2's path levels).  *bound = NULL when a job is not a contraction the
 * generator takes (the generic pgm_batch_run stays); else prepare / run / destroy it with
 * pgm_pm_prepare, pgm_pm_bound_run, pgm_pm_bound_destroy (not pgm_pm_merge).  The batch's pointers
 * must stay valid; the batch handle itself may be destroyed.  Up to 512 job pointers travel as the
 * kernel's arguments; a batch of more (up to 8,192) gets its pointer array copied into device memory
 * here and the kernel reads them from that table (freed with the bound launch); *bound = NULL above
 * 8,192 (split the batch). */
int pgm_batch_specialise(void *handle, void **bound);
int pgm_batch_destroy(void *handle);


/* ---------------------------------------------------------------- fused row plan
 * The batched-evidence hot path (DiscreteBayesianNetwork.predict /
 * predict_probability, DiscreteBayesianNetwork.py:731-989; the per-row
 * VariableElimination.query / map_query of ExactInference.py:246-624): per
 * evidence row, the whole reduce -> sum-product -> normalize ->
 * marginalize/argmax chain of one evidence pattern in ONE kernel, one lane per
 * row, CPT values staged in LDS, no HBM intermediates.
 *
 * After evidence reduction the factor graph over the unobserved variables splits
 * into independent COMPONENTS; each is summed over its own (query x hidden)
 * index space, so the joint is never expanded across components.  Loop dims are
 * grouped per component: [comp_loop_begin, +comp_n_query) are query dims,
 * [.., comp_loop_end) hidden (summed) dims.  Factor f (in component c, factors
 * of c are [comp_fac_begin, comp_fac_end)) evaluated at a loop point is
 *   values[fac_base[f] + sum_j code_j(row) * ev_stride_j + sum_k digit_k * fac_stride[f][k]]
 * Outputs follow the reference exactly: marginal = component marginal / its
 * mass; if the product of all component masses is 0 (impossible evidence) every
 * marginal is NaN (0/0 of DiscreteFactor.normalize, DiscreteFactor.py:530) and the
 * MAP index is 0 (np.argmax of an all-NaN joint).
 */
#define PGM_ROWS_MAX_LOOP 12
#define PGM_ROWS_MAX_FAC 16
#define PGM_ROWS_MAX_EV 48
#define PGM_ROWS_MAX_COMP 12
#define PGM_ROWS_MAX_MARG 192

enum pgm_rows_mode {
  PGM_ROWS_MARGINALS = 1, /* per query var normalized marginal (predict_probability) */
  PGM_ROWS_JOINT = 2,     /* normalized joint over the query dims (query joint=True); n_comp == 1 only */
  PGM_ROWS_MAP = 4,       /* first-index argmax of the joint (map_query / predict)  */
  PGM_ROWS_MAPGAP = 8,    /* also (best - second best) / best of the joint, for tie screening */
  PGM_ROWS_VALUES_GLOBAL = 16, /* tuning: read CPT values through L1/L2 instead of staging them in LDS */
  PGM_ROWS_ONE_GROUP = 32,     /* tuning: one 64-row group per workgroup (no staging amortisation) */
  PGM_ROWS_GENERIC = 64,       /* tuning: table-driven kernel even for all-affine plans (testing)  */
  PGM_ROWS_NO_JIT = 128,       /* testing: skip the plan-specialised (hipRTC) kernel, run the AOT ones */
  PGM_ROWS_FLOOR = 256         /* measurement (pgm_rows_plan_bind only): the plan's dispatch floor — same grid,
                                  same evidence-column loads and output stores as the specialised kernel, no
                                  CPT staging or arithmetic; the outputs are NOT results */
};

typedef struct {
  int32_t n_loop;
  int32_t n_query;  /* total query dims */
  int32_t n_fac;
  int32_t n_ev;
  int32_t n_values; /* packed CPT values (doubles) */
  int32_t n_comp;
  int32_t n_marg;   /* rows of the marginal output = sum of query cardinalities */
  int32_t n_joint;  /* entries of the joint = prod of query cardinalities */
  int32_t loop_card[PGM_ROWS_MAX_LOOP];
  int32_t loop_marg_off[PGM_ROWS_MAX_LOOP];   /* query dim: first marginal row of its variable (-1 hidden) */
  int32_t loop_map_stride[PGM_ROWS_MAX_LOOP]; /* query dim: stride in the flat joint / MAP index (0 hidden) */
  int32_t comp_loop_begin[PGM_ROWS_MAX_COMP];
  int32_t comp_n_query[PGM_ROWS_MAX_COMP];
  int32_t comp_loop_end[PGM_ROWS_MAX_COMP];
  int32_t comp_fac_begin[PGM_ROWS_MAX_COMP];
  int32_t comp_fac_end[PGM_ROWS_MAX_COMP];
  int32_t fac_base[PGM_ROWS_MAX_FAC];
  int32_t fac_stride[PGM_ROWS_MAX_FAC][PGM_ROWS_MAX_LOOP];
  int32_t fac_ev_begin[PGM_ROWS_MAX_FAC]; /* evidence terms of factor f: [begin, end) */
  int32_t fac_ev_end[PGM_ROWS_MAX_FAC];
  int32_t ev_col[PGM_ROWS_MAX_EV];
  int32_t ev_stride[PGM_ROWS_MAX_EV];
  int32_t ev_card[PGM_ROWS_MAX_EV];
} pgm_rows_plan;

int pgm_rows_plan_create(const pgm_rows_plan *plan, const double *host_values, void **handle);
int pgm_rows_plan_destroy(void *handle);
/* Source of the plan-specialised row kernel (hipRTC, compiled for gfx950 on the first run of an
 * all-affine plan: one query variable and no hidden variable per component).  Writes at most len
 * bytes (NUL-terminated) and the full size + 1 to *needed.  No device needed (tests, inspection). */
int pgm_rows_plan_source(const pgm_rows_plan *plan, char *buf, size_t len, size_t *needed);
/* Rows [row0, row0 + n_rows) of codes.  Outputs are column-major with leading dim ld_out (>= n_rows) and
 * row r written at column r (not row0 + r); any may be NULL unless its mode bit is set:
 *   marg [n_marg][ld_out] f64   joint [n_joint][ld_out] f64   map [n_rows] int32   gap [n_rows] f64 */
int pgm_rows_plan_run(void *handle, int32_t mode, const uint8_t *codes, int64_t ld_codes, int64_t row0,
                      int64_t n_rows, double *marg, double *joint, int64_t ld_out, int32_t *map,
                      double *gap, int32_t *err_flag, void *stream);

/* Prepared launch: validates the same arguments as pgm_rows_plan_run once and binds them; each
 * pgm_rows_bound_run then launches that pass (same result as the unbound call).  The buffers and the
 * plan handle must outlive the bound handle.  Replaces the per-batch Python call of predict()'s
 * inner loop (pgmpy/models/DiscreteBayesianNetwork.py:867-910) for repeated batches. */
int pgm_rows_plan_bind(void *handle, int32_t mode, const uint8_t *codes, int64_t ld_codes, int64_t row0,
                       int64_t n_rows, double *marg, double *joint, int64_t ld_out, int32_t *map,
                       double *gap, int32_t *err_flag, void *stream, void **bound);
int pgm_rows_bound_run(void *bound);
int pgm_rows_bound_destroy(void *bound);
/* which kernel a bound launch runs: "pgm_rows_jit" (one row per thread), "pgm_rows_jit2" (two rows
 * per thread, 16-B stores), "pgm_rows_floor" / "pgm_rows_floor2" (PGM_ROWS_FLOOR), or "" (an AOT kernel), with its grid and workgroup size */
int pgm_rows_bound_kernel(void *bound, char *name, size_t cap, uint32_t *blocks, uint32_t *wg);

/* Rows sharded over several GPUs from host buffers: the data-parallel axis of predict /
 * predict_probability (pgmpy/models/DiscreteBayesianNetwork.py:867-910, 912-989) split into n_shards
 * contiguous row blocks (shard i = rows [i n / S, (i + 1) n / S), as pgmpy_amd.distributed.shard_bounds),
 * shard i run by handles[i] on the HIP device that was current when that handle was created
 * (pgm_rows_plan_create once per device; the handles must describe the same plan).  One host thread per
 * shard: the shard's rows of the evidence columns the plan reads in (host_codes column-major uint8 with
 * columns [0, n_cols), leading dim ld_codes, the plan's column numbering), the plan's pass, its outputs
 * out to the caller's host arrays at the shard's columns — the gather of every shard's result is that
 * copy, each GPU's over its own host link.  A shard runs in chunks of 256 K rows (PGM_SHARD_CHUNK)
 * alternating between two streams and device buffers the handle keeps from its first call (no
 * allocation after it), so a chunk's copy-in and pass overlap the previous chunk's copy-out when the host
 * arrays are pinned (pgm_host_alloc); pageable arrays work and are staged by HIP.  One call at a time
 * per handle.  mode: PGM_ROWS_MARGINALS
 * (host_marg [n_marg][ld_out] f64) and / or PGM_ROWS_MAP (host_map [n_rows] int32).  *err_any is ORed
 * with the kernels' evidence-error flag (PGM_ROWS error semantics of pgm_rows_plan_run).  Returns when
 * every shard is done; the first failing shard's status otherwise.  Outputs equal one
 * pgm_rows_plan_run over all rows bit for bit.  (the multi-GPU entry a non-Python
 * FFI caller uses; the Python path shards with torch.distributed, pgmpy_amd/distributed.py.) */
int pgm_rows_shard_run(void *const *handles, int32_t n_shards, int32_t mode, const uint8_t *host_codes,
                       int64_t ld_codes, int64_t n_cols, int64_t n_rows, double *host_marg, int64_t ld_out,
                       int32_t *host_map, int32_t *err_any);

/* Host-side scan for evidence ingestion (no device needed): out[j] = 1 when any of the n int8 cells of
 * column cols[j] is negative (a pandas Categorical NaN code), else 0; up to `threads` host threads.
 * Finds the NaN-holding columns of a categorical frame in one native pass, so rows are grouped by
 * missing-column pattern from those columns only (predict's per-row NaN handling,
 * pgmpy/models/DiscreteBayesianNetwork.py:862-878). */
int pgm_host_any_negative_i8(const int8_t *const *cols, int32_t n_cols, int64_t n, uint8_t *out, int32_t threads);
/* r06 (pgmhost.cpp, one persistent pool of at most 16 host threads): the same scan as a job fed column by
 * column — begin (n rows, room for `capacity` columns), push column pointers as they become known (each
 * push is scanned on the pool while the caller goes on), end (waits, out[j] = 1 when pushed column j holds a
 * negative code; *n_cols = columns pushed; frees the job).  The caller keeps the columns alive until end.
 * pgm_host_lut_map_u8: dst[j * ld + i] = luts[j][(uint8_t)src[j][i]] (luts[j] NULL: the byte itself), on
 * the pool — the plan's evidence columns from category codes to state codes (state_name.py:71-84 per
 * cell in the reference). */
int pgm_host_scan_begin(int64_t n, int32_t capacity, int32_t threads, void **job);
int pgm_host_scan_push(void *job, const int8_t *const *cols, int32_t count);
int pgm_host_scan_end(void *job, uint8_t *out, int32_t *n_cols);
int pgm_host_lut_map_u8(const int8_t *const *src, const uint8_t *const *luts, int32_t n_cols, int64_t n, uint8_t *dst,
                        int64_t ld, int32_t threads);

/* Resident ring of row batches (streaming predict_probability / predict): one launch of the
 * plan-specialised two-rows-per-lane kernel ("pgm_rows_ring") stays resident while the host publishes
 * batches, so consecutive batches overlap on the chip instead of each paying a dispatch.  Replaces the
 * reference's per-batch caller loop (pgmpy/models/DiscreteBayesianNetwork.py:867-910, 912-989) for a
 * stream of equally sized batches.
 *   create: n_slots buffer sets; batch b reads codes[b % n_slots] (rows [row0, row0 + n_rows), leading
 *           dim ld_codes) and writes marg / map / gap[b % n_slots] (leading dim ld_out), as
 *           pgm_rows_plan_run.  mode: PGM_ROWS_MARGINALS | PGM_ROWS_MAP | PGM_ROWS_MAPGAP only; the
 *           two-rows-per-lane contract holds per slot (even n_rows / row0 / leading dims, 16-B aligned
 *           outputs) else PGM_EINVAL.  Needs the plan-specialised kernel (hipRTC).
 *   start:  launches the resident grid on `stream` for n_batches batches (the ring must not be
 *           running); waves that reach a batch not yet posted wait, and give up after timeout_s
 *           seconds (PGM_EDEVICE from finish).
 *   post:   publishes batches [0, n_posted) (monotone, <= n_batches).  A batch's inputs must be
 *           complete in device memory, and its slot's previous batch finished, before it is posted.
 *   finish: all n_batches posted -> waits for the launch (stream synchronize) and checks it.
 *   cancel: stops the launch early (waves exit at their next unposted batch) and waits.
 * Outputs of batch b equal pgm_rows_plan_run's on the same rows bit for bit. */
int pgm_rows_ring_create(void *handle, int32_t mode, int32_t n_slots, const uint8_t *const *codes,
                         const int64_t *ld_codes, const int64_t *row0, int64_t n_rows, double *const *marg,
                         int64_t ld_out, int32_t *const *map, double *const *gap, int32_t *err_flag, void *stream,
                         void **ring);
int pgm_rows_ring_start(void *ring, uint32_t n_batches, double timeout_s);
/* start_ready: start, then wait (up to ready_timeout_s) until every workgroup of the resident grid is
 * running with its CPT staged, so that what follows (posts, completions) no longer includes the launch
 * itself; PGM_EDEVICE (and the launch cancelled) if the grid does not come up in time */
int pgm_rows_ring_start_ready(void *ring, uint32_t n_batches, double timeout_s, double ready_timeout_s);
int pgm_rows_ring_post(void *ring, uint32_t n_posted);
int pgm_rows_ring_finish(void *ring);
int pgm_rows_ring_cancel(void *ring);
/* the ring's batch counter in pinned host memory and this launch's base: storing base + k (a plain,
 * aligned 32-bit store, monotone, k <= n_batches) publishes batches [0, k) exactly as
 * pgm_rows_ring_post(ring, k) does, without a library call per batch (finish then needs
 * pgm_rows_ring_post(ring, n_batches) or the store of base + n_batches) */
int pgm_rows_ring_counter(void *ring, uint32_t **counter, uint32_t *base);
/* the ring's kernel name ("pgm_rows_ring"), resident grid and workgroup size */
int pgm_rows_ring_kernel(void *ring, char *name, size_t cap, uint32_t *blocks, uint32_t *wg);
int pgm_rows_ring_destroy(void *ring);

/* Direct AQL dispatch (pgmpy_amd/csrc/pgmdq.cpp).  A user-mode HSA queue on the GPU agent of a HIP
 * device; a bound launch of the plan-specialised kernel (pgm_rows_plan_bind) is re-bound to it and
 * each pgm_dq_launch writes one kernel-dispatch packet (barrier bit set) and rings the doorbell — no
 * HIP runtime on the launch path.  Same kernel, same arguments, same results as pgm_rows_bound_run.
 * Ordering: pgm_dq_bind_rows waits for the device (inputs complete); dispatches on one queue run in
 * order; inputs may change only between pgm_dq_sync and the next launch (that launch first drains the
 * device with hipDeviceSynchronize, so HIP work issued in between is complete); call
 * pgm_dq_sync (a system-scope release barrier + wait) before HIP work reads the outputs.  The timer reports
 * the GPU span (queue profiling timestamps) from the first dispatch after pgm_dq_timer_start to the
 * last one issued.  The queue must outlive its bound launches.  Serves the same caller as
 * pgm_rows_bound_run (pgmpy/models/DiscreteBayesianNetwork.py:867-910, repeated batches). */
int pgm_dq_create(int hip_device, void **dq);
int pgm_dq_destroy(void *dq);
int pgm_dq_bind_rows(void *dq, void *bound, void **dbound);
int pgm_dq_launch(void *dbound);
/* a group of bound launches on one queue whose outputs are pairwise distinct (independent batches):
 * the first waits for everything before it (barrier bit), the others may overlap it and each other;
 * the next launch or sync waits for the whole group.  At most 128 launches, no launch repeated. */
int pgm_dq_launch_group(void *const *dbounds, int32_t n);
/* one dispatch whose own completion releases at system scope (its packet's release fence): the last
 * dispatch before the host or HIP reads the outputs, instead of a separate pgm_dq_sync barrier packet;
 * wait for it with pgm_dq_wait.  Like pgm_dq_sync, the next dispatch acquires at system scope. */
int pgm_dq_launch_release(void *dbound);
int pgm_dq_sync(void *dq);
/* the first half of pgm_dq_sync: append the system-scope release barrier packet without waiting for
 * it (pgm_dq_wait then waits for it with the dispatches), so several queues release in parallel */
int pgm_dq_release(void *dq);
/* wait until every dispatch issued on the queue has completed (no release barrier: call pgm_dq_sync
 * before HIP work reads the outputs) */
int pgm_dq_wait(void *dq);
int pgm_dq_timer_start(void *dq);
int pgm_dq_timer_stop_ms(void *dq, float *ms);
/* the same span as raw HSA system timestamps (start of the first timed dispatch, latest end) and their
 * frequency, so spans of several queues can be joined */
int pgm_dq_timer_stop_ticks(void *dq, uint64_t *start, uint64_t *end, uint64_t *freq);
/* after a timer stop: the sum of the timed dispatches' own durations (end - start, in the ticks of
 * pgm_dq_timer_stop_ticks) and how many were summed (those still in the 256-signal ring) — the
 * per-launch duration a kernel trace reports, which exceeds span / launches when queues overlap */
int pgm_dq_timer_dispatch_stats(void *dq, uint64_t *sum_ticks, uint64_t *count);
/* r06: after a timer stop, each timed dispatch's own start / end (HSA system ticks, the frequency of
 * pgm_dq_timer_stop_ticks) in issue order, at most cap of them (those still in the signal ring);
 * *count = how many were written.  The raw timestamps behind the C3 line's span-based frac. */
int pgm_dq_timer_dispatch_times(void *dq, uint64_t *start, uint64_t *end, int32_t cap, int32_t *count);
int pgm_dq_bound_destroy(void *dbound);
/* r05 (ABI 22): a compiled query's steps on the queue (VariableElimination.query through a captured
 * plain Program, pgmpy/inference/ExactInference.py:349-440, C1 / C2).  pgm_dq_bind_pm re-binds one
 * plan-specialised launch (pgm_pm_bound_* handle: a fused product step, a merged level or a specialised
 * contraction batch) to the queue; pgm_dq_run_chain writes the n launches as one dependent chain (each
 * packet's barrier bit set unless independent[i] is 1 — launch i reads nothing launch i-1 writes; the last
 * packet always waits for every earlier one — and
 * agent-scope fences on every packet, the last releasing at system scope — inputs the host writes between
 * chains must be in coherent host memory (pgm_host_alloc), which the kernels read uncached; independent
 * may be NULL), rings the doorbell once and returns when the last has completed — the outputs are then
 * visible to the host.  Contract: no HIP work that writes the chain's inputs may be pending (the chain
 * does not drain the device; the host writes inputs through mapped memory).  At most 128 launches.  All n
 * slots are reserved at once after every check that can fail (no half-written chain is left on the
 * queue).  Refused (PGM_EINVAL) while a pgm_dq_timer span is open on the queue: only the last packet
 * carries a completion signal, so there are no per-dispatch timestamps to report.
 * pgm_dq_profiling turns the queue's dispatch timestamps on or off (pgm_dq_timer_* need them).  Leave it
 * on for a queue a profiler may intercept (r06): a kernel-tracing tool reads every dispatch's timestamps
 * from its own completion signals, which needs the queue's profiling enabled — r05 turned it off on the
 * query queue and rocprofv3 crashed on the chain. */
int pgm_dq_bind_pm(void *dq, void *pm_bound, void **dbound);
int pgm_dq_run_chain(void *const *dbounds, const uint8_t *independent, int32_t n);
int pgm_dq_profiling(void *dq, int32_t on);

#ifdef __cplusplus
}
#endif
#endif /* PGMHIP_H */

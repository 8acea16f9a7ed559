// pgm_internal.h — private interface between pgmhip.hip (kernels, C-ABI), pgmdq.cpp (direct AQL
// dispatch) and pgmpm.cpp (plan-specialised batched-BP steps).  Not part of the C-ABI of
// include/pgmhip.h.
#pragma once
#include <cstddef>
#include <cstdint>

extern "C" {

typedef struct {
  const void *code;    // hipRTC code object of the plan-specialised kernel
  size_t code_size;
  const char *kernel;  // pgm_rows_jit or pgm_rows_jit2
  const void *args;    // packed explicit argument segment
  size_t args_size;
  unsigned blocks;     // workgroups (1-D grid)
  unsigned wg;         // work-items per workgroup
  const void *owner;   // the plan handle the code object belongs to
  int write_through;   // every output store of the kernel is write-through (sc1): no release needed
} pgmi_jit_launch;

int pgmi_rows_bound_jit(void *bound, pgmi_jit_launch *out);
int pgmi_pm_bound_jit(void *bound, pgmi_jit_launch *out);  // pgmpm.cpp: a specialised step / batch
int pgmi_fail(int code, const char *msg);  // set pgm_last_error, return code
int pgmi_failf(int code, const char *fmt, ...);  // printf-style pgmi_fail
}

#ifdef __cplusplus
#include <string>
#include <vector>

#include "pgmhip.h"

#define KMAX 12  // dims of a contraction / fused-step index space (incl. the row dim)
#define MOPS 8   // operands of a fused product + marginal step (r05: 4 -> 8, so a clique's pass reads its
                 // child messages directly instead of pre-multiplied aggregates)

// n / d for n < 2^31 with one mul-hi and one shift (Granlund-Montgomery round-up method)
struct FDiv {
  uint32_t d, m, s;
};

// a planned contraction (pgmhip.hip plan_contract; the generic kernels read it, pgmpm.cpp compiles a
// batch of them into a specialised kernel)
struct ContractK {
  int32_t nk, nr, g_log2, n_split;
  uint32_t n_out, n_red, red_chunk, row_mode;  // red_chunk: reduction-OUTER indices per split
  uint32_t n_ro, ri_card;                       // reduction = n_ro outer x ri_card innermost
  int64_t ri_sa, ri_sb;                         // strides of the innermost reduction dim
  uint32_t ri_chunk, ri_nb;                     // row mode: innermost dim cut in ri_nb chunks of ri_chunk
  uint32_t n_v, _pad2;                          // row mode: virtual reduction-outer count n_ro * ri_nb
  FDiv kdiv[KMAX];
  int64_t ksa[KMAX], ksb[KMAX], ksc[KMAX];
  FDiv rdiv[KMAX];
  int64_t rsa[KMAX], rsb[KMAX];
};

// a planned per-row evidence gather (pgm_gather: C[out] = A[out's offset + sum of codes x strides])
struct GatherK {
  int32_t nk, n_ev, batch_dim, _pad;
  uint32_t n_out, _pad2;
  int64_t ld, row0;
  FDiv kdiv[KMAX];
  int64_t ksa[KMAX], ksc[KMAX];
  int64_t ev_col[PGM_MAX_DIMS], ev_stride[PGM_MAX_DIMS];
  int32_t ev_card[PGM_MAX_DIMS];
};

// a planned n-ary contraction (pgm_batch_add_contract_n: C[keep] = reduce over red of prod_t X_t; r06):
// several pairwise steps of a contraction path done as ONE job, so the path has fewer dependency levels
struct ContractNK {
  int32_t n_ops, nk, nr, red, g_log2, _pad;
  uint32_t n_out, n_red;
  uint32_t kcard[KMAX], rcard[KMAX];
  int64_t ksc[KMAX];
  int64_t ks[MOPS][KMAX], rs[MOPS][KMAX];
};

// one job of a batch (pgm_batch_*) as the specialiser sees it: blocks [block0, block0 + nblocks) of
// the batch's 256-thread blocks; kind 0: C[keep] = reduce(combine(A, B)) (k), 1: an evidence gather (g),
// 2: an n-ary contraction (n, operands ops[0 .. n.n_ops))
struct pgmi_cs_job {
  int32_t kind, cmb, red;
  uint32_t block0, nblocks;
  const double *A, *B;
  double *C;
  const uint8_t *codes;
  int32_t *err;
  ContractK k;
  GatherK g;
  ContractNK n;
  const double *ops[MOPS];
};

// a plan-specialised kernel for a batch of contraction jobs (pgmpm.cpp): one_wg = 0: one launch of
// the batch's blocks (one level); 1: the single-workgroup levelled form (level_off: first block of
// each level + the end).  *bound = NULL when a job is not one it takes (the generic kernel runs).
int pgmi_cs_bind(const pgmi_cs_job *jobs, int n, const uint32_t *level_off, int n_levels, int one_wg, void **bound);

// the fused product + marginal step's plan (pgmhip.hip plans it and runs the generic kernels;
// pgmpm.cpp compiles it into specialised kernels)
struct ProdMK {
  int32_t n_ops, nk, nr, n_red;  // nk: kept outer dims + the row dim (last); nr: reduced dims
  int32_t mdiv;                  // >= 0: the marginal is stored divided by this operand (0/0 -> 0; PGM_PRODN_MDIV)
  int32_t kind[MOPS];
  int32_t vec[MOPS];             // operand has the row axis (stride 1) / is broadcast over rows
  int32_t jvar[MOPS];            // operand varies over the reduced entries (else loaded once per outer)
  uint32_t n_outer, NP;          // kept outer index space; row pairs
  FDiv kdiv[KMAX];
  int64_t ksc[KMAX], ksm[KMAX], ks[MOPS][KMAX];
  FDiv rdiv[KMAX];
  int64_t rsc[KMAX], rs[MOPS][KMAX];
  const double *ops[MOPS];
};

struct dim3;
int pgmi_plan_product_marg(const pgm_productn_desc *d, const double *const *ops, const double *C,
                           const int64_t *marg_s, const double *M, ProdMK &k, dim3 &grid);
void pgmi_appendf(std::string &o, const char *fmt, ...);  // printf into a growing source string
void pgmi_stale_probe(const char *fn);                   // PGM_STALE_PROBE=1 debugging aid
// gfx950 code object of a generated kernel source: the on-disk cache, else hipRTC (then cached)
bool pgmi_rtc_code(const std::string &src, const char *what, std::vector<char> &code);
#define STALE_PROBE() pgmi_stale_probe(__func__)
#endif

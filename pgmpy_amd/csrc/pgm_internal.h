// pgm_internal.h — private interface between pgmhip.hip (kernels, C-ABI) and pgmdq.cpp (direct AQL
// dispatch).  Not part of the C-ABI of include/pgmhip.h.
#pragma once
#include <cstddef>

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
int pgmi_fail(int code, const char *msg);  // set pgm_last_error, return code
}

// Internal interface between the fused-program interpreter (bq_fused.hip)
// and its native compiled form (bq_fused_jit.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "binquant_amd.h"

#define BQ_STR_(x) #x
#define BQ_STR(x) BQ_STR_(x)

namespace bq {
// opcode / index / operand checks of a bq_fused_program (BQ_OK or BQ_EINVAL)
int fused_validate(const bq_fused_program& P);
// native path on (BQ_FUSED_NATIVE unset or non-zero, or bq_fused_set_native(1))
bool fused_native_enabled();
// launch the program's compiled kernel (compiling it on first use)
int fused_native_eval(const bq_fused_program& P, int64_t S, int64_t T, hipStream_t stream);
}  // namespace bq

// Operand layout TT (A M-contiguous, B K-contiguous) of the MFMA GEMM
// (gemm_impl.h): its kernel instantiations in a translation unit of their own.
#include "gemm_impl.h"

TDG_GEMM_LAYOUT(tt, false, true)

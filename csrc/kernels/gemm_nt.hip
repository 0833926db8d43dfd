// Operand layout NT (A K-contiguous, B K-contiguous) of the MFMA GEMM
// (gemm_impl.h): its kernel instantiations in a translation unit of their own.
#include "gemm_impl.h"

TDG_GEMM_LAYOUT(nt, true, true)

// Operand layout NN (A K-contiguous, B N-contiguous) of the MFMA GEMM
// (gemm_impl.h): its kernel instantiations in a translation unit of their own.
#include "gemm_impl.h"

TDG_GEMM_LAYOUT(nn, true, false)

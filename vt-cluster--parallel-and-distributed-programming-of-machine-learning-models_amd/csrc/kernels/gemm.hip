// translation unit 0 of the GEMM kernels (see gemm_impl.h)
#define MIFT_GEMM_PART 0
#include "gemm_impl.h"

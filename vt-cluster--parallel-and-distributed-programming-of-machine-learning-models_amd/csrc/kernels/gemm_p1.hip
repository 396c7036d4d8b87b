// translation unit 1 of the GEMM kernels (see gemm_impl.h)
#define MIFT_GEMM_PART 1
#include "gemm_impl.h"

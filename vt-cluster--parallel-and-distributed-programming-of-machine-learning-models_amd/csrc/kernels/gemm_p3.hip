// translation unit 3 of the GEMM kernels (see gemm_impl.h)
#define MIFT_GEMM_PART 3
#include "gemm_impl.h"

// translation unit 2 of the GEMM kernels (see gemm_impl.h)
#define MIFT_GEMM_PART 2
#include "gemm_impl.h"

// combine_t_int.hip -- the fold kernels for int elements (combine_kernels.h), one
// translation unit per element type so the instantiations compile in parallel.
#include "combine_kernels.h"

MI355_COMBINE_TYPE(int32_t, int)

// combine_t_long.hip -- the fold kernels for long elements (combine_kernels.h), one
// translation unit per element type so the instantiations compile in parallel.
#include "combine_kernels.h"

MI355_COMBINE_TYPE(int64_t, long)

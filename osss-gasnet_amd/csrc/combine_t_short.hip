// combine_t_short.hip -- the fold kernels for short elements (combine_kernels.h), one
// translation unit per element type so the instantiations compile in parallel.
#include "combine_kernels.h"

MI355_COMBINE_TYPE(int16_t, short)

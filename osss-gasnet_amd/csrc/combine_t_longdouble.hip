// combine_t_longdouble.hip -- the fold kernels for longdouble elements (combine_kernels.h), one
// translation unit per element type so the instantiations compile in parallel.
#include "combine_kernels.h"

MI355_COMBINE_TYPE(x80, longdouble)

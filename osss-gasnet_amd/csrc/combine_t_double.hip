// combine_t_double.hip -- the fold kernels for double elements (combine_kernels.h), one
// translation unit per element type so the instantiations compile in parallel.
#include "combine_kernels.h"

MI355_COMBINE_TYPE(double, double)

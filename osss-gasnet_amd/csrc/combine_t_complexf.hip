// combine_t_complexf.hip -- the fold kernels for complexf elements (combine_kernels.h), one
// translation unit per element type so the instantiations compile in parallel.
#include "combine_kernels.h"

MI355_COMBINE_TYPE(cplxf, complexf)

// combine_t_complexd.hip -- the fold kernels for complexd elements (combine_kernels.h), one
// translation unit per element type so the instantiations compile in parallel.
#include "combine_kernels.h"

MI355_COMBINE_TYPE(cplxd, complexd)

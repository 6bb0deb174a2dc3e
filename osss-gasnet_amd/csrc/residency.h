// residency.h -- blocks per CU the spin-waiting grids are sized for.
//
// Every block of a fused_allreduce / fused_server / fused_pull grid waits for
// the grid's last block and for the other members, so all of them must be
// resident at once (fused.hip, coresident_grid). A launch takes at most
// min(occupancy API, MI355_FUSED_RESIDENT_PER_CU) - 1 blocks per CU. The API
// ignores the SGPR admission limit of 256-thread blocks,
// floor(800 / (ceil(sgpr / 16) * 16 + 16)) per CU (MI355X_MICROARCH.md
// "Residency"), so the build checks the compiled kernels against this
// constant: tools/check_residency.py reads every such kernel's .sgpr_count /
// .vgpr_count / LDS size from the code object and fails the build when one
// admits fewer blocks per CU than this.
#pragma once
#define MI355_FUSED_RESIDENT_PER_CU 6

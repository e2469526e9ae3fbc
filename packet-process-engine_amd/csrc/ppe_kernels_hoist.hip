// The stateless hoisted-fetch classify kernels over an LDS-resident image (C1's variant), built from
// csrc/ppe_kernels.hip with LLVM's iterative-ILP machine scheduler (Makefile); the default build routes those launches
// and occupancy queries here (ppe_launch_classify_hoist_lds / ppe_occupancy_hoist_lds).
#define PPE_TU_HOIST 1
#include "ppe_kernels.hip"

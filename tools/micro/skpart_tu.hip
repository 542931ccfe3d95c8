// resource usage of k_skpart_w alone (hipcc -Rpass-analysis=kernel-resource-usage): quick
// register / LDS checks while reshaping the partition kernel, without compiling assemble.hip
#include "../../pycuda-euler_amd/csrc/common.h"
#include "../../pycuda-euler_amd/csrc/count_sk2.h"
template __global__ void ec::k_skpart_w<7, 17, true>(const uint8_t *__restrict__, const uint64_t *__restrict__, uint64_t,
                                                     ec::MinCfg, uint32_t, uint64_t, uint32_t, uint64_t, uint32_t,
                                                     uint4 *, unsigned int *, uint8_t *, unsigned long long *,
                                                     unsigned int *, unsigned int *, unsigned long long *, uint32_t);
template __global__ void ec::k_skpart_w<7, 17, false>(const uint8_t *__restrict__, const uint64_t *__restrict__, uint64_t,
                                                      ec::MinCfg, uint32_t, uint64_t, uint32_t, uint64_t, uint32_t,
                                                      uint4 *, unsigned int *, uint8_t *, unsigned long long *,
                                                      unsigned int *, unsigned int *, unsigned long long *, uint32_t);

// K-streamed fused 1x1 convolutions (csrc/conv/conv1x1_ks.hip): the deep-reduction (K 1024 /
// 2048) sibling of conv1x1_bn, with the same operand prologues (codes 0 none, 2 BN backward,
// 3 block-output BN + shortcut + ReLU) and epilogues (forward: the consuming BN's statistics
// partials; dgrad: the output BN's backward reduction with the ReLU mask recomputed).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace apex_amd {

bool conv1x1_ks_supported(int64_t m, int k, int ncols);
// rows G of the [2][G][ncols] statistics / reduction partials
int conv1x1_ks_partials(int64_t m, int k, int ncols, int cus, int pro);
void conv1x1_ks(const void* a, const void* w, void* y, int64_t m, int k, int ncols, bool wt, int dtype,
                const float* pcoef, int pro, bool pc_split, const float* pc_res, const float* shift, float* part,
                const void* py, void* aout, uint8_t* bout, const float* rcoef, const void* rx, const float* rmean,
                int cus, hipStream_t s);

}  // namespace apex_amd

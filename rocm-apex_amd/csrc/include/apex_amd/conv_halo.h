// Halo-tile 3x3 stride-1 convolution (csrc/conv/conv3x3_halo.hip): C % 64 == 0, K % 128 == 0, no
// fused epilogue but the BN statistics; optional operand prologue relu(x * pcoef[c] + pcoef[C + c])
// (the producing batch norm + ReLU, applied to the staged input, padding kept zero).  The default
// engine of conv_tap_fprop where it applies (APEX_AMD_CONV_HFP=0 disables).
#pragma once
#include "apex_amd/conv_api.h"

namespace apex_amd {

bool conv_hfp_supported(const ConvTapArgs& a);
// 0: never, 1: small images (the default), 2: wherever supported; -1: back to APEX_AMD_CONV_HFP
void conv_hfp_set_mode(int mode);
bool conv_hfp_default(const ConvTapArgs& a);
int conv_hfp_stats_rows(const ConvTapArgs& a, int cus);  // statistics partial rows (workgroups per k-block)
void conv_hfp(const ConvTapArgs& a, const float* pcoef, int cus, hipStream_t s);

// the halo-tile 3x3 weight gradient (conv3x3_wgrad.hip) with its input through the producing BN
// + ReLU, x' = relu(x * xcoef[c] + xcoef[C + c]) (xcoef fp32 [2][C], null = plain); same support
// and workspace as conv_hwgrad
void conv_hwgrad_pro(const ConvTapArgs& a, const void* dy, void* dw_out, int out_dtype, float* ws, int cus,
                     hipStream_t s, const float* xcoef);

// the spatial-tile 64 -> 64 3x3 forward (conv3x3_sp.hip) with the same input prologue (pcoef fp32
// [2][64], null = plain; padding stays zero)
void conv_sp_fprop_pro(const ConvTapArgs& a, const float* pcoef, int cus, hipStream_t s);

}  // namespace apex_amd

// The single native extension of the package: apex._C (file rocm-apex_amd/_C*.so).
// Each subsystem registers a submodule; python code imports e.g. `apex._C.amp_C`.
#include "common.h"

namespace apex_amd {
void bind_amp_C(pybind11::module_& m);
void bind_norm(pybind11::module_& m);
void bind_softmax(pybind11::module_& m);
void bind_syncbn(pybind11::module_& m);
void bind_gemm(pybind11::module_& m);
void bind_xentropy(pybind11::module_& m);
void bind_attn(pybind11::module_& m);
void bind_contrib(pybind11::module_& m);
void bind_bn_nhwc(pybind11::module_& m);
void bind_conv(pybind11::module_& m);
}  // namespace apex_amd

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "MI355X (gfx950) native kernels for the apex-compatible framework";
  m.attr("arch") = "gfx950";
  apex_amd::bind_amp_C(m);
#ifdef APEX_AMD_WITH_NORM
  apex_amd::bind_norm(m);
#endif
#ifdef APEX_AMD_WITH_SOFTMAX
  apex_amd::bind_softmax(m);
#endif
#ifdef APEX_AMD_WITH_SYNCBN
  apex_amd::bind_syncbn(m);
#endif
#ifdef APEX_AMD_WITH_GEMM
  apex_amd::bind_gemm(m);
#endif
#ifdef APEX_AMD_WITH_XENTROPY
  apex_amd::bind_xentropy(m);
#endif
#ifdef APEX_AMD_WITH_ATTN
  apex_amd::bind_attn(m);
#endif
#ifdef APEX_AMD_WITH_BN_NHWC
  apex_amd::bind_bn_nhwc(m);
#endif
#ifdef APEX_AMD_WITH_CONV
  apex_amd::bind_conv(m);
#endif
#ifdef APEX_AMD_WITH_CONTRIB
  apex_amd::bind_contrib(m);
#endif
}

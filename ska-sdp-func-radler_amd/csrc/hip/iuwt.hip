// IUWT à-trous B3-spline decomposition (IuwtDecomposition,
// cpp/algorithms/iuwt/iuwt_decomposition.{h,cc}). Placeholder until the
// separable LDS-tiled kernels land; fails loudly.
#include "rdl_internal.h"

extern "C" {
int rdl_iuwt_decompose(rdl_session* s, const float*, uint32_t, uint32_t,
                       uint32_t, float*, float*, int) {
  (void)s;
  rdl::SetError("rdl_iuwt_decompose: not implemented yet");
  return RDL_ERR_UNSUPPORTED;
}
int rdl_iuwt_recompose(rdl_session* s, const float*, uint32_t, uint32_t,
                       uint32_t, float*, float*, int) {
  (void)s;
  rdl::SetError("rdl_iuwt_recompose: not implemented yet");
  return RDL_ERR_UNSUPPORTED;
}
}

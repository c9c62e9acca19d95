// Two-stage pipeline instantiations, fp32 S = 17..32,
// per-step and sum form, wrap (1x1 periodic) and ghost-ring forms.
#include "stencil_pipe.hpp"

namespace mxs {
namespace kernels {
namespace detail {

template <typename T, int S, bool WRAP, bool SUM, int XB>
void launch_pipe(const T* in, T* out, const TileGeom& g, index_t x0, index_t x1, index_t y0, index_t y1, T c0, T c1,
                 T sc, hipStream_t s) {
  launch_pipe_impl<T, S, WRAP, SUM, XB>(in, out, g, x0, x1, y0, y1, c0, c1, sc, s);
}

#define MXS_INST_LAUNCH(S, WRAP, SUM)                                                                \
  template void launch_pipe<float, S, WRAP, SUM>(const float*, float*, const TileGeom&, index_t, index_t, index_t, \
                                               index_t, float, float, float, hipStream_t);
#define MXS_INST_PIPE(S)      \
  MXS_INST_LAUNCH(S, true, false)  \
  MXS_INST_LAUNCH(S, true, true)   \
  MXS_INST_LAUNCH(S, false, false) \
  MXS_INST_LAUNCH(S, false, true)

MXS_INST_PIPE(17)
MXS_INST_PIPE(18)
MXS_INST_PIPE(19)
MXS_INST_PIPE(20)
MXS_INST_PIPE(21)
MXS_INST_PIPE(22)
MXS_INST_PIPE(23)
MXS_INST_PIPE(24)
MXS_INST_PIPE(25)
MXS_INST_PIPE(26)
MXS_INST_PIPE(27)
MXS_INST_PIPE(28)
MXS_INST_PIPE(29)
MXS_INST_PIPE(30)
MXS_INST_PIPE(31)
MXS_INST_PIPE(32)

#undef MXS_INST_PIPE
#undef MXS_INST_LAUNCH

// The scaled form (any c_center, c_neighbor != 0) at the solver's depths.
template void launch_pipe<float, 20, true, true, kScaledBody>(const float*, float*, const TileGeom&, index_t, index_t,
                                                           index_t, index_t, float, float, float, hipStream_t);
template void launch_pipe<float, 20, false, true, kScaledBody>(const float*, float*, const TileGeom&, index_t, index_t,
                                                           index_t, index_t, float, float, float, hipStream_t);
template void launch_pipe<float, 24, true, true, kScaledBody>(const float*, float*, const TileGeom&, index_t, index_t,
                                                           index_t, index_t, float, float, float, hipStream_t);
template void launch_pipe<float, 24, false, true, kScaledBody>(const float*, float*, const TileGeom&, index_t, index_t,
                                                           index_t, index_t, float, float, float, hipStream_t);


}  // namespace detail
}  // namespace kernels
}  // namespace mxs

// Two-stage pipeline instantiations, fp64 S = 9..16 (wide-lane body),
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

template <typename T, int S, bool WRAP>
bool wide_pipe_ok(const TileGeom& g, index_t x0, index_t x1, index_t y0, index_t y1) {
  return wide_pipe_ok_impl<T, S, WRAP>(g, x0, x1, y0, y1);
}

#define MXS_INST_LAUNCH(S, WRAP, SUM)                                                                \
  template void launch_pipe<double, S, WRAP, SUM>(const double*, double*, const TileGeom&, index_t, index_t, index_t, \
                                               index_t, double, double, double, hipStream_t);
#define MXS_INST_PIPE(S)                                                                                 \
  MXS_INST_LAUNCH(S, true, false)                                                                        \
  MXS_INST_LAUNCH(S, true, true)                                                                         \
  MXS_INST_LAUNCH(S, false, false)                                                                       \
  MXS_INST_LAUNCH(S, false, true)                                                                        \
  template bool wide_pipe_ok<double, S, true>(const TileGeom&, index_t, index_t, index_t, index_t);      \
  template bool wide_pipe_ok<double, S, false>(const TileGeom&, index_t, index_t, index_t, index_t);

MXS_INST_PIPE(9)
MXS_INST_PIPE(10)
MXS_INST_PIPE(11)
MXS_INST_PIPE(12)
MXS_INST_PIPE(13)
MXS_INST_PIPE(14)
MXS_INST_PIPE(15)
MXS_INST_PIPE(16)

#undef MXS_INST_PIPE
#undef MXS_INST_LAUNCH

// The scaled form (any c_center, c_neighbor != 0) at the solver's depths.
template void launch_pipe<double, 16, true, true, kScaledBody>(const double*, double*, const TileGeom&, index_t, index_t,
                                                           index_t, index_t, double, double, double, hipStream_t);
template void launch_pipe<double, 16, false, true, kScaledBody>(const double*, double*, const TileGeom&, index_t, index_t,
                                                           index_t, index_t, double, double, double, hipStream_t);


}  // namespace detail
}  // namespace kernels
}  // namespace mxs

// Host API of the hand-written CDNA4 (gfx950) kernels. Every launcher is
// stream-ordered, allocation-free and synchronisation-free, so any sequence of
// them can be captured into a hipGraph (cdna_hip_programming.md Guideline 9).
//
// Kernel inventory:
//   K1/K3  fill, fill_region, fill_random       kernels/fill.hip
//   K10    stencil5_rows / stencil5_rect         kernels/stencil.hip
//          stencil_box (LDS-tiled (2R+1)^2)      kernels/stencil.hip
//   K11/12 copy2d_batch (halo pack/unpack/self)  kernels/halo.hip
//   K2/4/5/8 dot_atomic, dot_partials, reduce_partials, dot_single_pass, dot_racy
//                                                kernels/dot.hip
#pragma once

#include <hip/hip_runtime_api.h>

#include <cmath>
#include <cstdint>
#include <limits>

#include "mxs/grid/layout.hpp"
#include "mxs/kernels/chunk_schedule.hpp"

namespace mxs {
namespace kernels {

// ---------------------------------------------------------------- fill (K1/K3)
template <typename T>
void fill(T* p, index_t n, T value, hipStream_t s);
// Fill a window of a buffer (reference InitKernel, stencil2d/mpi-2d-stencil-subarray-cuda.cu:17-28,
// which launched one thread per block).
template <typename T>
void fill_region(T* base, const Array2D& region, T value, hipStream_t s);
// Deterministic pseudo-random init of the core of a tile in [lo, hi): the value of
// a cell depends only on its *global* coordinates and the seed, so any domain
// decomposition of the same global grid starts from bit-identical data.
template <typename T>
void fill_random(T* tile, const TileGeom& g, index_t global_x0, index_t global_y0,
                 index_t global_width, std::uint64_t seed, T lo, T hi, hipStream_t s);

// ------------------------------------------------------------- stencil (K10)
// out = c_center * u[y][x] + c_neighbor * ((u[y-1][x] + u[y+1][x]) + (u[y][x-1] + u[y][x+1]))
// evaluated as fma(c_neighbor, (n + s) + (w + e), c_center * c) in the element type, so
// every kernel variant and the host reference agree bit for bit.
struct Stencil5Coeffs {
  double center = 0.2;
  double neighbor = 0.2;
  // With center == neighbor (= c, the 5-point average) the S-step kernels may
  // run the sum form: each pass accumulates plain 5-point sums and scales by
  // c^S once when it stores (8 instead of 11 VALU issue slots per 4 fp32 cells
  // and step; stencil_device.hpp). Equal to the per-step evaluation up to
  // rounding (a few ulp), not bit for bit. With center != neighbor (neighbor
  // != 0) the pipeline passes run the scaled form instead: v' = (n + s + w + e)
  // + (center / neighbor) v per level, neighbor^S once per pass (9 instead of 11
  // slots). false = always the per-step form.
  bool sum_form = true;
  // Bound on max|u| of a pass's input field (the solver passes its measured,
  // agreed absmax), or < 0: unknown. See fast_form_safe().
  double range = -1.0;
};
inline bool uses_sum_form(const Stencil5Coeffs& c) { return c.sum_form && c.center == c.neighbor; }
// The scaled form (stencil_device.hpp): unequal coefficients, c_neighbor != 0,
// in the fp32 pipeline (20 / 24) and balanced stream kernel (2-16) and the fp64
// wide pipeline (16); other depths and kernel forms run per step.
inline bool uses_scaled_form(const Stencil5Coeffs& c) {
  return c.sum_form && c.center != c.neighbor && c.neighbor != 0.0;
}
// The kernel layer's guard of both fast forms for an S-level pass in element
// type T (stencil5_tb and the chunk pass choose their form through it; the
// solver's range guard is the measured, collective version of the same bounds,
// and passes its bound in `range`):
//   * |c_center| + 4 |c_neighbor| <= 1: the operator is bounded by the field;
//   * c_neighbor^S is a normal number of T (it scales the stored result);
//   * inside a pass the carried values grow by up to (4 + |k|)^S (k =
//     c_center / c_neighbor; 5^S for the sum form): range (4 + |k|)^S < max/4.
// With the range unknown (range < 0) only a form that grows no faster than the
// sum form (|k| <= 1) is taken, under the sum form's documented contract
// (max|u| 5^S < max/4 is the caller's); a faster-growing scaled form runs per
// step (c_center 0.9, c_neighbor 0.013 grows as 73^S: 2e37 at S = 20).
template <typename T>
inline bool fast_form_safe(const Stencil5Coeffs& c, int S) {
  if (!(uses_sum_form(c) || uses_scaled_form(c))) return false;
  if (!(std::fabs(c.center) + 4.0 * std::fabs(c.neighbor) <= 1.0 + 1e-6)) return false;
  if (!(std::fabs(double(T(std::pow(c.neighbor, double(S))))) >= double(std::numeric_limits<T>::min()))) return false;
  const double k = std::fabs(c.center / c.neighbor);
  if (c.range < 0.0) return k <= 1.0;
  return std::isfinite(c.range) && c.range * std::pow(4.0 + k, double(S)) < double(std::numeric_limits<T>::max()) / 4.0;
}

enum class StencilVariant : int {
  Auto = 0,        // tuned default
  RegisterRoll = 1,  // rolling 3-row register window, x-neighbours by wave shuffles
  LdsTile = 2,       // LDS-staged 2D tile with a 1-cell ring
};

// Update core rows [row_begin, row_end) over the full core width. Columns 0 and
// width-1 read the ghost columns, so the result is only final once the halo for
// the current iteration has landed (see StencilSolver for the overlap schedule).
template <typename T>
void stencil5_rows(const T* in, T* out, const TileGeom& g, index_t row_begin, index_t row_end,
                   Stencil5Coeffs c, hipStream_t s, StencilVariant v = StencilVariant::Auto);

// Full-tile update of a 1x1 periodic grid with the self-exchange fused into the
// addressing (row -1 reads row H-1, column W reads column 0, ...): one launch per
// iteration, no ghost traffic. Needs width % (16 / sizeof(T)) == 0.
template <typename T>
void stencil5_periodic(const T* in, T* out, const TileGeom& g, Stencil5Coeffs c, hipStream_t s);
template <typename T>
bool stencil5_periodic_supported(const TileGeom& g);

// Temporal blocking: `steps` (S) Jacobi iterations in one launch over the core
// rectangle [x0, x1) x [y0, y1): every input byte crosses HBM once per S
// iterations. The source must hold valid data S cells around the rectangle: a
// ghost ring >= S deep exchanged for this super-step, or `wrap` (1x1 periodic
// grid: reads wrap around the tile). Bitwise identical to S single steps (same
// per-cell fma sequence). Variants:
//   Auto         wave-streaming kernel (register windows per time level, no LDS)
//                for the bulk, LDS tiles of matching shape for thin strips;
//   LdsTile      LDS-tiled (each workgroup stages its tile plus an S-deep apron,
//                iterates in LDS; S <= 8 for the bulk tile);
//   RegisterRoll same as Auto.
constexpr int kMaxTimeBlock = 16;
// fp32 blocks of 17..32 steps run on the two-stage wave pipeline
// (stencil5_stream_pipe_kernel: two waves per column strip, levels split
// between them and handed over through LDS). Needs fp32, x0 and x1 multiples
// of 4 (whole vectors); see stencil5_deep_supported().
constexpr int kMaxTimeBlockDeep = 32;
// Largest chunk (rows x pitch bytes) one workgroup of the streaming kernels
// stores through a single buffer descriptor: below 2^31 with room for the
// drop offsets of stencil_device.hpp (a sum of two never wraps).
constexpr index_t kMaxChunkBytes = 0x7F000000;
// The wave pipelines walk a longer share in pieces of at most kMaxChunkBytes;
// rows must be narrow enough that a piece holds at least this many (each piece
// pays its own pipeline fill of S rows).
constexpr index_t kMinChunkRows = 64;
// Measured default S for a w x h tile of `elem_bytes`-byte cells
// (profiles/stencil_tuning/tunes_*, profiles/r02_deep/pipe*_*, profiles/r02_f64,
// profiles/r02_sum): fp32 takes the two-stage pipeline at S = 20 (sum form,
// split 10 + 10: 32768^2 9.96 T cells/s, 16384 x 8192 9.18, 8192^2 7.79; the
// per-step form 11 + 9: 8.27 / 7.56 / 6.46; S = 24-28 adds 2-4% at 32768^2
// only); fp64 the wide-lane pipeline at S = 16 in the sum form (8 + 8: 3.5 /
// 4.05 T cells/s at 8192^2 / 16384^2) or S = 12 per step (6 + 6: 3.0 / 3.3);
// the fp32 single-wave kernels (small tiles): S = 16 from 2^27 cells, S = 12
// below (the pass is VALU-bound beyond S ~ 8, so a deeper block only pays
// where the chunk / strip aprons are small against the tile).
inline int auto_time_block(index_t w, index_t h, int elem_bytes = 4, bool sum_form = true) {
  // Rows too wide for kMinChunkRows per descriptor-sized piece (beyond ~8.3 M
  // fp32 columns; the padded pitch is at most w + 256): the fp32 pipelines
  // cannot take them, the single-wave kernels can (their non-descriptor body).
  if (elem_bytes == 4 && (w + 256) * 4 * kMinChunkRows > kMaxChunkBytes) return kMaxTimeBlock;
  if (elem_bytes == 4 && w >= 1024 && h >= 1024) {
    // The pipeline runs workgroups of 4 strips; with joint stage-1 windows a
    // group stores 912 columns at S = 20 (12 + 8) and 904 at S = 24 (12 + 12),
    // and a partial last group costs a whole one. S = 24 when it needs no more
    // groups than S = 20 (4096 wide: 5 and 5); otherwise the extra group costs
    // more than the deeper block saves (8192^2 sum form: 9 vs 10 groups,
    // 8.6-8.9 T cells/s at S = 20 vs 8.4 at 24; 16384 wide: 18 vs 19 groups,
    // 9.8-10.0 vs 9.4; profiles/r02_joint).
    auto groups = [&](int owg) { return (w + owg - 1) / owg; };
    if (sum_form && groups(904) <= groups(912)) return 24;
    // Tiles of >= 2^30 cells (chunks of ~4800 rows, warm-up negligible): the
    // deeper block relieves HBM and wins even at one group more, 32768^2 sum
    // form 11.1 T cells/s at S = 24 vs 10.9 at 20 (37 vs 36 groups). A 20-step
    // run is still one S = 20 pass (run(K) splits K near-equally).
    if (sum_form && w * h >= (index_t(1) << 30)) return 24;
    return 20;
  }
  if (elem_bytes == 8) return sum_form ? 16 : 12;
  return w * h >= (index_t(1) << 27) ? 16 : 12;
}
// Whether a `steps`-step stencil5_tb launch over [x0, x1) can run: every
// steps <= kMaxTimeBlock; deeper blocks only for fp32 on whole vectors.
template <typename T>
constexpr bool stencil5_deep_supported(int steps, index_t x0, index_t x1) {
  return steps <= kMaxTimeBlock || (steps <= kMaxTimeBlockDeep && sizeof(T) == 4 && x0 % 4 == 0 && x1 % 4 == 0);
}
template <typename T>
void stencil5_tb(const T* in, T* out, const TileGeom& g, int steps, index_t x0, index_t x1, index_t y0, index_t y1,
                 Stencil5Coeffs c, bool wrap, hipStream_t s, StencilVariant v = StencilVariant::Auto);

// ------------------------------------- chunk-list pass (interior-first super-step)
// The S-step pass over chunks of the core of a ghost-ring tile (no wrap) on the
// two-stage pipeline: workgroup w runs the chunk list table[w * entries ..]
// (kernels/chunk_schedule.hpp). Bitwise identical, per cell, to stencil5_tb
// over the same core (same per-cell arithmetic and kernel body; only the
// workgroup-to-chunk assignment differs).
struct ChunkPassShape {
  int steps = 0;
  bool sum = false;   // sum form (c_center == c_neighbor and allowed)
  bool scaled = false;  // scaled form (c_center != c_neighbor, c_neighbor != 0, allowed)
  int js0 = 0;        // stage-0 levels of the joint windows
  int lag1 = 0;       // level-order mask (stencil_pipe.hpp)
  int blocks = 0;     // resident workgroups (one per CU)
  index_t groups = 0;  // column groups of OWG output columns over the core width
  index_t owg = 0;
  index_t fill = 0;    // pipeline-fill row iterations per chunk
  // Input columns a group's joint windows read: [x - read_lead, x - read_lead +
  // read_span) for a group whose first output column is x (its chunks read the
  // ghost columns when that range leaves [0, width)).
  index_t read_lead = 0, read_span = 0;
};
// False when `steps` has no chunk-list form here (fp32 S = 20 / 24, fp64
// S = 16 on whole lane vectors; other depths keep the one-launch pass). The
// caller still has to keep every chunk of its schedule within kMaxChunkBytes
// (rows x pitch: the kernel's buffer-descriptor stores).
template <typename T>
bool chunk_pass_shape(const TileGeom& g, int steps, const Stencil5Coeffs& c, ChunkPassShape* out);
// table: shape.blocks x entries chunks in device memory (ChunkSchedule::table).
template <typename T>
void stencil5_chunk_pass(const T* in, T* out, const TileGeom& g, const Stencil5Coeffs& c, const ChunkPassShape& shape,
                         const PassChunk* table, int entries, hipStream_t s);

// max |x[i]| over n elements into *out (device pointer, overwritten; NaN if
// any element is NaN): the range check of the sum form.
template <typename T>
void absmax(const T* x, index_t n, T* out, hipStream_t s);
// Whether work on stream b runs while a kernel on stream a still runs (the two
// sit on different hardware queues): one bounded ~0.8 ms sleeping wave on a, a
// no-op kernel on b (kernels/queue_probe.hip). Synchronises both streams.
bool streams_concurrent(hipStream_t a, hipStream_t b);
// One single-wave kernel that holds stream s for `us` microseconds (capped at
// 10 ms) of the GPU's constant-rate wall clock (kernels/queue_probe.hip): the
// wire time an RCCL-loopback rehearsal adds after each transfer.
void spin_delay(double us, hipStream_t s);
// kClockStampWgs triples (XCD << 16 | SE/SH/CU id, shader clock counter — SCLK
// cycles, its rate follows DVFS —, constant-rate wall clock) at out[3 b ..],
// one per one-wave workgroup: two stamps around a launch, matched CU by CU,
// give the clock the launch ran at (device pointer).
constexpr int kClockStampWgs = 512;
void clock_stamp(unsigned long long* out, hipStream_t s);
// Number of 32-bit words that differ between a and b (bytes % 4 == 0) into
// *out (device pointer, overwritten): the direct halo's bitwise validation.
void count_diff(const void* a, const void* b, index_t bytes, unsigned* out, hipStream_t s);

// Update an arbitrary core rectangle [x0, x1) x [y0, y1) (scalar path; used for the
// boundary columns of the overlapped schedule and for tiny tiles).
template <typename T>
void stencil5_rect(const T* in, T* out, const TileGeom& g, index_t x0, index_t x1, index_t y0,
                   index_t y1, Stencil5Coeffs c, hipStream_t s);

// Processes sharing this GPU (ranks of one node bound to the same device, the
// IPC configuration). The persistent stencil kernels size their grid to the
// resident capacity of the chip divided by this, so the kernels of all sharing
// ranks are co-resident instead of queueing in rounds behind each other.
void set_gpu_share(int processes);
int gpu_share();

// Joint stage-1 windows in the fp32 two-stage pipeline (stencil_device.hpp:
// JointShape): on by default for time blocks that split into two multiples of
// 4 levels (S = 20, 24, 28, 32); off runs the per-strip layout (bitwise equal
// output). MXS_PIPE_JOINT=0 in the environment turns it off at start-up.
void set_pipe_joint(bool on);
bool pipe_joint();
// Ascending level order (one row of lag per level) in the joint fp32 pipeline
// where it measured faster: S = 20 on chunks of <= 768 rows (small and
// multi-GPU tiles), S = 24 everywhere (stencil_pipe.hpp). Bitwise equal output.
// MXS_PIPE_LAG1=0 in the environment turns it off at start-up.
void set_pipe_lag1(bool on);
bool pipe_lag1();
// Whether the most recent stencil launch was a pipeline pass in that order.
bool last_pipe_lag1();
// Fill-aware workgroup shares of the pipeline passes (chunk_schedule.hpp:
// balanced_starts; default on): a share that crosses a column-group boundary
// pays a second pipeline fill, and with equal row shares those workgroups set
// the pass time. MXS_PIPE_BALANCED=0 restores equal shares. Bitwise equal output.
void set_pipe_balanced(bool on);
bool pipe_balanced_on();

// Kernel form chosen by the most recent stencil launcher on this host process:
// "stream_pipe" (the two-stage pipeline: fp32 blocks > 16 steps, the one the
// benchmarks time, and fp64 blocks of 12 / 16 on whole lane vectors), "stream_balanced_rot" (persistent single-wave fp32
// rotated-pair kernel), "stream_balanced", "stream_grid_rot", "stream_grid", "tb_tile",
// "roll", "roll_wrap", "lds", "rect" or "box". A record of the host-side
// dispatch decision, for tests and result records; graph replays do not update it.
const char* last_stencil_dispatch();

// (2R+1)^2 box stencil with arbitrary weights (row-major, (2R+1)^2 entries), R in {1, 2}.
// Needs a ghost ring of at least R cells. LDS-tiled: each workgroup stages a
// (64+2R) x (16+2R) input tile once and reads the (2R+1)^2 taps from LDS.
constexpr int kMaxBoxRadius = 2;
struct BoxWeights {
  int radius = 1;
  float w[(2 * kMaxBoxRadius + 1) * (2 * kMaxBoxRadius + 1)] = {};
};
template <typename T>
void stencil_box(const T* in, T* out, const TileGeom& g, index_t x0, index_t x1, index_t y0,
                 index_t y1, const BoxWeights& w, hipStream_t s);

// ------------------------------------------------------ halo pack/unpack (K11/K12)
// A batch of strided 2D copies between up to three base pointers
// (slot 0 = tile, 1 = send buffer, 2 = recv buffer). One launch moves every
// segment of a halo exchange: gridDim.y indexes the copy.
constexpr int kMaxCopies = 24;
struct Copy2D {
  index_t src_off = 0, src_stride = 0;
  index_t dst_off = 0, dst_stride = 0;
  index_t width = 0, height = 0;
  int src_slot = 0, dst_slot = 0;
};
struct Copy2DBatch {
  int n = 0;
  Copy2D op[kMaxCopies];
};
// grid_x: workgroups per copy (0 = sized from the largest copy; tuning only).
// block: threads per workgroup (0 = 256). One-wave (64) workgroups are the
// ones the hardware places beside a running pipeline workgroup (the
// interior-first super-step's copies); 256 is faster alone.
// kind: which kernel symbol the launch uses (same body): halo_pack_kernel,
// halo_unpack_kernel or copy2d_batch_kernel, so kernel traces separate the
// exchange's two sides.
enum class CopyKind : int { Copy = 0, Pack = 1, Unpack = 2 };
template <typename T>
void copy2d_batch(T* slot0, T* slot1, T* slot2, const Copy2DBatch& b, hipStream_t s, int grid_x = 0, int block = 0,
                  CopyKind kind = CopyKind::Copy);

// ---------------------------------------------------------------- dot (K2-K8)
enum class DotReduce : int {
  Atomic = 0,      // per-block partial, one device atomic per block (mpicuda2.cu:65-81)
  TwoPass = 1,     // per-block partials + 1-block finisher kernel (mpicuda4.cu:71-88 + device finish)
  SinglePass = 2,  // last-block-done reduction with agent-scope release/acquire (mpicuda4.cu:157-185)
  HostPartials = 3,  // per-block partials, summed on the host in f64 (REDUCE_CPU)
  Racy = 4,        // NO_SYNC demonstrator: non-atomic `*out += partial` (ref_parallel-dot-product-atomics.cu:26-32)
};

// Scratch needed by the dot kernels: `partials` holds >= grid Acc values
// (dot_grid_size(n, kDotBlock) when grid <= 0: one workgroup per CU), `counter`
// one unsigned int (zeroed by the launcher every call).
int dot_grid_size(index_t n, int block);
constexpr int kDotBlock = 256;

// result = sum(x[i] * y[i]) accumulated in Acc (double or float). Writes the
// scalar into *out (device pointer). For HostPartials the partials are left in
// `partials[0..grid)` and *out is not written.
template <typename T, typename Acc>
void dot(const T* x, const T* y, index_t n, Acc* out, Acc* partials, unsigned* counter,
         DotReduce mode, int grid, hipStream_t s);

}  // namespace kernels
}  // namespace mxs

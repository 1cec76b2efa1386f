// rowgroup.hpp -- "row group" work decomposition for channel-last row kernels.
//
// A row (one spatial position, C contiguous fp32 channels) is handled by G consecutive lanes
// of a wave, each lane owning V float4 chunks at c4 = lane_in_group + j*G (j < V).  G is a
// power of two so row reductions are xor-shuffles inside the group; 64/G rows are in flight
// per wave.  C = 48*2^k (every WaveFormer width) maps to V = 3 with no idle lane.
#pragma once
#include <type_traits>

#include "wf_common.hpp"

namespace wf {

template <int N>
using ic = std::integral_constant<int, N>;

// Calls f(ic<G>, ic<V>) for the (G, V) that covers C4 = C/4 float4 chunks per row.
// Returns WF_E_SHAPE for unsupported widths (C4 > 256).
template <class F>
int dispatch_gv(int64_t C4, F&& f) {
  if (C4 % 3 == 0) {
    switch (C4 / 3) {
      case 1: return f(ic<1>{}, ic<3>{});
      case 2: return f(ic<2>{}, ic<3>{});
      case 4: return f(ic<4>{}, ic<3>{});
      case 8: return f(ic<8>{}, ic<3>{});
      case 16: return f(ic<16>{}, ic<3>{});
      case 32: return f(ic<32>{}, ic<3>{});
      case 64: return f(ic<64>{}, ic<3>{});
      default: break;
    }
  }
  if (C4 <= 1) return f(ic<1>{}, ic<1>{});
  if (C4 <= 2) return f(ic<2>{}, ic<1>{});
  if (C4 <= 4) return f(ic<4>{}, ic<1>{});
  if (C4 <= 8) return f(ic<8>{}, ic<1>{});
  if (C4 <= 16) return f(ic<16>{}, ic<1>{});
  if (C4 <= 32) return f(ic<32>{}, ic<1>{});
  if (C4 <= 64) return f(ic<64>{}, ic<1>{});
  if (C4 <= 128) return f(ic<64>{}, ic<2>{});
  if (C4 <= 256) return f(ic<64>{}, ic<4>{});
  return fail(WF_E_SHAPE, "channel count > 1024 is not supported");
}

// Mean / rstd of one row held as V float4 per lane (chunks with c4 >= C4 must be zero and
// are excluded through the count C).  Two-pass (mean, then centred sum of squares), like
// PyTorch's LayerNorm, so large means do not cancel.
template <int G, int V>
__device__ __forceinline__ void row_stats(const f32x4 (&v)[V], const bool (&live)[V], float C,
                                          float eps, float& mean, float& rstd) {
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < V; ++j) s += (v[j].x + v[j].y) + (v[j].z + v[j].w);
  mean = group_sum<G>(s) / C;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < V; ++j) {
    if (live[j]) {
      f32x4 d = v[j] - mean;
      q += (d.x * d.x + d.y * d.y) + (d.z * d.z + d.w * d.w);
    }
  }
  float var = group_sum<G>(q) / C;
  rstd = rsqrtf(var + eps);
}

}  // namespace wf

// spf_update.hip — incremental updates of the resident graph and the
// affected-run test (include/openr_spf.h: ospf_update_links,
// ospf_affected_roots).
//
// The reference recomputes every SPF after a topology change (LinkState
// clears spfResults_, openr/decision/LinkState.cpp:751-754; Decision rebuilds
// routes per debounced batch, Decision.cpp:918-996). A run of root r is
// unchanged by a batch that only changes link metrics / up state / overload
// bits when no changed link is on r's shortest-path DAG before the batch and
// none reaches or ties a shortest distance after it; runSpf's result (dist,
// nextHops, pathLinks, LinkState.cpp:836-911) is then bit-identical, so only
// the flagged runs need to be re-run.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "spf_kernels.h"

namespace ospf {
namespace {

constexpr uint32_t kInf = 0xFFFFFFFFu;
constexpr uint32_t kDown = 0x80000000u;

__global__ void scatter_kernel(uint32_t* base, const uint32_t* idx, const uint32_t* val,
                               uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) base[idx[i]] = val[i];
}

// can `x`'s relaxations matter to the run whose distance row is `d`?
__device__ bool node_matters(const DevGraph& g, const uint32_t* d, uint32_t x, bool hop) {
  const uint32_t dx = d[x];
  if (dx == kInf || dx == 0) return false;  // unreached, or the root (always relaxes)
  for (uint32_t e = g.row_ptr[x]; e < g.row_ptr[x + 1]; ++e) {
    const uint32_t cx = g.colx[e];
    if (cx & kDown) continue;
    const uint64_t nd = (uint64_t)dx + (hop ? 1u : g.w[e]);
    if (nd <= d[cx]) return true;
  }
  return false;
}

__global__ void affected_kernel(DevGraph g, const uint32_t* dist, uint32_t n_roots, uint32_t hop,
                                const ospf_change* ch, uint32_t n_ch, uint8_t* out) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_roots) return;
  const uint32_t* d = dist + (size_t)r * g.V;
  uint8_t hit = 0;
  for (uint32_t k = 0; k < n_ch && !hit; ++k) {
    const ospf_change c = ch[k];
    if (c.kind == OSPF_CHANGE_NODE) {
      hit = node_matters(g, d, c.a, hop != 0);
      continue;
    }
    const uint64_t da = d[c.a], db = d[c.b];
    const uint64_t w0ab = hop ? 1 : c.w_ab0, w0ba = hop ? 1 : c.w_ba0;
    const uint64_t w1ab = hop ? 1 : c.w_ab1, w1ba = hop ? 1 : c.w_ba1;
    // tight before (its head's dist / next hops / pathLinks used it)
    if (c.up0 && da != kInf && da + w0ab == db) hit = 1;
    if (c.up0 && db != kInf && db + w0ba == da) hit = 1;
    // shortens or ties a distance after
    if (c.up1 && da != kInf && da + w1ab <= db) hit = 1;
    if (c.up1 && db != kInf && db + w1ba <= da) hit = 1;
  }
  out[r] = hit;
}

}  // namespace

hipError_t launch_scatter(uint32_t* base, const uint32_t* idx, const uint32_t* val, uint32_t n,
                          hipStream_t s) {
  if (n) hipLaunchKernelGGL(scatter_kernel, dim3((n + 255) / 256), dim3(256), 0, s, base, idx, val, n);
  return hipGetLastError();
}

hipError_t launch_affected(const DevGraph& g, const uint32_t* dist, uint32_t n_roots, bool hop,
                           const ospf_change* ch, uint32_t n_ch, uint8_t* out, hipStream_t s) {
  if (n_roots)
    hipLaunchKernelGGL(affected_kernel, dim3((n_roots + 255) / 256), dim3(256), 0, s, g, dist,
                       n_roots, hop ? 1u : 0u, ch, n_ch, out);
  return hipGetLastError();
}

}  // namespace ospf

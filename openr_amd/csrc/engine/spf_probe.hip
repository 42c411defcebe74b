// spf_probe.hip — store-bandwidth probes (gfx950): the box's own HBM store
// rate, measured in the bench's process beside the sweep, so that a launch's
// roofline fraction can be quoted against what this box's HBM accepts and a
// slow box is told apart from a code regression.
//
// Patterns (same bytes written, 16-B non-temporal stores, 1 KB per wave
// instruction, like store_row16 in the derive kernels):
//   0 STREAM       one buffer swept in address order (grid-stride)
//   1 ROWS_CHUNK   the leaf launch's shape: two [rows][V] u32 arrays (next-hop
//                  and dist rows), a block = a group of `group` consecutive
//                  rows x a chunk of 1,024-node tiles, each tile's 4 KB written
//                  in every row of the group; blocks chunk-major (consecutive
//                  blocks = different groups, the same chunk), the leaf
//                  kernel's r05 order
//   2 ROWS_GROUP   the same blocks, group-major (consecutive blocks = one
//                  group's chunks): the rows in flight at once span a few
//                  groups instead of one chunk of every group
//   3 ROWS_WALK    persistent blocks (ctiles per CU), items = (group, tile)
//                  group-major, grid-stride: the whole chip walks the rows in
//                  order, a few groups in flight
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <vector>

#include "spf_internal.h"
#include "spf_kernels.h"

namespace ospf {
namespace {

__global__ void __launch_bounds__(256) probe_stream_kernel(uint4* p, size_t n16, uint32_t val) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  const uint4 v = make_uint4(val, val ^ 1u, val ^ 2u, val ^ 3u);
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride)
    store_row16(p + i, v);
}

__global__ void __launch_bounds__(256)
    probe_rows_kernel(uint32_t* a, uint32_t* b, uint32_t V, uint32_t rows, uint32_t group,
                      uint32_t ngroups, uint32_t tiles, uint32_t ctiles, uint32_t chunks,
                      uint32_t group_major, uint32_t val) {
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint32_t gr = group_major ? blockIdx.x / chunks : blockIdx.x % ngroups;
  const uint32_t ci = group_major ? blockIdx.x % chunks : blockIdx.x / ngroups;
  const uint32_t r0 = gr * group, nr = min(group, rows - r0);
  const uint32_t t0 = ci * ctiles, t1 = min(tiles, t0 + ctiles);
  const uint4 v = make_uint4(val, val ^ 1u, val ^ 2u, val ^ 3u);
  for (uint32_t t = t0; t < t1; ++t) {
    const uint32_t v0 = t * 1024u + wave * 256u + 4u * lane;
    if (v0 >= V) continue;
    for (uint32_t j = 0; j < nr; ++j) {
      store_row16(a + (size_t)(r0 + j) * V + v0, v);
      store_row16(b + (size_t)(r0 + j) * V + v0, v);
    }
  }
}

// persistent blocks, items = (group of `group` rows, one 1,024-node tile),
// group-major, handed out grid-stride: the chip's in-flight writes stay in a
// window of a few groups' rows (the whole chip walks the rows in order)
__global__ void __launch_bounds__(256)
    probe_rows_walk_kernel(uint32_t* a, uint32_t* b, uint32_t V, uint32_t rows, uint32_t group,
                           uint32_t ngroups, uint32_t tiles, uint32_t val) {
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint4 v = make_uint4(val, val ^ 1u, val ^ 2u, val ^ 3u);
  const uint64_t items = (uint64_t)ngroups * tiles;
  for (uint64_t it = blockIdx.x; it < items; it += gridDim.x) {
    const uint32_t gr = (uint32_t)(it / tiles), t = (uint32_t)(it % tiles);
    const uint32_t r0 = gr * group, nr = min(group, rows - r0);
    const uint32_t v0 = t * 1024u + wave * 256u + 4u * lane;
    if (v0 >= V) continue;
    for (uint32_t j = 0; j < nr; ++j) {
      store_row16(a + (size_t)(r0 + j) * V + v0, v);
      store_row16(b + (size_t)(r0 + j) * V + v0, v);
    }
  }
}

}  // namespace
}  // namespace ospf

int ospf_probe_store(ospf_ctx* c, uint32_t pattern, uint32_t V, uint32_t rows, uint32_t group,
                     uint32_t ctiles, uint32_t reps, float* ms_out) {
  if (!c || !ms_out || reps == 0) return OSPF_E_INVAL;
  if (pattern > 3) return ospf_int::fail(c, OSPF_E_INVAL, "probe: pattern 0..3");
  if (V == 0 || (V & 3u) || rows == 0 || group == 0)
    return ospf_int::fail(c, OSPF_E_INVAL, "probe: V a positive multiple of 4, rows, group > 0");
  const size_t row_bytes = (size_t)V * 4u, half = row_bytes * rows;
  HIPCHK(c, hipSetDevice(c->device));
  char* buf = nullptr;
  if (ospf_int::dev_malloc(c, (void**)&buf, 2 * half) != hipSuccess || !buf) {
    return ospf_int::fail(c, OSPF_E_NOMEM, "probe: no room for the probe buffer");
  }
  hipStream_t s = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  int rc = OSPF_OK;
  auto done = [&](int r) {
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (s) (void)hipStreamDestroy(s);
    (void)hipFree(buf);
    return r;
  };
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess)
    return done(ospf_int::hip_fail(c, hipGetLastError(), "probe: stream / events"));
  const uint32_t tiles = (V + 1023u) / 1024u;
  const uint32_t ngroups = (rows + group - 1) / group;
  const uint32_t ct = ctiles ? std::min(ctiles, tiles) : tiles;
  const uint32_t chunks = (tiles + ct - 1) / ct;
  for (uint32_t i = 0; i <= reps && rc == OSPF_OK; ++i) {  // rep 0 warms up (first touch)
    hipError_t e = hipEventRecord(e0, s);
    if (pattern == 0) {
      const size_t n16 = 2 * half / 16u;
      hipLaunchKernelGGL(ospf::probe_stream_kernel, dim3(c->n_cu * 8u), dim3(256), 0, s,
                         reinterpret_cast<uint4*>(buf), n16, 0x5A5A0000u + i);
    } else if (pattern == 3) {
      hipLaunchKernelGGL(ospf::probe_rows_walk_kernel, dim3(c->n_cu * (ctiles ? ctiles : 8u)),
                         dim3(256), 0, s, reinterpret_cast<uint32_t*>(buf),
                         reinterpret_cast<uint32_t*>(buf + half), V, rows, group, ngroups, tiles,
                         0x5A5A0000u + i);
    } else {
      hipLaunchKernelGGL(ospf::probe_rows_kernel, dim3(ngroups * chunks), dim3(256), 0, s,
                         reinterpret_cast<uint32_t*>(buf), reinterpret_cast<uint32_t*>(buf + half),
                         V, rows, group, ngroups, tiles, ct, chunks, pattern == 2 ? 1u : 0u,
                         0x5A5A0000u + i);
    }
    if (e == hipSuccess) e = hipGetLastError();
    if (e == hipSuccess) e = hipEventRecord(e1, s);
    if (e == hipSuccess) e = hipEventSynchronize(e1);
    float ms = 0.f;
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
    if (e != hipSuccess) rc = ospf_int::hip_fail(c, e, "probe launch");
    else if (i) ms_out[i - 1] = ms;
  }
  return done(rc);
}

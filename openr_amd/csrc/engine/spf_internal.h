// spf_internal.h — the engine context shared by the C ABI translation units
// (spf_engine.hip: graph, batches, derive, KSP2, updates; spf_sweep.cpp:
// all-sources sweeps and the multi-device context). Not a public header.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <map>
#include <string>
#include <system_error>
#include <thread>
#include <vector>

#include "host_pool.h"
#include "spf_kernels.h"

struct ospf_ctx {
  int device = 0;
  size_t lds_limit = 64 * 1024;
  int lds_attr = 0;
  int n_cu = 256;
  std::string err;
  uint64_t spf_runs = 0;
  uint32_t inject_after = 0;  // ospf_inject_error: calls until the injected failure (0 = off)
  uint64_t ksp_decr_stats[3] = {0, 0, 0};  // ospf_ksp2_stats
  // device blocks, streams and events of destroyed sweeps, taken again by the
  // next sweep (a graph patch drops the sweep; its successor reuses ~100 GB
  // of F100k rows instead of hipFree + hipMalloc, and its streams' scratch)
  std::multimap<size_t, void*> sweep_pool;
  size_t sweep_pool_bytes = 0;
  std::vector<hipStream_t> stream_pool;
  std::vector<hipEvent_t> event_pool;
  // sweeps created on this context and not yet destroyed: ospf_close
  // releases them first (a sweep destroyed after its context -- a caller's
  // GC order -- then frees only itself)
  std::vector<struct ospf_sweep*> live_sweeps;
  void (*release_sweep)(struct ospf_sweep*) = nullptr;
  // graph
  bool loaded = false;
  ospf_graph_info info{};
  std::vector<uint32_t> h_row_ptr, h_dn_off, h_dn;  // host copies for root queries
  // host shadows of the padded device arrays patched by ospf_update_*
  std::vector<uint32_t> h_prow, h_pcolx, h_pw, h_prw, h_nt, h_link_e, h_plink;
  // allocated capacity of the per-entry arrays (entries), of dn and of link_e
  // (link ids): the reserves of ospf_update_rows
  size_t cap_e = 0, cap_dn = 0, cap_lid = 0;
  uint64_t non_unit = 0;  // usable entries with metric != 1 (exact unit_metric under patches)
  void* d_graph = nullptr;
  ospf::DevGraph g{};
  const uint32_t* ew_base = nullptr;  // packed entries (g.ew) as words, for patches
  uint32_t max_dn = 0;
  uint32_t depth_bound = 2;  // BFS levels any root can reach (unit metric / hop count)
  uint32_t exact_bound = 2;  // depth_bound as last computed in full (patches may raise depth_bound)
  // >= every shortest distance: sum over nodes of the largest usable out-metric
  // (a simple path leaves each node once); patches only add to it
  uint64_t dist_bound = 0;
  std::vector<uint32_t> h_rowmax;  // largest usable out-metric per node (dist_bound = sum)
  std::vector<uint32_t> h_lvl;  // scratch of transit_detour (all UINT32_MAX between calls)
  // scratch per stream: batches queued on different streams run concurrently
  struct Scratch {
    void* p = nullptr;
    size_t bytes = 0;
  };
  std::map<void*, Scratch> scratch;
  void* d_stage = nullptr;
  size_t stage_bytes = 0;
  uint32_t* d_err = nullptr;
  // KSP2: traces run on an engine stream, overlapping later reruns
  hipStream_t aux = nullptr;
  // KSP2: the decremental kernels beside the pre-split runs' full reruns
  hipStream_t ksp_aux = nullptr, ksp_hi = nullptr;  // low / high priority
  hipEvent_t ksp_ev[4] = {nullptr, nullptr, nullptr, nullptr};
  // derive phase 1: rows kernels of one round beside the next round's levels
  hipStream_t lv_aux = nullptr;
  hipEvent_t lv_ev[4] = {nullptr, nullptr, nullptr, nullptr};  // traversed[2], rows done[2]
  // contracted cover graph (ospf_cover_prepare), valid for graph version cover_ver
  void* d_cover = nullptr;
  ospf::CoverGraph cover{};
  uint64_t cover_ver = ~0ull;
  bool cover_ok = false;
  // host copy of the contracted graph, and its closure split (when one
  // exists): seeds = the cover nodes of largest degree, every other cover
  // node in a component of C minus the seeds of <= kClosureMaxK nodes
  std::vector<uint32_t> h_ccv, h_ccrow, h_cctr;  // cover index -> node id, CSR, transit bits
  std::vector<uint32_t> h_cix, h_lrow, h_ladj;   // node -> cover index / leaf word, leaf in-links
  std::vector<uint2> h_cedge;
  std::vector<uint32_t> cl_seed;               // cover indices of the seeds
  std::vector<uint32_t> cl_comp_of;            // per cover index: component, or ~0u (seed)
  std::vector<uint32_t> cl_comp_off, cl_comp_mem;  // members (cover indices) per component
  std::vector<hipEvent_t> ev;  // [2 * slots]: rerun done / trace done per slot
  uint64_t graph_gen = 0;      // bumped by every load / patch (sweeps check it)
  // ospf_links_mask: the entries and planner state it replaced (restored by
  // ospf_links_unmask)
  struct Mask {
    bool on = false;
    std::vector<uint32_t> lids;
    std::vector<uint32_t> up, mlo, mhi;  // per masked link, before
    uint32_t depth_bound, exact_bound, max_metric, unit_metric;
    uint64_t dist_bound, non_unit, version;
    bool cover_ok;
  } mask;
};

namespace ospf_int {

// fn(lo, hi) over [0, n) on up to 16 host threads, chunks of `grain` taken
// dynamically (a fabric's spines, first by name, have 20x the rows of the
// rest: static slices left one thread with most of the work, and so did
// 512-node chunks -- the 288 spines' 513 k entries in one); serial when
// threads are unavailable. Chunks start at multiples of `grain` (64: whole
// words of per-node bitmaps).
template <class F>
void par_for(uint32_t n, F fn, uint32_t grain = 64) {
  const uint32_t hw = std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
  const uint32_t T = std::min(hw, (n + grain - 1) / grain);
  if (T <= 1) {
    fn(0u, n);
    return;
  }
  // the persistent pool (host_pool.h); threads of its own when it is busy
  if (host_pool::Pool::get().run(n, grain, T, [&](uint32_t lo, uint32_t hi) { fn(lo, hi); }))
    return;
  std::atomic<uint32_t> next{0};
  auto work = [&]() {
    for (;;) {
      const uint32_t lo = next.fetch_add(grain);
      if (lo >= n) return;
      fn(lo, std::min(n, lo + grain));
    }
  };
  std::vector<std::thread> th;
  try {
    for (uint32_t t = 1; t < T; ++t) th.emplace_back(work);
  } catch (const std::system_error&) {  // fewer threads: the rest share the work
  }
  work();
  for (auto& x : th) x.join();
}


// fn(lo, hi) over items [0, n) in chunks of about `target` units of work,
// item i weighing off[i + 1] - off[i] (a row's entries), and of at most 256
// items: a fabric's spines (1,781 entries each, first by name) spread over
// many chunks instead of loading one, and the light rows share few chunks
// (one atomic claim each). Chunk starts are multiples of `align`.
template <class F>
void par_for_rows(uint32_t n, const uint32_t* off, F fn, uint32_t target = 8192, uint32_t align = 1) {
  if (!n) return;
  const uint64_t total = (uint64_t)off[n] - off[0];
  const uint32_t want = (uint32_t)std::min<uint64_t>(n, std::max<uint64_t>(1, total / std::max(1u, target)));
  std::vector<uint32_t> cut{0u};
  for (uint32_t k = 1; k < want; ++k) {
    const uint64_t at = off[0] + total * k / want;
    uint32_t i = (uint32_t)(std::lower_bound(off, off + n, (uint32_t)at) - off);
    i = i / align * align;
    if (i > cut.back() && i < n) cut.push_back(i);
  }
  cut.push_back(n);
  std::vector<uint32_t> all;
  for (size_t k = 0; k + 1 < cut.size(); ++k) {
    all.push_back(cut[k]);
    const uint32_t step = std::max<uint32_t>(align, 256u / align * align);
    for (uint32_t x = cut[k] + step; x < cut[k + 1]; x += step) all.push_back(x);
  }
  all.push_back(n);
  par_for((uint32_t)all.size() - 1, [&](uint32_t clo, uint32_t chi) {
    for (uint32_t k = clo; k < chi; ++k) fn(all[k], all[k + 1]);
  }, 1);
}

int fail(ospf_ctx* c, int code, const std::string& msg);
// hipMalloc on the context's device; when it fails and destroyed sweeps'
// blocks are pooled (sweep_pool), the pool is freed and the allocation tried
// once more (the pool is never counted as used memory)
hipError_t dev_malloc(ospf_ctx* c, void** p, size_t bytes);
void pool_release(ospf_ctx* c);
// ospf_inject_error's hook at an entry point: true (and the error recorded)
// when this call is the one to fail
bool injected(ospf_ctx* c);
int hip_fail(ospf_ctx* c, hipError_t e, const char* what);
inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }
// the scratch of `stream`, grown to `need` bytes (a grown buffer replaces the
// old one only after the stream's queued work is done with it); `slot` 1 is a
// second buffer of the same stream (KSP2 state around nested batch calls)
char* stream_scratch(ospf_ctx* c, void* stream, size_t need, int* rc, int slot = 0);
// frees the scratch of `stream` (both slots); the stream must be idle
void release_stream_scratch(ospf_ctx* c, void* stream);

// Host plan of twin levels (spf_twin.hip twin_levels_kernel) for `roots` in
// order, cut into the caller's groups (offsets; empty = one root per group):
// per root its usable distinct neighbours (ascending) and the level-row
// positions (pos[rep[class]]) of its usable transit neighbours' classes, per
// group the union of those rows. OSPF_E_RANGE when a root has more than 128
// usable neighbours, a group more than kTwinMaxC class rows, or a class row
// is missing.
struct TwinLvHost {
  std::vector<uint32_t> grp, grow, nbo, nbl;
  std::vector<uint4> rinfo;
  uint32_t gmax = 0;  // largest group
};
int twin_lv_build(ospf_ctx* c, const std::vector<uint32_t>& roots, const std::vector<uint32_t>& groups,
                  const std::vector<uint32_t>& pos, const std::vector<uint32_t>& cls,
                  const std::vector<uint32_t>& rep, TwinLvHost& out);
// queue a planned twin-levels launch (device copies of the plan's arrays)
int twin_lv_launch(ospf_ctx* c, const ospf::TwinLvPlan& p, void* stream);
// ospf_nh_derive_twin_dev + the roots' own dist rows (d_dist at d_lev_pos;
// null: not written)
int nh_derive_twin_launch(ospf_ctx* c, const uint32_t* d_roots, uint32_t n, uint32_t nh_words,
                          uint32_t max_root_neighbors, const uint8_t* d_lev, uint32_t lev_pitch,
                          const uint32_t* d_lev_pos, const ospf_digest* d_lev_digest,
                          const uint32_t* d_twin_class, const uint32_t* d_twin_rep,
                          const uint32_t* d_twin_second, uint32_t* d_nh, ospf_digest* d_digest,
                          uint32_t* d_dist, void* stream, uint32_t dist_pitch = 0,
                          uint32_t nh_pitch = 0);
// ospf_levels_dev / ospf_leaf_derive2_dev with row pitches (words; 0 = V)
// for the dist and next-hop rows: the sweep keeps its rows 128-B aligned
// (depth_cap: levels launched 1 .. min(cap, depth bound) when non-zero -- a
// sweep's seed BFS at the depth its first run reached; d_maxd: that depth,
// atomicMax'ed by the rows kernel)
int levels_dev(ospf_ctx* c, const uint32_t* d_roots, uint32_t n, uint32_t flags,
               uint32_t* d_dist, uint32_t dist_pitch, uint8_t* d_lev, uint32_t lev_pitch,
               ospf_digest* d_lev_digest, void* stream, uint32_t depth_cap = 0,
               uint32_t* d_maxd = nullptr);
int leaf_derive(ospf_ctx* c, const uint32_t* d_roots, uint32_t n, const uint32_t* d_groups,
                uint32_t n_groups, uint32_t max_root_neighbors, uint8_t* d_lev,
                uint32_t lev_pitch, const uint32_t* d_pos, const uint32_t* d_lev_out,
                uint32_t* d_dist, uint32_t dist_pitch, uint32_t* d_nh, uint32_t nh_pitch,
                ospf_digest* d_digest, void* stream, int group_major = -1);

// Host plan of the cover closure (spf_cover.hip closure_kernel) for the
// closure roots `roots` (node ids, non-seed cover nodes; dc row i = roots[i])
// with the seeds' cover columns at seedC row seed_row[cover index] (~0u: not
// given -> OSPF_E_INVAL). KW = 8 or 16 (largest component, padded).
// NW > 0 (<= kClMaxNW, components of <= 8): also the next-hop masks -- fh
// [term][member][NW] the first hops of the member's shortest paths to the
// term's seed inside the component, fhloc [component][member][member][NW]
// those to each member -- so the closure writes the next hops of its cover
// columns (bit k = the root's k-th distinct neighbour).
struct ClosureHost {
  uint32_t KW = 8, NW = 0;
  std::vector<uint2> comp;
  std::vector<uint32_t> jl, cst, mem, dloc, out, fh, fhloc;
};
int closure_build(ospf_ctx* c, const std::vector<uint32_t>& roots,
                  const std::vector<uint32_t>& seed_row, ClosureHost& h, uint32_t NW = 0);

// ospf_wderive_wide_dev with a chunk size (256-node tiles per block; 0: the
// launcher's default) -- the sweep's wide cover roots run beside the leaves
// with larger chunks (fewer blocks, so the leaves keep most of the GPU)
int wderive_wide(ospf_ctx* c, const uint32_t* d_roots, uint32_t n, uint32_t flags,
                 uint32_t nh_words, const uint32_t* d_src, uint64_t src_pitch,
                 const uint32_t* d_pos, uint32_t* d_nh, ospf_digest* d_digest, void* stream,
                 uint32_t ctiles);

}  // namespace ospf_int

#define HIPCHK(ctx, call)                                            \
  do {                                                               \
    hipError_t e_ = (call);                                          \
    if (e_ != hipSuccess) return ospf_int::hip_fail(ctx, e_, #call); \
  } while (0)

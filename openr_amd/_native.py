"""ctypes bindings for the in-tree native libraries.

Loading fails loudly (ImportError) when a library is missing: there is no
Python or CPU fallback for the SPF path.
"""
from __future__ import annotations

import ctypes as C
import os

from .build import DECISION_SO, ENGINE_SO

vp, cp, u32, i32, u64, i64 = C.c_void_p, C.c_char_p, C.c_uint32, C.c_int, C.c_uint64, C.c_int64

OSPF_OK = 0
OSPF_E_INVAL = -1
OSPF_E_NOGRAPH = -2
OSPF_E_DEVICE = -3
OSPF_E_RANGE = -4
OSPF_E_NOMEM = -5
OSPF_DIST_INF = 0xFFFFFFFF
OSPF_HOP_COUNT = 0x1
OSPF_WANT_DIST = 0x2
OSPF_WANT_NH = 0x4
OSPF_WANT_DIGEST = 0x8
OSPF_SWEEP_DEFER = 0x100
OSPF_SWEEP_EARLY_START = 0x200

ENGINE_SYMBOLS = [
    "ospf_open", "ospf_close", "ospf_last_error", "ospf_load_graph", "ospf_graph_info_get",
    "ospf_root_neighbors", "ospf_sssp_batch", "ospf_sssp_batch_dev", "ospf_sync",
    "ospf_plan_variant", "ospf_plan", "ospf_plan_n", "ospf_spf_runs", "ospf_run_batch_dev",
    "ospf_ksp2_run", "ospf_ksp2_dev", "ospf_ksp2_stats", "ospf_update_links", "ospf_update_nodes", "ospf_update_rows",
    "ospf_levels_dev", "ospf_nh_derive_dev", "ospf_leaf_derive_dev",
    "ospf_nh_derive_twin_dev", "ospf_leaf_derive2_dev", "ospf_wderive_dev", "ospf_wderive_wide_dev",
    "ospf_lds_sweep_dev", "ospf_lds_sweep_fits", "ospf_twin_levels_dev",
    "ospf_cover_prepare", "ospf_cover_dist_dev",
    "ospf_affected_roots", "ospf_repair_runs", "ospf_links_mask", "ospf_links_unmask",
    "ospf_sweep_create", "ospf_sweep_destroy", "ospf_sweep_last_error", "ospf_sweep_get_info",
    "ospf_sweep_roots", "ospf_sweep_run", "ospf_sweep_digests", "ospf_sweep_digests_host",
    "ospf_sweep_poison",
    "ospf_sweep_row", "ospf_sweep_copy_rows", "ospf_sweep_profile", "ospf_sweep_graph_memsets",
    "ospf_multi_open", "ospf_multi_close", "ospf_multi_last_error", "ospf_multi_size",
    "ospf_multi_ctx", "ospf_multi_load_graph", "ospf_msweep_create", "ospf_msweep_destroy",
    "ospf_msweep_run", "ospf_msweep_digests", "ospf_msweep_part", "ospf_msweep_owner",
    "ospf_msweep_gather_backend", "ospf_probe_store", "ospf_inject_error",
]
DECISION_SYMBOLS = [
    "odl_create", "odl_create_multi", "odl_all_sources_prefetch", "odl_all_sources_digests",
    "odl_sweep_stats", "odl_destroy", "odl_last_error", "odl_free", "odl_apply", "odl_apply_hold", "odl_decrement_holds", "odl_has_holds", "odl_spf_text",
    "odl_kth_paths_text", "odl_links_text", "odl_link_keys_text", "odl_metric_a_to_b", "odl_is_overloaded",
    "odl_spf_runs", "odl_set_incremental", "odl_set_host_spf", "odl_incremental_stats", "odl_topology_stats", "odl_num_nodes", "odl_num_links", "odl_spf_digests", "odl_spf_prefetch",
    "odl_ksp2_text", "odl_route_text", "odl_route_db_text", "odl_route_db_bin", "odl_free_buf", "odl_path_a_in_b", "odl_ucmp_text", "odl_csr_size", "odl_csr_export", "odl_node_name", "odl_node_id",
    "odl_apply_kvs", "odl_apply_publication", "odl_node_patches", "odl_shard_stats", "odl_route_db_multi_text", "odl_adjdbs_decode", "odl_adjdbs_stream", "odl_adjdbs_error", "odl_adjdbs_free",
    "odl_last_decode_error", "odl_get_counters", "odl_last_engine_error", "odl_inject_engine_error",
    "odl_set_degrade",
]


class ospf_csr(C.Structure):  # noqa: N801
    _fields_ = [("n_nodes", u32), ("n_edges", u32), ("row_ptr", vp), ("col", vp),
                ("metric", vp), ("link_id", vp), ("twin", vp), ("edge_up", vp),
                ("no_transit", vp), ("link_rank", vp)]


class ospf_ignore(C.Structure):  # noqa: N801
    _fields_ = [("offsets", vp), ("link_ids", vp)]


class ospf_digest(C.Structure):  # noqa: N801
    _fields_ = [("reached", u64), ("sum_dist", u64), ("hash", u64)]


class ospf_batch(C.Structure):  # noqa: N801
    _fields_ = [("d_roots", vp), ("n_roots", u32), ("d_ign_offsets", vp), ("d_ign_ids", vp),
                ("max_ignored", u32), ("flags", u32), ("nh_words", u32),
                ("max_root_neighbors", u32), ("d_dist", vp), ("d_nh", vp), ("d_digest", vp)]


class ospf_ksp2(C.Structure):  # noqa: N801
    _fields_ = [("src", u32), ("dsts", vp), ("n", u32), ("path_cap", u32), ("k1", vp),
                ("k2", vp), ("status", vp)]


OSPF_KSP_RERUN, OSPF_KSP_OVF1, OSPF_KSP_OVF2 = 0x1, 0x2, 0x4


class ospf_link_update(C.Structure):  # noqa: N801
    _fields_ = [("link_id", u32), ("up", u32), ("metric_lo", u32), ("metric_hi", u32)]


OSPF_CHANGE_LINK, OSPF_CHANGE_NODE = 0, 1


class ospf_change(C.Structure):  # noqa: N801
    _fields_ = [("kind", u32), ("a", u32), ("b", u32), ("up0", u32), ("w_ab0", u32),
                ("w_ba0", u32), ("up1", u32), ("w_ab1", u32), ("w_ba1", u32)]


class ospf_plan_info(C.Structure):  # noqa: N801
    _fields_ = [("variant", C.c_int32), ("block", u32), ("lds_bytes", u32), ("slices", u32)]


OSPF_SWEEP_AUTO, OSPF_SWEEP_DERIVE, OSPF_SWEEP_WCOVER, OSPF_SWEEP_WDERIVE, OSPF_SWEEP_BATCH = \
    0, 1, 2, 3, 4
SWEEP_MODES = {"auto": 0, "derive": 1, "wcover": 2, "wderive": 3, "batch": 4, "lds": 5,
               "wmulti": 6}
SWEEP_MODE_NAMES = {v: k for k, v in SWEEP_MODES.items()}


class ospf_sweep_opts(C.Structure):  # noqa: N801
    _fields_ = [("flags", u32), ("mode", u32), ("part", u32), ("n_parts", u32),
                ("hip_graph", u32)]


class ospf_sweep_info(C.Structure):  # noqa: N801
    _fields_ = [("mode", u32), ("n_roots", u32), ("n_rows", u32), ("n_launches", u32),
                ("hip_graph", u32), ("max_nh_words", u32), ("device_bytes", u64),
                ("step_compulsory_bytes", u64), ("step_traversed_edges", u64)]


class ospf_sweep_launch(C.Structure):  # noqa: N801
    _fields_ = [("name", C.c_char * 32), ("kernel", C.c_char * 112), ("n_roots", u32),
                ("nh_words", u32), ("compulsory_bytes", u64), ("ms_median", C.c_double),
                ("ms_min", C.c_double)]


class odl_counters(C.Structure):  # noqa: N801
    _fields_ = [("spf_runs", u64), ("spf_ms_samples", u64), ("spf_ms_sum", C.c_double),
                ("ucmp_runs", u64), ("ucmp_ms_sum", C.c_double), ("route_build_runs", u64),
                ("route_build_ms_sum", C.c_double), ("engine_errors", u64),
                ("engine_degraded", u32)]


class ospf_graph_info(C.Structure):  # noqa: N801
    _fields_ = [("n_nodes", u32), ("n_edges", u32), ("n_links", u32), ("max_degree", u32),
                ("max_metric", u32), ("unit_metric", u32), ("version", u64),
                ("device_bytes", u64)]


_engine = None
_decision = None


def _load(path: str) -> C.CDLL:
    if not os.path.exists(path):
        raise ImportError(f"{path} is not built; run `python -m openr_amd.build` "
                          "(there is no CPU fallback for the SPF engine)")
    return C.CDLL(path, mode=C.RTLD_GLOBAL)


def engine() -> C.CDLL:
    global _engine
    if _engine is None:
        # OPENR_SPF_ENGINE_SO: another build of the same ABI (A/B experiments)
        L = _load(os.environ.get("OPENR_SPF_ENGINE_SO") or ENGINE_SO)
        L.ospf_open.argtypes = [i32, C.POINTER(vp)]
        L.ospf_close.argtypes = [vp]
        L.ospf_last_error.argtypes = [vp]
        L.ospf_last_error.restype = cp
        L.ospf_load_graph.argtypes = [vp, C.POINTER(ospf_csr), u64]
        L.ospf_graph_info_get.argtypes = [vp, C.POINTER(ospf_graph_info)]
        L.ospf_root_neighbors.argtypes = [vp, u32, vp, u32, C.POINTER(u32)]
        L.ospf_sssp_batch.argtypes = [vp, vp, u32, C.POINTER(ospf_ignore), u32, u32, vp, vp, vp]
        L.ospf_sssp_batch_dev.argtypes = [vp, vp, u32, vp, vp, u32, u32, u32, vp, vp, vp, vp]
        L.ospf_sync.argtypes = [vp, vp]
        L.ospf_plan_variant.argtypes = [vp, u32, u32, C.POINTER(C.c_int)]
        L.ospf_plan.argtypes = [vp, u32, u32, u32, C.POINTER(ospf_plan_info)]
        L.ospf_plan_n.argtypes = [vp, u32, u32, u32, u32, u32, C.POINTER(ospf_plan_info)]
        L.ospf_run_batch_dev.argtypes = [vp, C.POINTER(ospf_batch), vp]
        L.ospf_ksp2_run.argtypes = [vp, C.POINTER(ospf_ksp2)]
        L.ospf_ksp2_dev.argtypes = [vp, C.POINTER(ospf_ksp2), vp]
        L.ospf_ksp2_stats.argtypes = [vp, vp]
        L.ospf_levels_dev.argtypes = [vp, vp, u32, u32, vp, vp, u32, vp, vp]
        L.ospf_nh_derive_dev.argtypes = [vp, vp, u32, u32, u32, vp, u32, vp, vp, vp, vp, vp]
        L.ospf_nh_derive_twin_dev.argtypes = [vp, vp, u32, u32, u32, vp, u32, vp, vp, vp, vp, vp,
                                              vp, vp, vp]
        L.ospf_leaf_derive_dev.argtypes = [vp, vp, u32, vp, u32, u32, vp, u32, vp, vp, vp, vp, vp]
        L.ospf_lds_sweep_dev.argtypes = [vp, vp, u32, u32, u32, vp, vp, vp, vp]
        L.ospf_lds_sweep_fits.argtypes = [vp, u32, u32]
        L.ospf_twin_levels_dev.argtypes = [vp, vp, u32, vp, u32, vp, u32, vp, vp, vp, vp, vp, vp]
        L.ospf_leaf_derive2_dev.argtypes = [vp, vp, u32, vp, u32, u32, vp, u32, vp, vp, vp, vp,
                                            vp, vp]
        L.ospf_wderive_dev.argtypes = [vp, vp, u32, u32, u32, vp, u64, vp, vp, vp, vp, vp]
        L.ospf_wderive_wide_dev.argtypes = [vp, vp, u32, u32, u32, vp, u64, vp, vp, vp, vp]
        L.ospf_cover_prepare.argtypes = [vp, vp]
        L.ospf_cover_dist_dev.argtypes = [vp, vp, u32, vp, vp]
        L.ospf_update_links.argtypes = [vp, vp, u32, u64]
        L.ospf_update_nodes.argtypes = [vp, vp, vp, u32, u64]
        L.ospf_update_rows.argtypes = [vp, C.POINTER(ospf_csr), vp, u32, u64]
        L.ospf_affected_roots.argtypes = [vp, vp, u32, u32, vp, u32, vp, vp]
        L.ospf_repair_runs.argtypes = [vp, vp, u32, u32, u32, vp, vp, vp, u32, vp, vp]
        L.ospf_spf_runs.argtypes = [vp]
        L.ospf_spf_runs.restype = u64
        L.ospf_links_mask.argtypes = [vp, vp, u32, u64]
        L.ospf_links_unmask.argtypes = [vp]
        L.ospf_sweep_create.argtypes = [vp, C.POINTER(ospf_sweep_opts), C.POINTER(vp)]
        L.ospf_sweep_destroy.argtypes = [vp]
        L.ospf_sweep_last_error.argtypes = [vp]
        L.ospf_sweep_last_error.restype = cp
        L.ospf_sweep_get_info.argtypes = [vp, C.POINTER(ospf_sweep_info)]
        L.ospf_sweep_roots.argtypes = [vp, vp]
        L.ospf_sweep_run.argtypes = [vp, vp]
        L.ospf_sweep_digests.argtypes = [vp, vp, vp]
        L.ospf_sweep_digests_host.argtypes = [vp, vp]
        L.ospf_sweep_poison.argtypes = [vp, vp]
        L.ospf_sweep_row.argtypes = [vp, u32, C.POINTER(vp), C.POINTER(vp), C.POINTER(u32)]
        L.ospf_sweep_copy_rows.argtypes = [vp, vp, u32, u32, vp, vp]
        L.ospf_sweep_profile.argtypes = [vp, u32, vp, u32]
        L.ospf_sweep_graph_memsets.argtypes = [vp, C.POINTER(u32), C.POINTER(u32), C.POINTER(u32)]
        L.ospf_multi_open.argtypes = [vp, u32, C.POINTER(vp)]
        L.ospf_multi_close.argtypes = [vp]
        L.ospf_multi_last_error.argtypes = [vp]
        L.ospf_multi_last_error.restype = cp
        L.ospf_multi_size.argtypes = [vp]
        L.ospf_multi_size.restype = u32
        L.ospf_multi_ctx.argtypes = [vp, u32]
        L.ospf_multi_ctx.restype = vp
        L.ospf_multi_load_graph.argtypes = [vp, C.POINTER(ospf_csr), u64]
        L.ospf_msweep_create.argtypes = [vp, C.POINTER(ospf_sweep_opts), C.POINTER(vp)]
        L.ospf_msweep_destroy.argtypes = [vp]
        L.ospf_msweep_run.argtypes = [vp]
        L.ospf_msweep_digests.argtypes = [vp, vp]
        L.ospf_msweep_part.argtypes = [vp, u32]
        L.ospf_msweep_part.restype = vp
        L.ospf_msweep_owner.argtypes = [vp, u32, C.POINTER(u32)]
        L.ospf_msweep_gather_backend.argtypes = [vp]
        L.ospf_msweep_gather_backend.restype = u32
        L.ospf_probe_store.argtypes = [vp, u32, u32, u32, u32, u32, u32, vp]
        L.ospf_inject_error.argtypes = [vp, u32]
        _engine = L
    return _engine


def decision() -> C.CDLL:
    global _decision
    if _decision is None:
        engine()
        L = _load(os.environ.get("OPENR_DECISION_SO") or DECISION_SO)
        L.odl_create.argtypes = [cp, i32, C.POINTER(vp)]
        L.odl_create_multi.argtypes = [cp, vp, u32, C.POINTER(vp)]
        L.odl_all_sources_prefetch.argtypes = [vp, i32]
        L.odl_all_sources_digests.argtypes = [vp, i32, vp]
        L.odl_sweep_stats.argtypes = [vp, vp]
        L.odl_sweep_stats.restype = None
        L.odl_destroy.argtypes = [vp]
        L.odl_last_error.argtypes = [vp]
        L.odl_last_error.restype = cp
        L.odl_free.argtypes = [vp]
        L.odl_apply.argtypes = [vp, vp, u32, u32, vp]
        L.odl_apply_hold.argtypes = [vp, vp, u32, u32, vp, u64, u64]
        L.odl_decrement_holds.argtypes = [vp]
        L.odl_has_holds.argtypes = [vp]
        for f in ("odl_spf_text", "odl_kth_paths_text", "odl_links_text", "odl_ksp2_text",
                  "odl_route_text", "odl_route_db_text", "odl_ucmp_text",
                  "odl_link_keys_text"):
            getattr(L, f).restype = C.POINTER(C.c_char)
        L.odl_spf_text.argtypes = [vp, cp, i32]
        L.odl_kth_paths_text.argtypes = [vp, cp, cp, i32]
        L.odl_links_text.argtypes = [vp, cp]
        L.odl_link_keys_text.argtypes = [vp]
        L.odl_ksp2_text.argtypes = [vp, cp, cp, u32]
        L.odl_route_text.argtypes = [vp, cp, cp, u32, i32]
        L.odl_route_db_text.argtypes = [vp, cp, u32, cp, u32, i32]
        L.odl_route_db_bin.argtypes = [vp, cp, u32, cp, u32, i32, C.POINTER(vp), C.POINTER(u64)]
        L.odl_route_db_bin.restype = i32
        L.odl_free_buf.argtypes = [vp]
        L.odl_free_buf.restype = None
        L.odl_path_a_in_b.argtypes = [cp, u32, cp, u32]
        L.odl_path_a_in_b.restype = i32
        L.odl_ucmp_text.argtypes = [vp, cp, cp, u32, i32, i32]
        L.odl_metric_a_to_b.argtypes = [vp, cp, cp, i32]
        L.odl_metric_a_to_b.restype = i64
        L.odl_is_overloaded.argtypes = [vp, cp]
        L.odl_spf_runs.argtypes = [vp]
        L.odl_spf_runs.restype = u64
        L.odl_set_incremental.argtypes = [vp, i32]
        L.odl_set_incremental.restype = None
        L.odl_route_db_multi_text.argtypes = [vp, u32, cp, u32, cp, u32, i32]
        L.odl_route_db_multi_text.restype = C.POINTER(C.c_char)
        L.odl_node_patches.argtypes = [vp]
        L.odl_shard_stats.argtypes = [vp, vp]
        L.odl_shard_stats.restype = None
        L.odl_node_patches.restype = u64
        L.odl_apply_kvs.argtypes = [vp, u32, vp, vp, vp, u32, vp, cp, vp]
        L.odl_apply_kvs.restype = i32
        L.odl_apply_publication.argtypes = [vp, vp, u64, cp, vp, u32, vp]
        L.odl_apply_publication.restype = i32
        L.odl_adjdbs_decode.argtypes = [vp, vp, u32]
        L.odl_adjdbs_decode.restype = vp
        L.odl_adjdbs_stream.argtypes = [vp]
        L.odl_adjdbs_stream.restype = vp
        L.odl_adjdbs_error.argtypes = []
        L.odl_adjdbs_error.restype = cp
        L.odl_adjdbs_free.argtypes = [vp]
        L.odl_adjdbs_free.restype = None
        L.odl_last_decode_error.argtypes = [vp, C.POINTER(u64)]
        L.odl_last_decode_error.restype = cp
        L.odl_get_counters.argtypes = [vp, vp]
        L.odl_get_counters.restype = None
        L.odl_last_engine_error.argtypes = [vp]
        L.odl_last_engine_error.restype = cp
        L.odl_inject_engine_error.argtypes = [vp, u32]
        L.odl_inject_engine_error.restype = i32
        L.odl_set_degrade.argtypes = [vp, i32]
        L.odl_set_degrade.restype = None
        L.odl_set_host_spf.argtypes = [vp, i32]
        L.odl_set_host_spf.restype = None
        L.odl_incremental_stats.argtypes = [vp, vp]
        L.odl_incremental_stats.restype = None
        L.odl_topology_stats.argtypes = [vp, vp]
        L.odl_topology_stats.restype = None
        L.odl_num_nodes.argtypes = [vp]
        L.odl_num_nodes.restype = u32
        L.odl_num_links.argtypes = [vp]
        L.odl_num_links.restype = u32
        L.odl_spf_digests.argtypes = [vp, cp, u32, i32, vp]
        L.odl_spf_prefetch.argtypes = [vp, cp, u32, i32]
        L.odl_csr_size.argtypes = [vp, C.POINTER(u32), C.POINTER(u32)]
        L.odl_csr_export.argtypes = [vp] + [vp] * 8
        L.odl_node_name.argtypes = [vp, u32]
        L.odl_node_name.restype = cp
        L.odl_node_id.argtypes = [vp, cp]
        L.odl_node_id.restype = i64
        _decision = L
    return _decision

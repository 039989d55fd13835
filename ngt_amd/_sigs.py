"""ctypes signatures for libngt_amd.so (include/ngt_amd.h and include/NGT/Capi.h)."""
from ctypes import (POINTER, Structure, c_bool, c_char_p, c_double, c_float, c_int, c_int16, c_int32,
                    c_int64, c_size_t, c_uint, c_uint8, c_uint32, c_uint64, c_void_p)


class SearchParams(Structure):
    _fields_ = [("k", c_uint32), ("epsilon", c_float), ("radius", c_float), ("edge_size", c_int64),
                ("seed_mode", c_int32), ("all_leaf_nodes", c_int32),
                ("visited_hash_log2", c_int32), ("distance_filter", c_int32)]


class QgSearchParams(Structure):
    _fields_ = [("k", c_uint32), ("epsilon", c_float), ("result_expansion", c_float), ("radius", c_float),
                ("seed_mode", c_int32), ("visited_hash_log2", c_int32)]


class NgtqSearchParams(Structure):
    _fields_ = [("size", c_uint32), ("expansion", c_float), ("epsilon", c_float), ("mode", c_int32)]


class BuildParams(Structure):
    _fields_ = [("edge_size_for_creation", c_int32), ("edge_size_for_search", c_int32),
                ("batch_size_for_creation", c_int32), ("seed_size", c_int32), ("epsilon_for_creation", c_float),
                ("reserved", c_int32)]


class NGTQGQuery(Structure):
    _fields_ = [("query", POINTER(c_float)), ("size", c_size_t), ("epsilon", c_float),
                ("result_expansion", c_float), ("radius", c_float)]


class NGTQGQuantizationParameters(Structure):
    _fields_ = [("dimension_of_subvector", c_float), ("max_number_of_edges", c_size_t)]


class ObjectDistance(Structure):
    _fields_ = [("id", c_uint), ("distance", c_float)]

    def __repr__(self):
        return "%d %g" % (self.id, self.distance)


class NGTQuery(Structure):
    _fields_ = [("query", POINTER(c_float)), ("size", c_size_t), ("epsilon", c_float),
                ("accuracy", c_float), ("radius", c_float), ("edge_size", c_size_t)]


def declare(L):
    vp = c_void_p
    u32p, u64p, f32p = POINTER(c_uint32), POINTER(c_uint64), POINTER(c_float)
    sig = {
        # ---- include/ngt_amd.h
        "ngt_amd_last_error": (c_char_p, []),
        "ngt_amd_device_count": (c_int, []),
        "ngt_amd_index_create": (c_int, [POINTER(vp), c_int, c_int, c_int, c_uint32]),
        "ngt_amd_index_destroy": (None, [vp]),
        "ngt_amd_index_padded_dimension": (c_uint32, [vp]),
        "ngt_amd_index_set_objects": (c_int, [vp, vp, c_uint64, vp]),
        "ngt_amd_index_set_objects_device": (c_int, [vp, vp, c_uint64]),
        "ngt_amd_index_set_graph": (c_int, [vp, vp, vp, c_uint64]),
        "ngt_amd_index_set_graph_device": (c_int, [vp, vp, vp, c_uint64]),
        "ngt_amd_index_set_tree": (c_int, [vp, vp, c_uint32, vp, vp, c_uint32, c_uint32, vp, c_uint32, vp,
                                           c_uint64]),
        "ngt_amd_index_set_search_property": (c_int, [vp, c_int32, c_int32, c_int32, c_int32, c_int32]),
        "ngt_amd_resolve_edge_size": (c_uint64, [vp, c_int64, c_float]),
        "ngt_amd_search": (c_int, [vp, POINTER(SearchParams), vp, c_uint32, vp, vp, vp, vp, vp, vp]),
        "ngt_amd_tree_seeds_device": (c_int, [vp, vp, c_uint64, c_uint32, c_uint32, vp, c_uint32, vp, vp]),
        "ngt_amd_search_served": (c_int, [vp, POINTER(SearchParams), vp, vp, vp, vp, vp]),
        "ngt_amd_serve_stop": (c_int, [vp]),
        "ngt_amd_serve_stats": (c_int, [vp, vp, vp]),
        "ngt_amd_last_search_lookahead": (c_int, [vp]),
        "ngt_amd_qg_train_local_ngt": (c_int, [vp, c_uint64, c_uint32, c_uint32, vp]),
        "ngt_amd_search_device": (c_int, [vp, POINTER(SearchParams), vp, c_uint64, c_uint32, vp, vp, vp, vp,
                                          vp, vp, vp]),
        "ngt_amd_linear_search": (c_int, [vp, vp, c_uint32, c_uint32, c_double, vp, vp, vp]),
        "ngt_amd_linear_search_device": (c_int, [vp, vp, c_uint64, c_uint32, c_uint32, c_double, vp, vp, vp,
                                                 vp]),
        "ngt_amd_distances": (c_int, [vp, vp, c_uint32, vp, vp, c_uint64, vp]),
        "ngt_amd_prepare_queries_device": (c_int, [vp, vp, c_uint32, vp, vp]),
        "ngt_amd_srand": (None, [c_uint]),
        "ngt_amd_last_search_kernel_ms": (c_float, [vp]),
        "ngt_amd_last_search_slots": (c_uint32, [vp]),
        "ngt_amd_stream_error_word": (c_int, [vp, vp, vp]),
        "ngt_amd_last_search_budget": (c_uint32, [vp]),
        "ngt_amd_last_search_filtered": (c_int, [vp]),
        "ngt_amd_build_begin": (c_int, [vp, POINTER(BuildParams)]),
        "ngt_amd_build_insert": (c_int, [vp, c_uint64, c_uint64]),
        "ngt_amd_build_graph_size": (c_int, [vp, u64p, u64p]),
        "ngt_amd_build_get_graph": (c_int, [vp, vp, vp, vp]),
        "ngt_amd_build_tree_size": (c_int, [vp, u32p, u32p, u64p]),
        "ngt_amd_build_get_tree": (c_int, [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
        "ngt_amd_build_set_graph": (c_int, [vp, vp, vp, vp, c_uint64]),
        "ngt_amd_build_set_tree": (c_int, [vp, vp, vp, vp, vp, vp, vp, c_uint32, vp, vp, vp, vp, c_uint32,
                                           c_uint32]),
        "ngt_amd_merge_results_device": (c_int, [c_int, vp, vp, vp, c_uint32, c_uint32, c_uint32, vp, vp, vp, vp,
                                                 vp]),
        "ngt_amd_pack_results_device": (c_int, [c_int, vp, vp, vp, c_uint32, c_uint32, vp, vp]),
        "ngt_amd_merge_packed_device": (c_int, [c_int, vp, c_uint32, c_uint32, c_uint32, vp, vp, vp, vp, vp]),
        "ngt_amd_shard_unique_id": (c_int, [vp, c_uint64]),
        "ngt_amd_shard_comm_create": (c_int, [vp, c_int, c_int, c_int, vp, c_uint64]),
        "ngt_amd_shard_comm_destroy": (c_int, [vp]),
        "ngt_amd_shard_comm_set_offsets": (c_int, [vp, vp]),
        "ngt_amd_shard_comm_synchronize": (c_int, [vp, vp]),
        "ngt_amd_sharded_search_device": (c_int, [vp, vp, vp, vp, c_uint64, c_uint32, vp, vp, vp, vp, vp, vp, vp]),
        "ngt_amd_sharded_qg_search_device": (c_int, [vp, vp, vp, vp, c_uint64, c_uint32, vp, vp, vp, vp, vp, vp,
                                                     vp]),
        "ngt_amd_qg_set_quantizer": (c_int, [vp, vp, vp, c_uint32, c_uint32]),
        "ngt_amd_qg_build_graph": (c_int, [vp, vp, c_uint32]),
        "ngt_amd_qg_encode": (c_int, [vp, vp]),
        "ngt_amd_qg_train": (c_int, [vp, c_uint32, c_uint32, c_uint32, vp, vp]),
        "ngt_amd_qg_set_graph": (c_int, [vp, vp, vp, vp, vp]),
        "ngt_amd_qg_max_degree": (c_uint32, [vp]),
        "ngt_amd_qg_code_stride": (c_uint64, [vp]),
        "ngt_amd_qg_record_bytes": (c_uint64, [vp]),
        "ngt_amd_qg_get_graph": (c_int, [vp, vp, vp]),
        "ngt_amd_qg_lut": (c_int, [vp, vp, c_uint32, vp, vp, vp]),
        "ngt_amd_qg_adc": (c_int, [vp, vp, vp, vp, c_uint32, vp, vp, c_uint64, vp, vp]),
        "ngt_amd_qg_search": (c_int, [vp, POINTER(QgSearchParams), vp, c_uint32, vp, vp, vp, vp, vp, vp]),
        "ngt_amd_qg_search_device": (c_int, [vp, POINTER(QgSearchParams), vp, c_uint64, c_uint32, vp, vp, vp,
                                             vp, vp, vp, vp]),
        "ngt_amd_ngtq_open": (c_int, [c_char_p, c_int, POINTER(vp)]),
        "ngt_amd_ngtq_set": (c_int, [vp, vp, c_uint32, c_uint32, vp, c_uint64, vp, vp, c_uint64, vp, c_uint64]),
        "ngt_amd_ngtq_search": (c_int, [vp, POINTER(NgtqSearchParams), vp, c_uint32, vp, vp, vp]),
        "ngt_amd_ngtq_search_device": (c_int, [vp, POINTER(NgtqSearchParams), vp, c_uint64, c_uint32, vp, vp, vp,
                                               vp]),
        # ---- include/NGT/Capi.h
        "ngt_open_index": (vp, [c_char_p, vp]),
        "ngt_create_graph_and_tree": (vp, [c_char_p, vp, vp]),
        "ngt_create_graph_and_tree_in_memory": (vp, [vp, vp]),
        "ngt_create_property": (vp, [vp]),
        "ngt_save_index": (c_bool, [vp, c_char_p, vp]),
        "ngt_get_property": (c_bool, [vp, vp, vp]),
        "ngt_get_property_dimension": (c_int32, [vp, vp]),
        "ngt_set_property_dimension": (c_bool, [vp, c_int32, vp]),
        "ngt_set_property_edge_size_for_creation": (c_bool, [vp, c_int16, vp]),
        "ngt_set_property_edge_size_for_search": (c_bool, [vp, c_int16, vp]),
        "ngt_get_property_object_type": (c_int32, [vp, vp]),
        "ngt_is_property_object_type_float": (c_bool, [c_int32]),
        "ngt_is_property_object_type_integer": (c_bool, [c_int32]),
        "ngt_set_property_object_type_float": (c_bool, [vp, vp]),
        "ngt_set_property_object_type_integer": (c_bool, [vp, vp]),
        "ngt_set_property_distance_type_l1": (c_bool, [vp, vp]),
        "ngt_set_property_distance_type_l2": (c_bool, [vp, vp]),
        "ngt_set_property_distance_type_angle": (c_bool, [vp, vp]),
        "ngt_set_property_distance_type_hamming": (c_bool, [vp, vp]),
        "ngt_set_property_distance_type_jaccard": (c_bool, [vp, vp]),
        "ngt_set_property_distance_type_cosine": (c_bool, [vp, vp]),
        "ngt_set_property_distance_type_normalized_angle": (c_bool, [vp, vp]),
        "ngt_set_property_distance_type_normalized_cosine": (c_bool, [vp, vp]),
        "ngt_set_property_distance_type_normalized_l2": (c_bool, [vp, vp]),
        "ngt_set_property_distance_type_sparse_jaccard": (c_bool, [vp, vp]),
        "ngt_create_empty_results": (vp, [vp]),
        "ngt_search_index": (c_bool, [vp, POINTER(c_double), c_int32, c_size_t, c_float, c_float, vp, vp]),
        "ngt_search_index_as_float": (c_bool, [vp, f32p, c_int32, c_size_t, c_float, c_float, vp, vp]),
        "ngt_search_index_with_query": (c_bool, [vp, NGTQuery, vp, vp]),
        "ngt_linear_search_index": (c_bool, [vp, POINTER(c_double), c_int32, c_size_t, vp, vp]),
        "ngt_linear_search_index_as_float": (c_bool, [vp, f32p, c_int32, c_size_t, vp, vp]),
        "ngt_linear_search_index_with_query": (c_bool, [vp, NGTQuery, vp, vp]),
        "ngt_get_size": (c_int32, [vp, vp]),
        "ngt_get_result_size": (c_uint32, [vp, vp]),
        "ngt_get_result": (ObjectDistance, [vp, c_uint32, vp]),
        "ngt_insert_index": (c_uint, [vp, POINTER(c_double), c_uint32, vp]),
        "ngt_append_index": (c_uint, [vp, POINTER(c_double), c_uint32, vp]),
        "ngt_insert_index_as_float": (c_uint, [vp, f32p, c_uint32, vp]),
        "ngt_append_index_as_float": (c_uint, [vp, f32p, c_uint32, vp]),
        "ngt_batch_append_index": (c_bool, [vp, f32p, c_uint32, vp]),
        "ngt_batch_insert_index": (c_bool, [vp, f32p, c_uint32, u32p, vp]),
        "ngt_create_index": (c_bool, [vp, c_uint32, vp]),
        "ngt_remove_index": (c_bool, [vp, c_uint, vp]),
        "ngt_get_object_space": (vp, [vp, vp]),
        "ngt_get_object_as_float": (f32p, [vp, c_uint, vp]),
        "ngt_get_object_as_integer": (POINTER(c_uint8), [vp, c_uint, vp]),
        "ngt_destroy_results": (None, [vp]),
        "ngt_destroy_property": (None, [vp]),
        "ngt_close_index": (None, [vp]),
        "ngt_get_property_edge_size_for_creation": (c_int16, [vp, vp]),
        "ngt_get_property_edge_size_for_search": (c_int16, [vp, vp]),
        "ngt_get_property_distance_type": (c_int32, [vp, vp]),
        "ngt_create_error_object": (vp, []),
        "ngt_get_error_string": (c_char_p, [vp]),
        "ngt_clear_error_string": (None, [vp]),
        "ngt_destroy_error_object": (None, [vp]),
        "ngt_get_edges": (c_bool, [vp, c_uint, vp, vp]),
        "ngt_get_object_repository_size": (c_uint32, [vp, vp]),
        "ngt_batch_search_index": (c_bool, [vp, f32p, c_uint32, c_int32, c_size_t, c_float, c_float, c_int64,
                                            u32p, f32p, u32p, vp]),
        "ngt_batch_search_index_using_only_graph": (c_bool, [vp, f32p, c_uint32, c_int32, c_size_t, c_float,
                                                             c_float, c_int64, u32p, f32p, u32p, vp]),
        "ngt_batch_linear_search_index": (c_bool, [vp, f32p, c_uint32, c_int32, c_size_t, u32p, f32p, u32p,
                                                   vp]),
        "ngt_batch_linear_search_index_with_radius": (c_bool, [vp, f32p, c_uint32, c_int32, c_size_t, c_float,
                                                               u32p, f32p, u32p, vp]),
        "ngt_get_last_search_counters": (c_bool, [vp, u64p, vp]),
        "ngt_get_coalesce_stats": (c_bool, [vp, u64p, u64p, vp]),
        "ngt_get_device_index": (vp, [vp, vp]),
        "ngt_set_property_value": (c_bool, [vp, c_char_p, c_char_p, vp]),
        "ngt_get_property_value": (c_int32, [vp, c_char_p, c_char_p, c_size_t, vp]),
        # ---- include/NGT/NGTQ/Capi.h
        "ngtqg_open_index": (vp, [c_char_p, vp]),
        "ngtqg_open_index_with_max_edges": (vp, [c_char_p, c_uint32, vp]),
        "ngtqg_close_index": (None, [vp]),
        "ngtqg_initialize_quantization_parameters": (None, [POINTER(NGTQGQuantizationParameters)]),
        "ngtqg_quantize": (c_bool, [c_char_p, NGTQGQuantizationParameters, vp]),
        "ngtqg_initialize_query": (None, [POINTER(NGTQGQuery)]),
        "ngtqg_search_index": (c_bool, [vp, NGTQGQuery, vp, vp]),
        "ngtqg_batch_search_index": (c_bool, [vp, f32p, c_uint32, c_int32, c_size_t, c_float, c_float, c_float,
                                              u32p, f32p, u32p, vp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
